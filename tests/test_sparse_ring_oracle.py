"""The sparse ring mode on the CPU: oracle restatement, stand-in sampler and
the reference-style CPU ring workers (no GPU).

Reference behaviour restated (see oracle/ono_oracle.c ono_ref_ring_pull_grads_sparse):
  * SparseCapable{r} pushes a SparseGrad of the chunk's values with
    |g| >= calculate_threshold(chunk, r) (comms/src/sparse/protocol.rs:33-86,
    compressor.rs:71-98);
  * scatter zeroes only the sent values (worker_ring.rs:126-133); gather keeps
    only the sent values in grad (:177-193);
  * a receiver lifts a SparseGrad into a zero-filled buffer, then adds
    (scatter) or copies (gather) it (comms/src/handles/worker.rs:102-108).
Parity status: the threshold, codec and frames are pinned by the reference's
KATs (protocol.rs:150-223, sparse/tests.rs:13-59); the sparse ring's
composition has no reference test (parity unpinned, like the dense ring), and
above 16384 values the sample comes from a stand-in sampler, not rand 0.9.4.
"""
import numpy as np
import pytest

import ono_amd
from conftest import SEED, assert_bitexact
from oracle import oracle as O


def test_threshold_sample_matches_full_and_kat():
    g = np.arange(16, dtype=np.float32)  # sparse/tests.rs:13-59: r = 0.4 -> 9..15 survive
    assert O.sparse_threshold_sample(g, 0.4) == 9.0
    x = O.synth(12000, SEED, 1)
    for r in (0.1, 0.4, 0.9, 1.0):
        full = O.sparse_threshold(x, r)
        assert O.sparse_threshold_sample(x, r) == full
        perm = np.random.default_rng(3).permutation(x.size).astype(np.uint32)
        assert O.sparse_threshold_sample(x, r, perm) == full  # the sample's order is irrelevant


def test_threshold_floor_and_nan():
    # f32::max with f16::MIN_POSITIVE: tiny and NaN order statistics give the floor
    assert O.sparse_threshold_sample(np.full(100, 1e-9, np.float32), 0.5) == np.float32(6.103515625e-05)
    x = np.full(10, np.nan, np.float32)
    assert O.sparse_threshold_sample(x, 0.5) == np.float32(6.103515625e-05)


@pytest.mark.parametrize("length,amount,state", [(20000, 16384, 5), (1 << 20, 16384, 123), (16384, 16384, 7),
                                                 (16385, 16384, 9), (100, 100, 1)])
def test_default_sampler_product_equals_oracle(length, amount, state):
    """ono_sparse_sample_default (host code of the product) and the oracle's
    independent restatement draw the same indices and advance the same state."""
    a, sa = O.sample_default(state, length, amount)
    b, sb = ono_amd.sparse.sample_default(state, length, amount)
    assert np.array_equal(a, b) and sa == sb
    assert len(set(a.tolist())) == amount and int(a.max()) < length
    if amount == length:
        assert sa == state and np.array_equal(a, np.arange(length, dtype=np.uint32))  # no draws


@pytest.mark.parametrize("n,length", [(1, 500), (2, 109386), (3, 4099), (5, 70001)])
def test_sparse_ring_all_base_is_the_dense_ring(n, length):
    x = [O.synth(length, SEED + 2, r) for r in range(n)]
    g, res, st = O.ring_pull_grads_sparse(x, [0.0] * n, [11] * n)
    eg, er = O.ring_pull_grads(x, "f16")
    for r in range(n):
        assert_bitexact(g[r], eg[r], f"grad {r}")
        assert_bitexact(res[r], er[r], f"residual {r}")
    assert st == [11] * n


@pytest.mark.parametrize("n,length,ratios", [(2, 20000, [0.4, 0.4]), (3, 40000, [0.25, 0.0, 0.9]),
                                             (4, 4099, [1.0, 0.5, 0.5, 0.1])])
def test_sparse_ring_semantics(n, length, ratios):
    """Properties of the restated sparse round that hold whatever the sample:
    a sparse worker's residual keeps exactly what it did not send, values
    below f16::MIN_POSITIVE are never sent, every replica of a chunk holds
    values that are f16-exact (after the ÷n) or the owner's f32, and a worker
    whose serializer is Base zeroes what it sent."""
    x = [O.synth(length, SEED + 5, r) for r in range(n)]
    g, res, _ = O.ring_pull_grads_sparse(x, ratios, list(range(n)))
    chunks = O.split_chunks(length, n)
    for r in range(n):
        own = (r + 1) % n
        a, b = chunks[own]
        assert not res[r][a:b].any(), "the owned chunk's residual is reset at gather j = 0"
        if ratios[r] == 0.0:
            assert not res[r].any(), "Base serializer: every sent chunk is zeroed"
        else:
            tiny = np.abs(x[r]) < np.float32(6.103515625e-05)
            sent_chunk = chunks[r]  # scatter step 0 sends the rank's own-index chunk unchanged
            sl = slice(*sent_chunk)
            assert_bitexact(res[r][sl][tiny[sl]], x[r][sl][tiny[sl]], "sub-f16 values stay in the residual")
            kept = res[r][sl] != 0
            assert_bitexact(res[r][sl][kept], x[r][sl][kept], "unsent values stay as they were")


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,length,ratios", [(2, 40000, [0.4, 0.4]), (3, 10007, [0.25, 0.0, 0.6]),
                                             (4, 70001, [0.0, 0.3, 0.0, 1.0])])
def test_cpu_ring_workers_sparse_match_oracle(n, length, ratios):
    """Reference-style CPU workers (one process per rank) with sparse and dense
    serializers in one loopback ring, two rounds (the samplers' streams carry
    over): bit-exact with the in-memory restatement.  These are the peers the
    GPU tests mix MI355X workers with."""
    seeds = [1000 + r for r in range(n)]
    p0 = free_port()
    ws = {}
    nxt = p0
    for r in range(n - 1, -1, -1):
        ws[r] = O.CpuRingWorker(r, n, length, nxt, rounds=2, seed=SEED + 9, sparse=ratios[r], sparse_seed=seeds[r],
                                listen_port=p0 if r == 0 else 0)
        nxt = ws[r].port
    got = {r: w.result() for r, w in ws.items()}
    x = [O.synth(length, SEED + 9, r) for r in range(n)]
    _, _, st = O.ring_pull_grads_sparse(x, ratios, seeds)  # round 1 advances the samplers
    eg, er, _ = O.ring_pull_grads_sparse(x, ratios, st)
    for r in range(n):
        assert_bitexact(got[r][0], eg[r], f"grad rank {r}")
        assert_bitexact(got[r][1], er[r], f"residual rank {r}")
