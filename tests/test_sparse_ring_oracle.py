"""The sparse ring mode on the CPU: oracle restatements, stand-in sampler and
the reference-style CPU ring workers (no GPU).

Reference behaviour (read from the reference for round 3; restated twice, in
C — oracle/ono_oracle.c ono_ref_ring_pull_grads_sparse — and independently in
numpy — oracle/oracle_np.py ring_pull_grads_sparse, written line by line from
worker_ring.rs:112-204 and compressor.rs:71-98):
  * SparseCapable{r}'s push computes t = calculate_threshold(chunk, r) and the
    grad_drop stream of the values with |g| >= t (comms/src/sparse/protocol.rs:
    33-86); the stream goes out as a SparseGrad only when it is no longer than
    the chunk's f16 payload, 2 bytes per value (compressor.rs:79); otherwise the
    push is a DenseGrad of f16(chunk) (:84-89) and push_grad returns None
    (handles/worker.rs:157-174);
  * after a SparseGrad the scatter zeroes only the sent values
    (worker_ring.rs:126-132) and the gather keeps only the sent values in grad
    while the owned residual chunk is left as it is (:177-190; the reset at
    :178-184 is commented out); after a DenseGrad the scatter zeroes the chunk
    (:133) and the gather zeroes the owned residual at j == 0 (:191-193);
  * a receiver lifts a SparseGrad into a zero-filled buffer, then adds
    (scatter) or copies (gather) it (comms/src/handles/worker.rs:102-108).
Parity status: the threshold, codec and frames are pinned by the reference's
KATs (protocol.rs:150-223, sparse/tests.rs:13-59); the sparse ring's
composition has no reference test (parity unpinned, like the dense ring), and
above 16384 values the sample comes from a stand-in sampler, not rand 0.9.4.
Round 2's restatement missed the dense fallback and reset the owned residual
after a sparse push; both restatements here were rewritten from the reference
text and agree bit for bit.
"""
import numpy as np
import pytest

import ono_amd
from conftest import SEED, assert_bitexact
from oracle import oracle as O
from oracle import oracle_np as N


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


@pytest.mark.parametrize("r,kind", [(0.1, 3), (0.3, 1), (0.4, 1), (0.6, 1), (0.9, 1), (1.0, 1)])
def test_push_kind_on_the_synthetic_distribution(r, kind):
    """The config-1 chunk (54,693 values of the §8(d) distribution): only r = 0.1
    keeps the stream under 2 bytes per value; every larger ratio goes out as a
    DenseGrad (compressor.rs:79-89).  Both restatements agree."""
    x = O.synth(109386, SEED, 0)[:54693]
    sparse, t, _ = O.sparse_push(x, r, 0)
    _, sent, _, k = N.push_grad(x, r, 0)
    assert k == kind and sparse == (kind == 3)
    assert (sent is None) == (kind == 1)
    drop = O.grad_drop(x, t)
    assert (len(drop) <= 2 * x.size) == (kind == 3)
    assert drop == N.grad_drop(x, t)


def test_push_kat_alternating_goes_dense():
    """A hand-built chunk whose every other value reaches the threshold: each
    kept value costs a 10-byte run (8 B header + 2 B), 8 + 5 L bytes > 2 L, so
    the SparseCapable push is a DenseGrad of f16(chunk); with the runs joined
    (a kept block) the same values fit and go sparse."""
    L = 64
    alt = np.where(np.arange(L) % 2 == 0, 1.0, 0.25).astype(np.float32)
    # r = 0.5: k = 32 -> the 33rd smallest |g| = 1.0 is the threshold
    assert O.sparse_threshold(alt, 0.5) == 1.0
    assert len(O.grad_drop(alt, 1.0)) == 8 + 32 * 10 > 2 * L
    sparse, t, _ = O.sparse_push(alt, 0.5, 0)
    assert not sparse and t == 1.0
    block = np.sort(alt)[::-1].copy()  # 32 x 1.0 then 32 x 0.25: one run
    assert len(O.grad_drop(block, 1.0)) == 8 + 8 + 64 <= 2 * L
    sparse, t, _ = O.sparse_push(block, 0.5, 0)
    assert sparse and t == 1.0
    # the ring: rank 0's first push of the alternating chunk is dense, so the
    # chunk is zeroed whole (worker_ring.rs:133), unlike a sparse push
    x = [np.concatenate([alt, alt]), np.concatenate([block, block])]
    g, res, _ = O.ring_pull_grads_sparse(x, [0.5, 0.5], [0, 0])
    g2, res2, _ = N.ring_pull_grads_sparse(x, [0.5, 0.5], [0, 0])
    for r in range(2):
        assert_bitexact(g[r], g2[r], f"grad {r}")
        assert_bitexact(res[r], res2[r], f"residual {r}")
    assert not res[0][:L].any(), "a DenseGrad push zeroes the whole chunk"
    assert res[1][L:].any(), "a SparseGrad push leaves the unsent values"


@pytest.mark.parametrize("n,length,ratios", [(2, 109386, [0.1, 0.1]), (2, 109386, [0.3, 0.9]),
                                             (2, 20000, [0.4, 0.4]), (3, 40000, [0.25, 0.0, 0.9]),
                                             (4, 4099, [1.0, 0.5, 0.5, 0.1]), (4, 70001, [0.0, 0.3, 0.0, 1.0]),
                                             (5, 4099, [0.5, 0.0, 0.0, 0.2, 0.7]), (3, 60000, [0.05, 0.1, 0.15])])
def test_sparse_ring_c_equals_numpy(n, length, ratios):
    """The C restatement and the independent numpy one (written from the
    reference text) agree bit for bit on grads, residuals and sampler states."""
    seeds = [7 * r + 1 for r in range(n)]
    x = [O.synth(length, SEED + 5, r) for r in range(n)]
    g, res, st = O.ring_pull_grads_sparse(x, ratios, seeds)
    g2, res2, st2 = N.ring_pull_grads_sparse(x, ratios, seeds)
    for r in range(n):
        assert_bitexact(g[r], g2[r], f"grad {r}")
        assert_bitexact(res[r], res2[r], f"residual {r}")
    assert st == st2


@pytest.mark.parametrize("n,length,ratios", [(2, 20000, [0.1, 0.1]), (3, 40000, [0.05, 0.0, 0.1]),
                                             (4, 4099, [1.0, 0.5, 0.5, 0.1]), (2, 20000, [0.4, 0.4])])
def test_sparse_ring_semantics(n, length, ratios):
    """Properties of the round that hold whatever the sample: after a sparse
    gather push the owned residual chunk still holds the reduced sum (it is not
    reset); after a dense one it is zero; a sparse scatter push leaves exactly
    the unsent values; a Base worker ends with a zero residual."""
    x = [O.synth(length, SEED + 5, r) for r in range(n)]
    g, res, _ = O.ring_pull_grads_sparse(x, ratios, list(range(n)))
    chunks = O.split_chunks(length, n)
    st = list(range(n))
    for r in range(n):
        own = (r + 1) % n
        a, b = chunks[own]
        if ratios[r] == 0.0:
            assert not res[r].any(), "Base serializer: every sent chunk is zeroed"
            continue
        # the scatter's first push is the rank's own-index chunk, unchanged
        sl = slice(*chunks[r])
        first_sparse, _, _ = O.sparse_push(x[r][sl], ratios[r], st[r])
        if first_sparse:
            tiny = np.abs(x[r]) < np.float32(6.103515625e-05)
            assert_bitexact(res[r][sl][tiny[sl]], x[r][sl][tiny[sl]], "sub-f16 values stay in the residual")
            kept = res[r][sl] != 0
            assert_bitexact(res[r][sl][kept], x[r][sl][kept], "unsent values stay as they were")
        else:
            assert not res[r][sl].any(), "a dense push zeroes the chunk"
        # the owner's chunk: grad = sum / n (f32) before the gather's mask; the
        # residual keeps the sum after a sparse push, zero after a dense one
        owned_sum = res[r][a:b]
        if owned_sum.any():
            kept = g[r][a:b] != 0
            assert_bitexact(g[r][a:b][kept], (owned_sum / np.float32(n)).astype(np.float32)[kept],
                            "the owner's kept values are the residual's sum / n")


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
