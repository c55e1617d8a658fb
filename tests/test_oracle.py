"""The CPU oracle pinned against the reference's own known-answer tests and
the committed golden vectors (CPU only).

KATs restated from the reference (lminervino18/oxidized-neural-orchestra):
  f16 wire bytes       comms/src/sparse/protocol.rs:150-223, sparse/tests.rs:13-59
  BlockingShard        parameter_server/src/storage/blocking/shard.rs:132-185
  BlockingStore        parameter_server/src/storage/blocking/store.rs:156-243
  lineal convergence   parameter_server/src/test.rs:85-126 (asserts nothing there;
                       here: converges to the 1.0 fixed point)
"""
import numpy as np
import pytest

from conftest import SEED, assert_bitexact
from oracle import oracle as O
from oracle import oracle_np as N

IMPLS = {"c": O, "numpy": N}


# --------------------------------------------------------------- f16 KATs
@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_f16_reference_bytes(impl):
    # sparse/protocol.rs:158-167: 1.0 -> [0, 60], -1.0 -> [0, 188], 2.0 -> [0, 64] (LE)
    x = np.array([1.0, -1.0, 2.0], np.float32)
    h = O.f16_encode(x) if impl == "c" else N.f32_to_f16_bits(x)
    assert list(h.astype("<u2").view(np.uint8)) == [0, 60, 0, 188, 0, 64]


def test_grad_drop_kat():  # sparse/protocol.rs:150-170
    buf = O.grad_drop(np.array([1.0, -1.0, 0.0, 2.0], np.float32), 1.0)
    assert list(buf) == [4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188,
                         1, 0, 0, 0, 1, 0, 0, 0, 0, 64]


def test_grad_lift_kat():  # sparse/protocol.rs:172-190, :207-222
    buf = bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188,
                 1, 0, 0, 0, 1, 0, 0, 0, 0, 64])
    assert list(O.grad_lift(buf)) == [1.0, -1.0, 0.0, 2.0]
    short = bytes([3, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188])
    assert list(O.grad_lift(short)) == [0.0, 1.0, -1.0]


def test_sparse_gradient_kat():  # sparse/tests.rs:13-59: r = 0.4, 16 values -> 9..15 survive
    g = np.arange(16, dtype=np.float32)
    t = O.sparse_threshold(g, 0.4)
    assert t == 9.0
    out = O.grad_lift(O.grad_drop(g, t))
    assert list(out) == [0.0] * 9 + [9.0, 10.0, 11.0, 12.0, 13.0, 14.0, 15.0]


def test_frame_layout():  # msg.rs:136-149 + sink.rs:41-50: [u64 BE len][u32 BE kind][f16 LE]
    h = O.f16_encode(np.array([1.0, -1.0], np.float32))
    assert O.frame_dense(h) == bytes([0, 0, 0, 0, 0, 0, 0, 8, 0, 0, 0, 1, 0, 60, 0, 188])
    assert O.frame_dense(h, True)[8:12] == bytes([0, 0, 0, 2])


def test_f16_golden(golden):
    g = golden("f16")
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    assert_bitexact(O.f16_decode(h), g["decode_all_out"], "decode")
    assert np.array_equal(O.f16_encode(g["encode_in"]), g["encode_out"])
    assert np.array_equal(N.f32_to_f16_bits(g["encode_in"]), g["encode_out"])


def test_f16_rne_edges():
    enc = lambda v: int(O.f16_encode(np.array([v], np.float32))[0])  # noqa: E731
    assert enc(65504.0) == 0x7BFF
    assert enc(65519.99) == 0x7BFF           # below the halfway point to 2^16
    assert enc(65520.0) == 0x7C00            # tie rounds to even -> inf
    assert enc(2.0 ** -24) == 0x0001         # smallest subnormal
    assert enc(2.0 ** -25) == 0x0000         # tie -> even (zero)
    assert enc(3 * 2.0 ** -26) == 0x0001     # above the tie
    assert enc(1.0 + 2.0 ** -11) == 0x3C00   # tie between 1 and 1+2^-10 -> even
    assert enc(1.0 + 3 * 2.0 ** -11) == 0x3C02
    assert enc(float("-inf")) == 0xFC00
    nan = np.array([0x7F812345], np.uint32).view(np.float32)
    assert int(O.f16_encode(nan)[0]) == 0x7C00 | 0x0200 | (0x012345 >> 13)


# ----------------------------------------------------------- chunking
@pytest.mark.parametrize("length,n,expect", [
    (109386, 2, [54693, 54693]),
    (2 ** 26 + 5, 8, [8388609] * 5 + [8388608] * 3),
    (10, 3, [4, 3, 3]),
    (2, 3, [1, 1]),        # iterator stops on the empty slice: fewer chunks than ranks
    (0, 4, []),
])
def test_split_chunks(length, n, expect):
    for impl in (O, N):
        ch = impl.split_chunks(length, n)
        assert [b - a for a, b in ch] == expect


# --------------------------------------------------- ring vs golden
def _ring_cases(g):
    return sorted({k.rsplit("_", 1)[0] for k in g.files if k.endswith("_in")})


@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_ring_golden(golden, impl):
    g = golden("ring")
    for key in _ring_cases(g):
        wire = key.rsplit("_", 1)[1]
        ins = list(g[key + "_in"])
        grads, res = IMPLS[impl].ring_pull_grads(ins, wire)
        for r in range(len(ins)):
            assert_bitexact(grads[r], g[key + "_grad"][r], f"{impl} {key} rank {r}")
            assert not np.any(bits_nonzero(res[r])), "residual must be zeroed"


def bits_nonzero(a):
    return np.asarray(a, np.float32).view(np.uint32) != 0


def test_ring_semantics_f16():
    """Owner keeps f32 sum / n, replicas hold f16(sum) / n (worker_ring.rs:166 vs :200)."""
    n, length = 3, 999
    ins = [O.synth(length, SEED, r) for r in range(n)]
    grads, _ = O.ring_pull_grads(ins, "f16")
    chunks = O.split_chunks(length, n)
    for c, (lo, hi) in enumerate(chunks):
        owner = (c - 1) % n
        # chunk c summed in order c, c+1, ..., c+n-1 with f16 re-quantised partials
        p = ins[c][lo:hi].copy()
        for k in range(1, n):
            p = (ins[(c + k) % n][lo:hi] + N.quantize_f16(p)).astype(np.float32)
        assert_bitexact(grads[owner][lo:hi], p / np.float32(n), "owner")
        for r in range(n):
            if r != owner:
                assert_bitexact(grads[r][lo:hi], N.quantize_f16(p) / np.float32(n), "replica")


def test_ring_f32_wire_equals_sum_in_chunk_order():
    n, length = 4, 1001
    ins = [O.synth(length, SEED + 5, r) for r in range(n)]
    grads, _ = O.ring_pull_grads(ins, "f32")
    for c, (lo, hi) in enumerate(O.split_chunks(length, n)):
        order = [ins[(c + k) % n][lo:hi] for k in range(n)]
        expect = O.sum_scale(order, float(n))
        for r in range(n):
            assert_bitexact(grads[r][lo:hi], expect, f"chunk {c} rank {r}")


def test_ring_panics_like_reference():
    with pytest.raises(ValueError):
        O.ring_pull_grads([np.ones(2, np.float32)] * 3, "f16")


def test_ring_n1_is_copy():
    x = O.synth(100, SEED, 0)
    grads, res = O.ring_pull_grads([x], "f16")
    assert_bitexact(grads[0], x)  # no f16 rounding and no division for one worker
    assert not res[0].any()


def test_sum_scale_golden(golden):
    g = golden("sum_scale")
    for key in [k[:-3] for k in g.files if k.endswith("_in")]:
        d = float(key.split("_d")[1])
        assert_bitexact(O.sum_scale(list(g[key + "_in"]), d), g[key + "_out"], key)


# -------------------------------------------------------- CPU TCP ring
@pytest.mark.parametrize("n,length", [(1, 100), (2, 109386), (3, 4099), (4, 1001)])
def test_cpu_tcp_ring_matches_oracle(n, length):
    """The reference-style TCP loopback ring (the CPU baseline) is bit-exact
    with the in-memory restatement."""
    r = O.cpu_ring(n, length, 2, check=True, pin=False, timeout=120)
    assert r["check"] == 1


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,length", [(2, 5003), (3, 10007)])
def test_cpu_ring_single_worker_processes(n, length):
    """The single-worker mode (one process per rank, the peer the TCP-edge GPU
    tests mix into their rings) forms a ring with itself and is bit-exact."""
    p0 = free_port()
    ws = {}
    nxt = p0
    for r in range(n - 1, 0, -1):
        ws[r] = O.CpuRingWorker(r, n, length, nxt, rounds=2, seed=SEED + 3)
        nxt = ws[r].port
    ws[0] = O.CpuRingWorker(0, n, length, nxt, rounds=2, seed=SEED + 3, listen_port=p0)
    got = {r: w.result() for r, w in ws.items()}
    eg, er = O.ring_pull_grads([O.synth(length, SEED + 3, r) for r in range(n)], "f16")
    for r in range(n):
        assert_bitexact(got[r][0], eg[r], f"grad rank {r}")
        assert_bitexact(got[r][1], er[r], f"residual rank {r}")


# --------------------------------------------------------- store KATs
def _store(impl, params, shard, nworkers, kind="add", **hp):
    if impl == "c":
        return O.Store(params, shard, nworkers, kind, **hp)
    return N.BlockingStore(params, shard, nworkers, kind, **hp)


@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_shard_accumulation_and_update(impl):  # shard.rs:131-152
    s = _store(impl, np.zeros(3), 3, 1)
    s.accumulate([1.0, 2.0, 3.0])
    s.accumulate([1.0, 1.0, 1.0])
    s.update_params()
    assert list(s.pull_params()) == [2.0, 3.0, 4.0]


@pytest.mark.parametrize("impl", ["c", "numpy"])
def test_shard_gradient_is_averaged_across_workers(impl):  # shard.rs:170-185
    s = _store(impl, np.zeros(2), 2, 2)
    s.accumulate([2.0, 4.0])
    s.accumulate([2.0, 4.0])
    s.update_params()
    assert list(s.pull_params()) == [2.0, 4.0]


def test_store_handle_ragged_shards():  # store.rs:175-188
    s = O.Store(np.zeros(15), 8, 1, "add")
    assert s.nshards == 2
    s.accumulate(np.ones(15))
    s.update_params()
    assert list(s.pull_params()) == [1.0] * 15


def test_store_handle_buffer_swap():  # store.rs:190-207 (also shard.rs:154-168 double buffering)
    s = O.Store(np.zeros(10), 1, 1, "add")
    s.accumulate(np.ones(10))
    s.update_params()
    assert s.active_idx == 1
    s.accumulate(np.full(10, 5.0))
    assert list(s.pull_params()) == [1.0] * 10
    s.update_params()
    assert list(s.pull_params()) == [6.0] * 10


def test_store_update_locking_mechanism():  # store.rs:209-222
    s = O.Store(np.zeros(10), 1, 1, "add")
    s.set_updating(True)
    before = s.active_idx
    s.update_params()
    assert s.active_idx == before
    s.set_updating(False)
    s.update_params()
    assert s.active_idx != before


@pytest.mark.parametrize("params,shard", [(100, 25), (105, 10)])
def test_store_flow_and_ragged_edge(params, shard):  # store.rs:224-243
    s = O.Store(np.zeros(params), shard, 1, "add")
    s.accumulate(np.ones(params))
    s.update_params()
    out = s.pull_params()
    assert out.size == params and np.all(out == 1.0)


def test_store_size_mismatch():
    s = O.Store(np.zeros(4), 2, 1, "gd")
    with pytest.raises(ValueError):
        s.accumulate(np.ones(5))


def test_store_golden(golden):
    g = golden("store")
    for kind in ("gd", "momentum", "adam"):
        for nworkers in (1, 3):
            params = g[f"{kind}_w{nworkers}_init"]
            s = O.Store(params, 100, nworkers, kind, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
            for rnd in range(4):
                for w in range(nworkers):
                    s.accumulate(N.synth(1031, SEED + 1000 * rnd + w, w + 1))
                s.update_params()
                assert_bitexact(s.pull_params(), g[f"{kind}_w{nworkers}_traj"][rnd], f"{kind} w{nworkers} r{rnd}")


def test_lineal_convergence():
    """parameter_server/src/test.rs:85-126: 1 worker, BlockingStore, GD lr 0.1,
    params start at 0.5, worker sends grad = p - 1 on the f16 wire."""
    s = O.Store(np.full(2, 0.5, np.float32), 1, 1, "gd", lr=0.1)
    for _ in range(100):
        p = s.pull_params()
        g = N.quantize_f16((p - np.float32(1.0)).astype(np.float32))
        s.accumulate(g)
        s.update_params()
    assert np.all(np.abs(s.pull_params() - 1.0) < 1e-3)


def test_synth_generators_agree():
    for seed, rank, n, off in [(SEED, 0, 10000, 0), (1, 7, 4099, 123456789), (SEED, 3, 1031, 2 ** 33)]:
        assert_bitexact(O.synth(n, seed, rank, off), N.synth(n, seed, rank, off))
    x = O.synth(200000, SEED, 0)
    assert 0.005 < np.mean(x == 0) < 0.016
    assert np.all(np.abs(x) < 16)
