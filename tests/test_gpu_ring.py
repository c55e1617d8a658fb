"""GPU parity of the ring all-reduce (WorkerRingManager) against the oracle.

* The co-resident local ring executes the reference hop schedule on one
  device for n virtual ranks: bit-exact with the oracle for both wires.
* The RCCL ring at n = 1 (the only size a one-GPU box can host; n > 1 is
  exercised by bench.py's multi-GPU runs): pull_grads semantics on owned,
  external and host buffers.
* Full-size (256 MiB) properties: residual zeroed, replicas agree where the
  reference says they agree, values equal the oracle on a sample.
"""
import numpy as np
import pytest
import torch

import ono_amd
from conftest import SEED, assert_bitexact
from oracle import oracle as O
from oracle import oracle_np as N

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def run_local(ins, wire):
    res = [to_dev(x) for x in ins]
    grads = [torch.full_like(r, 7.0) for r in res]
    ono_amd.local_ring_pull_grads(res, grads, wire)
    return [host(g) for g in grads], [host(r) for r in res]


def test_local_ring_golden(golden):
    g = golden("ring")
    keys = sorted({k.rsplit("_", 1)[0] for k in g.files if k.endswith("_in")})
    for key in keys:
        wire = key.rsplit("_", 1)[1]
        ins = list(g[key + "_in"])
        grads, res = run_local(ins, wire)
        for r in range(len(ins)):
            assert_bitexact(grads[r], g[key + "_grad"][r], f"{key} rank {r}")
            assert not res[r].view(np.uint32).any()


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 16])
@pytest.mark.parametrize("length", [109386, 2 ** 18 + 5, 65536])
@pytest.mark.parametrize("wire", ["f16", "f32"])
def test_local_ring_vs_oracle(n, length, wire):
    ins = [O.synth(length, SEED + 11, r) for r in range(n)]
    grads, res = run_local(ins, wire)
    eg, _ = O.ring_pull_grads(ins, wire)
    for r in range(n):
        assert_bitexact(grads[r], eg[r], f"rank {r}")
        assert not res[r].view(np.uint32).any()


def test_local_ring_errors():
    with pytest.raises(ono_amd.SizeMismatch):
        run_local([np.ones(2, np.float32)] * 3, "f16")


@pytest.mark.parametrize("wire", ["f32", "f16"])
def test_ring_n1_owned_buckets(wire):
    size = 100003
    ring = ono_amd.WorkerRingManager(0, ["127.0.0.1:40000"], size, wire=wire)
    x = O.synth(size, SEED, 0)
    ring.residual.copy_(torch.from_numpy(x))
    pm = ring.pull_grads()
    assert_bitexact(host(pm.grad), x)           # n == 1: copy, no f16, no division
    assert not host(ring.residual).view(np.uint32).any()
    # the producer side: acc_residual
    g = to_dev(O.synth(size, SEED, 1))
    ring.acc_residual(g)
    ring.acc_residual(g)
    g1 = O.synth(size, SEED, 1)
    e = ((np.zeros(size, np.float32) + g1) + g1).astype(np.float32)  # residual starts at +0
    assert_bitexact(host(ring.residual), e)
    ring.close()


def test_ring_buckets_zero_at_creation_on_any_stream():
    """A ring's owned buckets are zero when ono_ring_create returns, as seen from a non-blocking stream the
    creation never touched (the fill runs on the ring's stream and is waited for).
    Rings come and go over memory the previous ones used (and dirtied: each round leaves its grad), and
    the first acc_residual on the new stream starts from +0."""
    size = (1 << 20) + 3
    s = torch.cuda.Stream()
    for k in range(6):
        ring = ono_amd.WorkerRingManager(0, 1, size)
        with torch.cuda.stream(s):
            res0, grad0 = ring.residual.clone(), ring.grad.clone()
        s.synchronize()
        assert not host(res0).view(np.uint32).any(), f"ring {k}: residual not zero at creation"
        assert not host(grad0).view(np.uint32).any(), f"ring {k}: grad not zero at creation"
        g = O.synth(size, SEED + k, 2)
        gd = to_dev(g)
        torch.cuda.synchronize()
        ring.acc_residual(gd, stream=s)
        pm = ring.pull_grads(stream=s)
        s.synchronize()
        assert_bitexact(host(pm.grad), (np.zeros(size, np.float32) + g).astype(np.float32))
        ring.close()


def test_ring_n1_dev_and_host_forms():
    size = 4099
    ring = ono_amd.WorkerRingManager(0, 1, size)
    x = O.synth(size, SEED, 5)
    res, grad = to_dev(x), torch.zeros(size, device=DEV)
    ring.pull_grads_dev(res, grad)
    assert_bitexact(host(grad), x)
    assert not host(res).any()
    hr, hg = x.copy(), np.zeros(size, np.float32)
    ring.pull_grads_host(hr, hg)
    assert_bitexact(hg, x)
    assert not hr.any()
    with pytest.raises(ono_amd.SizeMismatch):
        ring.pull_grads_dev(res[:10], grad[:10])
    buf = to_dev(x)
    ring.allreduce_avg_(buf)
    assert_bitexact(host(buf), x)
    ring.close()


def test_ring_timing_and_abort():
    size = 1 << 20
    ring = ono_amd.WorkerRingManager(0, 1, size)
    ring.timing(True)
    for _ in range(3):
        ring.pull_grads()
    t = ring.timing_read()
    assert t["kernels"] == 3 and t["kernel_ms"] > 0
    ring.abort()
    with pytest.raises(ono_amd.Aborted):
        ring.pull_grads()
    ring.close()


def test_full_size_256mib_local_ring_f32_n2():
    """BASELINE config 3 shape (256 MiB, n = 2) on one device: with two ranks
    the f32 reduction is a single commutative add, so every element equals
    (a + b) / 2 and both replicas are identical; residuals are zeroed."""
    n_el = 1 << 26
    a = torch.empty(n_el, dtype=torch.float32, device=DEV)
    b = torch.empty_like(a)
    ono_amd.kernels.synth(a, SEED, 0)
    ono_amd.kernels.synth(b, SEED, 1)
    expect = torch.empty_like(a)
    ono_amd.kernels.sum_scale(expect, [a, b], 2.0)
    ga, gb = torch.empty_like(a), torch.empty_like(a)
    ono_amd.local_ring_pull_grads([a, b], [ga, gb], "f32")
    torch.cuda.synchronize()
    assert torch.equal(ga.view(torch.int32), expect.view(torch.int32))
    assert torch.equal(gb.view(torch.int32), expect.view(torch.int32))
    assert int(torch.count_nonzero(a.view(torch.int32))) == 0
    assert int(torch.count_nonzero(b.view(torch.int32))) == 0
    # oracle spot check on a strided sample
    idx = np.arange(0, n_el, 65537)
    sa, sb = O.synth(n_el, SEED, 0)[idx], O.synth(n_el, SEED, 1)[idx]
    assert_bitexact(host(ga)[idx], O.sum_scale([sa, sb], 2.0))


def test_full_size_256mib_local_ring_f16_n8_properties():
    """256 MiB per rank, n = 8, f16 wire: every replica of chunk c equals
    f16(owner value * n) / n, the owner's chunk is the f32 chain, the
    residuals are zeroed, and a sample matches the oracle's chain."""
    n, n_el = 8, (1 << 26) + 5
    res = [torch.empty(n_el, dtype=torch.float32, device=DEV) for _ in range(n)]
    for r, t in enumerate(res):
        ono_amd.kernels.synth(t, SEED, r)
    grads = [torch.empty_like(res[0]) for _ in range(n)]
    ono_amd.local_ring_pull_grads(res, grads, "f16")
    torch.cuda.synchronize()
    for t in res:
        assert int(torch.count_nonzero(t.view(torch.int32))) == 0
    chunks = O.split_chunks(n_el, n)
    for c, (lo, hi) in enumerate(chunks[:3]):
        owner = (c - 1) % n
        sl = slice(lo, lo + 4096)
        ins = [O.synth(4096, SEED, r, lo) for r in range(n)]
        p = ins[c].copy()
        for k in range(1, n):
            p = (ins[(c + k) % n] + N.quantize_f16(p)).astype(np.float32)
        assert_bitexact(host(grads[owner][sl]), p / np.float32(n), f"owner chunk {c}")
        rep = N.quantize_f16(p) / np.float32(n)
        for r in range(n):
            if r != owner:
                assert_bitexact(host(grads[r][sl]), rep, f"replica {r} chunk {c}")
    del res, grads
    torch.cuda.empty_cache()


def test_unique_id_roundtrip():
    uid = ono_amd.unique_id()
    assert isinstance(uid, bytes) and len(uid) == 128


@pytest.mark.parametrize("register", [False, True])
@pytest.mark.parametrize("size", [4099, (5 << 20) + 3, (12 << 20) + 7])
def test_host_fed_pipeline(register, size):
    """ono_ring_pull_grads_host: chunked H2D -> reduce -> D2H (16 MiB chunks,
    ragged last chunk), registered in-place DMA and pinned bounce slots."""
    ring = ono_amd.WorkerRingManager(0, 1, size)
    x = O.synth(size, SEED, 7)
    res, grad = x.copy(), np.full(size, 3.0, np.float32)
    if register:
        ring.register_host(res)
        ring.register_host(grad)
    for _ in range(2):
        res[:] = x
        ring.pull_grads_host(res, grad)
        assert_bitexact(grad, x)
        assert not res.view(np.uint32).any()
    if register:
        ring.unregister_host(res)
        ring.unregister_host(grad)
        with pytest.raises(ono_amd.InvalidArgument):
            ring.unregister_host(res)
    ring.close()


def run_local_direct(ins, wire):
    res = [to_dev(x) for x in ins]
    grads = [torch.full_like(r, 7.0) for r in res]
    ono_amd.local_ring_pull_grads(res, grads, wire, algo="direct")
    return [host(g) for g in grads], [host(r) for r in res]


def test_local_direct_golden(golden):
    """The direct schedule's fused owner kernel (all-to-all order, one pass)
    reproduces the reference hop ring bit for bit on every golden case."""
    g = golden("ring")
    keys = sorted({k.rsplit("_", 1)[0] for k in g.files if k.endswith("_in")})
    for key in keys:
        wire = key.rsplit("_", 1)[1]
        ins = list(g[key + "_in"])
        grads, res = run_local_direct(ins, wire)
        for r in range(len(ins)):
            assert_bitexact(grads[r], g[key + "_grad"][r], f"{key} rank {r}")
            assert not res[r].view(np.uint32).any()


@pytest.mark.parametrize("n", [2, 3, 5, 8, 16])
@pytest.mark.parametrize("length", [109386, 2 ** 18 + 5])
@pytest.mark.parametrize("wire", ["f16", "f32"])
def test_local_direct_vs_oracle(n, length, wire):
    ins = [O.synth(length, SEED + 13, r) for r in range(n)]
    grads, res = run_local_direct(ins, wire)
    eg, _ = O.ring_pull_grads(ins, wire)
    for r in range(n):
        assert_bitexact(grads[r], eg[r], f"rank {r}")
        assert not res[r].view(np.uint32).any()


def test_local_direct_full_size_f16_n8_equals_hops():
    """256 MiB per rank, n = 8, ragged: direct == hop schedule bit for bit."""
    n, n_el = 8, (1 << 26) + 5
    outs = {}
    for algo in ("hops", "direct"):
        res = [torch.empty(n_el, dtype=torch.float32, device=DEV) for _ in range(n)]
        for r, t in enumerate(res):
            ono_amd.kernels.synth(t, SEED, r)
        grads = [torch.empty_like(res[0]) for _ in range(n)]
        ono_amd.local_ring_pull_grads(res, grads, "f16", algo=algo)
        torch.cuda.synchronize()
        for t in res:
            assert int(torch.count_nonzero(t.view(torch.int32))) == 0
        outs[algo] = grads
        del res
    for r in range(n):
        assert torch.equal(outs["hops"][r].view(torch.int32), outs["direct"][r].view(torch.int32)), r
    del outs
    torch.cuda.empty_cache()


def test_full_size_1gib_local_direct_f32_n8():
    """BASELINE config 4 shape: 1 GiB bucket per rank, n = 8 (16 GiB in HBM).
    Size-independent property: every rank's chunk c equals sum_scale of the
    n slices taken in the reference order c, c+1, ..., c+7, divided by 8;
    residuals are zeroed; a strided sample matches the oracle."""
    n, n_el = 8, 1 << 28
    res = [torch.empty(n_el, dtype=torch.float32, device=DEV) for _ in range(n)]
    for r, t in enumerate(res):
        ono_amd.kernels.synth(t, SEED + 5, r)
    chunks = O.split_chunks(n_el, n)
    expect = torch.empty(n_el, dtype=torch.float32, device=DEV)
    for c, (lo, hi) in enumerate(chunks):
        ono_amd.kernels.sum_scale(expect[lo:hi], [res[(c + k) % n][lo:hi] for k in range(n)], float(n))
    grads = [torch.empty_like(res[0]) for _ in range(n)]
    ono_amd.local_ring_pull_grads(res, grads, "f32", algo="direct")
    torch.cuda.synchronize()
    for r in range(n):
        assert torch.equal(grads[r].view(torch.int32), expect.view(torch.int32)), r
        assert int(torch.count_nonzero(res[r].view(torch.int32))) == 0
    idx = np.arange(0, n_el, 1 << 20)
    hs = [np.array([O.synth(1, SEED + 5, r, int(i))[0] for i in idx], np.float32) for r in range(n)]
    ge = host(grads[3])[idx]
    for j, i in enumerate(idx):
        c = next(k for k, (lo, hi) in enumerate(chunks) if lo <= i < hi)
        assert_bitexact(ge[j:j + 1], O.sum_scale([hs[(c + k) % n][j:j + 1] for k in range(n)], float(n)))
    del res, grads, expect
    torch.cuda.empty_cache()


@pytest.mark.parametrize("algo", ["allreduce", "hops", "direct"])
def test_ring_set_algo_n1(algo):
    ring = ono_amd.WorkerRingManager(0, 1, 1000, algo=algo)
    x = O.synth(1000, SEED, 3)
    ring.residual.copy_(torch.from_numpy(x))
    ring.pull_grads()
    assert_bitexact(host(ring.grad), x)
    ring.close()
    f16ring = ono_amd.WorkerRingManager(0, 1, 1000, wire="f16")
    with pytest.raises(ono_amd.InvalidArgument):
        f16ring.set_algo("allreduce")
    f16ring.close()


@pytest.mark.parametrize("segments", [1, 2, 4, 7])
def test_allreduce_pipeline_segments_n1(segments):
    """The segmented f32 all-reduce schedule (finaliser of segment j on a side
    stream, overlapping the all-reduce of segment j+1) through a real one-rank
    RCCL communicator: every round's grad is its own residual, bit for bit, and
    every residual ends zeroed — a finaliser that ran ahead of its all-reduce
    would leave zeros or a stale round in grad."""
    length = (1 << 25) + 37
    ring = ono_amd.WorkerRingManager(0, 1, length, algo="allreduce")
    ring.set_pipeline(segments)
    s = torch.cuda.Stream()
    grad = torch.full((length,), 7.0, device=DEV)
    xs = [to_dev(O.synth(length, SEED + 40 + k, 0)) for k in range(3)]
    res = [x.clone() for x in xs]
    try:
        with torch.cuda.stream(s):
            for k in range(3):
                ring.pull_grads_dev(res[k], grad, s)
                out = grad.clone()
                torch.cuda.current_stream().synchronize()
                assert torch.equal(out.view(torch.int32), xs[k].view(torch.int32)), f"round {k}"
                assert not res[k].view(torch.int32).any()
    finally:
        ring.close()


@pytest.mark.parametrize("algo", ["hops", "direct"])
@pytest.mark.parametrize("wire", ["f16", "f32"])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_local_ring_special_values(n, wire, algo):
    """NaN (with payloads), +-inf, -0, f16 overflow/underflow and f32 overflow
    through the whole round: bit-exact with the oracle wherever the oracle is
    not NaN, NaN exactly where the oracle is NaN (payload propagation through
    a + b is compiler-dependent in the reference itself)."""
    length = 100003
    ins = [O.synth_special(length, SEED + 17, r) for r in range(n)]
    eg, _ = O.ring_pull_grads(ins, wire)
    res = [to_dev(x) for x in ins]
    grads = [torch.full_like(r, 7.0) for r in res]
    ono_amd.local_ring_pull_grads(res, grads, wire, algo=algo)
    for r in range(n):
        got = host(grads[r])
        ok = O.same_or_both_nan(got, eg[r])
        assert ok.all(), f"rank {r}: {np.count_nonzero(~ok)} differ, first at {np.flatnonzero(~ok)[0]}"
        assert np.isnan(eg[r]).any() and np.isinf(eg[r]).any()  # the specials did reach the output
        assert not host(res[r]).view(np.uint32).any()
