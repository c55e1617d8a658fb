"""GPU parity of the elementwise kernels (through the C ABI) against the CPU
oracle: bit-exact (0 ulp) for every op, including misaligned chunk starts,
ragged lengths, f16 subnormals/ties/overflow/NaN, and every divisor class."""
import numpy as np
import pytest
import torch

import ono_amd
from ono_amd import kernels as K
from conftest import SEED, assert_bitexact
from oracle import oracle as O
from oracle import oracle_np as N

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

LENGTHS = [0, 1, 2, 3, 4, 5, 7, 63, 64, 65, 1023, 4099, 1 << 16, (1 << 20) + 3]
OFFSETS = [0, 1, 2, 3]


def dev(a: np.ndarray, offset: int = 0) -> torch.Tensor:
    """Copy a host array to the device at an element offset (misaligned start)."""
    t = torch.empty(a.size + offset + 4, dtype=torch.float32 if a.dtype == np.float32 else torch.int16,
                    device=DEV)
    v = t[offset:offset + a.size]
    v.copy_(torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a))
    return v


def host(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    a = t.cpu().numpy()
    return a.view(np.uint16) if a.dtype == np.int16 else a


def test_device_present():
    assert torch.cuda.is_available()
    assert "gfx950" in torch.cuda.get_device_properties(0).gcnArchName


@pytest.mark.parametrize("n", LENGTHS)
@pytest.mark.parametrize("k", [1, 2, 3, 4, 8, 16])
def test_sum_scale(n, k):
    ins = [O.synth(n, SEED + 3, r) for r in range(k)]
    for d in (1.0, float(k), 3.0, 7.0, 0.5):
        off = (n + k) % 4
        dins = [dev(x, off) for x in ins]
        out = dev(np.zeros(n, np.float32), off)
        K.sum_scale(out, dins, d)
        assert_bitexact(host(out), O.sum_scale(ins, d), f"n={n} k={k} d={d}")


def test_sum_scale_mixed_phases_falls_back_exactly():
    n = 4099
    ins = [O.synth(n, SEED, r) for r in range(3)]
    dins = [dev(x, o) for x, o in zip(ins, (0, 1, 3))]
    out = dev(np.zeros(n, np.float32), 2)
    K.sum_scale(out, dins, 3.0)
    assert_bitexact(host(out), O.sum_scale(ins, 3.0))


def test_sum_scale_golden(golden):
    g = golden("sum_scale")
    for key in [k[:-3] for k in g.files if k.endswith("_in")]:
        d = float(key.split("_d")[1])
        ins = [np.ascontiguousarray(x) for x in g[key + "_in"]]
        out = dev(np.zeros(ins[0].size, np.float32))
        K.sum_scale(out, [dev(x) for x in ins], d)
        assert_bitexact(host(out), g[key + "_out"], key)


def test_sum_scale_inplace_alias():
    n = 100003
    a, b = O.synth(n, SEED, 0), O.synth(n, SEED, 1)
    da, db = dev(a), dev(b)
    K.sum_scale(da, [da, db], 2.0)
    assert_bitexact(host(da), O.sum_scale([a, b], 2.0))


@pytest.mark.parametrize("n", LENGTHS)
@pytest.mark.parametrize("off", OFFSETS)
def test_acc_and_scale_zero(n, off):
    a, b = O.synth(n, SEED, 0), O.synth(n, SEED, 1)
    da, db = dev(a, off), dev(b, off)
    K.acc(da, db)
    ref = a.copy()
    O.lib().ono_ref_acc_residual(O._f(ref), O._f(b), n)
    assert_bitexact(host(da), ref)
    for d in (1.0, 2.0, 8.0, 3.0, 5.0):
        src, dst = dev(a, off), dev(np.zeros(n, np.float32), off)
        K.scale_zero(dst, src, d, src)
        assert_bitexact(host(dst), a / np.float32(d) if d != 1.0 else a)
        assert not host(src).view(np.uint32).any()


def test_f16_decode_exhaustive(golden):
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    out = dev(np.zeros(h.size, np.float32))
    K.f16_decode(out, dev(h))
    assert_bitexact(host(out), golden("f16")["decode_all_out"], "all 65536 f16 patterns")


def test_f16_encode_golden(golden):
    g = golden("f16")
    x = np.ascontiguousarray(g["encode_in"])
    out = dev(np.zeros(x.size, np.uint16))
    K.f16_encode(out, dev(x))
    assert np.array_equal(host(out), g["encode_out"])


def test_f16_encode_exhaustive():
    """Every one of the 2^32 f32 bit patterns (the device generates the
    patterns; the C oracle converts each chunk on the host)."""
    chunk = 1 << 28
    for start in range(0, 1 << 32, chunk):
        pat = torch.arange(start, start + chunk, dtype=torch.int64, device=DEV).to(torch.int32)
        x = pat.view(torch.float32)
        out = torch.empty(chunk, dtype=torch.int16, device=DEV)
        K.f16_encode(out, x)
        got = host(out)
        ref = O.f16_encode(np.arange(start, start + chunk, dtype=np.uint64).astype(np.uint32).view(np.float32))
        bad = np.flatnonzero(got != ref)
        assert bad.size == 0, f"pattern 0x{start + bad[0]:08x}: 0x{got[bad[0]]:04x} vs 0x{ref[bad[0]]:04x}"
        del pat, x, out


@pytest.mark.parametrize("n", LENGTHS)
@pytest.mark.parametrize("off", [0, 1, 3])
def test_hop_kernels(n, off):
    """encode_zero / decode_add / add_encode_zero / decode_scale vs oracle."""
    a = O.synth(n, SEED, 0)
    h = O.f16_encode(O.synth(n, SEED, 1))
    # encode_zero
    da, dh = dev(a, off), dev(np.zeros(n, np.uint16), off)
    K.f16_encode_zero(dh, da)
    assert np.array_equal(host(dh), O.f16_encode(a))
    assert not host(da).view(np.uint32).any()
    # decode_add
    da = dev(a, off)
    K.f16_decode_add(da, dev(h, off))
    ref = (a + O.f16_decode(h)).astype(np.float32)
    assert_bitexact(host(da), ref)
    # add_encode_zero
    da, dout = dev(a, off), dev(np.zeros(n, np.uint16), off)
    K.f16_add_encode_zero(dout, da, dev(h, off))
    assert np.array_equal(host(dout), O.f16_encode(ref))
    assert not host(da).view(np.uint32).any()
    # decode_scale
    for d in (1.0, 2.0, 3.0, 8.0):
        dout = dev(np.zeros(n, np.float32), off)
        K.f16_decode_scale(dout, dev(h, off), d)
        e = O.f16_decode(h)
        assert_bitexact(host(dout), e / np.float32(d) if d != 1.0 else e)


@pytest.mark.parametrize("n", [65, 71, 4099, (1 << 20) + 3])
@pytest.mark.parametrize("hoff,foff", [(0, 0), (1, 0), (0, 2), (5, 1), (7, 3)])
def test_f16_codec_operand_phases(n, hoff, foff):
    """encode / decode_scale with the f16 and f32 operands at equal and at
    different 4-element phases (vector body vs scalar fallback)."""
    x = O.synth(n, SEED, 2)
    h = O.f16_encode(x)
    out = dev(np.zeros(n, np.uint16), hoff)
    K.f16_encode(out, dev(x, foff))
    assert np.array_equal(host(out), h)
    for d in (1.0, 3.0):
        dout = dev(np.zeros(n, np.float32), foff)
        K.f16_decode_scale(dout, dev(h, hoff), d)
        e = O.f16_decode(h)
        assert_bitexact(host(dout), e / np.float32(d) if d != 1.0 else e)


def test_nan_inf_propagation():
    x = np.array([np.nan, -np.inf, np.inf, 1.0, -0.0], np.float32)
    x = np.concatenate([x, np.array([0x7FC00001, 0xFF812345, 0x7F800001], np.uint32).view(np.float32)])
    out = dev(np.zeros(x.size, np.uint16))
    K.f16_encode(out, dev(x))
    assert np.array_equal(host(out), O.f16_encode(x))
    dec = dev(np.zeros(x.size, np.float32))
    K.f16_decode(dec, out)
    assert_bitexact(host(dec), O.f16_decode(O.f16_encode(x)))


@pytest.mark.parametrize("n,seed,rank,offset", [(1, 1, 0, 0), (4099, SEED, 3, 0), (1 << 20, SEED, 0, 12345),
                                                (1031, 7, 1, 2 ** 33 + 1)])
def test_synth_matches_oracle(n, seed, rank, offset):
    for off in (0, 1):
        t = dev(np.zeros(n, np.float32), off)
        K.synth(t, seed, rank, offset)
        assert_bitexact(host(t), O.synth(n, seed, rank, offset))


@pytest.mark.parametrize("k", [2, 4, 8])
def test_full_size_sum_scale_property(k):
    """64 MiB bucket (BASELINE config 2), k = 2 / 4 / 8 inputs (each k its own
    SumScaleOp instantiation), divisor k: the kernel equals the oracle on a
    strided sample and then on all 16 M elements
    (worker_ring.rs:141-143 summed in input order, param_manager.rs:183-188 ÷n)."""
    n = 1 << 24
    ins = [torch.empty(n, dtype=torch.float32, device=DEV) for _ in range(k)]
    for r, t in enumerate(ins):
        K.synth(t, SEED, r)
    out = torch.empty(n, dtype=torch.float32, device=DEV)
    K.sum_scale(out, ins, float(k))
    idx = np.arange(0, n, 4097)
    got = host(out)[idx]
    hs = [host(t)[idx] for t in ins]
    assert_bitexact(got, O.sum_scale(hs, float(k)))
    full = [host(t) for t in ins]
    assert_bitexact(host(out), O.sum_scale(full, float(k)), f"all 16M elements, k = {k}")


@pytest.mark.parametrize("wire", ["f32", "f16"])
@pytest.mark.parametrize("n,length", [(2, 4099), (3, 1000003), (8, (1 << 20) + 5), (16, 65541)])
def test_direct_chain_is_the_owner_of_the_ring(wire, n, length):
    """ono_direct_chain over the slices of chunk c (rank c, c+1, ..., owner
    c-1 last) gives the owner's grad of the oracle ring, and its message is
    what every replica ends up with (f16: decode / n) — the DIRECT / XGMI owner
    kernel against worker_ring.rs:112-204 as restated by the oracle."""
    res = [O.synth(length, SEED + 11, r) for r in range(n)]
    grads, _ = O.ring_pull_grads(res, wire)
    for ci, (lo, hi) in enumerate(O.split_chunks(length, n)):
        if ci % max(1, n // 3):  # a few chunks per case
            continue
        owner = (ci - 1) % n
        off = (lo + ci) % 4
        ins = [dev(res[(ci + j) % n][lo:hi], off) for j in range(n)]
        g = dev(np.zeros(hi - lo, np.float32), off)
        out = (dev(np.zeros(hi - lo, np.uint16), off) if wire == "f16" else dev(np.zeros(hi - lo, np.float32), off))
        K.direct_chain(g, out, ins, float(n), wire)
        assert_bitexact(host(g), grads[owner][lo:hi], f"owner grad, chunk {ci}")
        other = (owner + 1) % n
        if wire == "f16":
            dec = O.f16_decode(host(out))
            assert_bitexact((dec / np.float32(n)).astype(np.float32), grads[other][lo:hi],
                            f"replica from the message, chunk {ci}")
        else:
            assert_bitexact(host(out), grads[owner][lo:hi], f"f32 message, chunk {ci}")
        assert not host(ins[-1]).any(), "own slice not zeroed"
        for j in range(n - 1):
            assert_bitexact(host(ins[j]), res[(ci + j) % n][lo:hi], "received slices must stay untouched")


def test_direct_chain_zero_all_and_no_out():
    n, length = 5, 4099
    ins_h = [O.synth(length, SEED + 12, r) for r in range(n)]
    ins = [dev(x) for x in ins_h]
    g = dev(np.zeros(length, np.float32))
    K.direct_chain(g, None, ins, 5.0, "f16", zero_all=True)
    p = ins_h[0].copy()
    for j in range(1, n):
        p = (ins_h[j] + O.f16_decode(O.f16_encode(p))).astype(np.float32)
    assert_bitexact(host(g), (p / np.float32(5.0)).astype(np.float32))
    for t in ins:
        assert not host(t).any()
