"""GPU parity of the sparse gradient codec (comms/src/sparse/protocol.rs)
against the reference's own KATs (protocol.rs:150-223, sparse/tests.rs:13-59)
and the C oracle: byte-exact encoding, exact decoding, reference errors."""
import numpy as np
import pytest
import torch

import ono_amd
from ono_amd import sparse as SP
from conftest import SEED, assert_bitexact
from oracle import oracle as O

pytestmark = pytest.mark.gpu

KAT_BUF = bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188,
                 1, 0, 0, 0, 1, 0, 0, 0, 0, 64])


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


@pytest.fixture(params=[0, 1], ids=["pattern_first", "walk_only"])
def lift_mode(request):
    """Each device-lift test runs with the pattern path first (the default) and
    with the walk path alone, so both parsers meet every case."""
    L = ono_amd.lib()
    assert L.ono_sparse_lift_set_mode(request.param) == 0
    yield request.param
    assert L.ono_sparse_lift_set_mode(0) == 0


def test_grad_drop_kat():  # protocol.rs:150-170
    assert SP.grad_drop(dev([1.0, -1.0, 0.0, 2.0]), 1.0) == KAT_BUF


def test_grad_lift_kat():  # protocol.rs:172-190, :207-222
    assert SP.grad_lift(KAT_BUF).cpu().tolist() == [1.0, -1.0, 0.0, 2.0]
    short = bytes([3, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188])
    assert SP.grad_lift(short).cpu().tolist() == [0.0, 1.0, -1.0]


def test_sparse_gradient_kat():  # sparse/tests.rs:13-59
    g = np.arange(16, dtype=np.float32)
    t = SP.threshold_full(g, 0.4)
    assert t == 9.0
    out = SP.grad_lift(SP.grad_drop(dev(g), t)).cpu().tolist()
    assert out == [0.0] * 9 + [9.0, 10.0, 11.0, 12.0, 13.0, 14.0, 15.0]


@pytest.mark.parametrize("n", [0, 1, 2, 7, 2047, 2048, 2049, 4099, 65536 + 17, (1 << 20) + 5])
@pytest.mark.parametrize("r", [0.0, 0.4, 0.9, 0.999])
def test_drop_matches_oracle_bytes(n, r):
    g = O.synth(n, SEED + 21, 1)
    if n > 3:
        g[3] = np.nan          # never kept (|NaN| >= t is false)
        g[n // 2] = np.inf     # always kept
    t = float(np.quantile(np.abs(g[np.isfinite(g)]), r)) if n > 3 else 0.0
    t = max(t, 6.103515625e-05) if r > 0 else 0.0
    got = SP.grad_drop(dev(g), t)
    assert got == O.grad_drop(g, t)
    back = SP.grad_lift(got, cap=n).cpu().numpy()
    assert_bitexact(back, O.grad_lift(O.grad_drop(g, t), cap=max(n, 1)))


def test_drop_alternating_runs_worst_case():
    n = 100001
    g = np.zeros(n, np.float32)
    g[::2] = 1.5  # n/2 runs of length 1: the largest encoding
    got = SP.grad_drop(dev(g), 1.0)
    assert got == O.grad_drop(g, 1.0)
    assert len(got) == 8 + 10 * ((n + 1) // 2)


def test_threshold_full_matches_oracle():
    for n, r in [(16, 0.4), (1000, 0.9), (16384, 0.5), (3, 1.0), (5, 0.0)]:
        g = O.synth(n, SEED, 2)
        assert SP.threshold_full(g, r) == O.sparse_threshold(g, r)


@pytest.mark.parametrize("buf,msg", [
    (b"\x04\x00\x00", "smaller than TOTAL_LEN_SIZE"),
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0]), "Missing index bytes"),
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0]), "Missing chunk length bytes"),
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 3, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188]), "exceeds target vector bounds"),
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 60]), "Truncated float data"),
])
def test_lift_errors(buf, msg):
    with pytest.raises(ono_amd.InvalidWorkerEvent, match=msg):
        SP.grad_lift(buf, cap=16)


def test_masks_match_ring_bookkeeping():
    g = O.synth(50001, SEED, 4)
    t = 0.01
    a, b = dev(g), dev(g)
    SP.mask_sent(a, t)
    SP.mask_unsent(b, t)
    torch.cuda.synchronize()
    e_sent = np.where(np.abs(g) >= t, np.float32(0), g)    # worker_ring.rs:128-131
    e_unsent = np.where(np.abs(g) < t, np.float32(0), g)   # worker_ring.rs:183-187
    assert_bitexact(a.cpu().numpy(), e_sent)
    assert_bitexact(b.cpu().numpy(), e_unsent)


@pytest.mark.parametrize("offset", [0, 1, 3])
def test_drop_exact_size_buffer_and_unaligned_input(offset):
    """The two host-visible paths of ono_sparse_drop: a buffer of exactly the
    encoded size (the counts come back to the host before the write pass) and
    one byte short (SizeMismatch), plus the worst-case buffer, on a 16-B aligned
    gradient and on unaligned views (scalar loads instead of 16-B vectors)."""
    import ctypes as C

    n = 65536 + 17
    g = O.synth(n, SEED + 5, 2)
    t = float(np.quantile(np.abs(g), 0.8))
    want = O.grad_drop(g, t)
    base = torch.zeros(n + 8, dtype=torch.float32, device="cuda")
    view = base[offset:offset + n]
    view.copy_(torch.from_numpy(g))
    assert SP.grad_drop(view, t) == want
    L = ono_amd.lib()
    for cap, ok in ((len(want), True), (len(want) - 1, False)):
        buf = torch.empty(cap + 8, dtype=torch.uint8, device="cuda")
        nb = C.c_size_t(0)
        rc = L.ono_sparse_drop(buf.data_ptr(), cap, C.byref(nb), view.data_ptr(), n, t,
                               torch.cuda.current_stream().cuda_stream)
        if ok:
            assert rc == 0 and nb.value == len(want)
            assert bytes(buf[: nb.value].cpu().numpy()) == want
        else:
            assert rc == 1  # ONO_E_SIZE


# ----------------------------------------------------------- device lift ----
def to_dev(b: bytes) -> torch.Tensor:
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda() if b else torch.empty(0, dtype=torch.uint8,
                                                                                            device="cuda")


def random_stream(rng, nrec: int, max_off: int, max_len: int, payload: str, min_off: int = 0) -> bytes:
    """A valid sparse stream of nrec records built directly (not by grad_drop):
    zero-length records, zero offsets and payloads chosen to look like record
    headers ("zeros", "small": f16 bit patterns < 0x40) stress the speculative
    record starts; "random": every f16 bit pattern."""
    offs = rng.integers(min_off, max_off + 1, nrec)
    lens = rng.integers(0, max_len + 1, nrec)
    total = int(offs.sum() + lens.sum()) + int(rng.integers(0, 5))
    parts = [np.uint64(total).tobytes()]
    for o, ln in zip(offs, lens):
        parts.append(np.array([o, ln], np.uint32).tobytes())
        if payload == "zeros":
            v = np.zeros(ln, np.uint16)
        elif payload == "small":
            v = rng.integers(0, 0x40, ln).astype(np.uint16)
        else:
            v = rng.integers(0, 1 << 16, ln).astype(np.uint16)
        parts.append(v.tobytes())
    return b"".join(parts)


@pytest.mark.usefixtures("lift_mode")
def test_lift_dev_kats():
    assert SP.grad_lift(to_dev(KAT_BUF)).cpu().tolist() == [1.0, -1.0, 0.0, 2.0]
    short = bytes([3, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188])
    assert SP.grad_lift(to_dev(short)).cpu().tolist() == [0.0, 1.0, -1.0]
    assert SP.grad_lift(to_dev(bytes(8))).numel() == 0


@pytest.mark.usefixtures("lift_mode")
@pytest.mark.parametrize("n", [2049, 65536 + 17, (1 << 20) + 5, 1 << 24])
@pytest.mark.parametrize("r", [0.0, 0.5, 0.9, 0.999])
def test_drop_lift_device_resident(n, r):
    """drop -> lift with the stream never leaving HBM (ono_sparse_lift_dev), and
    the host-stream lift over the same bytes: both equal the oracle's lift."""
    g = O.synth(n, SEED + 23, 3)
    t = float(np.quantile(np.abs(g), r)) if r > 0 else 0.0
    t = max(t, 6.103515625e-05) if r > 0 else 0.0
    wire = SP.grad_drop_dev(dev(g), t)
    host_bytes = bytes(wire.cpu().numpy())
    want = O.grad_lift(host_bytes, cap=n)
    assert_bitexact(SP.grad_lift_dev(wire, n).cpu().numpy(), want)
    assert_bitexact(SP.grad_lift(host_bytes, cap=n).cpu().numpy(), want)


@pytest.mark.usefixtures("lift_mode")
@pytest.mark.parametrize("payload", ["random", "small", "zeros"])
@pytest.mark.parametrize("nrec,max_off,max_len", [(1, 3, 5), (37, 2, 3), (5000, 4, 40), (200000, 1, 6),
                                                  (3000, 0, 2000)])
def test_lift_dev_random_streams(payload, nrec, max_off, max_len):
    """Streams written directly (arbitrary offsets/lengths, zero-length records,
    header-like payloads): the device parse equals the oracle whether its
    speculative record starts hold or are refuted (sequential fallback)."""
    rng = np.random.default_rng(nrec * 7 + max_len + len(payload))
    b = random_stream(rng, nrec, max_off, max_len, payload)
    total = int.from_bytes(b[:8], "little")
    want = O.grad_lift(b, cap=max(total, 1))
    assert_bitexact(SP.grad_lift_dev(to_dev(b), total).cpu().numpy(), want)
    assert_bitexact(SP.grad_lift(b, cap=total).cpu().numpy(), want)


def test_lift_dev_typical_stream_takes_the_parallel_parse():
    """The bench's stream (90th-percentile threshold, 16 M values) must not fall
    back to the sequential parse; neither must a drop-like stream (offsets >= 1)
    with random f16 payload."""
    L = ono_amd.lib()
    g = ono_amd.kernels.synth(torch.empty(1 << 24, dtype=torch.float32, device="cuda"), SEED, 7)
    t = float(torch.quantile(g[: 1 << 20].abs().float(), 0.9).item())
    wire = SP.grad_drop_dev(g, t)
    before = L.ono_sparse_lift_fallbacks()
    back = SP.grad_lift_dev(wire, g.numel())
    b2 = random_stream(np.random.default_rng(5), 100000, 3, 30, "random", min_off=1)  # drop-like: runs maximal
    SP.grad_lift_dev(to_dev(b2), int.from_bytes(b2[:8], "little"))
    assert L.ono_sparse_lift_fallbacks() == before
    keep = g.abs() >= t
    torch.cuda.synchronize()
    ref = torch.where(keep, g.half().float(), torch.zeros_like(g))  # RNE f16 of the kept values
    assert torch.equal(back.view(torch.int32), ref.view(torch.int32))


@pytest.mark.usefixtures("lift_mode")
@pytest.mark.parametrize("buf,msg", [
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0]), "Missing index bytes"),
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0]), "Missing chunk length bytes"),
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 3, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188]), "exceeds target vector bounds"),
    (bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 60]), "Truncated float data"),
])
def test_lift_dev_errors(buf, msg):
    with pytest.raises(ono_amd.InvalidWorkerEvent, match=msg):
        SP.grad_lift_dev(to_dev(buf), 16)


@pytest.mark.usefixtures("lift_mode")
def test_lift_dev_error_deep_in_a_long_stream():
    """A bounds error in record 150000 of a valid-looking stream: the parallel
    parse refutes itself and the sequential parse reports the reference's error."""
    rng = np.random.default_rng(11)
    b = bytearray(random_stream(rng, 200000, 2, 4, "random"))
    total = int.from_bytes(b[:8], "little")
    b[:8] = np.uint64(total // 2).tobytes()
    with pytest.raises(ono_amd.InvalidWorkerEvent, match="exceeds target vector bounds"):
        SP.grad_lift_dev(to_dev(bytes(b)), total)


@pytest.mark.usefixtures("lift_mode")
def test_lift_dev_size_error_and_short_cap():
    """total > cap: ONO_E_SIZE from the device-side check, nothing written."""
    import ctypes as C

    g = np.arange(64, dtype=np.float32)
    wire = SP.grad_drop_dev(dev(g), 10.0)
    out = torch.full((32,), 7.0, dtype=torch.float32, device="cuda")
    ln = C.c_size_t(0)
    rc = ono_amd.lib().ono_sparse_lift_dev(out.data_ptr(), 32, C.byref(ln), wire.data_ptr(), wire.numel(),
                                           torch.cuda.current_stream().cuda_stream)
    assert rc == 1  # ONO_E_SIZE
    assert torch.all(out == 7.0)
    back = SP.grad_lift_dev(wire, 100)  # larger cap: out_len is the stream's total
    assert back.numel() == 64
    assert_bitexact(back.cpu().numpy(), O.grad_lift(bytes(wire.cpu().numpy()), cap=64))


@pytest.mark.usefixtures("lift_mode")
@pytest.mark.parametrize("offset", [0, 1, 2])
def test_lift_dev_into_unaligned_gradient(offset):
    """g at a 4-B (not 16-B) boundary: the device zero-fill's scalar form."""
    import ctypes as C

    n = 70001
    g = O.synth(n, SEED + 29, 1)
    t = float(np.quantile(np.abs(g), 0.7))
    wire = SP.grad_drop_dev(dev(g), t)
    base = torch.full((n + 8,), 5.0, dtype=torch.float32, device="cuda")
    view = base[offset:offset + n]
    ln = C.c_size_t(0)
    rc = ono_amd.lib().ono_sparse_lift_dev(view.data_ptr(), n, C.byref(ln), wire.data_ptr(), wire.numel(),
                                           torch.cuda.current_stream().cuda_stream)
    assert rc == 0 and ln.value == n
    assert_bitexact(view.cpu().numpy(), O.grad_lift(bytes(wire.cpu().numpy()), cap=n))
    assert torch.all(base[:offset] == 5.0) and torch.all(base[offset + n:] == 5.0)


@pytest.mark.parametrize("pattern", ["far", "long_runs"])
def test_drop_headers_across_tiles_and_scan_chunks(pattern):
    """Run headers whose neighbour run is many tiles away, across the tile
    scan's 8192-tile chunks (n > 2^24): the offset / length carries."""
    n = 20_000_003
    g = np.zeros(n, np.float32)
    if pattern == "far":
        for i in (0, 5, 2047, 2048, 4_000_000, 16_777_215, 16_777_216, 16_777_218, n - 1):
            g[i] = 1.5
    else:  # kept runs spanning tiles and the chunk boundary, gaps spanning many tiles
        g[10_000:30_000] = -2.0
        g[16_770_000:16_790_000] = 3.0
        g[19_999_000:19_999_001] = 1.0
        g[n - 3000:] = 0.75
    got = SP.grad_drop_dev(dev(g), 0.5)
    want = O.grad_drop(g, 0.5)
    assert bytes(got.cpu().numpy()) == want
    assert_bitexact(SP.grad_lift_dev(got, n).cpu().numpy(), O.grad_lift(want, cap=n))


@pytest.mark.parametrize("first_unkept", [128 * 2048 * 2 + 5, 128 * 2048 * 3 - 1, 128 * 2048 * 4 + 77, None])
def test_drop_whole_chunks_kept(first_unkept):
    """Chunks of 128 tiles with every value kept: the last run's length in a
    tile comes from the first unkept value in a later chunk (two, three or
    more chunks on), or from n when there is none."""
    n = 128 * 2048 * 5 + 301
    g = np.full(n, 2.0, np.float32)
    if first_unkept is not None:
        g[first_unkept] = 0.0
        g[first_unkept + 1000::7] = 0.0
    got = SP.grad_drop_dev(dev(g), 0.5)
    want = O.grad_drop(g, 0.5)
    assert bytes(got.cpu().numpy()) == want
    assert_bitexact(SP.grad_lift_dev(got, n).cpu().numpy(), O.grad_lift(want, cap=n))


@pytest.mark.parametrize("pattern", ["all_kept", "none_kept", "tile_edges", "clustered", "single_tail"])
def test_drop_tile_boundary_patterns(pattern):
    """The encoder's cross-tile header fields (sp_move completes the first
    run's offset from the kept values before the tile and the last run's
    length from the unkept values after it): runs that start or end exactly at
    the 2048-value tile edges, one run over every tile, nothing kept, bursts of
    runs with long gaps, a lone value at the very end."""
    n = 3 * 2048 * 5 + 11
    g = np.zeros(n, np.float32)
    if pattern == "all_kept":
        g[:] = 2.0
    elif pattern == "tile_edges":
        for k in range(1, n // 2048 + 1):
            e = 2048 * k
            g[max(0, e - 3):e] = 1.0          # a run ending at the tile's end
            if e + 1 < n:
                g[e + 1:e + 4] = -1.0         # one starting just after the next tile's start
            if k % 3 == 0 and e < n:
                g[e - 1:e + 1] = 3.0          # one crossing the edge
    elif pattern == "clustered":
        rng = np.random.default_rng(7)
        for c in rng.integers(0, n - 300, 40):
            m = rng.random(300) < 0.6
            g[c:c + 300] = np.where(m, rng.standard_normal(300).astype(np.float32) + 3.0, 0.0)
    elif pattern == "single_tail":
        g[-1] = -7.0
    got = SP.grad_drop_dev(dev(g), 0.5)
    want = O.grad_drop(g, 0.5)
    assert bytes(got.cpu().numpy()) == want
    assert_bitexact(SP.grad_lift_dev(got, n).cpu().numpy(), O.grad_lift(want, cap=n))


@pytest.mark.parametrize("n", [0, 5, 2048, (1 << 20) + 3])
def test_drop_async_matches_blocking(n):
    """ono_sparse_drop_async: the same bytes as the blocking drop, the length
    in device memory, several drops queued back to back on one stream with
    no host wait between them; a buffer below the worst case is refused."""
    L = ono_amd.lib()
    cap = L.ono_sparse_max_bytes(n)
    gs = [O.synth(n, SEED + 40 + k, 1) for k in range(3)]
    ts = [float(np.quantile(np.abs(x), 0.9)) if n else 0.0 for x in gs]
    bufs = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in gs]
    nbs = torch.zeros(len(gs), dtype=torch.int64, device="cuda")
    dgs = [dev(x) for x in gs]
    torch.cuda.synchronize()
    for k in range(len(gs)):
        SP.grad_drop_async(dgs[k], ts[k], bufs[k], nbs[k:k + 1])
    torch.cuda.synchronize()
    for k in range(len(gs)):
        want = O.grad_drop(gs[k], ts[k])
        assert int(nbs[k].item()) == len(want)
        assert bytes(bufs[k][: len(want)].cpu().numpy()) == want
    with pytest.raises(ono_amd.OnoError):
        SP.grad_drop_async(dgs[0], ts[0], bufs[0][: max(cap - 1, 0)], nbs[:1])


# ------------------------------------------------ calculate_threshold on the device
def _threshold_inputs(n, seed):
    x = O.synth(n, seed, 0)
    rng = np.random.default_rng(seed)
    k = max(1, n // 50)
    x[rng.integers(0, n, k)] = 0.0
    x[rng.integers(0, n, k)] = -0.0
    x[rng.integers(0, n, k)] = np.float32(6.103515625e-05)          # the floor itself
    x[rng.integers(0, n, k)] = x[rng.integers(0, n, k)]           # ties
    x[rng.integers(0, n, max(1, k // 4))] = np.inf
    x.view(np.uint32)[rng.integers(0, n, max(1, k // 4))] = 0xFFC01234  # -NaN with a payload
    return x


@pytest.mark.parametrize("n", [1, 2, 17, 1000, 16384])
@pytest.mark.parametrize("r", [0.05, 0.4, 0.9, 1.0])
def test_threshold_full_sample_vs_oracle(n, r):
    """sp_threshold (radix select over the |g| bit patterns in LDS) equals the
    restated calculate_threshold (sort in total_cmp order, k-th, max with
    f16::MIN_POSITIVE) — NaN, inf, signed zeros and ties included."""
    x = _threshold_inputs(n, SEED + n)
    got = SP.threshold(torch.from_numpy(x).cuda(), r)
    want = O.sparse_threshold_sample(x, r)
    assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32), (got, want)


@pytest.mark.parametrize("n,r", [(16385, 0.4), (100000, 0.1), (1 << 22, 0.9)])
def test_threshold_drawn_sample_vs_oracle(n, r):
    """Above 16384 values the sample is the caller's indices (a duplicate-free
    draw); the device gathers them from HBM."""
    x = _threshold_inputs(n, SEED + 7)
    idx, _ = O.sample_default(99, n, 16384)
    got = SP.threshold(torch.from_numpy(x).cuda(), r, idx)
    assert np.float32(got).view(np.uint32) == np.float32(O.sparse_threshold_sample(x, r, idx)).view(np.uint32)


@pytest.mark.parametrize("kind", ["all_equal", "two_values", "all_nan", "denormals", "every_rank", "wide_exponents",
                                  "one_bit_apart"])
def test_threshold_adversarial_samples(kind):
    """The bit-sliced select (two key bits per step over transposed bit
    planes) against the restated calculate_threshold on samples that stress
    each digit path: all keys equal (every step keeps all candidates), two
    values, all NaN, denormals (the high bits all zero), every rank of one
    sample, keys spread over every exponent, keys one ulp apart."""
    rng = np.random.default_rng(5)
    n = 16384
    if kind == "all_equal":
        xs = [np.full(n, 0.3, np.float32), np.full(777, -2.5, np.float32)]
    elif kind == "two_values":
        xs = [np.where(rng.random(n) < 0.37, 1.0, 2.0).astype(np.float32)]
    elif kind == "all_nan":
        x = np.empty(n, np.float32)
        x.view(np.uint32)[:] = 0x7FC00000 | rng.integers(0, 1 << 22, n).astype(np.uint32)
        xs = [x]
    elif kind == "denormals":
        x = np.empty(n, np.float32)
        x.view(np.uint32)[:] = rng.integers(0, 1 << 23, n).astype(np.uint32)
        xs = [x]
    elif kind == "wide_exponents":
        x = np.empty(n, np.float32)
        x.view(np.uint32)[:] = rng.integers(0, 0x7F800000, n).astype(np.uint32) | (rng.integers(0, 2, n) << 31).astype(np.uint32)
        xs = [x]
    elif kind == "one_bit_apart":
        base = np.uint32(0x3F800000)
        x = np.empty(n, np.float32)
        x.view(np.uint32)[:] = base + rng.integers(0, 4, n).astype(np.uint32)
        xs = [x]
    else:  # every rank: r from 0 to 1 in fine steps over one sample of 513 values (a partial last lane column)
        xs = [O.synth(513, SEED + 3, 0)]
    rs = [0.001, 0.1, 0.5, 0.9, 1.0] if kind != "every_rank" else [i / 512 for i in range(1, 513)]
    for x in xs:
        xd = torch.from_numpy(x).cuda()
        for r in rs:
            got = SP.threshold(xd, r)
            want = O.sparse_threshold_sample(x, r)
            assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32), (kind, len(x), r, got, want)


def test_threshold_argument_errors():
    g = torch.zeros(20000, device="cuda")
    with pytest.raises(ono_amd.InvalidArgument):
        SP.threshold(g, 0.4)  # above 16384 values a sample is required
    with pytest.raises(ono_amd.InvalidArgument):
        SP.threshold(g[:10], 1.5)
    with pytest.raises(ono_amd.InvalidArgument):
        SP.threshold(g[:10], 0.4, np.array([3, 10], np.uint32))  # index out of range


# ------------------------------------------------- lift: three-launch paths ----
def _lift_into(buf_dev: torch.Tensor, out: torch.Tensor, cap: int) -> int:
    import ctypes as C

    ln = C.c_size_t(0)
    rc = ono_amd.lib().ono_sparse_lift_dev(out.data_ptr(), cap, C.byref(ln), buf_dev.data_ptr(), buf_dev.numel(),
                                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rc == 0, ono_amd.lib().ono_last_error()
    return ln.value


@pytest.mark.usefixtures("lift_mode")
@pytest.mark.parametrize("n,r", [(70001, 0.9), (1 << 20, 0.5), (4099, 0.0)])
def test_lift_dev_leaves_values_past_total_untouched(n, r):
    """cap > total: g[0, total) is the lift (zeros between the runs), g[total, cap) keeps what it held
    (protocol.rs:96-144 resizes the caller's vector to total)."""
    g = O.synth(n, SEED + 41, 2)
    t = max(float(np.quantile(np.abs(g), r)), 6.103515625e-05) if r > 0 else 0.0
    wire = SP.grad_drop_dev(dev(g), t)
    cap = n + 3000
    out = torch.full((cap,), 9.0, dtype=torch.float32, device="cuda")
    assert _lift_into(wire, out, cap) == n
    assert_bitexact(out[:n].cpu().numpy(), O.grad_lift(bytes(wire.cpu().numpy()), cap=n))
    assert torch.all(out[n:] == 9.0)


@pytest.mark.usefixtures("lift_mode")
@pytest.mark.parametrize("lens", [[4096], [4097], [8192 + 33], [33, 32, 31, 4096 * 3 + 1], [1, 2, 3] * 50])
def test_lift_dev_long_runs_across_chunks(lens):
    """Runs longer than one lane's share (> 32 values) go through the chunk queue, including runs that
    are whole multiples of the 4096-value chunk and one value past it."""
    rng = np.random.default_rng(sum(lens))
    parts, total = [], 0
    body = []
    for ln in lens:
        off = int(rng.integers(1, 40))
        body.append(np.array([off, ln], np.uint32).tobytes())
        body.append(rng.integers(0, 0x7C00, ln).astype(np.uint16).tobytes())  # finite f16 values
        total += off + ln
    total += 7
    b = np.uint64(total).tobytes() + b"".join(body)
    want = O.grad_lift(b, cap=total)
    out = torch.full((total,), 5.0, dtype=torch.float32, device="cuda")
    assert _lift_into(to_dev(b), out, total) == total
    assert_bitexact(out.cpu().numpy(), want)


def test_lift_dev_walks_longer_than_the_noted_records():
    """Offsets of 0 after the first record refuse every speculative start, so segment 0's walk spans the
    whole stream: records past the 32 it notes are walked again by sl_place's overflow path."""
    rng = np.random.default_rng(3)
    nrec = 3000
    lens = rng.integers(1, 4, nrec)
    offs = np.zeros(nrec, np.int64)
    offs[0] = 5
    body = []
    for o, ln in zip(offs, lens):
        body.append(np.array([o, ln], np.uint32).tobytes())
        body.append(rng.integers(0, 0x7C00, ln).astype(np.uint16).tobytes())
    total = int(offs.sum() + lens.sum()) + 11
    b = np.uint64(total).tobytes() + b"".join(body)
    L = ono_amd.lib()
    before = L.ono_sparse_lift_fallbacks()
    out = torch.empty(total, dtype=torch.float32, device="cuda")
    assert _lift_into(to_dev(b), out, total) == total
    assert L.ono_sparse_lift_fallbacks() == before  # the parallel parse held (one walk, verified)
    assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


@pytest.mark.usefixtures("lift_mode")
@pytest.mark.parametrize("offs,lens,tail", [
    ([], [], 3_000_000),                                   # no records: g is all tail (queued zero chunks)
    ([1_500_000, 2_000_000, 10], [5, 40, 1], 2_500_000),  # gaps wider than a workgroup zeroes itself
    ([200_000, 300_000, 7, 1], [3, 50, 2, 4100], 90_000),  # a group zeroed by its workgroup, then scattered
    ([3, 1, 4, 1, 5], [9, 2, 6, 5, 3], 5),                  # a small range built in LDS
])
def test_lift_dev_range_modes(offs, lens, tail):
    """Every element of g[0, total) is written exactly once, whatever a group's range: an LDS image for
    small ranges, zero-then-scatter for medium ones, queued zero chunks for wide gaps and tails."""
    rng = np.random.default_rng(len(offs) + tail)
    body, total = [], 0
    for o, ln in zip(offs, lens):
        body.append(np.array([o, ln], np.uint32).tobytes())
        body.append(rng.integers(0, 0x7C00, ln).astype(np.uint16).tobytes())
        total += o + ln
    total += tail
    b = np.uint64(total).tobytes() + b"".join(body)
    want = O.grad_lift(b, cap=total)
    out = torch.full((total + 64,), 3.0, dtype=torch.float32, device="cuda")
    assert _lift_into(to_dev(b), out, total + 64) == total
    assert_bitexact(out[:total].cpu().numpy(), want)
    assert torch.all(out[total:] == 3.0)


_ONE_LAUNCH_CHILD = r"""
import sys
sys.path[:0] = {paths!r}
import numpy as np, torch
from ono_amd import sparse as SP
from oracle import oracle as O

def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()

cases = []
if {small!r}:
    g = O.synth(300_001, 5, 1); cases.append((g, float(np.quantile(np.abs(g), 0.9))))
    n = 64 * 2048 * 3 + 77                 # > 3 look-back groups, ragged
    g = np.zeros(n, np.float32)
    g[10:70_000] = 1.0                     # a run over 34 tiles and into the second group
    g[131_071:131_074] = -2.0              # one across the first group edge
    for k in range(1, n // 2048, 5):
        g[2048 * k - 2:2048 * k + 1] = 3.0  # runs across tile edges
    g[-1] = 4.0
    cases.append((g, 0.5))
    cases.append((np.full(5 * 2048, 2.0, np.float32), 1.0))   # all kept
    cases.append((np.zeros(9 * 2048 + 3, np.float32), 1.0))   # none kept
else:  # more than 64 groups: several level-1 windows; runs and gaps across many tiles and groups
    n = 20_000_003
    g = np.zeros(n, np.float32)
    for i in (0, 5, 2047, 2048, 4_000_000, 8_388_607, 8_388_608, 16_777_215, 16_777_216, n - 1):
        g[i] = 1.5
    g[10_000:300_000] = -2.0
    g[16_770_000:16_790_000] = 3.0
    cases.append((g, 0.5))
    g = O.synth(9_000_001, 7, 1); cases.append((g, float(np.quantile(np.abs(g), 0.9))))
for g, t in cases:
    got = SP.grad_drop_dev(dev(g), t)
    assert bytes(got.cpu().numpy()) == O.grad_drop(g, t), (len(g), t)
print("ok", len(cases))
"""


@pytest.mark.parametrize("polls,small", [("0", True), ("1", True), ("96", False)],
                         ids=["fallback_always", "fallback_after_one_poll", "large_one_launch"])
def test_drop_one_launch_matches_oracle(polls, small):
    """sp_drop1 forced for every size (ONO_DROP_ONE_LAUNCH_TILES): its decoupled
    fallback (ONO_DROP_FALLBACK_POLLS=0: every look-back descriptor not there at
    the first read is computed by the waiting wave from the gradient itself, a
    group's from its tiles) and, at 20 M values, look-backs over more than 64
    groups: the same bytes as the oracle over runs across tile and group edges,
    all and none kept."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    paths = [root, os.path.join(root, "oxidized-neural-orchestra_amd")]
    env = dict(os.environ, ONO_DROP_FALLBACK_POLLS=polls, ONO_DROP_ONE_LAUNCH_TILES="1000000000")
    r = subprocess.run([sys.executable, "-c", _ONE_LAUNCH_CHILD.format(paths=paths, small=small)], capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip() == "ok %d" % (4 if small else 2)


IMAGE_FORM_WORKER = r"""
import sys
import numpy as np
import torch
sys.path[:0] = [{root!r}, {root!r} + "/oxidized-neural-orchestra_amd", {root!r} + "/tests"]
from ono_amd import sparse as SP
from oracle import oracle as O
rng = np.random.default_rng(11)
for n, r in [(256 * 2048 + 1, 0.9), (1 << 20, 0.5), (3 * 128 * 2048 + 77, 0.0), (5_000_003, 0.99)]:
    g = rng.standard_normal(n).astype(np.float32)
    t = float(np.quantile(np.abs(g), r))
    got = bytes(SP.grad_drop_dev(torch.from_numpy(g).cuda(), t).cpu().numpy())
    assert got == O.grad_drop(g, t), (n, r)
print("ok")
"""


def test_drop_image_form_matches_oracle():
    """The round-4 form (sp_image + sp_move, ONO_DROP_FORM=image, read once per
    process) still gives the reference's bytes above the one-launch size."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ONO_DROP_FORM="image")
    r = subprocess.run([sys.executable, "-c", IMAGE_FORM_WORKER.format(root=root)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_drop_past_256_chunks():
    """A gradient of more than 256 chunks of 128 tiles (n > 2^26): the
    aggregates before the tile's chunk past the first 256, read in blocks of
    64, and the next chunk's first unkept value past 256; runs across the chunk
    edges there."""
    n = (1 << 26) + 3 * 128 * 2048 + 999
    g = np.zeros(n, np.float32)
    chunk = 128 * 2048
    for c in (0, 255, 256, 257, 300):
        e = c * chunk
        g[max(0, e - 5):e + 7] = 1.25 + c
    g[260 * chunk:262 * chunk + 3] = -0.75          # a run over two whole chunks
    g[n - 10:] = 2.5
    got = SP.grad_drop_dev(dev(g), 0.5)
    want = O.grad_drop(g, 0.5)
    assert bytes(got.cpu().numpy()) == want
    assert_bitexact(SP.grad_lift_dev(got, n).cpu().numpy(), O.grad_lift(want, cap=n))
