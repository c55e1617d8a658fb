"""CPU model of the device lift's pattern path (csrc/ono_sparse.hip, pl_index /
pl_place), checked against the reference's sequential parse
(oracle/oracle_np.py grad_lift, restating comms/src/sparse/protocol.rs:96-144).

The claim the GPU path rests on: whenever the pattern's checks all pass, its
records ARE the sequential parse's records, so the lift it writes is the
reference's; and every stream grad_drop_into produces (gaps and runs below
2^16) passes.  The model follows the kernels' decomposition — per tile the
candidates (units k+1 and k+3 zero), each candidate's successor checked inside
the tile, the tile's exit; across tiles the link from the nearest non-empty
tile before, the head, the last exit and the total — with a small tile so the
cross-tile rules are exercised, and is driven by hypothesis over adversarial
streams (zero payloads, header-like payloads, zero-length runs, offsets and
lengths at and above 2^16, truncations, wrong totals) as well as drop output.
No GPU: the device kernels are held to the same streams by
tests/test_gpu_sparse_pattern.py."""
import numpy as np
from hypothesis import HealthCheck, given, settings, strategies as st

from oracle import oracle_np as N

TILE = 16  # units per tile in the model (the kernels use 2048; the rules do not depend on it)


def pattern_parse(buf: bytes, tile: int = TILE):
    """The pattern path's decision: None when refuted, else the records
    [(unit, offset, length)] it would place.  Mirrors pl_index + pl_place."""
    if len(buf) < 8 or (len(buf) - 8) % 2:
        return None
    total = int.from_bytes(buf[:8], "little")
    u = np.frombuffer(buf[8:], dtype="<u2").astype(np.int64)
    M = u.size
    if M == 0:
        return None  # (empty streams take the walk path)
    pad = np.concatenate([u, np.ones(4, np.int64)])
    k = np.arange(M)
    cand = (pad[k + 1] == 0) & (pad[k + 3] == 0) & (k + 4 <= M)
    T = (M + tile - 1) // tile
    recs, tiles = [], []
    for t in range(T):
        lo, hi = t * tile, min((t + 1) * tile, M)
        cs = [int(c) for c in np.flatnonzero(cand[lo:hi]) + lo]
        exitv = None
        for i, c in enumerate(cs):  # pl_index: each successor inside the tile is the next candidate
            nx = c + 4 + int(u[c + 2])
            if nx > M:
                return None
            if nx < hi and nx < M:
                if i + 1 >= len(cs) or cs[i + 1] != nx:
                    return None
            else:
                if i + 1 != len(cs):
                    return None
                exitv = nx
        tiles.append((cs, exitv))
        recs += [(c, int(u[c]), int(u[c + 2])) for c in cs]
    prev_exit = None  # pl_place: the link into each non-empty tile, the head, the last exit
    for cs, exitv in tiles:
        if cs:
            if (prev_exit is None and cs[0] != 0) or (prev_exit is not None and prev_exit != cs[0]):
                return None
            prev_exit = exitv
    if prev_exit != M:
        return None
    if sum(o + ln for _, o, ln in recs) > total:
        return None
    return recs


def sequential_records(buf: bytes):
    """The reference's parse (protocol.rs:109-141) as records, or None on its errors."""
    try:
        N.grad_lift(buf)
    except ValueError:
        return None
    body = buf[8:]
    out, bi = [], 0
    while bi < len(body):
        off = int.from_bytes(body[bi:bi + 4], "little")
        ln = int.from_bytes(body[bi + 4:bi + 8], "little")
        out.append((bi // 2, off, ln))
        bi += 8 + 2 * ln
    return out


def check(buf: bytes):
    got = pattern_parse(buf)
    if got is not None:
        assert got == sequential_records(buf), "the pattern path accepted a stream it parses differently"
    return got


def build(recs, total_pad=0, total=None):
    parts = []
    for off, ln, vals in recs:
        parts.append(np.array([off, ln], "<u4").tobytes())
        parts.append(np.asarray(vals, "<u2").tobytes())
    tot = sum(o + n for o, n, _ in recs) + total_pad if total is None else total
    return np.uint64(tot).tobytes() + b"".join(parts)


def test_reference_kats():
    kat = bytes([4, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188, 1, 0, 0, 0, 1, 0, 0, 0, 0, 64])
    assert check(kat) == [(0, 0, 2), (6, 1, 1)]  # protocol.rs:150-190
    short = bytes([3, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 2, 0, 0, 0, 0, 60, 0, 188])
    assert check(short) == [(0, 1, 2)]           # protocol.rs:207-222


@settings(max_examples=120, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(n=st.integers(1, 3000), ratio=st.floats(0.0, 1.0), seed=st.integers(0, 2**31 - 1),
       special=st.sampled_from(["none", "zeros", "nan", "inf", "tiny"]))
def test_drop_output_is_accepted_and_exact(n, ratio, seed, special):
    """grad_drop's streams with gaps and runs below 2^16 pass, and their records are the sequential
    parse's (NaN is never kept, inf is, zeros and values under f16's range are dropped or kept by the
    threshold >= f16::MIN_POSITIVE)."""
    rng = np.random.default_rng(seed)
    g = rng.standard_normal(n).astype(np.float32)
    if special == "zeros":
        g[rng.random(n) < 0.3] = 0.0
    elif special == "nan":
        g[rng.random(n) < 0.1] = np.nan
    elif special == "inf":
        g[rng.random(n) < 0.05] = np.inf
    elif special == "tiny":
        g *= np.float32(1e-6)
    t = max(float(np.quantile(np.abs(np.nan_to_num(g)), ratio)), float(N.MIN_POSITIVE_F16))
    buf = N.grad_drop(g, t)
    if len(buf) == 8:
        return  # no records: the walk path lifts the empty stream
    assert check(buf) is not None


_u16 = st.integers(0, 0xFFFF)
_payload = st.one_of(st.just("random"), st.just("zero"), st.just("headerish"))


@st.composite
def streams(draw):
    nrec = draw(st.integers(1, 40))
    recs = []
    for i in range(nrec):
        off = draw(st.one_of(st.integers(0 if i == 0 else 1, 30), st.sampled_from([0, 65535, 65536, 70000])))
        ln = draw(st.one_of(st.integers(1, 8), st.sampled_from([0, 33, 65535, 65536])))
        ln = min(ln, 70)  # (values are bytes in the stream: keep the examples small)
        kind = draw(_payload)
        if kind == "random":
            vals = draw(st.lists(_u16, min_size=ln, max_size=ln))
        elif kind == "zero":
            vals = [0] * ln
        else:
            vals = ([3, 0, 1, 0] * ln)[:ln]
        recs.append((off, ln, vals))
    buf = bytearray(build(recs, total_pad=draw(st.integers(0, 5))))
    mut = draw(st.sampled_from(["none", "total_minus", "truncate", "append", "flip"]))
    if mut == "total_minus":
        tot = int.from_bytes(buf[:8], "little")
        buf[:8] = np.uint64(max(0, tot - draw(st.integers(1, 10)))).tobytes()
    elif mut == "truncate":
        del buf[len(buf) - draw(st.integers(1, min(6, len(buf) - 8))):]
    elif mut == "append":
        buf += bytes(draw(st.lists(st.integers(0, 255), min_size=1, max_size=9)))
    elif mut == "flip" and len(buf) > 8:
        i = draw(st.integers(8, len(buf) - 1))
        buf[i] ^= 1 << draw(st.integers(0, 7))
    return bytes(buf)


@settings(max_examples=1200, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(buf=streams())
def test_adversarial_streams_are_never_misparsed(buf):
    """Whatever the stream, acceptance implies the reference's parse, record for record."""
    check(buf)


def test_refused_shapes():
    """The shapes the pattern refuses (the walk path or the host parse them)."""
    v = [0x3C00]
    assert check(build([(0, 1, v), (70000, 1, v)])) is None      # an offset of 2^16 or more
    assert check(build([(0, 1, v), (1, 0, []), (1, 1, v)])) is None  # a zero-length run
    assert check(build([(0, 2, [0x3C00, 0]), (1, 1, v)])) is None    # a zero value before a header
    assert check(build([(0, 1, v), (2, 1, v)], total=2)) is None     # the sum exceeds total
    assert check(build([(5, 3, [1, 2, 3]), (1, 2, [4, 5])])) is not None
