"""The device lift's pattern path (round 3): drop-shaped streams parse with no
speculation and no walks, checked to be the reference's sequential parse
(comms/src/sparse/protocol.rs:96-144); every other stream is refuted by those
checks and parsed by the walk path or the host, never mis-parsed."""
import ctypes as C

import numpy as np
import pytest
import torch

import ono_amd
from ono_amd import sparse as SP
from conftest import SEED, assert_bitexact
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


def to_dev(b: bytes) -> torch.Tensor:
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()


def lift_into(buf_dev: torch.Tensor, out: torch.Tensor, cap: int) -> int:
    ln = C.c_size_t(0)
    rc = ono_amd.lib().ono_sparse_lift_dev(out.data_ptr(), cap, C.byref(ln), buf_dev.data_ptr(), buf_dev.numel(),
                                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rc == 0, ono_amd.lib().ono_last_error()
    return ln.value


def counters():
    L = ono_amd.lib()
    return L.ono_sparse_lift_pattern_misses(), L.ono_sparse_lift_fallbacks()


def pattern_stream(rng, nrec, off_range, len_range, pad=3):
    """A drop-shaped stream: offsets in off_range (>= 1 after the first), lengths >= 1, both < 2^16,
    nonzero finite f16 payloads of either sign."""
    offs = rng.integers(off_range[0], off_range[1] + 1, nrec).astype(np.int64)
    lens = rng.integers(len_range[0], len_range[1] + 1, nrec).astype(np.int64)
    total = int(offs.sum() + lens.sum()) + pad
    units = 4 + lens
    starts = np.concatenate([[0], np.cumsum(units)[:-1]])
    u = rng.integers(1, 0x7C00, int(units.sum())).astype(np.uint16)
    u |= rng.integers(0, 2, u.size).astype(np.uint16) << 15
    u[starts], u[starts + 1] = offs & 0xFFFF, offs >> 16
    u[starts + 2], u[starts + 3] = lens & 0xFFFF, lens >> 16
    return np.uint64(total).tobytes() + u.tobytes(), total


def header_positions(b: bytes, upto: int) -> list[int]:
    pos, out = 8, []
    while pos < len(b) and len(out) < upto:
        out.append(pos)
        pos += 8 + 2 * int.from_bytes(b[pos + 4:pos + 8], "little")
    return out


@pytest.mark.parametrize("n,r", [(1 << 24, 0.9), ((1 << 20) + 5, 0.5), (65536 + 17, 0.99), (4099, 0.1),
                                 (1 << 22, 0.999)])
def test_pattern_path_takes_drop_output(n, r):
    """grad_drop's output is parsed by the pattern path: no hand-over to the walk path, no host parse,
    bit-exact with the oracle's lift."""
    g = O.synth(n, SEED + 51, 5)
    t = max(float(np.quantile(np.abs(g), r)), 6.103515625e-05)
    wire = SP.grad_drop_dev(dev(g), t)
    before = counters()
    out = SP.grad_lift_dev(wire, n)
    assert counters() == before
    assert_bitexact(out.cpu().numpy(), O.grad_lift(bytes(wire.cpu().numpy()), cap=n))


@pytest.mark.parametrize("nrec,off_range,len_range", [
    (1, (0, 0), (1, 1)),                 # one record at offset 0
    (3, (1, 5), (1, 3)),
    (20000, (1, 30), (1, 12)),           # many tiles, short runs (one lane each)
    (3000, (1, 40), (33, 700)),          # long runs: the workgroup copies them
    (40, (1, 9), (20000, 65535)),        # runs longer than a tile: payloads read past the staged tile
    (2000, (50, 200), (1, 3)),           # tile ranges above the LDS image: zeroed in g, then scattered
    (1200, (60000, 65535), (1, 2)),      # wide tile ranges: zero chunks queued for sl_long's grid
    (3_600_000, (1, 9), (1, 2)),         # more than 4096 tiles: the element prefixes from pl_scan
])
def test_pattern_path_range_shapes(nrec, off_range, len_range):
    """Drop-shaped streams of every range shape stay on the pattern path, are exact, and leave
    g[total, cap) untouched."""
    rng = np.random.default_rng(nrec + off_range[1] + len_range[1])
    b, total = pattern_stream(rng, nrec, off_range, len_range)
    before = counters()
    out = torch.full((total + 16,), 4.0, dtype=torch.float32, device="cuda")
    assert lift_into(to_dev(b), out, total + 16) == total
    assert counters() == before
    assert_bitexact(out[:total].cpu().numpy(), O.grad_lift(b, cap=total))
    assert torch.all(out[total:] == 4.0)


@pytest.mark.parametrize("offset", [1, 2, 3])
def test_pattern_path_into_unaligned_gradient(offset):
    """g at a 4-B (not 16-B) boundary: the image's scalar store form."""
    rng = np.random.default_rng(offset)
    b, total = pattern_stream(rng, 9000, (1, 12), (1, 5))
    base = torch.full((total + 8,), 5.0, dtype=torch.float32, device="cuda")
    view = base[offset:offset + total]
    before = counters()
    assert lift_into(to_dev(b), view, total) == total
    assert counters() == before
    assert_bitexact(view.cpu().numpy(), O.grad_lift(b, cap=total))
    assert torch.all(base[:offset] == 5.0) and torch.all(base[offset + total:] == 5.0)


@pytest.mark.parametrize("case", ["zero_payload", "zero_length_run", "gap_2_16", "run_2_16", "header_like",
                                  "odd_tail", "total_too_small", "truncated"])
def test_pattern_refuted_streams_are_never_misparsed(case):
    """Streams outside the pattern's shape fail its checks (never a wrong parse): the walk path or the
    host parse gives the oracle's result or the reference's error."""
    rng = np.random.default_rng(sum(map(ord, case)))
    b, total = pattern_stream(rng, 5000, (1, 20), (1, 6))
    b = bytearray(b)
    rec = header_positions(bytes(b), 2001)[2000]  # a header deep in the stream (tile 2 or so)
    ln = int.from_bytes(b[rec + 4:rec + 8], "little")
    if case == "zero_payload":  # 0x0000 values: false candidates where a header follows a 1-value run
        for p in header_positions(bytes(b), 5000)[::7]:
            b[p + 8:p + 10] = b"\x00\x00"
    elif case == "zero_length_run":  # a record with no values (the reference lifts it)
        b[rec + 8 + 2 * ln:rec + 8 + 2 * ln] = np.array([3, 0], np.uint32).tobytes()
        total += 3
    elif case == "gap_2_16":  # an offset of 2^16 or more: its header's high half is not zero
        off = int.from_bytes(b[rec:rec + 4], "little") + 70000
        b[rec:rec + 4] = np.uint32(off).tobytes()
        total += 70000
    elif case == "run_2_16":
        b[rec + 4:rec + 8] = np.uint32(ln + 70000).tobytes()
        b[rec + 8 + 2 * ln:rec + 8 + 2 * ln] = rng.integers(1, 0x7C00, 70000).astype(np.uint16).tobytes()
        total += 70000
    elif case == "header_like":  # payload values that read as a plausible header pair
        b[rec + 8:rec + 8] = np.array([2, 0, 1, 0], np.uint16).tobytes()
        b[rec + 4:rec + 8] = np.uint32(ln + 4).tobytes()
        total += 4
    elif case == "odd_tail":
        b += b"\x01"
    elif case == "total_too_small":
        total -= 10
    elif case == "truncated":  # the last run's length points past the stream
        last = header_positions(bytes(b), 5000)[-1]
        b[last + 4:last + 8] = np.uint32(int.from_bytes(b[last + 4:last + 8], "little") + 2).tobytes()
    b[:8] = np.uint64(total).tobytes()
    b = bytes(b)
    m0, _ = counters()
    errors = {"odd_tail": "Missing index bytes", "total_too_small": "exceeds target vector bounds",
              "truncated": "Truncated float data"}
    if case in errors:
        with pytest.raises(ono_amd.InvalidWorkerEvent, match=errors[case]):
            SP.grad_lift_dev(to_dev(b), total + 16)
        assert counters()[0] == m0 + (0 if case == "odd_tail" else 1)
        return
    out = SP.grad_lift_dev(to_dev(b), total)
    if case != "zero_payload":
        assert counters()[0] == m0 + 1
    assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


def test_pattern_path_many_lifts_reuse_scratch():
    """Lifts of growing and shrinking streams back to back (scratch regrown, epochs advancing): each
    exact, none handed over."""
    rng = np.random.default_rng(77)
    before = counters()
    for nrec in (10, 40000, 500, 120000, 1):
        b, total = pattern_stream(rng, nrec, (1, 15), (1, 4))
        out = SP.grad_lift_dev(to_dev(b), total)
        assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))
    assert counters() == before


@pytest.mark.parametrize("shift", [2, 4, 6])
def test_pattern_path_stream_at_a_2_byte_boundary(shift):
    """The stream itself at 2 / 4 / 6 bytes past an 8-byte boundary (a frame inside a larger receive
    buffer): the unit loads take their 2-byte form; exact, no hand-over."""
    rng = np.random.default_rng(shift)
    b, total = pattern_stream(rng, 7000, (1, 12), (1, 5))
    raw = torch.zeros(len(b) + 16, dtype=torch.uint8, device="cuda")
    raw[shift:shift + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
    view = raw[shift:shift + len(b)]
    assert view.data_ptr() % 8 == shift
    before = counters()
    out = torch.empty(total, dtype=torch.float32, device="cuda")
    assert lift_into(view, out, total) == total
    assert counters() == before
    assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


# ---- the stream-ordered lift (ono_sparse_lift_dev_async)

def lift_async(b: bytes, cap: int, status: torch.Tensor, fill: float = 6.0):
    buf = to_dev(b)
    out = torch.full((cap + 8,), fill, dtype=torch.float32, device="cuda")
    ticket = SP.grad_lift_dev_async(buf, out[:cap], status)
    torch.cuda.synchronize()
    return out, ticket, int(status.item()) == ticket


@pytest.mark.parametrize("n,r", [(1 << 24, 0.9), ((1 << 20) + 5, 0.5), (4099, 0.1)])
def test_async_lift_of_drop_output(n, r):
    """Stream-ordered, drop output: not refused, bit-exact, g[total, cap) untouched."""
    g = O.synth(n, SEED + 61, 6)
    t = max(float(np.quantile(np.abs(g), r)), 6.103515625e-05)
    b = bytes(SP.grad_drop_dev(dev(g), t).cpu().numpy())
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    out, ticket, refused = lift_async(b, n + 5, status)
    assert ticket != 0 and not refused
    assert_bitexact(out[:n].cpu().numpy(), O.grad_lift(b, cap=n))
    assert torch.all(out[n:] == 6.0)


@pytest.mark.parametrize("nrec,off_range,len_range", [
    (2000, (50, 200), (1, 3)),          # wide tile ranges: placed in windows by pl_place itself
    (1200, (60000, 65535), (1, 2)),     # very wide: every window in turn (no queue in this form)
    (3000, (1, 40), (33, 700)),         # long runs
    (3_600_000, (1, 9), (1, 2)),        # more than 4096 tiles: pl_scan
])
def test_async_lift_range_shapes(nrec, off_range, len_range):
    rng = np.random.default_rng(nrec + 17)
    b, total = pattern_stream(rng, nrec, off_range, len_range)
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    out, ticket, refused = lift_async(b, total, status)
    assert not refused
    assert_bitexact(out[:total].cpu().numpy(), O.grad_lift(b, cap=total))


@pytest.mark.parametrize("case", ["zero_length_run", "gap_2_16", "odd_tail", "empty", "total_over_cap",
                                  "truncated"])
def test_async_lift_refuses_what_the_pattern_cannot_take(case):
    """Refused calls say so through the status word (the blocking lift then parses them or reports the
    reference's error); total > cap writes nothing."""
    rng = np.random.default_rng(5)
    b, total = pattern_stream(rng, 3000, (1, 20), (1, 6))
    b = bytearray(b)
    rec = header_positions(bytes(b), 1001)[1000]
    ln = int.from_bytes(b[rec + 4:rec + 8], "little")
    cap = total
    if case == "zero_length_run":
        b[rec + 8 + 2 * ln:rec + 8 + 2 * ln] = np.array([3, 0], np.uint32).tobytes()
        total += 3
        cap = total
    elif case == "gap_2_16":
        b[rec:rec + 4] = np.uint32(int.from_bytes(b[rec:rec + 4], "little") + 70000).tobytes()
        total += 70000
        cap = total
    elif case == "odd_tail":
        b += b"\x01"
    elif case == "empty":
        b = bytearray(np.uint64(17).tobytes())
        total = cap = 17
    elif case == "total_over_cap":
        cap = total - 1
    elif case == "truncated":
        last = header_positions(bytes(b), 3000)[-1]
        b[last + 4:last + 8] = np.uint32(int.from_bytes(b[last + 4:last + 8], "little") + 2).tobytes()
    b[:8] = np.uint64(total).tobytes()
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    out, ticket, refused = lift_async(bytes(b), cap, status, fill=2.0)
    assert refused
    if case == "total_over_cap":
        assert torch.all(out == 2.0)


def test_async_lifts_back_to_back_on_one_stream():
    """Several stream-ordered lifts queued without a wait, one status word per call: each call's ticket
    is new, the refused one (a zero-length run) is the only one flagged, the others exact."""
    rng = np.random.default_rng(9)
    streams, outs, statuses, tickets = [], [], [], []
    for i in range(4):
        b, total = pattern_stream(rng, 5000 + 1000 * i, (1, 15), (1, 4))
        if i == 2:
            bb = bytearray(b)
            rec = header_positions(b, 11)[10]
            ln = int.from_bytes(bb[rec + 4:rec + 8], "little")
            bb[rec + 8 + 2 * ln:rec + 8 + 2 * ln] = np.array([1, 0], np.uint32).tobytes()
            total += 1
            bb[:8] = np.uint64(total).tobytes()
            b = bytes(bb)
        buf = to_dev(b)
        out = torch.empty(total, dtype=torch.float32, device="cuda")
        st = torch.zeros(1, dtype=torch.int64, device="cuda")
        tickets.append(SP.grad_lift_dev_async(buf, out, st))
        streams.append((b, buf, total))
        outs.append(out)
        statuses.append(st)
    torch.cuda.synchronize()
    assert len(set(tickets)) == 4
    for i, ((b, _, total), out, st, tk) in enumerate(zip(streams, outs, statuses, tickets)):
        assert (int(st.item()) == tk) == (i == 2)
        if i != 2:
            assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


def test_async_lifts_on_two_streams_concurrently():
    """Per-stream scratch: stream-ordered lifts queued on two streams at once (no wait between them) are
    each exact and not refused."""
    rng = np.random.default_rng(21)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    prep = []
    for k in range(6):
        b, total = pattern_stream(rng, 20000 + 3000 * k, (1, 15), (1, 4))
        prep.append((b, total, to_dev(b), torch.empty(total, dtype=torch.float32, device="cuda"),
                     torch.zeros(1, dtype=torch.int64, device="cuda")))
    torch.cuda.synchronize()  # inputs in place; then every lift queued with no wait in between
    jobs = []
    for k, (b, total, buf, out, st) in enumerate(prep):
        s = s1 if k % 2 == 0 else s2
        jobs.append((b, total, out, st, SP.grad_lift_dev_async(buf, out, st, s)))
    torch.cuda.synchronize()
    for b, total, out, st, tk in jobs:
        assert int(st.item()) != tk
        assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


# ---- the one-launch stream-ordered lift (pl_fused: an 8-B aligned stream of at most 4096 tiles; one
# tile per workgroup up to 2048 tiles, three above, each tile's range from a look-back over the tiles
# published before it)

def tiles_of(b: bytes) -> int:
    return ((len(b) - 8) // 2 + 2047) // 2048


@pytest.mark.parametrize("target", [1, 2, 63, 64, 65, 2047, 2048, 2049, 2050, 3001, 4096])
def test_async_lift_one_launch_at_tile_counts(target):
    """Tile counts at the one-launch form's edges (chunks of 64 tiles, one and three tiles per
    workgroup, the last tile ragged or whole): not refused, bit-exact."""
    rng = np.random.default_rng(1000 + target)
    # ~6.5 units a record (lengths 1-4): enough records to fill `target` tiles, the last one partly
    nrec = max(1, int((target - 0.5) * 2048 / 6.5))
    b, total = pattern_stream(rng, nrec, (1, 15), (1, 4))
    assert abs(tiles_of(b) - target) <= 1
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    out, ticket, refused = lift_async(b, total + 3, status)
    assert not refused
    assert_bitexact(out[:total].cpu().numpy(), O.grad_lift(b, cap=total))
    assert torch.all(out[total:] == 6.0)  # nothing written past the stream's total


@pytest.mark.parametrize("where", [0.02, 0.4, 0.7, 0.99])
def test_async_lift_one_launch_refuses_a_late_fault(where):
    """A zero-length run in a tile of the first, second or third stripe of a three-tiles-per-workgroup
    launch: the call is refused (every other tile still publishes, nobody waits forever)."""
    rng = np.random.default_rng(77)
    b, total = pattern_stream(rng, 900_000, (1, 15), (1, 4))
    assert 2048 < tiles_of(b) <= 4096
    bb = bytearray(b)
    heads = header_positions(b, 900_000)
    rec = heads[int(where * (len(heads) - 2))]
    ln = int.from_bytes(bb[rec + 4:rec + 8], "little")
    bb[rec + 8 + 2 * ln:rec + 8 + 2 * ln] = np.array([2, 0], np.uint32).tobytes()
    total += 2
    bb[:8] = np.uint64(total).tobytes()
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    _, _, refused = lift_async(bytes(bb), total, status)
    assert refused


def test_async_lift_of_an_unaligned_stream():
    """A stream at a 2-B (not 8-B) boundary takes the two-launch form: exact, not refused."""
    rng = np.random.default_rng(31)
    b, total = pattern_stream(rng, 700_000, (1, 15), (1, 4))
    raw = torch.zeros(len(b) + 8, dtype=torch.uint8, device="cuda")
    raw[2:2 + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()
    buf = raw[2:2 + len(b)]
    assert buf.data_ptr() % 8 == 2
    out = torch.empty(total, dtype=torch.float32, device="cuda")
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    ticket = SP.grad_lift_dev_async(buf, out, status)
    torch.cuda.synchronize()
    assert int(status.item()) != ticket
    assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


def test_async_lift_one_launch_back_to_back_sizes():
    """One-launch lifts of different tile counts queued back to back on one stream (the chunk lines
    alternate between two arrays, each zeroed by the launch before): all exact."""
    rng = np.random.default_rng(44)
    jobs = []
    for nrec in (700_000, 30_000, 1_200_000, 5_000, 900_000, 700_000):
        b, total = pattern_stream(rng, nrec, (1, 15), (1, 4))
        buf, out = to_dev(b), torch.empty(total, dtype=torch.float32, device="cuda")
        st = torch.zeros(1, dtype=torch.int64, device="cuda")
        jobs.append((b, total, buf, out, st))
    torch.cuda.synchronize()
    tickets = [SP.grad_lift_dev_async(buf, out, st) for _, _, buf, out, st in jobs]
    torch.cuda.synchronize()
    for (b, total, _, out, st), tk in zip(jobs, tickets):
        assert int(st.item()) != tk
        assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


def test_async_lift_one_launch_after_an_over_cap_lift():
    """an over-cap one-launch lift returns before its workgroups reach the end of the
    kernel, where the next launch's chunk lines are zeroed; the host flips the pair anyway.  Queued on
    one stream (the default one, as the other one-launch tests): a lift of > 64 tiles (its counts land
    in one array of the pair), an over-cap lift (uses the other, must zero the first), then another lift
    of > 64 tiles of the same shape (uses the first again).  The third must not see the first one's
    complete chunk counts: exact and not refused; the over-cap one refused, g untouched."""
    rng = np.random.default_rng(4242)
    jobs = []
    for k in range(3):
        b, total = pattern_stream(rng, 700_000, (1, 15), (1, 4))
        assert 64 < tiles_of(b) <= 4096
        cap = total - 1 if k == 1 else total
        buf = to_dev(b)
        out = torch.full((cap + 8,), 3.0, dtype=torch.float32, device="cuda")
        st = torch.zeros(1, dtype=torch.int64, device="cuda")
        jobs.append((b, total, cap, buf, out, st))
    torch.cuda.synchronize()
    tickets = [SP.grad_lift_dev_async(buf, out[:cap], st) for _, _, cap, buf, out, st in jobs]
    torch.cuda.synchronize()
    for k, ((b, total, cap, _, out, st), tk) in enumerate(zip(jobs, tickets)):
        if k == 1:
            assert int(st.item()) == tk
            assert torch.all(out == 3.0)
        else:
            assert int(st.item()) != tk, f"lift {k} refused"
            assert_bitexact(out[:total].cpu().numpy(), O.grad_lift(b, cap=total))


def same_size_stream(rng, units: int, total: int) -> bytes:
    """A drop-shaped stream of exactly `units` u16 after the total and the given total: records of
    lengths 1-4 until the units are filled (the last record's length takes the rest), offsets 1-15
    lowered where needed to fit the total, the rest of the total as the tail."""
    lens = []
    left = units
    while left >= 9:
        ln = int(rng.integers(1, 5))
        if left - (4 + ln) < 5 and left - (4 + ln) != 0:
            ln = left - 4
        lens.append(ln)
        left -= 4 + ln
    if left:
        lens.append(left - 4)  # (left >= 5 here)
    lens = np.array(lens, np.int64)
    offs = rng.integers(1, 16, lens.size).astype(np.int64)
    excess = int(offs.sum() + lens.sum()) - total
    if excess > 0:  # lower offsets towards 1
        room = offs - 1
        take = np.minimum(room, np.ceil(room * excess / max(int(room.sum()), 1)).astype(np.int64))
        offs -= take
        extra = int(offs.sum() + lens.sum()) - total
        i = 0
        while extra > 0:
            if offs[i] > 1:
                offs[i] -= 1
                extra -= 1
            i = (i + 1) % offs.size
    assert offs.min() >= 1 and int(offs.sum() + lens.sum()) <= total
    u_units = 4 + lens
    starts = np.concatenate([[0], np.cumsum(u_units)[:-1]])
    u = rng.integers(1, 0x7C00, int(u_units.sum())).astype(np.uint16)
    u |= rng.integers(0, 2, u.size).astype(np.uint16) << 15
    u[starts], u[starts + 1] = offs & 0xFFFF, offs >> 16
    u[starts + 2], u[starts + 3] = lens & 0xFFFF, lens >> 16
    assert u.size == units
    return np.uint64(total).tobytes() + u.tobytes()


def test_async_lift_under_graph_capture_replays_new_streams():
    """Captured in a graph (the epoch frozen at capture), the stream-ordered lift takes the two launches,
    which carry no per-call state: replays over new stream contents of the same length stay exact."""
    rng = np.random.default_rng(88)
    b, total = pattern_stream(rng, 700_000, (1, 15), (1, 4))
    buf = to_dev(b)
    out = torch.empty(total, dtype=torch.float32, device="cuda")
    st = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        SP.grad_lift_dev_async(buf, out, st)  # scratch allocated before the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        ticket = SP.grad_lift_dev_async(buf, out, st)
    for k in range(3):  # other records (the tiles' sums and links all change), the same length and total
        b2 = same_size_stream(np.random.default_rng(500 + k), (len(b) - 8) // 2, total)
        assert len(b2) == len(b) and b2[:8] == b[:8] and b2 != b
        buf.copy_(torch.frombuffer(bytearray(b2), dtype=torch.uint8).cuda())
        st.zero_()
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        assert int(st.item()) != ticket
        assert_bitexact(out.cpu().numpy(), O.grad_lift(b2, cap=total))


def test_async_lifts_of_large_streams_on_two_streams_concurrently():
    """Two lifts whose one-launch grids would each need most of the device, queued on two streams at
    once: the second takes the two launches while the first may still run, so neither waits on slots
    the other holds — both exact and not refused."""
    rng = np.random.default_rng(61)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    prep = []
    for k in range(4):
        b, total = pattern_stream(rng, 1_150_000 + 10_000 * k, (1, 15), (1, 4))
        assert 3 * 1536 // 2 < tiles_of(b) <= 4096
        prep.append((b, total, to_dev(b), torch.empty(total, dtype=torch.float32, device="cuda"),
                     torch.zeros(1, dtype=torch.int64, device="cuda")))
    torch.cuda.synchronize()
    jobs = [(b, total, out, st, SP.grad_lift_dev_async(buf, out, st, s1 if k % 2 == 0 else s2))
            for k, (b, total, buf, out, st) in enumerate(prep)]
    torch.cuda.synchronize()
    for b, total, out, st, tk in jobs:
        assert int(st.item()) != tk
        assert_bitexact(out.cpu().numpy(), O.grad_lift(b, cap=total))


def test_async_lift_one_launch_with_cu_slots_held_by_another_process():
    """the one-launch lift needs its whole grid resident (tiles wait on tiles of other
    workgroups).  Another process holds three quarters of the CUs (every LDS byte of each) for 400 ms
    while a ~4000-tile lift (~1350 workgroups of three tiles) is queued: the workgroups that start count
    themselves in, find the count stalled short of the grid for ~100 us and give the call up; the rest
    start in the freed slots, see the refusal and end.  So the call is refused quickly instead of polling ~10 ms per wave
    (and waiting for the other process), and the blocking lift that follows is exact."""
    import os
    import subprocess
    import time
    hog = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "cu_hog")
    if not os.path.exists(hog):
        pytest.skip("tests/native/cu_hog not built")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(4096)
    b, total = pattern_stream(rng, 1_280_000, (1, 15), (1, 4))
    assert 3900 <= tiles_of(b) <= 4096
    buf = to_dev(b)
    out = torch.full((total + 8,), 3.0, dtype=torch.float32, device="cuda")
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    p = subprocess.Popen([hog, str(3 * cus // 4), "400"], stdout=subprocess.PIPE, text=True)
    try:
        assert p.stdout.readline().startswith("running")
        t0 = time.perf_counter()
        ticket = SP.grad_lift_dev_async(buf, out[:total], status)
        torch.cuda.synchronize()
        took = time.perf_counter() - t0
        refused = int(status.item()) == ticket
        if refused:
            out[:total] = SP.grad_lift_dev(buf, total)
        assert p.poll() is None, "the other process ended before the lift (timing void)"
    finally:
        p.wait(timeout=30)
    assert_bitexact(out[:total].cpu().numpy(), O.grad_lift(b, cap=total))
    print(f"lift with 3/4 of the CUs held elsewhere: {took * 1e3:.2f} ms, refused={refused}")
    assert took < 0.005, f"the one-launch lift took {took * 1e3:.1f} ms while CU slots were held elsewhere"


def test_stream_lift_one_launch_after_another_streams_lift():
    """A stream-ordered lift made while its stream was the device's only lifting one is not recorded; once
    another stream lifts, that launch must not keep counting as running (round 6's late session: every
    64 MiB lift of the bench's codec leg then took the two launches, 1.07 instead of 0.023 ms).  After a lift
    on stream A and 60 ms, twelve back-to-back lifts on stream B run at the one-launch rate, and are exact."""
    n = 1 << 24
    g = O.synth(n, SEED + 57, 2)
    t = max(float(np.quantile(np.abs(g), 0.9)), 6.103515625e-05)
    wire = SP.grad_drop_dev(dev(g), t)
    want = O.grad_lift(bytes(wire.cpu().numpy()), cap=n)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3)]
    st = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    SP.grad_lift_dev_async(wire, outs[0], st, sa)
    torch.cuda.synchronize()
    import time
    time.sleep(0.06)
    for i in range(4):  # (warm: the stream's scratch)
        SP.grad_lift_dev_async(wire, outs[i % 3], st, sb)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(sb)
    tickets = [SP.grad_lift_dev_async(wire, outs[i % 3], st, sb) for i in range(12)]
    e1.record(sb)
    e1.synchronize()
    per_ms = e0.elapsed_time(e1) / 12
    assert int(st.item()) != tickets[-1]  # not refused
    assert_bitexact(outs[11 % 3].cpu().numpy(), want)
    assert per_ms < 0.3, per_ms  # one launch: ~0.023 ms; the two launches measured 1.07
