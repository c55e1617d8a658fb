"""The sparse drop under HIP graph capture, and its writers' bounds (VERDICT r5
item 1).

grad_drop_into (comms/src/sparse/protocol.rs:57-86) grows its Vec, so it can
never write out of bounds; the device encoder writes into a caller's buffer at
offsets derived from chunk aggregates, so every writer checks its range against
the buffer and an aggregate that disagrees with its tile records is an error,
not a store.  The captured drop keeps its only state between calls — which of
the two aggregate arrays a call sums into — on the device, so a replayed graph
follows it as an uncaptured call does."""
import numpy as np
import pytest
import torch

import ono_amd
from ono_amd import sparse as SP
from conftest import SEED
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _buf(n):
    return torch.empty(ono_amd.lib().ono_sparse_max_bytes(n), dtype=torch.uint8, device="cuda")


def _fresh_stream():
    """A HIP stream no earlier test has used (hipStreamCreate; torch.cuda.Stream
    hands out pooled streams)."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    h = C.c_void_p()
    assert hip.hipStreamCreate(C.byref(h)) == 0
    return torch.cuda.ExternalStream(h.value)


def _wire(buf, nbd):
    nb = int(nbd.item())
    return bytes(buf[:nb].cpu().numpy())


@pytest.mark.parametrize("tiles", [300, 40])
def test_drop_async_captured_in_a_graph(tiles):
    """ono_sparse_drop_async captured in a HIP graph and replayed over new
    contents of the same gradient: every replay gives the oracle's bytes, and an
    uncaptured drop afterwards still does.  300 tiles: the two launches as
    uncaptured; 40 tiles: uncaptured the one launch, captured the two."""
    n = tiles * 2048 + 77
    rng = np.random.default_rng(SEED + 41)
    g = torch.empty(n, dtype=torch.float32, device="cuda")
    buf = _buf(n)
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
    t = 1.2
    s = torch.cuda.Stream()
    x = rng.standard_normal(n).astype(np.float32)
    g.copy_(torch.from_numpy(x))
    torch.cuda.synchronize()
    SP.grad_drop_async(g, t, buf, nbd, stream=s)
    s.synchronize()
    assert _wire(buf, nbd) == O.grad_drop(x, t)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        SP.grad_drop_async(g, t, buf, nbd, stream=s)
    for k in range(4):
        x = rng.standard_normal(n).astype(np.float32) * (1.0 + k)
        g.copy_(torch.from_numpy(x))
        nbd.zero_()
        torch.cuda.synchronize()
        gr.replay()
        torch.cuda.synchronize()
        assert _wire(buf, nbd) == O.grad_drop(x, t), f"replay {k}"
    SP.drop_check(s)
    x = rng.standard_normal(n).astype(np.float32)
    g.copy_(torch.from_numpy(x))
    torch.cuda.synchronize()
    SP.grad_drop_async(g, t, buf, nbd, stream=s)
    s.synchronize()
    assert _wire(buf, nbd) == O.grad_drop(x, t)
    # replays and uncaptured calls interleaved on the capture stream
    for k in range(3):
        x = rng.standard_normal(n).astype(np.float32)
        g.copy_(torch.from_numpy(x))
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            gr.replay()
        s.synchronize()
        assert _wire(buf, nbd) == O.grad_drop(x, t), f"interleaved replay {k}"
        SP.grad_drop_async(g, 0.7, buf, nbd, stream=s)
        s.synchronize()
        assert _wire(buf, nbd) == O.grad_drop(x, 0.7), f"interleaved call {k}"
    SP.drop_check(s)
    del gr


def test_drop_capture_refusals():
    """Under capture: the blocking drop and a drop whose scratch does not exist
    yet are refused (ONO_E_ARG) before anything is enqueued, and the capture
    goes on; an empty gradient is captured (the total alone)."""
    n = 300 * 2048
    g = torch.zeros(n, dtype=torch.float32, device="cuda")
    buf = _buf(n)
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = _fresh_stream()  # (torch's pooled streams may already carry a drop's scratch)
    e = torch.empty(0, dtype=torch.float32, device="cuda")
    b0 = _buf(0)
    nb0 = torch.full((1,), 99, dtype=torch.int64, device="cuda")
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        with pytest.raises(ono_amd.InvalidArgument, match="outside the capture"):
            SP.grad_drop_async(g, 0.5, buf, nbd, stream=s)
        with pytest.raises(ono_amd.InvalidArgument, match="blocking"):
            SP.grad_drop(g, 0.5, stream=s)
        SP.grad_drop_async(e, 0.5, b0, nb0, stream=s)
    b0.fill_(0xAB)
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    assert int(nb0.item()) == 8 and bytes(b0[:8].cpu().numpy()) == bytes(8)


@pytest.mark.parametrize("add", [3, 1 << 28])
def test_stale_aggregates_are_an_error_not_a_store(add):
    """Chunk aggregates that are not zero when the call begins (the hook adds
    `add` to every chunk's counts): small — the wire would be misplaced inside
    the buffer; huge — every later tile's range would pass the buffer's end.
    Either way nothing is stored past the buffer (its guard bytes keep their
    value), the blocking call raises IoError, the stream-ordered call's length
    reads ~0 for the huge case and drop_check raises; the next drop on the
    stream is exact again."""
    n = 300 * 2048 + 5
    rng = np.random.default_rng(SEED + 43)
    x = rng.standard_normal(n).astype(np.float32)
    g = torch.from_numpy(x).cuda()
    cap = ono_amd.lib().ono_sparse_max_bytes(n)
    guard = 1 << 20
    big = torch.full((cap + guard,), 0x5A, dtype=torch.uint8, device="cuda")
    buf = big[:cap]
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    want = O.grad_drop(x, 1.0)
    SP.grad_drop_async(g, 1.0, buf, nbd, stream=s)
    s.synchronize()
    assert _wire(buf, nbd) == want
    # stream-ordered
    SP.drop_debug_stale(add, stream=s)
    SP.grad_drop_async(g, 1.0, buf, nbd, stream=s)
    with pytest.raises(ono_amd.IoError, match="aggregates"):
        SP.drop_check(s)
    if add >= 1 << 20:
        assert int(nbd.item()) == -1  # ~0 as int64
    assert bool((big[cap:] == 0x5A).all()), "a store past the buffer"
    SP.drop_check(s)  # cleared
    SP.grad_drop_async(g, 1.0, buf, nbd, stream=s)
    s.synchronize()
    assert _wire(buf, nbd) == want
    # blocking (the two launches: above 256 tiles)
    SP.drop_debug_stale(add, stream=s)
    with pytest.raises(ono_amd.IoError, match="aggregates"):
        SP.grad_drop(g, 1.0, stream=s)
    assert bool((big[cap:] == 0x5A).all())
    assert SP.grad_drop(g, 1.0, stream=s) == want
    SP.drop_check(s)


def test_stale_aggregates_under_replay():
    """The hook between two replays of a captured drop: that replay is
    reported, the following one is exact (the device parity moved on)."""
    n = 280 * 2048 + 3
    rng = np.random.default_rng(SEED + 44)
    g = torch.empty(n, dtype=torch.float32, device="cuda")
    buf = _buf(n)
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.Stream()
    x = rng.standard_normal(n).astype(np.float32)
    g.copy_(torch.from_numpy(x))
    torch.cuda.synchronize()
    SP.grad_drop_async(g, 0.9, buf, nbd, stream=s)
    s.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        SP.grad_drop_async(g, 0.9, buf, nbd, stream=s)
    SP.drop_debug_stale(7, stream=s)
    with torch.cuda.stream(s):
        gr.replay()
    with pytest.raises(ono_amd.IoError):
        SP.drop_check(s)
    with torch.cuda.stream(s):
        gr.replay()
    SP.drop_check(s)
    assert _wire(buf, nbd) == O.grad_drop(x, 0.9)
