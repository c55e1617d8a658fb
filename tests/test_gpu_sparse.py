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
