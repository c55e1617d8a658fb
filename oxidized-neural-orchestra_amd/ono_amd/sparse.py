"""Sparse top-(1-r) gradient codec on the device (comms/src/sparse/protocol.rs).

grad_drop(g, threshold) -> bytes   (protocol.rs:57-86, byte-exact wire format)
grad_lift(buf) -> device tensor     (protocol.rs:96-144)
mask_sent / mask_unsent             (the ring's sparse bookkeeping, worker_ring.rs:128-131, 183-187)
The threshold is the caller's: the reference draws it from a rand 0.9.4 StdRng
sample (protocol.rs:33-49); for gradients of <= 16384 values that sample is
the whole gradient and `threshold_full` reproduces it exactly.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import kernels
from ._lib import call, lib

SAMPLE_SIZE_MAX = 1 << 14
MIN_POSITIVE_F16 = np.float32(6.103515625e-05)


def threshold_full(g: np.ndarray, r: float) -> float:
    """calculate_threshold for len(g) <= 16384 (sample = every value)."""
    g = np.asarray(g, dtype=np.float32)
    if g.size == 0:
        return 0.0
    if g.size > SAMPLE_SIZE_MAX:
        raise ValueError("above 16384 values the reference threshold depends on rand 0.9.4 StdRng sampling")
    a = np.sort(np.abs(g).view(np.uint32)).view(np.float32)   # total_cmp order of non-negative floats
    k = int(np.float32(g.size) * (np.float32(1.0) - np.float32(r)))
    k = min(max(k, 0), g.size - 1)
    return float(max(a[k], MIN_POSITIVE_F16))


def threshold(g: torch.Tensor, r: float, idx=None, stream=None) -> float:
    """calculate_threshold on the device (ono_sparse_threshold): over every
    value (len <= 16384, idx None) or the sample indices `idx` (<= 16384)."""
    n = g.numel()
    t = C.c_float()
    if idx is None:
        call("ono_sparse_threshold", C.byref(t), kernels.f32_ptr(g), n, None, n, float(r), kernels.stream_handle(stream))
    else:
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        call("ono_sparse_threshold", C.byref(t), kernels.f32_ptr(g), n, ix.ctypes.data, ix.size, float(r),
             kernels.stream_handle(stream))
    return t.value


def sample_default(state: int, length: int, amount: int) -> tuple[np.ndarray, int]:
    """The default threshold sampler (ono_sparse_sample_default): (indices,
    next state).  Host code — no device needed."""
    st = C.c_uint64(state & (2 ** 64 - 1))
    out = np.empty(amount, dtype=np.uint32)
    call("ono_sparse_sample_default", C.byref(st), length, out.ctypes.data if amount else None, amount)
    return out, st.value


def grad_drop(g: torch.Tensor, threshold: float, stream=None) -> bytes:
    n = g.numel()
    cap = lib().ono_sparse_max_bytes(n)
    buf = torch.empty(cap + 8, dtype=torch.uint8, device=g.device)
    nb = C.c_size_t(0)
    call("ono_sparse_drop", buf.data_ptr(), cap, C.byref(nb), kernels.f32_ptr(g), n, float(threshold),
         kernels.stream_handle(stream))
    return bytes(buf[: nb.value].cpu().numpy())


def grad_lift(buf, cap: int | None = None, device: str = "cuda", stream=None) -> torch.Tensor:
    """buf: the wire bytes (host) or a device uint8 tensor holding them."""
    if isinstance(buf, torch.Tensor) and buf.is_cuda:
        return grad_lift_dev(buf, cap, stream)
    b = np.frombuffer(bytes(buf), dtype=np.uint8)
    total = int.from_bytes(bytes(buf[:8]), "little") if len(buf) >= 8 else 0
    cap = total if cap is None else cap
    out = torch.empty(max(cap, 1), dtype=torch.float32, device=device)
    ln = C.c_size_t(0)
    call("ono_sparse_lift", kernels.f32_ptr(out), cap, C.byref(ln), b.ctypes.data if b.size else None, b.size,
         kernels.stream_handle(stream))
    torch.cuda.synchronize()
    return out[: ln.value]


def grad_drop_dev(g: torch.Tensor, threshold: float, stream=None) -> torch.Tensor:
    """grad_drop leaving the wire bytes in HBM (a uint8 device tensor)."""
    n = g.numel()
    cap = lib().ono_sparse_max_bytes(n)
    buf = torch.empty(cap + 8, dtype=torch.uint8, device=g.device)
    nb = C.c_size_t(0)
    call("ono_sparse_drop", buf.data_ptr(), cap, C.byref(nb), kernels.f32_ptr(g), n, float(threshold),
         kernels.stream_handle(stream))
    return buf[: nb.value]


def grad_drop_async(g: torch.Tensor, threshold: float, buf: torch.Tensor, nbytes: torch.Tensor,
                    stream=None) -> None:
    """Stream-ordered grad_drop (ono_sparse_drop_async): buf (uint8, at least
    ono_sparse_max_bytes(n)) receives the wire bytes and nbytes (one int64 on
    the device) their length, when the stream gets there; nothing waits."""
    n = g.numel()
    assert buf.is_cuda and buf.dtype == torch.uint8 and nbytes.is_cuda and nbytes.dtype == torch.int64
    call("ono_sparse_drop_async", buf.data_ptr(), buf.numel(), nbytes.data_ptr(), kernels.f32_ptr(g), n,
         float(threshold), kernels.stream_handle(stream))


def drop_check(stream=None) -> None:
    """ono_sparse_drop_check: synchronizes the stream and raises IoError if a
    stream-ordered drop on it found a range past its buffer or stale chunk
    aggregates (nothing was stored out of bounds either way)."""
    call("ono_sparse_drop_check", kernels.stream_handle(stream))


def drop_debug_stale(add: int, stream=None) -> None:
    """Test hook (ono_sparse_drop_debug_stale): the stream's next two-launch
    drop starts from chunk aggregates that are not zero."""
    call("ono_sparse_drop_debug_stale", kernels.stream_handle(stream), int(add))


def lift_debug_refuse(count: int) -> int:
    """Test hook (ono_sparse_lift_debug_refuse): the process's next `count`
    one-launch stream-ordered lifts are refused; 0 clears it.  Returns the
    refusals of the previous setting not yet taken."""
    return int(lib().ono_sparse_lift_debug_refuse(int(count)))


def grad_lift_dev(buf: torch.Tensor, cap: int | None = None, stream=None) -> torch.Tensor:
    """grad_lift of wire bytes already in HBM (ono_sparse_lift_dev)."""
    assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
    nb = buf.numel()
    if cap is None:
        cap = int.from_bytes(bytes(buf[:8].cpu().numpy()), "little") if nb >= 8 else 0
    out = torch.empty(max(cap, 1), dtype=torch.float32, device=buf.device)
    ln = C.c_size_t(0)
    call("ono_sparse_lift_dev", kernels.f32_ptr(out), cap, C.byref(ln), buf.data_ptr() if nb else None, nb,
         kernels.stream_handle(stream))
    return out[: ln.value]


def grad_lift_dev_async(buf: torch.Tensor, out: torch.Tensor, status: torch.Tensor, stream=None) -> int:
    """Stream-ordered grad_lift (ono_sparse_lift_dev_async) of wire bytes in HBM
    into out[0, total): returns the ticket; once the stream has passed the call,
    status (one int64 on the device) equals it iff the lift was refused (then
    use grad_lift_dev)."""
    assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
    assert status.is_cuda and status.dtype == torch.int64 and out.is_cuda and out.dtype == torch.float32
    ticket = C.c_uint64(0)
    call("ono_sparse_lift_dev_async", kernels.f32_ptr(out), out.numel(), buf.data_ptr(), buf.numel(),
         status.data_ptr(), C.byref(ticket), kernels.stream_handle(stream))
    return ticket.value


def mask_sent(g: torch.Tensor, threshold: float, stream=None) -> torch.Tensor:
    """Scatter side: the values just sent (|g| >= t) leave the residual."""
    call("ono_sparse_mask", kernels.f32_ptr(g), g.numel(), float(threshold), 1, kernels.stream_handle(stream))
    return g


def mask_unsent(g: torch.Tensor, threshold: float, stream=None) -> torch.Tensor:
    """Gather side: only the values that were sent (|g| >= t) stay."""
    call("ono_sparse_mask", kernels.f32_ptr(g), g.numel(), float(threshold), 0, kernels.stream_handle(stream))
    return g
