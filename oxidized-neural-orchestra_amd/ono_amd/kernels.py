"""Elementwise kernels of the reduction path, on device tensors.

Thin wrappers over the C-ABI (include/ono_reduce.h); torch is only used to
hold device memory and to name the HIP stream.  Each function launches one
gfx950 kernel of libono_reduce.so on `stream` (default: torch's current
stream) and returns immediately (stream-ordered).
"""
from __future__ import annotations

import ctypes as C

import torch

from ._lib import MAX_INPUTS, call


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def f32_ptr(t: torch.Tensor) -> int:
    if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
        raise ValueError("expected a contiguous float32 device tensor")
    return t.data_ptr()


def u16_ptr(t: torch.Tensor) -> int:
    if not (t.is_cuda and t.dtype in (torch.int16, torch.uint16) and t.is_contiguous()):
        raise ValueError("expected a contiguous 16-bit device tensor (f16 wire bits)")
    return t.data_ptr()


def sum_scale(out: torch.Tensor, ins: list[torch.Tensor], divisor: float = 1.0, stream=None) -> torch.Tensor:
    """out = (((ins[0] + ins[1]) + ...) / divisor — worker_ring.rs:141-143 + param_manager.rs:183-188."""
    k = len(ins)
    if not 1 <= k <= MAX_INPUTS:
        raise ValueError(f"1 <= k <= {MAX_INPUTS}")
    n = out.numel()
    if any(x.numel() != n for x in ins):
        raise ValueError("all buckets must have the same length")
    arr = (C.c_void_p * k)(*[f32_ptr(x) for x in ins])
    call("ono_sum_scale_f32", f32_ptr(out), arr, k, n, float(divisor), stream_handle(stream))
    return out


def direct_chain(grad: torch.Tensor, out, ins: list[torch.Tensor], divisor: float, wire: str = "f32",
                 zero_all: bool = False, stream=None) -> torch.Tensor:
    """The DIRECT / XGMI owner's fused chain (worker_ring.rs:122-143, :166,
    :101-105): p = ins[0]; p = ins[j] + wire(p); grad = p / divisor; out =
    f16(p) (f16 wire) or grad (f32 wire) when given; the last input (or all,
    zero_all) zeroed."""
    k = len(ins)
    if not 1 <= k <= MAX_INPUTS:
        raise ValueError(f"1 <= k <= {MAX_INPUTS}")
    n = grad.numel()
    if any(x.numel() != n for x in ins) or (out is not None and out.numel() != n):
        raise ValueError("all operands must have the same length")
    if out is not None and out.element_size() != (2 if wire == "f16" else 4):
        raise ValueError("out element size does not match the wire")
    arr = (C.c_void_p * k)(*[f32_ptr(x) for x in ins])
    optr = None if out is None else (u16_ptr(out) if wire == "f16" else f32_ptr(out))
    call("ono_direct_chain", f32_ptr(grad), optr, arr, k, n, float(divisor),
         1 if wire == "f16" else 0, int(zero_all), stream_handle(stream))
    return grad


def acc(acc: torch.Tensor, x: torch.Tensor, stream=None) -> torch.Tensor:
    """acc += x — ParamManager::acc_residual (param_manager.rs:191-197)."""
    if acc.numel() != x.numel():
        raise ValueError("length mismatch")
    call("ono_acc_f32", f32_ptr(acc), f32_ptr(x), acc.numel(), stream_handle(stream))
    return acc


def scale_zero(dst: torch.Tensor, src: torch.Tensor, divisor: float, zero: torch.Tensor | None = None,
               stream=None) -> torch.Tensor:
    """dst = src / divisor (copy for 1), then zero[:] = 0."""
    n = dst.numel()
    if src.numel() != n or (zero is not None and zero.numel() != n):
        raise ValueError("length mismatch")
    call("ono_scale_zero_f32", f32_ptr(dst), f32_ptr(src), n, float(divisor),
         f32_ptr(zero) if zero is not None else None, stream_handle(stream))
    return dst


def copy(dst: torch.Tensor, src: torch.Tensor, stream=None) -> torch.Tensor:
    """dst = src — the library's own 1R1W stream (no overlap)."""
    if src.numel() != dst.numel():
        raise ValueError("length mismatch")
    call("ono_copy_f32", f32_ptr(dst), f32_ptr(src), dst.numel(), stream_handle(stream))
    return dst


def fill(dst: torch.Tensor, value: float = 0.0, stream=None) -> torch.Tensor:
    """dst[:] = value — the library's own write-only stream."""
    call("ono_fill_f32", f32_ptr(dst), float(value), dst.numel(), stream_handle(stream))
    return dst


def f16_encode(out: torch.Tensor, x: torch.Tensor, stream=None) -> torch.Tensor:
    call("ono_f16_encode", u16_ptr(out), f32_ptr(x), x.numel(), stream_handle(stream))
    return out


def f16_decode(out: torch.Tensor, h: torch.Tensor, stream=None) -> torch.Tensor:
    call("ono_f16_decode", f32_ptr(out), u16_ptr(h), h.numel(), stream_handle(stream))
    return out


def f16_encode_zero(out: torch.Tensor, chunk: torch.Tensor, stream=None) -> torch.Tensor:
    call("ono_f16_encode_zero", u16_ptr(out), f32_ptr(chunk), chunk.numel(), stream_handle(stream))
    return out


def f16_decode_add(acc: torch.Tensor, h: torch.Tensor, stream=None) -> torch.Tensor:
    call("ono_f16_decode_add", f32_ptr(acc), u16_ptr(h), acc.numel(), stream_handle(stream))
    return acc


def f16_add_encode_zero(out: torch.Tensor, acc: torch.Tensor, h: torch.Tensor, stream=None) -> torch.Tensor:
    call("ono_f16_add_encode_zero", u16_ptr(out), f32_ptr(acc), u16_ptr(h), acc.numel(), stream_handle(stream))
    return out


def f16_decode_scale(out: torch.Tensor, h: torch.Tensor, divisor: float, stream=None) -> torch.Tensor:
    call("ono_f16_decode_scale", f32_ptr(out), u16_ptr(h), h.numel(), float(divisor), stream_handle(stream))
    return out


def synth(out: torch.Tensor, seed: int, rank: int, offset: int = 0, stream=None) -> torch.Tensor:
    """Fill with the §8(d) synthetic gradient distribution (bit-identical to the oracle's)."""
    call("ono_synth_f32", f32_ptr(out), out.numel(), int(seed), int(rank), int(offset), stream_handle(stream))
    return out
