"""Exchange plans: the N > 1 schedules as data (ono_plan_*, ono_plan.cpp).

The RCCL schedules of pull_grads (ALLREDUCE + segments, HOPS, DIRECT) and of
the sharded PS step are built per rank by pure host functions and executed by
one interpreter in the library; these wrappers hand the same step lists to
Python so tests can check and run them without GPUs.
"""
from __future__ import annotations

import ctypes as C

from ._lib import ALGO, WIRE, PlanStep, call
from . import kernels

KIND = ("group_begin", "send", "recv", "group_end", "allreduce", "reduce_scatter", "all_gather", "kernel",
        "memset", "copy", "fork", "join")
OP = ("encode_zero", "add_encode_zero", "add_finish", "decode_scale", "direct", "scale_zero", "opt_update")
BUF = ("residual", "grad", "wire0", "wire1", "rbuf", "gstage", "msg", "gin", "gpad", "gshard", "ppad", "params")


def _steps(fn, *args) -> list[dict]:
    n = C.c_size_t(0)
    call(fn, *args, None, 0, C.byref(n))
    arr = (PlanStep * max(n.value, 1))()
    call(fn, *args, arr, n.value, C.byref(n))
    out = []
    for st in arr[: n.value]:
        refs = [(BUF[st.buf[i]] if st.buf[i] >= 0 else None, int(st.off[i])) for i in range(st.nref)]
        out.append({"kind": KIND[st.kind], "op": OP[st.op] if st.kind == 7 else None, "peer": st.peer,
                    "dtype": "f16" if st.dtype == 1 else "f32", "stream": st.stream, "flag": st.flag,
                    "divisor": st.divisor, "count": int(st.count), "refs": refs})
    return out


def pull_grads(algo: str, wire: str, pos: int, nranks: int, size: int, segments: int = 1) -> list[dict]:
    return _steps("ono_plan_pull_grads", ALGO[algo], WIRE[wire], pos, nranks, size, segments)


def pull_grads_sub(algo: str, wire: str, pos: int, nranks: int, size: int, sub_elems: int, j: int) -> list[dict]:
    """Sub-round j of a host-fed HOPS / DIRECT round (ono_plan_pull_grads_sub)."""
    return _steps("ono_plan_pull_grads_sub", ALGO[algo], WIRE[wire], pos, nranks, size, sub_elems, j)


def sub_rounds(nranks: int, size: int, sub_elems: int) -> int:
    from ._lib import lib
    return int(lib().ono_plan_sub_rounds(nranks, size, sub_elems))


def ps_step(pos: int, nranks: int, nparams: int) -> list[dict]:
    return _steps("ono_plan_ps_step", pos, nranks, nparams)


def buffers(nranks: int, size: int, nparams: int = 0) -> dict:
    c = (C.c_uint64 * len(BUF))()
    call("ono_plan_buffers", nranks, size, nparams, c)
    return {BUF[i]: int(c[i]) for i in range(len(BUF))}


def _ptrs(ts):
    return (C.c_void_p * len(ts))(*[kernels.f32_ptr(t) for t in ts])


def run_local(algo: str, wire: str, residuals, grads, segments: int = 1, stream=None) -> None:
    """Every rank's pull_grads plan run by co-resident ranks on one device
    (ono_plan_run_local): the N > 1 schedules' device work without RCCL."""
    n = len(residuals)
    size = residuals[0].numel()
    call("ono_plan_run_local", ALGO[algo], WIRE[wire], n, size, segments, _ptrs(residuals), _ptrs(grads),
         kernels.stream_handle(stream))


def run_local_sub(algo: str, wire: str, residuals, grads, sub_elems: int, stream=None) -> None:
    """The host-fed sub-rounds (ono_plan_run_local_sub) by co-resident ranks."""
    n = len(residuals)
    size = residuals[0].numel()
    call("ono_plan_run_local_sub", ALGO[algo], WIRE[wire], n, size, sub_elems, _ptrs(residuals), _ptrs(grads),
         kernels.stream_handle(stream))


def run_local_ps(grads, params, shards, opt, step_size: float = 0.0, v=None, s=None, stream=None) -> None:
    """ono_ps_step's plan for co-resident ranks (ono_plan_run_local_ps); opt
    is an ono_amd optimizer (its spec()), shards / v / s are per-rank shard
    tensors updated in place."""
    n = len(grads)
    nul = (C.c_void_p * n)()
    call("ono_plan_run_local_ps", n, grads[0].numel(), _ptrs(grads), _ptrs(params), _ptrs(shards),
         _ptrs(v) if v is not None else nul, _ptrs(s) if s is not None else nul, C.byref(opt.spec()),
         float(step_size), kernels.stream_handle(stream))
