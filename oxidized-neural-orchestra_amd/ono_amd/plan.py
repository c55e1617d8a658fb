"""Exchange plans: the N > 1 schedules as data (ono_plan_*, ono_plan.cpp).

The RCCL schedules of pull_grads (ALLREDUCE + segments, HOPS, DIRECT) and of
the sharded PS step are built per rank by pure host functions and executed by
one interpreter in the library; these wrappers hand the same step lists to
Python so tests can check and run them without GPUs.
"""
from __future__ import annotations

import ctypes as C

from ._lib import ALGO, WIRE, PlanStep, call

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


def ps_step(pos: int, nranks: int, nparams: int) -> list[dict]:
    return _steps("ono_plan_ps_step", pos, nranks, nparams)


def buffers(nranks: int, size: int, nparams: int = 0) -> dict:
    c = (C.c_uint64 * len(BUF))()
    call("ono_plan_buffers", nranks, size, nparams, c)
    return {BUF[i]: int(c[i]) for i in range(len(BUF))}
