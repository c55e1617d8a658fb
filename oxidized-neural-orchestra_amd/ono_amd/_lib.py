"""ctypes binding of libono_reduce.so (include/ono_reduce.h).

The library is the product: every call here goes straight to the HIP/RCCL
code.  There is no fallback — if the shared object is missing or fails to
load, importing ono_amd raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libono_reduce.so")
HEADER = os.path.normpath(os.path.join(HERE, "..", "..", "include", "ono_reduce.h"))

(ONO_OK, ONO_E_SIZE, ONO_E_PROTO, ONO_E_HIP, ONO_E_RCCL, ONO_E_ABORTED, ONO_E_ARG, ONO_E_OTHER,
 ONO_E_IO) = range(9)
WIRE = {"f32": 0, "f16": 1}
ALGO = {"auto": 0, "allreduce": 1, "hops": 2, "direct": 3, "xgmi": 4}
OPT_KIND = {"gd": 0, "momentum": 1, "adam": 2, "add": 3}
STORE_KIND = {"blocking": 0, "wild": 1}
SYNC_KIND = {"barrier": 0, "nonblocking": 1}
UID_BYTES = 128
XGMI_HANDLE_BYTES = 128
MAX_INPUTS = 16
PHASES = ("kernel", "rccl", "xgmi_scatter", "xgmi_barrier", "xgmi_gather", "sparse_codec")  # ono_phase


class OnoError(RuntimeError):
    """Base error; `.code` is the ono_status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[ono {code}] {msg}")
        self.code = code


class SizeMismatch(OnoError):
    """ParamServerErr::SizeMismatch (parameter_server/src/storage/error.rs:13-17)."""


class InvalidWorkerEvent(OnoError):
    """io::Error "Received an invalid worker event" (worker_ring.rs:136-138)."""


class HipError(OnoError):
    pass


class RcclError(OnoError):
    pass


class Aborted(OnoError):
    pass


class InvalidArgument(OnoError, ValueError):
    pass


class IoError(OnoError, OSError):
    """Socket failure on a TCP ring (the reference's io::Error from comms/)."""


_ERR = {ONO_E_SIZE: SizeMismatch, ONO_E_PROTO: InvalidWorkerEvent, ONO_E_HIP: HipError,
        ONO_E_RCCL: RcclError, ONO_E_ABORTED: Aborted, ONO_E_ARG: InvalidArgument,
        ONO_E_IO: IoError}


PLAN_REFS = MAX_INPUTS + 2


class PlanStep(C.Structure):
    """ono_plan_step (include/ono_reduce.h): one step of an exchange plan."""
    _fields_ = [("kind", C.c_int32), ("op", C.c_int32), ("peer", C.c_int32), ("dtype", C.c_int32),
                ("stream", C.c_int32), ("nref", C.c_int32), ("flag", C.c_int32), ("divisor", C.c_float),
                ("count", C.c_uint64), ("buf", C.c_int32 * PLAN_REFS), ("off", C.c_uint64 * PLAN_REFS)]


class OptSpec(C.Structure):
    _fields_ = [("kind", C.c_int), ("lr", C.c_float), ("momentum", C.c_float),
                ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float)]


LEADER_FN = C.CFUNCTYPE(None, C.c_void_p)
# ono_sample_fn: int (*)(void *ctx, size_t len, uint32_t *idx, size_t amount)
SAMPLE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_uint32), C.c_size_t)

_vp, _fp, _sz, _i, _u64 = C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_uint64

# name -> (restype, argtypes)
_SIGS = {
    "ono_last_error": (C.c_char_p, []),
    "ono_abi_version": (_i, []),
    "ono_device_count": (_i, [C.POINTER(C.c_int)]),
    "ono_sum_scale_f32": (_i, [_fp, C.POINTER(C.c_void_p), _i, _sz, C.c_float, _vp]),
    "ono_acc_f32": (_i, [_fp, _fp, _sz, _vp]),
    "ono_scale_zero_f32": (_i, [_fp, _fp, _sz, C.c_float, _fp, _vp]),
    "ono_copy_f32": (_i, [_fp, _fp, _sz, _vp]),
    "ono_fill_f32": (_i, [_fp, C.c_float, _sz, _vp]),
    "ono_f16_encode": (_i, [_vp, _fp, _sz, _vp]),
    "ono_f16_decode": (_i, [_fp, _vp, _sz, _vp]),
    "ono_f16_encode_zero": (_i, [_vp, _fp, _sz, _vp]),
    "ono_f16_decode_add": (_i, [_fp, _vp, _sz, _vp]),
    "ono_f16_add_encode_zero": (_i, [_vp, _fp, _vp, _sz, _vp]),
    "ono_f16_decode_scale": (_i, [_fp, _vp, _sz, C.c_float, _vp]),
    "ono_synth_f32": (_i, [_fp, _sz, _u64, _u64, _sz, _vp]),
    "ono_direct_chain": (_i, [_fp, _vp, C.POINTER(C.c_void_p), _i, _sz, C.c_float, _i, _i, _vp]),
    "ono_sparse_max_bytes": (_sz, [_sz]),
    "ono_sparse_drop": (_i, [_vp, _sz, C.POINTER(C.c_size_t), _fp, _sz, C.c_float, _vp]),
    "ono_sparse_drop_async": (_i, [_vp, _sz, _vp, _fp, _sz, C.c_float, _vp]),
    "ono_sparse_drop_check": (_i, [_vp]),
    "ono_sparse_drop_debug_stale": (_i, [_vp, C.c_uint32]),
    "ono_sparse_lift": (_i, [_fp, _sz, C.POINTER(C.c_size_t), _vp, _sz, _vp]),
    "ono_sparse_lift_dev": (_i, [_fp, _sz, C.POINTER(C.c_size_t), _vp, _sz, _vp]),
    "ono_sparse_lift_fallbacks": (_sz, []),
    "ono_sparse_lift_debug_refuse": (_i, [C.c_uint32]),
    "ono_sparse_lift_pattern_misses": (_sz, []),
    "ono_sparse_lift_dev_async": (_i, [_fp, _sz, _vp, _sz, _vp, C.POINTER(C.c_uint64), _vp]),
    "ono_sparse_lift_set_mode": (_i, [_i]),
    "ono_sparse_mask": (_i, [_fp, _sz, C.c_float, _i, _vp]),
    "ono_sparse_threshold": (_i, [C.POINTER(C.c_float), _fp, _sz, _vp, _sz, C.c_float, _vp]),
    "ono_sparse_sample_default": (_i, [C.POINTER(C.c_uint64), _sz, _vp, _sz]),
    "ono_ring_set_sparse": (_i, [_vp, C.c_float, _u64]),
    "ono_worker_event_check": (_i, [C.c_uint32, C.c_char_p, _sz]),
    "ono_ring_set_sampler": (_i, [_vp, _vp, _vp]),
    "ono_ring_unique_id": (_i, [C.c_char_p]),
    "ono_ring_create": (_i, [C.POINTER(C.c_void_p), _i, _i, _sz, _i, C.c_char_p, _i]),
    "ono_ring_create_tcp": (_i, [C.POINTER(C.c_void_p), _i, _i, _sz, _i, _i, _i]),
    "ono_ring_create_xgmi": (_i, [C.POINTER(C.c_void_p), _i, _i, _sz, _i, _i]),
    "ono_ring_xgmi_handle": (_i, [_vp, C.c_char_p]),
    "ono_ring_xgmi_connect": (_i, [_vp, C.c_char_p]),
    "ono_ring_set_xgmi_timeout": (_i, [_vp, C.c_double]),
    "ono_xgmi_pool_release": (_i, [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "ono_xgmi_pool_close_imports": (_i, [C.POINTER(C.c_size_t)]),
    "ono_xgmi_pool_free_exports": (_i, [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t), C.c_double]),
    "ono_xgmi_pool_stats": (_i, [C.POINTER(C.c_size_t)] * 4),
    "ono_ring_check": (_i, [_vp]),
    "ono_ring_destroy": (_i, [_vp]),
    "ono_ring_set_pipeline": (_i, [_vp, _i]),
    "ono_ring_grad": (C.c_void_p, [_vp]),
    "ono_ring_residual": (C.c_void_p, [_vp]),
    "ono_ring_size": (_sz, [_vp]),
    "ono_ring_acc_residual": (_i, [_vp, _fp, _vp]),
    "ono_ring_pull_grads": (_i, [_vp, _vp]),
    "ono_ring_pull_grads_dev": (_i, [_vp, _fp, _fp, _sz, _vp]),
    "ono_ring_pull_grads_host": (_i, [_vp, _fp, _fp, _sz]),
    "ono_ring_register_host": (_i, [_vp, _vp, _sz]),
    "ono_ring_unregister_host": (_i, [_vp, _vp]),
    "ono_ring_allreduce_avg_dev": (_i, [_vp, _fp, _sz, _vp]),
    "ono_ring_set_algo": (_i, [_vp, _i]),
    "ono_ring_abort": (_i, [_vp]),
    "ono_ring_timing_enable": (_i, [_vp, _i]),
    "ono_ring_timing_read": (_i, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                  C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "ono_ring_timing_phases": (_i, [_vp, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "ono_local_ring_pull_grads": (_i, [C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), _i, _sz, _i, _vp]),
    "ono_local_direct_pull_grads": (_i, [C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), _i, _sz, _i, _vp]),
    "ono_optimizer_create": (_i, [C.POINTER(C.c_void_p), C.POINTER(OptSpec), _sz, _i]),
    "ono_optimizer_destroy": (_i, [_vp]),
    "ono_optimizer_step": (_i, [_vp, _fp, _fp, _fp, _sz, _vp]),
    "ono_store_create":(_i, [C.POINTER(C.c_void_p), _i, _fp, _sz, _sz, _sz, C.POINTER(OptSpec), _i]),
    "ono_store_destroy": (_i, [_vp]),
    "ono_store_len": (_sz, [_vp]),
    "ono_store_accumulate": (_i, [_vp, _fp, _sz]),
    "ono_store_accumulate_dev": (_i, [_vp, _fp, _sz]),
    "ono_store_accumulate_f16": (_i, [_vp, _vp, _sz]),
    "ono_store_accumulate_f16_dev": (_i, [_vp, _vp, _sz]),
    "ono_store_update_params": (_i, [_vp]),
    "ono_store_pull_params": (_i, [_vp, _fp, _sz]),
    "ono_store_pull_params_dev": (_i, [_vp, _fp, _sz]),
    "ono_store_active_idx": (_i, [_vp]),
    "ono_store_set_updating": (_i, [_vp, _i]),
    "ono_sync_create": (_i, [C.POINTER(C.c_void_p), _i, _sz]),
    "ono_sync_clone": (_i, [_vp]),
    "ono_sync_release": (_i, [_vp]),
    "ono_sync_step": (_i, [_vp, _vp, _fp, _fp, _sz]),
    "ono_sync_step_f16": (_i, [_vp, _vp, _vp, _fp, _sz]),
    "ono_barrier_create": (_i, [C.POINTER(C.c_void_p), _sz]),
    "ono_barrier_destroy": (_i, [_vp]),
    "ono_barrier_wait_with": (_i, [_vp, LEADER_FN, _vp]),
    "ono_barrier_acquire": (_i, [_vp]),
    "ono_ps_create": (_i, [C.POINTER(C.c_void_p), _vp, _fp, _sz, C.POINTER(OptSpec)]),
    "ono_ps_destroy": (_i, [_vp]),
    "ono_ps_step": (_i, [_vp, _fp, _fp, _vp]),
    "ono_plan_pull_grads": (_i, [_i, _i, _i, _i, _sz, _i, _vp, _sz, C.POINTER(C.c_size_t)]),
    "ono_plan_ps_step": (_i, [_i, _i, _sz, _vp, _sz, C.POINTER(C.c_size_t)]),
    "ono_plan_pull_grads_sub": (_i, [_i, _i, _i, _i, _sz, _sz, _sz, _vp, _sz, C.POINTER(C.c_size_t)]),
    "ono_plan_sub_rounds": (_sz, [_i, _sz, _sz]),
    "ono_plan_run_local_sub": (_i, [_i, _i, _i, _sz, _sz, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), _vp]),
    "ono_plan_buffers": (_i, [_i, _sz, _sz, C.POINTER(C.c_uint64)]),
    "ono_plan_run_local": (_i, [_i, _i, _i, _sz, _i, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), _vp]),
    "ono_plan_run_local_ps": (_i, [_i, _sz, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                   C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.POINTER(OptSpec), C.c_float, _vp]),
}

_lib = None


def header_functions() -> list[str]:
    """Every function declared in include/ono_reduce.h."""
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ono_[a-z0-9_]+)\s*\(", text)))


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `make -C oxidized-neural-orchestra_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.ono_abi_version() != 2:
            raise ImportError("libono_reduce.so ABI mismatch")
        _lib = L
    return _lib


def worker_event_check(kind: int, payload: bytes) -> None:
    """WorkerHandle::recv_event's verdict on one frame as the ring sees it
    (comms/src/handles/worker.rs:82-130): returns for a gradient, raises the
    reference's error class otherwise."""
    check(lib().ono_worker_event_check(kind, payload, len(payload)))


def check(rc: int) -> None:
    if rc != ONO_OK:
        msg = lib().ono_last_error().decode(errors="replace")
        raise _ERR.get(rc, OnoError)(rc, msg)


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args))
