"""Parameter-server store and synchronizers, MI355X-native.

Mirrors parameter_server/src/storage (trait Store: len / accumulate /
update_params / pull_params; BlockingStore, WildStore) and
parameter_server/src/synchronization (BarrierSync, NoBlockingSync,
DynBarrier).  Gradients and parameters cross the API as host float32 arrays
(the reference receives them from comms/); the store itself lives in HBM.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np
import torch

from ._lib import LEADER_FN, OPT_KIND, STORE_KIND, SYNC_KIND, OptSpec, call, lib

SHARD_AMOUNT_FACTOR = 2  # parameter_server/src/service/builder.rs (shards = 2 x cores)


def shard_size_for(nparams: int, cores: int | None = None) -> int:
    """ServerBuilder::resolve_store sizing (builder.rs:164-173)."""
    cores = cores or os.cpu_count() or 1
    n = max(nparams, 1)
    shards = min(n, cores * SHARD_AMOUNT_FACTOR)
    return -(-n // shards)


# ------------------------------------------------------------- optimizers
@dataclass
class GradientDescent:  # optimization/gradient_descent.rs
    learning_rate: float

    def spec(self) -> OptSpec:
        return OptSpec(OPT_KIND["gd"], self.learning_rate, 0.0, 0.0, 0.0, 0.0)


@dataclass
class GradientDescentWithMomentum:  # optimization/gradient_descent_with_momentum.rs
    learning_rate: float
    momentum: float

    def spec(self) -> OptSpec:
        return OptSpec(OPT_KIND["momentum"], self.learning_rate, self.momentum, 0.0, 0.0, 0.0)


@dataclass
class Adam:  # optimization/adam.rs
    learning_rate: float
    beta1: float = 0.9
    beta2: float = 0.999
    epsilon: float = 1e-8

    def spec(self) -> OptSpec:
        return OptSpec(OPT_KIND["adam"], self.learning_rate, 0.0, self.beta1, self.beta2, self.epsilon)


@dataclass
class AddOptimizer:
    """The reference unit tests' optimizer: w += g (blocking/shard.rs:117-128)."""

    def spec(self) -> OptSpec:
        return OptSpec(OPT_KIND["add"], 0.0, 0.0, 0.0, 0.0, 0.0)


def _f32(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


# ------------------------------------------------------------------ stores
class _Store:
    _kind = "blocking"

    def __init__(self, shard_size: int, nworkers: int, params, optimizer, device: int = 0):
        p = _f32(params)
        h = C.c_void_p()
        spec = optimizer.spec()
        call("ono_store_create", C.byref(h), STORE_KIND[self._kind], p.ctypes.data if p.size else None,
             p.size, shard_size, nworkers, C.byref(spec), device)
        self._h = h
        self.nparams = p.size

    def __len__(self) -> int:
        return self.nparams

    def len(self) -> int:
        return self.nparams

    def accumulate(self, grad) -> None:
        g = _f32(grad)
        call("ono_store_accumulate", self._h, g.ctypes.data if g.size else None, g.size)

    def accumulate_f16(self, grad_f16) -> None:
        """accumulate() from the reference's wire form: the worker's f16
        payload (uint16 bit patterns), decoded inside the accumulate kernel."""
        if isinstance(grad_f16, torch.Tensor):
            if grad_f16.dtype not in (torch.float16, torch.int16) or not grad_f16.is_cuda:
                raise ValueError("device payload must be a float16/int16 CUDA tensor")
            call("ono_store_accumulate_f16_dev", self._h, grad_f16.data_ptr(), grad_f16.numel())
            return
        h = np.ascontiguousarray(grad_f16)
        if h.dtype not in (np.uint16, np.float16):
            raise ValueError("host payload must be uint16 (f16 bit patterns) or float16")
        call("ono_store_accumulate_f16", self._h, h.ctypes.data if h.size else None, h.size)

    def update_params(self) -> None:
        call("ono_store_update_params", self._h)

    def pull_params(self, out: np.ndarray | None = None) -> np.ndarray:
        if out is None:
            out = np.empty(self.nparams, np.float32)
        if out.dtype != np.float32 or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous float32 array")
        call("ono_store_pull_params", self._h, out.ctypes.data if out.size else None, out.size)
        return out

    @property
    def active_idx(self) -> int:
        return lib().ono_store_active_idx(self._h)

    def set_updating(self, v: bool) -> None:
        call("ono_store_set_updating", self._h, int(v))

    def close(self) -> None:
        if getattr(self, "_h", None):
            call("ono_store_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BlockingStore(_Store):
    """storage/blocking/store.rs: double-buffered, CAS-guarded, averages by nworkers."""

    _kind = "blocking"


class WildStore(_Store):
    """storage/wild/store.rs: applies the optimizer to every gradient on arrival."""

    _kind = "wild"

    def __init__(self, shard_size: int, params, optimizer, device: int = 0):
        super().__init__(shard_size, 1, params, optimizer, device)


# --------------------------------------------------------- synchronization
class DynBarrier:
    """synchronization/dyn_barrier.rs (generation barrier, one leader)."""

    def __init__(self, size: int):
        h = C.c_void_p()
        call("ono_barrier_create", C.byref(h), size)
        self._h = h

    def wait_with(self, leader_fn) -> None:
        cb = LEADER_FN(lambda _ctx: leader_fn())
        call("ono_barrier_wait_with", self._h, cb, None)

    def acquire(self) -> None:
        call("ono_barrier_acquire", self._h)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ono_barrier_destroy(self._h)
            self._h = None


class _Sync:
    _kind = "barrier"

    def __init__(self, size: int = 1, _handle=None):
        if _handle is None:
            h = C.c_void_p()
            call("ono_sync_create", C.byref(h), SYNC_KIND[self._kind], size)
            _handle = h
        self._h = _handle

    def clone(self):
        """One handle per worker task (the Rust Arc clone)."""
        call("ono_sync_clone", self._h)
        return type(self)(_handle=self._h)

    def drop(self) -> None:
        """Drop of this clone (barrier.rs:30-38 shrinks the barrier)."""
        if self._h is not None:
            call("ono_sync_release", self._h)
            self._h = None

    def step(self, store: _Store, grad, params: np.ndarray) -> None:
        """Synchronizer::step: accumulate; [barrier, leader updates]; pull."""
        g = _f32(grad)
        if params.dtype != np.float32 or not params.flags.c_contiguous:
            raise ValueError("params must be a contiguous float32 array")
        call("ono_sync_step", self._h, store._h, g.ctypes.data if g.size else None,
             params.ctypes.data if params.size else None, g.size)

    def step_f16(self, store: _Store, grad_f16, params: np.ndarray) -> None:
        """step() with the gradient as the f16 payload it arrives in (uint16 bit patterns)."""
        h = np.ascontiguousarray(grad_f16)
        if h.dtype not in (np.uint16, np.float16):
            raise ValueError("payload must be uint16 (f16 bit patterns) or float16")
        if params.dtype != np.float32 or not params.flags.c_contiguous:
            raise ValueError("params must be a contiguous float32 array")
        call("ono_sync_step_f16", self._h, store._h, h.ctypes.data if h.size else None,
             params.ctypes.data if params.size else None, h.size)


class BarrierSync(_Sync):
    """synchronization/barrier.rs."""

    _kind = "barrier"


class NoBlockingSync(_Sync):
    """synchronization/non_blocking.rs."""

    _kind = "nonblocking"

    def __init__(self, _handle=None):
        super().__init__(1, _handle)
