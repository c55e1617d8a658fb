"""Multi-GPU parameter-server mode (BASELINE config 5).

The sharded synchronizer of parameter_server/ (BlockingStore + BarrierSync
across nworkers) as one RCCL reduce-scatter of the workers' gradients, a fused
(÷nworkers + optimizer) kernel on the shard each GPU owns, and one RCCL
all-gather of the parameters.  Every GPU is both a worker and a shard server.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import kernels
from ._lib import call
from .ring import WorkerRingManager


class ShardedParamServer:
    def __init__(self, ring: WorkerRingManager, params, optimizer):
        p = np.ascontiguousarray(params, dtype=np.float32)
        h = C.c_void_p()
        spec = optimizer.spec()
        call("ono_ps_create", C.byref(h), ring._h, p.ctypes.data, p.size, C.byref(spec))
        self._h, self.ring, self.nparams = h, ring, p.size

    def step(self, grad: torch.Tensor, params: torch.Tensor, stream=None) -> torch.Tensor:
        """accumulate (reduce-scatter) -> leader update on every shard -> pull (all-gather)."""
        if grad.numel() != self.nparams or params.numel() != self.nparams:
            raise ValueError("gradient/params length must equal the store length")
        call("ono_ps_step", self._h, kernels.f32_ptr(grad), kernels.f32_ptr(params),
             kernels.stream_handle(stream))
        return params

    def close(self) -> None:
        if getattr(self, "_h", None):
            call("ono_ps_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
