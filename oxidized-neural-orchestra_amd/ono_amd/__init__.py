"""ono_amd — MI355X-native gradient-bucket reduction for oxidized-neural-orchestra.

Host-side mirror of the reference's ring middleware (WorkerRingManager,
ParamManager) and parameter-server synchronizer/store (Store, BlockingStore,
WildStore, BarrierSync, NoBlockingSync, DynBarrier), over the C ABI of
libono_reduce.so (include/ono_reduce.h).

torch is imported first on purpose: it loads the process's HIP runtime
(libamdhip64.so.7) and RCCL, and libono_reduce.so then binds to those same
objects, so torch tensors, torch streams and the library share one runtime.
"""
import torch  # noqa: F401  (must precede the library load; see above)

from ._lib import (Aborted, HipError, InvalidArgument, InvalidWorkerEvent, IoError, OnoError,
                   RcclError, SizeMismatch, header_functions, lib, worker_event_check)
from . import kernels, plan, sparse
from .ring import (DeviceOptimizer, ParamManager, WorkerRingManager, local_ring_pull_grads, unique_id,
                   xgmi_pool_close_imports, xgmi_pool_free_exports, xgmi_pool_release, xgmi_pool_stats)
from .store import (Adam, AddOptimizer, BarrierSync, BlockingStore, DynBarrier, GradientDescent,
                    GradientDescentWithMomentum, NoBlockingSync, WildStore, shard_size_for)
from .ps import ShardedParamServer

lib()  # fail loudly at import when the native library is missing

__all__ = [
    "Aborted", "HipError", "InvalidArgument", "InvalidWorkerEvent", "IoError", "OnoError", "RcclError",
    "SizeMismatch", "header_functions", "lib", "kernels", "DeviceOptimizer", "ParamManager", "WorkerRingManager",
    "local_ring_pull_grads", "unique_id", "Adam", "AddOptimizer", "BarrierSync", "BlockingStore",
    "DynBarrier", "GradientDescent", "GradientDescentWithMomentum", "NoBlockingSync", "WildStore",
    "shard_size_for", "ShardedParamServer", "worker_event_check", "xgmi_pool_release", "xgmi_pool_stats",
    "xgmi_pool_close_imports", "xgmi_pool_free_exports",
]
