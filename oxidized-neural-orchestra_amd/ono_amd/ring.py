"""WorkerRingManager — the ring all-reduce middleware, MI355X-native.

Mirrors worker/src/middlewares/worker_ring.rs (WorkerRingManager::{new,
build_param_manager, pull_grads}) and the ParamManager view it hands back
(machine_learning/src/param_manager.rs:97-108, 183-197).  The manager owns the
`grad` and `residual` buckets (in HBM here); the caller owns `params`.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import kernels
from ._lib import ALGO, PHASES, SAMPLE_FN, UID_BYTES, WIRE, XGMI_HANDLE_BYTES, call, lib


class _DevArray:
    """__cuda_array_interface__ view of library-owned device memory."""

    def __init__(self, ptr: int, n: int):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False),
                                         "version": 2, "strides": None}


def unique_id() -> bytes:
    """Rank 0 generates the RCCL id; it reaches the other ranks out of band
    (the reference's ring TCP links, worker/src/builder.rs:272-311)."""
    buf = C.create_string_buffer(UID_BYTES)
    call("ono_ring_unique_id", buf)
    return buf.raw


class ParamManager:
    """The all-reduce ParamManager: one entity over (params, grad, residual)."""

    def __init__(self, params, grad: torch.Tensor, residual: torch.Tensor):
        self.params, self.grad, self.residual = params, grad, residual

    def acc_residual(self, stream=None) -> None:
        """residual += grad (param_manager.rs:191-197)."""
        kernels.acc(self.residual, self.grad, stream)

    def normalize_gradient(self, n: int, stream=None) -> None:
        """grad /= n (param_manager.rs:183-188)."""
        kernels.scale_zero(self.grad, self.grad, float(n), None, stream)

    def zero_grad(self) -> None:
        """param_manager.rs:168-172."""
        self.grad.zero_()

    def optimize(self, optimizer: "DeviceOptimizer", params_copy: torch.Tensor | None = None,
                 stream=None) -> None:
        """ParamManager::optimize + zero_grad + the optimization_params copy of
        all_reduce.rs:126-132, fused into one kernel."""
        optimizer.step(self.params, self.grad, params_copy, stream)


class DeviceOptimizer:
    """GradientDescent / WithMomentum / Adam for the all-reduce consumer, with
    its state in HBM (ono_optimizer_*)."""

    def __init__(self, optimizer, n: int, device: int | None = None):
        from ._lib import OptSpec  # noqa: F401
        spec = optimizer.spec()
        h = C.c_void_p()
        dev = torch.cuda.current_device() if device is None else device
        call("ono_optimizer_create", C.byref(h), C.byref(spec), n, dev)
        self._h, self.n = h, n

    def step(self, params: torch.Tensor, grad: torch.Tensor, params_copy: torch.Tensor | None = None,
             stream=None) -> None:
        call("ono_optimizer_step", self._h, kernels.f32_ptr(params), kernels.f32_ptr(grad),
             kernels.f32_ptr(params_copy) if params_copy is not None else None, params.numel(),
             kernels.stream_handle(stream))

    def close(self) -> None:
        if getattr(self, "_h", None):
            call("ono_optimizer_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class WorkerRingManager:
    """worker_ring.rs:10-56.  `addrs` is the worker list (only its length is
    used: the ring order is the list order); `wire` selects "f32" (RCCL
    all-reduce) or "f16" (the reference's exact f16 hop schedule)."""

    def __init__(self, pos: int, addrs, size: int, amount_of_layers: int = 1, *,
                 uid: bytes | None = None, wire: str = "f32", device: int | None = None,
                 algo: str = "auto"):
        nranks = addrs if isinstance(addrs, int) else len(addrs)
        self.pos, self.nranks, self.size = pos, nranks, size
        self.amount_of_layers = amount_of_layers
        self.device = torch.cuda.current_device() if device is None else device
        self.wire = wire
        self.algo = "auto"
        self._socks = ()
        h = C.c_void_p()
        if isinstance(uid, tuple):  # (fd_prev, fd_next): the TCP edge, see over_tcp()
            call("ono_ring_create_tcp", C.byref(h), pos, nranks, size, self.device, *uid)
        elif uid == "xgmi":  # no communicator, see over_xgmi()
            call("ono_ring_create_xgmi", C.byref(h), pos, nranks, size, self.device, WIRE[wire])
        else:
            call("ono_ring_create", C.byref(h), pos, nranks, size, self.device, uid, WIRE[wire])
        self._h = h
        if algo != "auto":
            self.set_algo(algo)
        self._bind()

    @classmethod
    def over_tcp(cls, pos: int, addrs, size: int, prev_sock, next_sock, amount_of_layers: int = 1,
                 *, device: int | None = None) -> "WorkerRingManager":
        """The TCP edge: the manager over the worker's own connections
        (worker/src/builder.rs:272-311 — `prev_sock` accepted from the previous
        worker, `next_sock` connected to the next), speaking the reference's
        frames byte for byte (comms/src/protocol/msg.rs:120-191).  Always the
        f16 wire and the hop schedule.  The sockets stay owned by the caller
        and must outlive the manager."""
        nranks = addrs if isinstance(addrs, int) else len(addrs)
        fds = (-1, -1) if nranks == 1 else (prev_sock.fileno(), next_sock.fileno())
        self = cls(pos, nranks, size, amount_of_layers, uid=fds, wire="f16", device=device)
        self._socks = (prev_sock, next_sock)
        self.algo = "hops"
        return self

    @classmethod
    def over_xgmi(cls, pos: int, addrs, size: int, allgather, amount_of_layers: int = 1, *,
                  wire: str = "f32", device: int | None = None) -> "WorkerRingManager":
        """The xGMI peer-access schedule with no collective library: every rank
        exports its exchange region and maps its peers' (ONO_ALGO_XGMI).
        `allgather(bytes) -> list[bytes]` moves the 128-byte handles between the
        ranks in rank order — any control channel (the reference's ring links,
        a gloo group, a pipe).  Every rank must construct (and close) together."""
        nranks = addrs if isinstance(addrs, int) else len(addrs)
        self = cls(pos, nranks, size, amount_of_layers, uid="xgmi", wire=wire, device=device)
        self.algo = "xgmi"
        if nranks > 1:
            buf = C.create_string_buffer(XGMI_HANDLE_BYTES)
            call("ono_ring_xgmi_handle", self._h, buf)
            handles = allgather(buf.raw)
            if len(handles) != nranks or any(len(x) != XGMI_HANDLE_BYTES for x in handles):
                raise ValueError(f"allgather must return one {XGMI_HANDLE_BYTES}-byte handle per rank")
            call("ono_ring_xgmi_connect", self._h, b"".join(handles))
        return self

    def _bind(self):
        h, size = self._h, self.size
        dev = f"cuda:{self.device}"
        self.grad = torch.as_tensor(_DevArray(lib().ono_ring_grad(h), size), device=dev)
        self.residual = torch.as_tensor(_DevArray(lib().ono_ring_residual(h), size), device=dev)

    # -- worker_ring.rs:65-72
    def build_param_manager(self, params) -> ParamManager:
        return ParamManager(params, self.grad, self.residual)

    # -- worker_ring.rs:82-94 (device resident; stream-ordered)
    def pull_grads(self, params=None, stream=None) -> ParamManager:
        call("ono_ring_pull_grads", self._h, kernels.stream_handle(stream))
        return self.build_param_manager(params)

    def pull_grads_dev(self, residual: torch.Tensor, grad: torch.Tensor, stream=None) -> None:
        call("ono_ring_pull_grads_dev", self._h, kernels.f32_ptr(residual), kernels.f32_ptr(grad),
             residual.numel(), kernels.stream_handle(stream))

    def pull_grads_host(self, residual: np.ndarray, grad: np.ndarray) -> None:
        """Host-fed round (the reference's buffers arrive from comms/): H2D,
        reduce, D2H; residual is zeroed in place, grad receives the average."""
        for a in (residual, grad):
            if a.dtype != np.float32 or not a.flags.c_contiguous or a.size != self.size:
                raise ValueError("expected contiguous float32 host buffers of ring size")
        call("ono_ring_pull_grads_host", self._h, residual.ctypes.data, grad.ctypes.data, self.size)

    def register_host(self, a: np.ndarray) -> None:
        """Page-lock a long-lived host bucket for in-place DMA by pull_grads_host."""
        call("ono_ring_register_host", self._h, a.ctypes.data, a.nbytes)

    def unregister_host(self, a: np.ndarray) -> None:
        call("ono_ring_unregister_host", self._h, a.ctypes.data)

    def allreduce_avg_(self, buf: torch.Tensor, stream=None) -> torch.Tensor:
        call("ono_ring_allreduce_avg_dev", self._h, kernels.f32_ptr(buf), buf.numel(),
             kernels.stream_handle(stream))
        return buf

    def acc_residual(self, grad: torch.Tensor, stream=None) -> None:
        call("ono_ring_acc_residual", self._h, kernels.f32_ptr(grad), kernels.stream_handle(stream))

    def set_algo(self, algo: str) -> None:
        """n > 1 exchange schedule: "allreduce" | "hops" | "direct" | "xgmi" | "auto"."""
        call("ono_ring_set_algo", self._h, ALGO[algo])
        self.algo = algo

    def set_sparse(self, r: float, seed: int = 0) -> None:
        """The SparseCapable{r} serializer (compressor.rs:71-98): SparseGrad
        frames of the values with |g| >= calculate_threshold(chunk, r), the
        ring's sparse branches (worker_ring.rs:126-133, :177-193).  r = 0
        returns to the Base (dense f16) serializer.  TCP rings only.  `seed`
        starts the default threshold sampler (used above 16384 values)."""
        call("ono_ring_set_sparse", self._h, float(r), int(seed) & (2 ** 64 - 1))

    def set_sampler(self, fn) -> None:
        """fn(length, amount) -> `amount` distinct indices of [0, length): the
        threshold sample of every sparse push (the reference draws it with
        rand::seq::index::sample on the Compressor's StdRng).  None restores
        the default sampler."""
        if fn is None:
            self._sampler = None
            call("ono_ring_set_sampler", self._h, None, None)
            return

        def tramp(_ctx, length, idx, amount):
            try:
                got = np.asarray(fn(int(length), int(amount)), dtype=np.uint32)
                if got.shape != (amount,):
                    return 1
                C.memmove(idx, got.ctypes.data, 4 * amount)
                return 0
            except Exception:  # reported to the ring as a sampler failure
                return 1
        self._sampler = SAMPLE_FN(tramp)  # kept alive as long as the ring
        call("ono_ring_set_sampler", self._h, C.cast(self._sampler, C.c_void_p), None)

    def set_pipeline(self, segments: int) -> None:
        """Segments of the f32 all-reduce schedule (finaliser of segment j
        overlaps the all-reduce of segment j+1); 1 = unsegmented, 0 = default."""
        call("ono_ring_set_pipeline", self._h, segments)

    def set_xgmi_timeout(self, seconds: float) -> None:
        """How long an xGMI barrier waits for a slow peer before the round
        fails with IoError (0 = env ONO_XGMI_TIMEOUT_S, else 600 s)."""
        call("ono_ring_set_xgmi_timeout", self._h, float(seconds))

    def check(self) -> None:
        """Raise if the rounds enqueued so far are invalid (synchronize first):
        IoError after an xGMI barrier timeout, Aborted after abort()."""
        call("ono_ring_check", self._h)

    def abort(self) -> None:
        call("ono_ring_abort", self._h)

    def timing(self, enable: bool) -> None:
        call("ono_ring_timing_enable", self._h, int(enable))

    def timing_read(self) -> dict:
        km, kn, cm, cn = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
        call("ono_ring_timing_read", self._h, C.byref(km), C.byref(kn), C.byref(cm), C.byref(cn))
        return {"kernel_ms": km.value, "kernels": kn.value, "collective_ms": cm.value, "collectives": cn.value}

    def timing_phases(self) -> dict:
        """{phase: (ms, launches)} — local kernels, RCCL calls, xGMI scatter /
        barrier / gather (ono_ring_timing_phases)."""
        ms, cnt = (C.c_double * len(PHASES))(), (C.c_int64 * len(PHASES))()
        call("ono_ring_timing_phases", self._h, ms, cnt)
        return {p: (ms[i], cnt[i]) for i, p in enumerate(PHASES)}

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.grad = self.residual = None
            call("ono_ring_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def xgmi_pool_close_imports() -> int:
    """Release, phase 1 (ono_xgmi_pool_close_imports): mark every peer region this
    process maps as closed and close the imports.  Every rank, once its xGMI rings
    are destroyed; then a collective step; then xgmi_pool_free_exports."""
    closed = C.c_size_t(0)
    call("ono_xgmi_pool_close_imports", C.byref(closed))
    return closed.value


def xgmi_pool_free_exports(wait_s: float = 60.0) -> dict:
    """Release, phase 2 (ono_xgmi_pool_free_exports): free every idle exchange
    region once all its importers have closed it (waits up to wait_s)."""
    freed, kept = C.c_size_t(0), C.c_size_t(0)
    call("ono_xgmi_pool_free_exports", C.byref(freed), C.byref(kept), float(wait_s))
    return {"freed_bytes": freed.value, "kept": kept.value}


def xgmi_pool_release() -> dict:
    """Both phases in one call (ono_xgmi_pool_release): close this process's peer
    imports, then free its idle exchange regions once their importers have closed
    them.  Only when no xGMI ring of the process is alive; multi-process callers
    should prefer the two phases with a barrier between."""
    freed, closed = C.c_size_t(0), C.c_size_t(0)
    call("ono_xgmi_pool_release", C.byref(freed), C.byref(closed))
    return {"freed_bytes": freed.value, "closed_imports": closed.value}


def xgmi_pool_stats() -> dict:
    v = [C.c_size_t(0) for _ in range(4)]
    call("ono_xgmi_pool_stats", *[C.byref(x) for x in v])
    return dict(zip(("regions", "region_bytes", "quarantined", "imports"), (x.value for x in v)))


def local_ring_pull_grads(residuals: list[torch.Tensor], grads: list[torch.Tensor], wire: str = "f16",
                          stream=None, algo: str = "hops") -> None:
    """Every rank of one pull_grads round, co-resident on one device (the
    device analog of the reference's loopback workers).  algo "hops" runs the
    reference hop schedule, "direct" the direct schedule's fused owner kernel."""
    n = len(residuals)
    size = residuals[0].numel()
    if len(grads) != n or any(t.numel() != size for t in residuals + grads):
        raise ValueError("one residual and one grad bucket of equal size per rank")
    rp = (C.c_void_p * n)(*[kernels.f32_ptr(t) for t in residuals])
    gp = (C.c_void_p * n)(*[kernels.f32_ptr(t) for t in grads])
    fn = {"hops": "ono_local_ring_pull_grads", "direct": "ono_local_direct_pull_grads"}[algo]
    call(fn, rp, gp, n, size, WIRE[wire], kernels.stream_handle(stream))
