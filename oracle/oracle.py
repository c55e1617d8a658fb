"""ctypes front-end for the C oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; it is the checker, never the thing measured or shipped.  The
library it loads (oracle/_build/libono_oracle.so) is built from
oracle/ono_oracle.c by ``make -C oracle`` (driven by __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
LIB_PATH = os.path.join(BUILD, "libono_oracle.so")
CPU_RING = os.path.join(BUILD, "ono_cpu_ring")

OPT = {"gd": 0, "momentum": 1, "adam": 2, "add": 3}

_lib = None
_fp = C.POINTER(C.c_float)
_u16p = C.POINTER(C.c_uint16)
_u8p = C.POINTER(C.c_uint8)


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or not os.path.exists(CPU_RING):
            build()
        L = C.CDLL(LIB_PATH)
        L.ono_ref_f32_to_f16.restype = C.c_uint16
        L.ono_ref_f32_to_f16.argtypes = [C.c_float]
        L.ono_ref_f16_to_f32.restype = C.c_float
        L.ono_ref_f16_to_f32.argtypes = [C.c_uint16]
        L.ono_ref_f16_encode.argtypes = [_u16p, _fp, C.c_size_t]
        L.ono_ref_f16_decode.argtypes = [_fp, _u16p, C.c_size_t]
        L.ono_ref_split_chunks.restype = C.c_size_t
        L.ono_ref_split_chunks.argtypes = [C.c_size_t, C.c_size_t, C.POINTER(C.c_size_t)]
        L.ono_ref_ring_pull_grads.restype = C.c_int
        L.ono_ref_ring_pull_grads.argtypes = [C.POINTER(_fp), C.POINTER(_fp), C.c_int, C.c_size_t, C.c_int]
        L.ono_ref_sum_scale.argtypes = [_fp, C.POINTER(_fp), C.c_int, C.c_size_t, C.c_float]
        L.ono_ref_normalize.argtypes = [_fp, C.c_size_t, C.c_size_t]
        L.ono_ref_acc_residual.argtypes = [_fp, _fp, C.c_size_t]
        L.ono_ref_store_new.restype = C.c_void_p
        L.ono_ref_store_new.argtypes = [_fp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int,
                                        C.c_float, C.c_float, C.c_float, C.c_float, C.c_float]
        L.ono_ref_store_free.argtypes = [C.c_void_p]
        L.ono_ref_store_accumulate.restype = C.c_int
        L.ono_ref_store_accumulate.argtypes = [C.c_void_p, _fp, C.c_size_t]
        L.ono_ref_store_update_params.argtypes = [C.c_void_p]
        L.ono_ref_store_pull_params.restype = C.c_int
        L.ono_ref_store_pull_params.argtypes = [C.c_void_p, _fp, C.c_size_t]
        L.ono_ref_store_active_idx.restype = C.c_int
        L.ono_ref_store_active_idx.argtypes = [C.c_void_p]
        L.ono_ref_store_set_updating.argtypes = [C.c_void_p, C.c_int]
        L.ono_ref_store_nshards.restype = C.c_size_t
        L.ono_ref_store_nshards.argtypes = [C.c_void_p]
        L.ono_ref_wild_new.restype = C.c_void_p
        L.ono_ref_wild_new.argtypes = [_fp, C.c_size_t, C.c_size_t, C.c_int,
                                       C.c_float, C.c_float, C.c_float, C.c_float, C.c_float]
        L.ono_ref_wild_free.argtypes = [C.c_void_p]
        L.ono_ref_wild_accumulate.restype = C.c_int
        L.ono_ref_wild_accumulate.argtypes = [C.c_void_p, _fp, C.c_size_t]
        L.ono_ref_wild_pull_params.restype = C.c_int
        L.ono_ref_wild_pull_params.argtypes = [C.c_void_p, _fp, C.c_size_t]
        L.ono_ref_sparse_threshold_full.restype = C.c_float
        L.ono_ref_sparse_threshold_full.argtypes = [_fp, C.c_size_t, C.c_float]
        L.ono_ref_grad_drop.restype = C.c_size_t
        L.ono_ref_grad_drop.argtypes = [_u8p, _fp, C.c_size_t, C.c_float]
        L.ono_ref_grad_lift.restype = C.c_int
        L.ono_ref_grad_lift.argtypes = [_fp, C.c_size_t, C.POINTER(C.c_size_t), _u8p, C.c_size_t]
        L.ono_ref_frame_dense.restype = C.c_size_t
        L.ono_ref_frame_dense.argtypes = [_u8p, _u16p, C.c_size_t, C.c_int]
        L.ono_ref_synth.argtypes = [_fp, C.c_size_t, C.c_uint64, C.c_uint64, C.c_size_t]
        L.ono_ref_sparse_threshold_sample.restype = C.c_float
        L.ono_ref_sparse_threshold_sample.argtypes = [_fp, C.c_size_t, C.POINTER(C.c_uint32), C.c_size_t, C.c_float]
        L.ono_ref_sample_default.argtypes = [C.POINTER(C.c_uint64), C.c_size_t, C.POINTER(C.c_uint32), C.c_size_t]
        L.ono_ref_ring_pull_grads_sparse.restype = C.c_int
        L.ono_ref_ring_pull_grads_sparse.argtypes = [C.POINTER(_fp), C.POINTER(_fp), C.c_int, C.c_size_t,
                                                     C.POINTER(C.c_float), C.POINTER(C.c_uint64)]
        L.ono_ref_sparse_push_is_sparse.restype = C.c_int
        L.ono_ref_sparse_push_is_sparse.argtypes = [_fp, C.c_size_t, C.c_float, C.POINTER(C.c_uint64),
                                                    C.POINTER(C.c_float)]
        _lib = L
    return _lib


def _f(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_fp)


def _u16(a: np.ndarray):
    assert a.dtype == np.uint16 and a.flags.c_contiguous
    return a.ctypes.data_as(_u16p)


# ----------------------------------------------------------------- functions
def f16_encode(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.size, np.uint16)
    lib().ono_ref_f16_encode(_u16(out), _f(x), x.size)
    return out


def f16_decode(h: np.ndarray) -> np.ndarray:
    h = np.ascontiguousarray(h, dtype=np.uint16)
    out = np.empty(h.size, np.float32)
    lib().ono_ref_f16_decode(_f(out), _u16(h), h.size)
    return out


def split_chunks(length: int, n: int) -> list[tuple[int, int]]:
    off = (C.c_size_t * (n + 1))()
    k = lib().ono_ref_split_chunks(length, n, off)
    return [(off[i], off[i + 1]) for i in range(k)]


def ring_pull_grads(residuals: list[np.ndarray], wire: str = "f16"):
    """All ranks' pull_grads() round; returns (grads, residuals_after)."""
    n = len(residuals)
    res = [np.array(r, dtype=np.float32, copy=True) for r in residuals]
    length = res[0].size
    grads = [np.zeros(length, np.float32) for _ in range(n)]
    rp = (_fp * n)(*[_f(r) for r in res])
    gp = (_fp * n)(*[_f(g) for g in grads])
    rc = lib().ono_ref_ring_pull_grads(rp, gp, n, length, 0 if wire == "f16" else 1)
    if rc != 0:
        raise ValueError("reference panics: fewer chunks than ranks")
    return grads, res


def ring_pull_grads_sparse(residuals: list[np.ndarray], ratios, states):
    """The round with per-worker serializers (ratio 0 = Base dense f16, else
    SparseCapable{ratio}; states = the default samplers' streams).  Returns
    (grads, residuals_after, states_after)."""
    n = len(residuals)
    res = [np.array(r, dtype=np.float32, copy=True) for r in residuals]
    length = res[0].size
    grads = [np.zeros(length, np.float32) for _ in range(n)]
    rp = (_fp * n)(*[_f(r) for r in res])
    gp = (_fp * n)(*[_f(g) for g in grads])
    rat = (C.c_float * n)(*[float(x) for x in ratios])
    st = (C.c_uint64 * n)(*[int(x) & (2 ** 64 - 1) for x in states])
    if lib().ono_ref_ring_pull_grads_sparse(rp, gp, n, length, rat, st) != 0:
        raise ValueError("reference panics: fewer chunks than ranks")
    return grads, res, [st[i] for i in range(n)]


def sparse_push(chunk: np.ndarray, ratio: float, state: int = 0):
    """What a SparseCapable{ratio} worker's push_grad sends for `chunk`
    (compressor.rs:71-98): (is_sparse, threshold, next sampler state)."""
    ch = np.ascontiguousarray(chunk, dtype=np.float32)
    st = C.c_uint64(state & (2 ** 64 - 1))
    t = C.c_float(0.0)
    sp = lib().ono_ref_sparse_push_is_sparse(_f(ch), ch.size, ratio, C.byref(st), C.byref(t))
    return bool(sp), float(t.value), st.value


def sample_default(state: int, length: int, amount: int):
    """The stand-in threshold sampler: (indices, next state)."""
    st = C.c_uint64(state & (2 ** 64 - 1))
    out = np.empty(max(amount, 1), np.uint32)
    lib().ono_ref_sample_default(C.byref(st), length, out.ctypes.data_as(C.POINTER(C.c_uint32)), amount)
    return out[:amount].copy(), st.value


def sparse_threshold_sample(g: np.ndarray, r: float, idx=None) -> float:
    """calculate_threshold over the sample idx (None: every value)."""
    g = np.ascontiguousarray(g, dtype=np.float32)
    if idx is None:
        return float(lib().ono_ref_sparse_threshold_sample(_f(g), g.size, None, g.size, r))
    ix = np.ascontiguousarray(idx, dtype=np.uint32)
    return float(lib().ono_ref_sparse_threshold_sample(_f(g), g.size, ix.ctypes.data_as(C.POINTER(C.c_uint32)),
                                                       ix.size, r))


def sum_scale(ins: list[np.ndarray], divisor: float) -> np.ndarray:
    ins = [np.ascontiguousarray(x, dtype=np.float32) for x in ins]
    out = np.empty(ins[0].size, np.float32)
    ip = (_fp * len(ins))(*[_f(x) for x in ins])
    lib().ono_ref_sum_scale(_f(out), ip, len(ins), out.size, divisor)
    return out


def synth(n: int, seed: int, rank: int, offset: int = 0) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().ono_ref_synth(_f(out), n, seed, rank, offset)
    return out


def synth_special(n: int, seed: int, rank: int) -> np.ndarray:
    """synth() with IEEE special values planted at rank-dependent strides:
    quiet NaNs with payloads, +-inf, -0, f16-overflowing 7e4, f16-subnormal /
    underflowing 1e-8 and 3e38 (an f32 sum of two overflows).  Test input."""
    x = synth(n, seed, rank)
    u = x.view(np.uint32)
    u[rank % 97::97] = 0x7FC01234 + rank
    x[(rank + 3) % 101::101] = np.inf if rank % 2 == 0 else -np.inf
    u[(rank + 5) % 103::103] = 0x80000000
    x[(rank + 7) % 107::107] = 7.0e4
    x[(rank + 11) % 109::109] = 1.0e-8
    x[(rank + 13) % 113::113] = 3.0e38
    return x


def same_or_both_nan(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Element mask: bit-identical, or NaN in both (NaN payload propagation
    through a + b is not pinned by IEEE-754 nor by the reference's compiler,
    which may commute the operands)."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def frame_dense(h: np.ndarray, is_last: bool = False) -> bytes:
    h = np.ascontiguousarray(h, dtype=np.uint16)
    buf = np.empty(12 + 2 * h.size, np.uint8)
    k = lib().ono_ref_frame_dense(buf.ctypes.data_as(_u8p), _u16(h), h.size, int(is_last))
    return bytes(buf[:k])


def sparse_threshold(g: np.ndarray, r: float) -> float:
    g = np.ascontiguousarray(g, dtype=np.float32)
    return float(lib().ono_ref_sparse_threshold_full(_f(g), g.size, r))


def grad_drop(g: np.ndarray, threshold: float) -> bytes:
    g = np.ascontiguousarray(g, dtype=np.float32)
    buf = np.empty(8 + 10 * max(g.size, 1), np.uint8)
    k = lib().ono_ref_grad_drop(buf.ctypes.data_as(_u8p), _f(g), g.size, threshold)
    return bytes(buf[:k])


def grad_lift(buf: bytes, cap: int = 1 << 20) -> np.ndarray:
    b = np.frombuffer(buf, dtype=np.uint8).copy()
    out = np.zeros(cap, np.float32)
    ln = C.c_size_t(0)
    rc = lib().ono_ref_grad_lift(_f(out), cap, C.byref(ln), b.ctypes.data_as(_u8p), b.size)
    if rc != 0:
        raise ValueError(f"grad_lift error {rc}")
    return out[: ln.value].copy()


class Store:
    """BlockingStore oracle."""

    def __init__(self, params, shard_size: int, nworkers: int, kind: str = "gd",
                 lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8):
        p = np.ascontiguousarray(params, dtype=np.float32)
        self.n = p.size
        self._h = lib().ono_ref_store_new(_f(p), p.size, shard_size, nworkers, OPT[kind],
                                          lr, momentum, beta1, beta2, eps)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ono_ref_store_free(self._h)
            self._h = None

    def accumulate(self, g) -> None:
        g = np.ascontiguousarray(g, dtype=np.float32)
        if lib().ono_ref_store_accumulate(self._h, _f(g), g.size):
            raise ValueError("SizeMismatch")

    def update_params(self) -> None:
        lib().ono_ref_store_update_params(self._h)

    def pull_params(self) -> np.ndarray:
        out = np.empty(self.n, np.float32)
        lib().ono_ref_store_pull_params(self._h, _f(out), self.n)
        return out

    @property
    def active_idx(self) -> int:
        return lib().ono_ref_store_active_idx(self._h)

    def set_updating(self, v: bool) -> None:
        lib().ono_ref_store_set_updating(self._h, int(v))

    @property
    def nshards(self) -> int:
        return lib().ono_ref_store_nshards(self._h)


class WildStore:
    def __init__(self, params, shard_size: int, kind: str = "gd",
                 lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8):
        p = np.ascontiguousarray(params, dtype=np.float32)
        self.n = p.size
        self._h = lib().ono_ref_wild_new(_f(p), p.size, shard_size, OPT[kind], lr, momentum,
                                         beta1, beta2, eps)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().ono_ref_wild_free(self._h)
            self._h = None

    def accumulate(self, g) -> None:
        g = np.ascontiguousarray(g, dtype=np.float32)
        if lib().ono_ref_wild_accumulate(self._h, _f(g), g.size):
            raise ValueError("SizeMismatch")

    def update_params(self) -> None:
        pass

    def pull_params(self) -> np.ndarray:
        out = np.empty(self.n, np.float32)
        lib().ono_ref_wild_pull_params(self._h, _f(out), self.n)
        return out


def build_native(out_dir: str) -> dict:
    """The -march=native variants of the CPU baselines ("also
    report a -march=native variant"), compiled on the host that runs them
    (a binary tuned for this container's CPU may not run on the GPU box's)."""
    os.makedirs(out_dir, exist_ok=True)
    flags = ["-O3", "-march=native", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-D_GNU_SOURCE"]
    exes = {}
    for name in ("ono_cpu_ring", "ono_cpu_ps"):
        exe = os.path.join(out_dir, name)
        subprocess.run(["gcc", *flags, "-o", exe, os.path.join(HERE, name + ".c"),
                        os.path.join(HERE, "ono_oracle.c"), "-lm", "-lpthread"], check=True)
        exes[name] = exe
    return exes


def cpu_ps(mode: str, length: int, threads: int = 16, workers: int = 2, rounds: int = 3,
           timeout: float = 600, exe: str | None = None) -> dict:
    """oracle/ono_cpu_ps.c: 'hop' = one scatter hop's compute on one core,
    'ps' = BlockingStore accumulate + update on `threads` cores (2 x threads shards)."""
    import json

    if exe is None:
        exe = os.path.join(BUILD, "ono_cpu_ps")
        if not os.path.exists(exe):
            build()
    cmd = [exe, "--mode", mode, "--len", str(length), "--threads", str(threads), "--workers", str(workers),
           "--rounds", str(rounds)]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout)
    return json.loads(out.stdout.strip().splitlines()[-1])


def cpu_ring(ranks: int, length: int, rounds: int, seed: int = 0x0402026, check: bool = False,
             pin: bool = True, timeout: float = 600, exe: str | None = None) -> dict:
    """Run the TCP-loopback reference-style CPU ring (oracle/ono_cpu_ring.c)."""
    import json

    if exe is None:
        exe = CPU_RING
        if not os.path.exists(CPU_RING):
            build()
    cmd = [exe, "--ranks", str(ranks), "--len", str(length), "--rounds", str(rounds),
           "--seed", str(seed)]
    if check:
        cmd.append("--check")
    if not pin:
        cmd.append("--no-pin")
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout)
    return json.loads(out.stdout.strip().splitlines()[-1])


class CpuRingWorker:
    """One reference-style ring worker as its own process (ono_cpu_ring.c single
    mode): listens on an ephemeral loopback port (`.port`), connects to
    `next_port`, runs `rounds` pull_grads rounds over the reference framing on
    input synth(length, seed, rank), and leaves grad and residual of the last
    round in `result()`.  Test infrastructure: the peer that proves an MI355X
    worker and a reference worker can share one ring."""

    def __init__(self, rank: int, ranks: int, length: int, next_port: int, rounds: int = 1,
                 seed: int = 0x0402026, listen_port: int = 0, sparse: float = 0.0, sparse_seed: int = 0):
        import json
        import tempfile

        if not os.path.exists(CPU_RING):
            build()
        self.length = length
        fd, self.out = tempfile.mkstemp(suffix=".bin")
        os.close(fd)
        self.proc = subprocess.Popen(
            [CPU_RING, "--rank", str(rank), "--ranks", str(ranks), "--len", str(length),
             "--next-port", str(next_port), "--listen-port", str(listen_port), "--rounds", str(rounds),
             "--seed", str(seed), "--out", self.out,
             # the ratio as the exact decimal of its f32 value (no double rounding in atof)
             "--sparse", repr(float(np.float32(sparse))), "--sparse-seed", str(sparse_seed)],
            stdout=subprocess.PIPE, text=True)
        self.port = json.loads(self.proc.stdout.readline())["port"]

    def result(self, timeout: float = 120):
        """(grad, residual) of the last round; raises if the worker failed."""
        import json

        try:
            tail = self.proc.stdout.read()
            rc = self.proc.wait(timeout)
            if rc != 0:
                raise RuntimeError(f"ono_cpu_ring worker exited with {rc}")
            data = np.fromfile(self.out, dtype=np.float32)
            info = json.loads(tail.strip().splitlines()[-1])
            return data[:self.length].copy(), data[self.length:].copy(), info
        finally:
            self.close()

    def close(self):
        if self.proc.poll() is None:
            self.proc.kill()
            self.proc.wait()
        if os.path.exists(self.out):
            os.unlink(self.out)
