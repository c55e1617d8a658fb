"""numpy restatement of the reference reduction path — TEST INFRASTRUCTURE ONLY.

An implementation independent of ``ono_oracle.c`` (vectorised numpy instead of
scalar C).  tests/golden/make_golden.py runs both and only writes fixtures when
they agree bit for bit.  Nothing in the product imports this module.

Reference (lminervino18/oxidized-neural-orchestra):
  chunking       worker/src/middlewares/mod.rs:15-59
  ring           worker/src/middlewares/worker_ring.rs:82-204
  f16 wire       comms/src/handles/compressor.rs:106-118, handles/worker.rs:84-101
                 (crate `half` 2.7.1: IEEE binary16, round-to-nearest-even)
  averaging      machine_learning/src/param_manager.rs:183-188
  store          parameter_server/src/storage/blocking/{store,shard}.rs
  optimizers     machine_learning/src/optimization/*.rs
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


# --------------------------------------------------------------------------- f16
def f32_to_f16_bits(x: np.ndarray) -> np.ndarray:
    """`half::f16::from_f32` bit patterns (uint16)."""
    x = np.ascontiguousarray(x, dtype=F32)
    with np.errstate(over="ignore", invalid="ignore"):
        h = x.astype(np.float16).view(np.uint16).copy()
    u = x.view(np.uint32)
    nan = np.isnan(x)
    if nan.any():  # half keeps the top payload bits and sets the quiet bit
        un = u[nan]
        h[nan] = (((un >> 16) & 0x8000) | 0x7C00 | 0x0200 | ((un & 0x7FFFFF) >> 13)).astype(np.uint16)
    return h


def f16_bits_to_f32(h: np.ndarray) -> np.ndarray:
    """`half::f16::to_f32` (exact widening; NaN gets the f32 quiet bit)."""
    h = np.ascontiguousarray(h, dtype=np.uint16)
    out = h.view(np.float16).astype(F32)
    nan = (h & 0x7C00) == 0x7C00
    nan &= (h & 0x03FF) != 0
    if nan.any():
        hn = h[nan].astype(np.uint32)
        out[nan] = (((hn & 0x8000) << 16) | 0x7FC00000 | ((hn & 0x3FF) << 13)).astype(np.uint32).view(F32)
    return out


def quantize_f16(x: np.ndarray) -> np.ndarray:
    return f16_bits_to_f32(f32_to_f16_bits(x))


# --------------------------------------------------------------------- chunking
def split_chunks(length: int, n: int) -> list[tuple[int, int]]:
    """SplitChunks::next — first length % n chunks get one extra element; stops
    as soon as the remaining slice is empty (so min(length, n) chunks)."""
    base, rem = divmod(length, n)
    out, pos = [], 0
    while pos < length and len(out) < n:
        ln = base + (1 if rem > 0 else 0)
        rem = max(rem - 1, 0)
        out.append((pos, pos + ln))
        pos += ln
    return out


# ------------------------------------------------------------------------- ring
def ring_pull_grads(residuals: list[np.ndarray], wire: str = "f16"):
    """One pull_grads() round of every rank; returns (grads, residuals_after).

    Chunk c's sum is formed in the order c, c+1, ..., c+n-1 with the running
    partial re-quantised to the wire type at every hop; its owner (rank c-1)
    keeps the f32 sum, every other rank a wire-decoded copy; then /n for n>1.
    """
    n = len(residuals)
    length = residuals[0].size
    chunks = split_chunks(length, n)
    if len(chunks) < n:
        raise ValueError("reference panics: fewer chunks than ranks")
    q = quantize_f16 if wire == "f16" else (lambda a: a.astype(F32, copy=True))
    res = [np.array(r, dtype=F32, copy=True) for r in residuals]
    grads = [np.zeros(length, dtype=F32) for _ in range(n)]
    idx = list(range(n))
    for _s in range(n - 1):
        msgs = []
        for r in range(n):
            lo, hi = chunks[idx[r]]
            msgs.append(q(res[r][lo:hi]))
            res[r][lo:hi] = 0
        for r in range(n):
            p = (r - 1) % n
            idx[r] = (idx[r] - 1) % n
            lo, hi = chunks[idx[r]]
            res[r][lo:hi] = res[r][lo:hi] + msgs[p]
    for r in range(n):
        idx[r] = (r + 1) % n
        lo, hi = chunks[idx[r]]
        grads[r][lo:hi] = res[r][lo:hi]
    if n == 1:
        lo, hi = chunks[idx[0]]
        res[0][lo:hi] = 0
        return grads, res
    for j in range(n - 1):
        msgs = []
        for r in range(n):
            lo, hi = chunks[idx[r]]
            msgs.append(q(grads[r][lo:hi]))
            if j == 0:
                res[r][lo:hi] = 0
        for r in range(n):
            p = (r - 1) % n
            idx[r] = (idx[r] - 1) % n
            lo, hi = chunks[idx[r]]
            grads[r][lo:hi] = msgs[p]
    f = F32(n)
    grads = [(g / f).astype(F32) for g in grads]
    return grads, res


def sum_scale(ins: list[np.ndarray], divisor: float) -> np.ndarray:
    acc = np.array(ins[0], dtype=F32, copy=True)
    for x in ins[1:]:
        acc = acc + x.astype(F32)
    if F32(divisor) != F32(1):
        acc = acc / F32(divisor)
    return acc.astype(F32)


# ------------------------------------------------------------------- optimizers
class Optimizer:
    """GradientDescent / WithMomentum / Adam / the tests' AddOptimizer."""

    def __init__(self, kind: str, length: int, lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8):
        self.kind = kind
        self.lr, self.mu = F32(lr), F32(momentum)
        self.b1, self.b2, self.eps = F32(beta1), F32(beta2), F32(eps)
        self.b1t, self.b2t = F32(1), F32(1)
        self.v = np.zeros(length, F32)
        self.s = np.zeros(length, F32)

    def update(self, g: np.ndarray, w: np.ndarray) -> None:
        g = g.astype(F32)
        if self.kind == "gd":
            w -= self.lr * g
        elif self.kind == "momentum":
            self.v[:] = (self.mu * self.v) + g
            w -= self.lr * self.v
        elif self.kind == "adam":
            self.b1t = F32(self.b1t * self.b1)
            self.b2t = F32(self.b2t * self.b2)
            bc1, bc2 = F32(F32(1) - self.b1t), F32(F32(1) - self.b2t)
            step = F32(self.lr * F32(np.sqrt(bc2) / bc1))
            self.v[:] = self.b1 * self.v + (F32(1) - self.b1) * g
            self.s[:] = self.b2 * self.s + (F32(1) - self.b2) * (g * g)
            w -= (step * self.v) / (np.sqrt(self.s) + self.eps)
        elif self.kind == "add":
            w += g
        else:
            raise ValueError(self.kind)


class BlockingStore:
    """BlockingStore + BlockingShard semantics (double buffer, CAS guard)."""

    def __init__(self, params, shard_size: int, nworkers: int, kind: str, **hp):
        self.params = np.array(params, dtype=F32, copy=True)
        self.n = self.params.size
        self.shard = shard_size
        self.nworkers = max(nworkers, 1)
        self.grads = [np.zeros(self.n, F32), np.zeros(self.n, F32)]
        self.active = 0
        self.updating = False
        self.bounds = [(lo, min(lo + shard_size, self.n)) for lo in range(0, self.n, shard_size)]
        self.opts = [Optimizer(kind, hi - lo, **hp) for lo, hi in self.bounds]

    def accumulate(self, g) -> None:
        g = np.asarray(g, dtype=F32)
        if g.size != self.n:
            raise ValueError("SizeMismatch")
        self.grads[self.active] += g

    def update_params(self) -> None:
        if self.updating:
            return
        self.updating = True
        frozen = self.active
        self.active ^= 1
        for (lo, hi), opt in zip(self.bounds, self.opts):
            g = self.grads[frozen][lo:hi]
            if self.nworkers > 1:
                g /= F32(self.nworkers)
            w = self.params[lo:hi]
            opt.update(g, w)
            g[:] = 0
        self.updating = False

    def pull_params(self) -> np.ndarray:
        return self.params.copy()


# ------------------------------------------------------------------ synthetic
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth(n: int, seed: int, rank: int, offset: int = 0) -> np.ndarray:
    """The §8(d) synthetic gradient generator (bit-identical to ono_ref_synth
    and to the device generator)."""
    g = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        key = _mix64(np.array([np.uint64(seed) + g * np.uint64(rank + 1)], dtype=np.uint64))[0]
        i = np.arange(offset, offset + n, dtype=np.uint64)
        h1 = _mix64(key + g * (i + np.uint64(1)))
        h2 = _mix64(h1 ^ np.uint64(0xD1B54A32D192ED03))
    cls = ((h1 >> np.uint64(32)) % np.uint64(100)).astype(np.uint32)
    sign = (h2 >> np.uint64(63)).astype(np.uint32)
    out = np.empty(n, dtype=F32)
    # normal class
    s4 = ((h2 & np.uint64(0xFFFF)) + ((h2 >> np.uint64(16)) & np.uint64(0xFFFF))
          + ((h2 >> np.uint64(32)) & np.uint64(0xFFFF)) + ((h2 >> np.uint64(48)) & np.uint64(0xFFFF)))
    scale = F32(float.fromhex("0x1.3c1a2ep-22"))
    out[:] = (s4.astype(np.int64) - 131070).astype(F32) * scale
    # f16-subnormal magnitudes
    m = cls == 1
    sub = ((h2 >> np.uint64(8)) & np.uint64(0x3FFFF)).astype(F32) * F32(2.0 ** -32)
    sub = np.where(sign == 1, -sub, sub)
    out[m] = sub[m]
    # exact f16 ties
    t = cls == 2
    e = ((h2 >> np.uint64(8)) % np.uint64(13)).astype(np.uint32)
    m10 = ((h2 >> np.uint64(16)) & np.uint64(0x3FF)).astype(np.uint32)
    tie = ((sign << 31) | ((e + 117) << 23) | (m10 << 13) | 0x1000).astype(np.uint32).view(F32)
    out[t] = tie[t]
    # signed zeros
    z = cls == 0
    out[z] = (sign[z] << 31).astype(np.uint32).view(F32)
    return out
