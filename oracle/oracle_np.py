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
  sparse codec   comms/src/sparse/protocol.rs:33-144
  serializer     comms/src/handles/compressor.rs:71-98, handles/worker.rs:157-174
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


# ------------------------------------------------------------------ sparse codec
SAMPLE_SIZE_MAX = 1 << 14                 # protocol.rs:21
MIN_POSITIVE_F16 = F32(6.103515625e-05)   # f16::MIN_POSITIVE (protocol.rs:22)
_G64 = 0x9E3779B97F4A7C15
_MASK64 = (1 << 64) - 1


def _mix64_int(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return z ^ (z >> 31)


def sample_default(state: int, length: int, amount: int):
    """The library's stand-in for rand's index::sample (Floyd over splitmix64):
    (indices in draw order, next state).  amount == length draws nothing."""
    if amount >= length:
        return np.arange(length, dtype=np.uint32), state
    seen, out = set(), []
    for j in range(length - amount, length):
        state = (state + _G64) & _MASK64
        t = _mix64_int(state) % (j + 1)
        if t in seen:
            t = j
        seen.add(t)
        out.append(t)
    return np.array(out, dtype=np.uint32), state


def calculate_threshold(residual: np.ndarray, r: float, sample_idx) -> F32:
    """protocol.rs:33-49 over the drawn sample (the k-th order statistic does
    not depend on the order the sample is drawn in)."""
    if residual.size == 0:
        return F32(0)
    bits = residual.view(np.uint32)[np.asarray(sample_idx, dtype=np.int64)] & np.uint32(0x7FFFFFFF)  # abs
    m = bits.size
    with np.errstate(invalid="ignore"):
        kf = F32(m) * (F32(1) - F32(r))          # f32 arithmetic
    k = 0 if not (kf > 0) else int(kf)            # `as usize`: truncates, saturates at 0 (NaN -> 0)
    k = min(max(k, 0), m - 1)
    # total_cmp on non-negative values (NaN above +inf) is the order of the bit patterns
    x = np.sort(bits)[k].view(F32)
    return F32(np.fmax(x, MIN_POSITIVE_F16))     # f32::max ignores NaN


def grad_drop(residual: np.ndarray, threshold) -> bytes:
    """grad_drop_into (protocol.rs:57-86): [u64 LE len] then, per run of
    |g| >= threshold, [u32 LE offset from the previous run's end][u32 LE run]
    [f16 LE values]."""
    g = np.ascontiguousarray(residual, dtype=F32)
    keep = np.abs(g) >= F32(threshold)
    edges = np.flatnonzero(np.diff(np.concatenate(([False], keep, [False])).astype(np.int8)))
    starts, ends = edges[0::2], edges[1::2]
    parts = [np.uint64(g.size).tobytes()]
    last_end = 0
    h = f32_to_f16_bits(g)
    for a, b in zip(starts.tolist(), ends.tolist()):
        parts.append(np.array([a - last_end, b - a], dtype="<u4").tobytes())
        parts.append(h[a:b].astype("<u2").tobytes())
        last_end = b
    return b"".join(parts)


def grad_lift(buf: bytes) -> np.ndarray:
    """grad_lift_into (protocol.rs:96-144) into a fresh buffer; raises the
    reference's error strings."""
    if len(buf) < 8:
        raise ValueError("The given sparse buffer is smaller than TOTAL_LEN_SIZE")
    total = int.from_bytes(buf[:8], "little")
    g = np.zeros(total, dtype=F32)
    body = buf[8:]
    gi = bi = 0
    while bi < len(body):
        if bi + 4 > len(body):
            raise ValueError("Missing index bytes at grad lift")
        gi += int.from_bytes(body[bi:bi + 4], "little")
        bi += 4
        if bi + 4 > len(body):
            raise ValueError("Missing chunk length bytes at grad lift")
        cl = int.from_bytes(body[bi:bi + 4], "little")
        bi += 4
        if gi > total or total - gi < cl:
            raise ValueError("Gradient chunk exceeds target vector bounds")
        if bi + 2 * cl > len(body):
            raise ValueError("Truncated float data")
        g[gi:gi + cl] = f16_bits_to_f32(np.frombuffer(body[bi:bi + 2 * cl], dtype="<u2"))
        bi += 2 * cl
        gi += cl
    return g


def push_grad(chunk: np.ndarray, ratio: float, state: int):
    """WorkerHandle::push_grad (handles/worker.rs:157-174) over
    Compressor::compress (compressor.rs:71-98): returns (what the receiver's
    recv_event hands its ring, Some(threshold) -> float or None -> None, the
    sampler state after the push, the wire payload's kind 1 or 3)."""
    if ratio > 0:
        m = min(chunk.size, SAMPLE_SIZE_MAX)
        if chunk.size > SAMPLE_SIZE_MAX:
            idx, state = sample_default(state, chunk.size, m)
        else:
            idx = np.arange(chunk.size)
        t = calculate_threshold(chunk, ratio, idx)
        buf = grad_drop(chunk, t)
        if len(buf) <= chunk.size * 2:          # compressor.rs:79
            return grad_lift(buf), t, state, 3
    return quantize_f16(chunk), None, state, 1


def ring_pull_grads_sparse(residuals: list[np.ndarray], ratios, states):
    """One pull_grads() round of every worker, each with its own serializer
    (ratio 0 = Base), written from worker_ring.rs:112-204 as the reference
    states it.  Returns (grads, residuals_after, states_after)."""
    n = len(residuals)
    length = residuals[0].size
    chunks = split_chunks(length, n)
    if len(chunks) < n:
        raise ValueError("reference panics: fewer chunks than ranks")
    res = [np.array(r, dtype=F32, copy=True) for r in residuals]
    grads = [np.zeros(length, dtype=F32) for _ in range(n)]
    st = list(states)
    i = list(range(n))
    for _ in range(n - 1):                       # scatter, :121-144
        events = []
        for r in range(n):
            lo, hi = chunks[i[r]]
            ev, sent, st[r], _ = push_grad(res[r][lo:hi], ratios[r], st[r])
            events.append(ev)
            ch = res[r][lo:hi]
            if sent is not None:                 # :126-132
                ch[np.abs(ch) >= sent] = F32(0)
            else:                                # :133
                ch[:] = F32(0)
        for r in range(n):
            i[r] = (i[r] + n - 1) % n            # :140
            lo, hi = chunks[i[r]]
            agg = events[(r - 1) % n]
            k = min(hi - lo, agg.size)           # the zip stops at the shorter
            res[r][lo:lo + k] += agg[:k]
    for r in range(n):                           # gather, :163-166
        i[r] = (r + 1) % n
        lo, hi = chunks[i[r]]
        grads[r][lo:hi] = res[r][lo:hi]
    if n == 1:                                   # :168-171
        lo, hi = chunks[i[0]]
        res[0][lo:hi] = F32(0)
        return grads, res, st
    for j in range(n - 1):                       # :173-201
        events = []
        for r in range(n):
            lo, hi = chunks[i[r]]
            ev, sent, st[r], _ = push_grad(grads[r][lo:hi], ratios[r], st[r])
            events.append(ev)
            if sent is not None:                 # :177-190 (the residual is not touched)
                ch = grads[r][lo:hi]
                ch[np.abs(ch) < sent] = F32(0)
            elif j == 0:                         # :191-193
                res[r][lo:hi] = F32(0)
        for r in range(n):
            i[r] = (i[r] + n - 1) % n            # :199
            lo, hi = chunks[i[r]]
            acc = events[(r - 1) % n]
            if acc.size != hi - lo:
                raise ValueError("copy_from_slice panics on a length mismatch")
            grads[r][lo:hi] = acc                # :200
    f = F32(n)                                   # :101-105
    grads = [(g / f).astype(F32) for g in grads]
    return grads, res, st


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
