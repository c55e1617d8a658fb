"""Generate tests/golden/*.npz — run from the repo root: python tests/golden/make_golden.py

Golden vectors for the reduction path.  The reference (Rust) cannot be built
or imported here (no cargo/rustc, no network), so the
expected outputs come from the numpy restatement (oracle/oracle_np.py) and are
written ONLY if the independent C restatement (oracle/ono_oracle.c) agrees bit
for bit.  Inputs are the §8(d) synthetic gradients.
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from oracle import oracle_np as N  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 0x0402026

RING_CASES = [(1, 16), (2, 37), (2, 1000), (3, 4099), (4, 4099), (5, 17), (8, 4099), (8, 8), (7, 1031)]
SUM_CASES = [(2, 4099, 2.0), (3, 1000, 3.0), (4, 513, 4.0), (8, 257, 8.0), (5, 100, 5.0), (2, 64, 1.0)]


def bits(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a).view(np.uint32)


def same(a, b) -> bool:
    return np.array_equal(bits(np.asarray(a, np.float32)), bits(np.asarray(b, np.float32)))


def ring_fixtures() -> dict:
    out = {}
    for n, length in RING_CASES:
        res = [N.synth(length, SEED, r) for r in range(n)]
        assert all(same(a, O.synth(length, SEED, r)) for r, a in enumerate(res))
        for wire in ("f16", "f32"):
            g_np, r_np = N.ring_pull_grads(res, wire)
            g_c, r_c = O.ring_pull_grads(res, wire)
            assert all(same(a, b) for a, b in zip(g_np, g_c)), (n, length, wire)
            assert all(same(a, b) for a, b in zip(r_np, r_c)), (n, length, wire)
            key = f"n{n}_len{length}_{wire}"
            out[f"{key}_in"] = np.stack(res)
            out[f"{key}_grad"] = np.stack(g_np)
    return out


def sum_fixtures() -> dict:
    out = {}
    for k, length, d in SUM_CASES:
        ins = [N.synth(length, SEED + 17, r) for r in range(k)]
        a = N.sum_scale(ins, d)
        b = O.sum_scale(ins, d)
        assert same(a, b), (k, length, d)
        out[f"k{k}_len{length}_d{d:g}_in"] = np.stack(ins)
        out[f"k{k}_len{length}_d{d:g}_out"] = a
    return out


def f16_fixtures() -> dict:
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16)
    dec_np, dec_c = N.f16_bits_to_f32(h), O.f16_decode(h)
    assert same(dec_np, dec_c)
    rng = np.random.default_rng(7)
    x = np.concatenate([
        rng.integers(0, 2**32, 60_000, dtype=np.uint64).astype(np.uint32).view(np.float32),
        N.synth(20_000, SEED, 0),
        np.array([0.0, -0.0, 1.0, -1.0, 2.0, 65504.0, 65519.996, 65520.0, 1e9, -1e9, np.inf, -np.inf,
                  2.0 ** -24, 2.0 ** -25, 3 * 2.0 ** -26, 2.0 ** -14, 6.1e-5], np.float32),
        np.array([0x7FC00001, 0xFF800001, 0x7F812345, 0x7FFFFFFF], np.uint32).view(np.float32),
    ]).astype(np.float32)
    enc_np, enc_c = N.f32_to_f16_bits(x), O.f16_encode(x)
    assert np.array_equal(enc_np, enc_c)
    return {"decode_all_out": dec_np, "encode_in": x, "encode_out": enc_np}


def store_fixtures() -> dict:
    out = {}
    for kind in ("gd", "momentum", "adam"):
        for nworkers in (1, 3):
            params = N.synth(1031, SEED + 99, 0)
            hp = dict(lr=0.1, momentum=0.9, beta1=0.9, beta2=0.999, eps=1e-8)
            s_np = N.BlockingStore(params, 100, nworkers, kind, **hp)
            s_c = O.Store(params, 100, nworkers, kind, **hp)
            traj = []
            for rnd in range(4):
                for w in range(nworkers):
                    g = N.synth(1031, SEED + 1000 * rnd + w, w + 1)
                    s_np.accumulate(g)
                    s_c.accumulate(g)
                s_np.update_params()
                s_c.update_params()
                p_np, p_c = s_np.pull_params(), s_c.pull_params()
                assert same(p_np, p_c), (kind, nworkers, rnd)
                traj.append(p_np)
            out[f"{kind}_w{nworkers}_init"] = params
            out[f"{kind}_w{nworkers}_traj"] = np.stack(traj)
    return out


def main() -> None:
    np.savez_compressed(os.path.join(OUT, "ring.npz"), **ring_fixtures())
    np.savez_compressed(os.path.join(OUT, "sum_scale.npz"), **sum_fixtures())
    np.savez_compressed(os.path.join(OUT, "f16.npz"), **f16_fixtures())
    np.savez_compressed(os.path.join(OUT, "store.npz"), **store_fixtures())
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
