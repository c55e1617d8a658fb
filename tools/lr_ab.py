"""Measurement tool (not part of the product): bench.py's local_reduce against
tools/sum_alloc_ab.py's loop in one process, interleaved, to find why the
bench's k = 8 figure sits below the standalone tools' (same kernel, same
rotation).  Variants of the bench loop:
  bench      bench.local_reduce as shipped (ono_amd.kernels.sum_scale per launch)
  raw        the same buffers, prebuilt ctypes argument arrays (no wrapper)
  fresh      raw over a newly allocated set of buffers each pass
  carved / carved_skew68k   raw over buffers carved from one allocation (each 68 KiB further)
  bench_k_only / bench_warm4 / bench_settle   bench.local_reduce for this k alone; with four
             rotations of warm-up; with a synchronised 0.5 s pause before the warm-up

usage: python tools/lr_ab.py [passes=3] [steps=40]
"""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oxidized-neural-orchestra_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import ono_amd  # noqa: E402

N = 16 << 20


def make_sets(k):
    nsets = 1536 // ((k + 1) * 64) + 2
    sets = []
    for si in range(nsets):
        ins = [ono_amd.kernels.synth(torch.empty(N, device="cuda"), 7 + si, r) for r in range(k)]
        sets.append((ins, torch.empty(N, device="cuda")))
    return sets


def carved_sets(k, skew_bytes=0):
    """every buffer of the rotation carved from ONE allocation (optionally each
    one `skew_bytes` further than the previous one's end)"""
    nsets = 1536 // ((k + 1) * 64) + 2
    per = N + skew_bytes // 4
    big = torch.empty(per * nsets * (k + 1), device="cuda")
    views = [big[i * per:i * per + N] for i in range(nsets * (k + 1))]
    for i, v in enumerate(views):
        ono_amd.kernels.synth(v, 7 + i // (k + 1), i % (k + 1))
    return [(views[s * (k + 1):s * (k + 1) + k], views[s * (k + 1) + k]) for s in range(nsets)], big


def raw(sets, k, steps, stream, warmup=3):
    lib = ono_amd.lib()
    args = [((C.c_void_p * k)(*[t.data_ptr() for t in ins]), C.c_void_p(out.data_ptr())) for ins, out in sets]
    sh = C.c_void_p(stream.cuda_stream)
    for i in range(warmup):
        a, o = args[i % len(args)]
        lib.ono_sum_scale_f32(o, a, k, N, C.c_float(float(k)), sh)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for i in range(steps):
        a, o = args[(warmup + i) % len(args)]
        lib.ono_sum_scale_f32(o, a, k, N, C.c_float(float(k)), sh)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


def wrapped(sets, k, steps, stream, warmup=3):
    for i in range(warmup):
        ins, dst = sets[i % len(sets)]
        ono_amd.kernels.sum_scale(dst, ins, float(k), stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for i in range(steps):
        ins, dst = sets[(warmup + i) % len(sets)]
        ono_amd.kernels.sum_scale(dst, ins, float(k), stream)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    stream = torch.cuda.Stream()
    res = {}
    for k in (8, 4, 2):
        sets = make_sets(k)
        for _ in range(passes):
            lr = bench.local_reduce(torch, ono_amd, steps, 3)
            res.setdefault((k, "bench"), []).append(lr[f"k{k}"]["us_per_launch"])
            lr = bench.local_reduce(torch, ono_amd, steps, 3, ks=(k,))
            res.setdefault((k, "bench_k_only"), []).append(lr[f"k{k}"]["us_per_launch"])
            lr = bench.local_reduce(torch, ono_amd, steps, 3, ks=(k,), warm_rotations=4)
            res.setdefault((k, "bench_warm4"), []).append(lr[f"k{k}"]["us_per_launch"])
            lr = bench.local_reduce(torch, ono_amd, steps, 3, ks=(k,), settle_s=0.5)
            res.setdefault((k, "bench_settle"), []).append(lr[f"k{k}"]["us_per_launch"])
            res.setdefault((k, "wrapped"), []).append(wrapped(sets, k, steps, stream))
            res.setdefault((k, "raw"), []).append(raw(sets, k, steps, stream))
            fresh = make_sets(k)
            res.setdefault((k, "fresh"), []).append(raw(fresh, k, steps, stream))
            del fresh
            cs, big = carved_sets(k)
            res.setdefault((k, "carved"), []).append(raw(cs, k, steps, stream))
            del cs, big
            cs, big = carved_sets(k, 4096 * 17)
            res.setdefault((k, "carved_skew68k"), []).append(raw(cs, k, steps, stream))
            del cs, big
            torch.cuda.empty_cache()
        del sets
        torch.cuda.empty_cache()
    for (k, kind), v in sorted(res.items()):
        us = statistics.median(v)
        print(f"k={k} {kind:8s} {us:8.2f} us  {(k + 1) * 4 * N / us / 1e3 / 8000:.3f} of 8 TB/s  "
              f"{[round(x, 2) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
