"""Measurement tool (not part of the product): ono_sum_scale_f32 at the
64 MiB config-2 bucket, the same launches timed over buffers from torch's
caching allocator and over buffers from hipMalloc directly, alternating in one
process (event span over L launches rotating over sets > 1.5 GiB), to tell a
placement effect from box-to-box and run-to-run drift.

usage: python tools/sum_alloc_ab.py [passes=3]
"""
import ctypes as C
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oxidized-neural-orchestra_amd")]

import torch  # noqa: E402

import ono_amd  # noqa: E402

N = 16 << 20
L = 40
hip = C.CDLL("libamdhip64.so")


def hip_bufs(count):
    out = []
    for _ in range(count):
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(N * 4)) == 0
        out.append(p.value)
    return out


def run(ptr_sets, k, stream):
    lib = ono_amd.lib()
    arrs = [((C.c_void_p * k)(*s[:k]), s[k]) for s in ptr_sets]
    for i in range(3):
        ins, out = arrs[i % len(arrs)]
        lib.ono_sum_scale_f32(C.c_void_p(out), ins, k, N, C.c_float(float(k)), C.c_void_p(stream.cuda_stream))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(stream)
    for i in range(L):
        ins, out = arrs[(3 + i) % len(arrs)]
        lib.ono_sum_scale_f32(C.c_void_p(out), ins, k, N, C.c_float(float(k)), C.c_void_p(stream.cuda_stream))
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / L


def main():
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    stream = torch.cuda.Stream()
    res = {}
    for k in (2, 4, 8):
        nsets = 1536 // ((k + 1) * 64) + 2
        tb = [torch.empty(N, dtype=torch.float32, device="cuda") for _ in range(nsets * (k + 1))]
        for i, t in enumerate(tb):
            ono_amd.kernels.synth(t, 7 + i, i % 9)
        tsets = [[t.data_ptr() for t in tb[s * (k + 1):(s + 1) * (k + 1)]] for s in range(nsets)]
        hb = hip_bufs(nsets * (k + 1))
        for i, p in enumerate(hb):
            ono_amd.lib().ono_synth_f32(C.c_void_p(p), N, 7 + i, i % 9, 0, None)
        hsets = [hb[s * (k + 1):(s + 1) * (k + 1)] for s in range(nsets)]
        for _ in range(passes):
            res.setdefault((k, "torch"), []).append(run(tsets, k, stream))
            res.setdefault((k, "hipMalloc"), []).append(run(hsets, k, stream))
        del tb
        for p in hb:
            hip.hipFree(C.c_void_p(p))
        torch.cuda.empty_cache()
    for (k, kind), v in sorted(res.items()):
        us = statistics.median(v)
        print(f"k={k} {kind:9s} {us:8.2f} us  {(k + 1) * 4 * N / us / 1e3 / 8000:.3f} of 8 TB/s  {[round(x, 2) for x in v]}")


if __name__ == "__main__":
    main()
