"""Where a SparseCapable TCP hop's codec time goes (round 5): each library call
the TCP ring makes per hop (ono_tcp.cpp out_sparse / incoming), timed alone on
one chunk of the config-1 bucket (54,693 values: 2 workers of the MLP
784-128-64-10) and of a 256 MiB bucket's half, host wall clock, median of 200
(20 for the large chunk) calls after warmup.

usage: python tools/sparse_call_costs.py [out.json]
"""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oxidized-neural-orchestra_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ono_amd  # noqa: E402
from ono_amd import kernels  # noqa: E402

L = ono_amd.lib()


def med_us(fn, reps, warm=5):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2)


def costs(n: int, r: float, reps: int) -> dict:
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    g = torch.empty(n, dtype=torch.float32, device="cuda")
    kernels.synth(g, 0x0402026, 0)
    torch.cuda.synchronize()
    m = min(n, 16384)
    idx = np.zeros(m, np.uint32)
    st = C.c_uint64(7)
    out = {"values": n, "r": r}
    if n > 16384:
        out["sample_default_host"] = med_us(
            lambda: L.ono_sparse_sample_default(C.byref(st), n, idx.ctypes.data, m), reps)
    t = C.c_float(0)
    ix = idx.ctypes.data if n > 16384 else None
    out["threshold"] = med_us(lambda: L.ono_sparse_threshold(C.byref(t), kernels.f32_ptr(g), n, ix, m, r, sh), reps)
    cap = L.ono_sparse_max_bytes(n)
    buf = torch.empty(cap + 8, dtype=torch.uint8, device="cuda")
    nb = C.c_size_t(0)
    out["drop_blocking"] = med_us(
        lambda: L.ono_sparse_drop(buf.data_ptr(), cap, C.byref(nb), kernels.f32_ptr(g), n, t, sh), reps)
    out["wire_bytes"] = nb.value
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")

    def drop_async_sync():
        L.ono_sparse_drop_async(buf.data_ptr(), cap, nbd.data_ptr(), kernels.f32_ptr(g), n, t, sh)
        s.synchronize()
    out["drop_async_then_sync"] = med_us(drop_async_sync, reps)
    host = bytes(buf[:nb.value].cpu().numpy())
    pinned = torch.empty(nb.value, dtype=torch.uint8).pin_memory()
    pinned.copy_(torch.frombuffer(bytearray(host), dtype=torch.uint8))
    dst = torch.empty(n, dtype=torch.float32, device="cuda")
    ln = C.c_size_t(0)
    out["lift_host_stream"] = med_us(
        lambda: L.ono_sparse_lift(kernels.f32_ptr(dst), n, C.byref(ln), pinned.data_ptr(), nb.value, sh), reps)
    out["lift_dev_blocking"] = med_us(
        lambda: L.ono_sparse_lift_dev(kernels.f32_ptr(dst), n, C.byref(ln), buf.data_ptr(), nb.value, sh), reps)
    status = torch.zeros(1, dtype=torch.int64, device="cuda")
    tk = C.c_uint64(0)

    def lift_async_sync():
        L.ono_sparse_lift_dev_async(kernels.f32_ptr(dst), n, buf.data_ptr(), nb.value, status.data_ptr(), C.byref(tk),
                                    sh)
        s.synchronize()
    out["lift_dev_async_then_sync"] = med_us(lift_async_sync, reps)

    def mask_sync():
        L.ono_sparse_mask(kernels.f32_ptr(dst), n, t, 1, sh)
        s.synchronize()
    out["mask_then_sync"] = med_us(mask_sync, reps)
    out["empty_sync"] = med_us(lambda: s.synchronize(), reps)
    return out


def main():
    torch.cuda.set_device(0)
    res = {"config1_chunk": costs(54693, 0.1, 200), "config1_chunk_r001": costs(54693, 0.01, 200),
           "256MiB_half": costs(1 << 25, 0.1, 20)}
    line = json.dumps(res)
    print(line)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
