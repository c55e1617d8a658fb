"""A/B of the stream-ordered 64 MiB sparse drop between library builds (round 6): each .so is loaded with
ctypes (RTLD_LOCAL: their symbols do not meet), and the passes alternate A, B, A, B ... over the same 6
rotating 64 MiB gradients (bench.py's sparse_codec shape: 24 drops back to back, one event pair).  Prints one
JSON line: per library the per-pass us per drop, the median, and whether its bytes equal the first library's.
usage: python tools/drop_lib_ab.py LIB_A LIB_B [passes]"""
import ctypes as C
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oxidized-neural-orchestra_amd"))
import ono_amd  # noqa: E402  (synth only: the gradients)


def main():
    libs = sys.argv[1:3]
    passes = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    L = [C.CDLL(os.path.abspath(p)) for p in libs]
    for l in L:
        l.ono_sparse_drop_async.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t, C.c_float,
                                            C.c_void_p]
        l.ono_sparse_max_bytes.argtypes = [C.c_size_t]
        l.ono_sparse_max_bytes.restype = C.c_size_t
    n, NG, K = 16 << 20, 6, 24
    gs = [ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), 1234 + i, 7) for i in range(NG)]
    tg = [float(torch.quantile(g[: 1 << 20].abs().float(), 0.9).item()) for g in gs]
    cap = L[0].ono_sparse_max_bytes(n)
    bufs = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in L]
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    h = s.cuda_stream

    def drop(li, i):
        rc = L[li].ono_sparse_drop_async(bufs[li].data_ptr(), cap, nbd.data_ptr(), gs[i % NG].data_ptr(), n,
                                         tg[i % NG], h)
        assert rc == 0, (libs[li], rc)

    wires = []
    for li in range(len(L)):
        drop(li, 0)
        torch.cuda.synchronize()
        nb = int(nbd.item())
        wires.append(bytes(bufs[li][:nb].cpu().numpy()))
    res = {p: [] for p in libs}
    for _ in range(passes):
        for li, p in enumerate(libs):
            for i in range(2 * NG):
                drop(li, i)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for i in range(K):
                drop(li, i)
            b.record(s)
            torch.cuda.synchronize()
            res[p].append(round(a.elapsed_time(b) * 1e3 / K, 2))
    out = {p: {"us_per_drop": v, "median": statistics.median(v), "bytes_equal_first": wires[i] == wires[0]}
           for i, (p, v) in enumerate(res.items())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
