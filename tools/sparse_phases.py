"""Phase timing of the one-pass sparse encoder (measurement tool): per-
workgroup wall-clock stamps (start, first tile counted, record published,
records scanned, end; 100 MHz) of one drop of the bench's 64 MiB workload."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oxidized-neural-orchestra_amd"))
import ono_amd  # noqa: E402

n = 16 << 20
g = ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), 1234, 7)
t = float(torch.quantile(g[: 1 << 20].abs().float(), 0.9).item())
L = ono_amd.lib()
L.ono_sparse_drop_debug.argtypes = [C.c_void_p]
dbg = torch.zeros(5 * 4096, dtype=torch.int64, device="cuda")
for it in range(3):
    dbg.zero_()
    L.ono_sparse_drop_debug(dbg.data_ptr())
    ono_amd.sparse.grad_drop_dev(g, t)
    L.ono_sparse_drop_debug(None)
    d = dbg.cpu().numpy().reshape(-1, 5)
    d = d[d[:, 0] > 0].astype(np.float64)
    t0 = d[:, 0].min()
    rel = (d - t0) / 100.0  # us
    print(f"drop {it}: {len(d)} workgroups")
    for k, name in enumerate(["start", "tile0 counted", "published", "scanned", "end"]):
        col = rel[:, k]
        print(f"  {name:14s} min {col.min():8.1f} med {np.median(col):8.1f} max {col.max():8.1f} us")
