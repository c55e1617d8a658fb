"""Drop + device lift of the bench's sparse workload (64 MiB gradient, 90th
percentile threshold), K times — a short program for rocprofv3 kernel stats."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oxidized-neural-orchestra_amd"))
import ono_amd  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = 16 << 20
g = ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), 1234, 7)
t = float(torch.quantile(g[: 1 << 20].abs().float(), 0.9).item())
L = ono_amd.lib()
wire = ono_amd.sparse.grad_drop_dev(g, t)
out = torch.empty(n, dtype=torch.float32, device="cuda")
ln = C.c_size_t(0)
s = torch.cuda.current_stream().cuda_stream
for _ in range(K):
    ono_amd._lib.call("ono_sparse_lift_dev", out.data_ptr(), n, C.byref(ln), wire.data_ptr(), wire.numel(), s)
torch.cuda.synchronize()
print("fallbacks", L.ono_sparse_lift_fallbacks(), "wire", wire.numel())
