"""The DIRECT schedule's owner-chain arithmetic on one GPU (ono_local_direct_pull_grads:
R ranks' 256 MiB buckets in one process), K rounds over rotating residual sets — a short
program for rocprofv3 kernel stats of DirectOp (the N > 1 compute kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oxidized-neural-orchestra_amd"))
import ono_amd  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
wire = sys.argv[3] if len(sys.argv) > 3 else "f16"
n = (64 << 20) if len(sys.argv) <= 4 else int(sys.argv[4])
sets = [[ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), 7 + s, r) for r in range(R)]
        for s in range(3)]
grads = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(R)]
torch.cuda.synchronize()
for k in range(K):
    res = sets[k % 3]
    ono_amd.ring.local_ring_pull_grads(res, grads, wire=wire, algo="direct")
    if k % 3 == 2:
        for s in range(3):
            for r in range(R):
                ono_amd.kernels.synth(sets[s][r], 7 + s + k, r)
torch.cuda.synchronize()
print("ok", R, K, wire, n)
