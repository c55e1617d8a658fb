"""Diagnose a sparse drop against the CPU oracle on the bench's workload
(64 MiB, synth(SEED, 7), threshold = 90th |g| percentile of the first 1 M)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "oxidized-neural-orchestra_amd"))
sys.path.insert(0, ROOT)
import ono_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker)

SEED = 0x0402026
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
seed = int(sys.argv[2], 0) if len(sys.argv) > 2 else SEED
g = ono_amd.kernels.synth(torch.empty(n, dtype=torch.float32, device="cuda"), seed, 7)
t = float(torch.quantile(g[: 1 << 20].abs().float(), 0.9).item())
got = ono_amd.sparse.grad_drop(g, t)
want = O.grad_drop(g.cpu().numpy(), t)
print("n", n, "t", t, "len got", len(got), "want", len(want))
if got == want:
    print("identical")
    sys.exit(0)
a, b = np.frombuffer(got, np.uint8), np.frombuffer(want, np.uint8)
m = min(len(a), len(b))
d = np.nonzero(a[:m] != b[:m])[0]
print("first diff at byte", d[0] if len(d) else m, "of", m, "ndiff", len(d))
# walk the reference stream to find the record holding that byte
pos, gi, rec = 8, 0, 0
while pos < len(b):
    off = int(np.frombuffer(b[pos:pos + 4].tobytes(), "<u4")[0]); ln = int(np.frombuffer(b[pos + 4:pos + 8].tobytes(), "<u4")[0])
    gi += off
    end = pos + 8 + 2 * ln
    if len(d) and end > d[0]:
        print("record", rec, "at byte", pos, "offset", off, "len", ln, "start elem", gi, "tile", gi // 2048,
              "elem in tile", gi % 2048)
        print("got  hdr", np.frombuffer(a[pos:pos + 8].tobytes(), "<u4"), "want hdr", (off, ln))
        break
    gi += ln
    pos = end
    rec += 1
sys.exit(1)
