"""Repeat the n == 1 host-fed registered round (ono_ring_pull_grads_host) and
count rounds whose grad differs from the input: a probe for the ordering of
the CPU residual reset against the in-flight H2D DMA (measurement tool)."""
import sys

import numpy as np

sys.path[:0] = [".", "oxidized-neural-orchestra_amd"]
import ono_amd  # noqa: E402
from oracle import oracle as O  # noqa: E402

size = (5 << 20) + 3
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
bad = 0
for register in (True, False):
    ring = ono_amd.WorkerRingManager(0, 1, size)
    x = O.synth(size, 0x0402026, 7)
    res, grad = x.copy(), np.full(size, 3.0, np.float32)
    if register:
        ring.register_host(res)
        ring.register_host(grad)
    nb = 0
    for i in range(reps):
        res[:] = x
        ring.pull_grads_host(res, grad)
        d = int((grad.view(np.uint32) != x.view(np.uint32)).sum())
        if d:
            nb += 1
            print(f"register={register} rep {i}: {d} elements differ, first {int(np.flatnonzero(grad != x)[0])}")
    print(f"register={register}: {nb} of {reps} rounds wrong", flush=True)
    bad += nb
    ring.close()
sys.exit(1 if bad else 0)
