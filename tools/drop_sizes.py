"""The drop's cost by size, one-launch encoder (sp_drop1) against the two launches (sp_image +
sp_move, ONO_DROP_FUSED=0), each form in its own process: blocking call (host wall clock, median)
and stream-ordered (ono_sparse_drop_async, K back to back between two events, over 6 gradients in
turn), ~10 % kept.  Picks the size up to which the one launch is used (kDropOneLaunchTiles).
usage: python tools/drop_sizes.py [out.json]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, json, time, statistics, ctypes as C
sys.path[:0] = [{root!r}, {pkg!r}]
import numpy as np, torch, ono_amd
from ono_amd import kernels
L = ono_amd.lib()
torch.cuda.set_device(0)
s = torch.cuda.current_stream(); sh = s.cuda_stream
out = {{}}
for n in {sizes!r}:
    gs = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(6)]
    for i, g in enumerate(gs):
        kernels.synth(g, 0x0402026 + i, 0)
    torch.cuda.synchronize()
    t = float(gs[0].abs().float().quantile(0.9).item()) if n <= 1 << 24 else float(gs[0][: 1 << 24].abs().quantile(0.9).item())
    cap = L.ono_sparse_max_bytes(n)
    buf = torch.empty(cap + 8, dtype=torch.uint8, device="cuda")
    nb = C.c_size_t(0)
    reps = 200 if n <= 1 << 20 else 30
    ts = []
    for r in range(reps + 5):
        g = gs[r % 6]
        t0 = time.perf_counter()
        assert L.ono_sparse_drop(buf.data_ptr(), cap, C.byref(nb), kernels.f32_ptr(g), n, C.c_float(t), sh) == 0
        if r >= 5:
            ts.append(time.perf_counter() - t0)
    nbd = torch.zeros(1, dtype=torch.int64, device="cuda")
    K = 48
    for r in range(8):
        L.ono_sparse_drop_async(buf.data_ptr(), cap, nbd.data_ptr(), kernels.f32_ptr(gs[r % 6]), n, C.c_float(t), sh)
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for r in range(K):
        L.ono_sparse_drop_async(buf.data_ptr(), cap, nbd.data_ptr(), kernels.f32_ptr(gs[r % 6]), n, C.c_float(t), sh)
    e1.record(); torch.cuda.synchronize()
    out[n] = {{"blocking_us": round(statistics.median(ts) * 1e6, 2), "stream_us": round(e0.elapsed_time(e1) * 1e3 / K, 2),
               "wire": nb.value}}
    del gs, buf
print(json.dumps(out))
"""
SIZES = [54_693, 262_144, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20]


def main():
    res = {}
    for name, env in (("one_launch", {"ONO_DROP_ONE_LAUNCH_TILES": "1000000000"}), ("two_launches", {"ONO_DROP_FUSED": "0"})):
        code = CHILD.format(root=ROOT, pkg=os.path.join(ROOT, "oxidized-neural-orchestra_amd"), sizes=SIZES)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=400,
                           env=dict(os.environ, **env))
        res[name] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-800:]
        print(name, json.dumps(res[name]), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
