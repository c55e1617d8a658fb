"""Measurement tool (not part of the product): the path's kernels as bench.py
times them (local_reduce, path_kernels) plus the pull_grads finaliser
(scale_zero at the 256 MiB headline bucket), printed as one JSON line for the
occupancy cap this process runs under (ONO_EW_OCC, read once by the library;
tools/occ_sweep.sh runs one process per cap).

usage: ONO_EW_OCC=<cap> python tools/occ_probe.py [steps=30] [rounds=1]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oxidized-neural-orchestra_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import ono_amd  # noqa: E402


def scale_zero(steps: int, warmup: int = 3) -> dict:
    n = 64 << 20  # 256 MiB: the headline bucket
    nsets = 4     # 4 x 768 MiB rotation
    sets = [(torch.empty(n, device="cuda"), ono_amd.kernels.synth(torch.empty(n, device="cuda"), 7 + i, 0),
             torch.empty(n, device="cuda")) for i in range(nsets)]
    stream = torch.cuda.current_stream()
    for i in range(warmup):
        d, s, z = sets[i % nsets]
        ono_amd.kernels.scale_zero(d, s, 2.0, z)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(stream)
    for i in range(steps):
        d, s, z = sets[(warmup + i) % nsets]
        ono_amd.kernels.scale_zero(d, s, 2.0, z)
    b.record(stream)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / steps * 1e3
    del sets
    torch.cuda.empty_cache()
    return {"us_per_launch": round(us, 2), "frac_of_hbm_peak": round(12 * n / us / 1e3 / bench.HBM_PEAK_GBS, 4)}


def ring_local(algo: str, wire: str, steps: int, ranks: int = 4) -> float:
    """us per pull_grads round of `ranks` co-resident ranks (ono_plan_run_local),
    64 MiB per rank; per-kernel times come from a rocprofv3 kernel trace."""
    n = 16 << 20
    res = [ono_amd.kernels.synth(torch.empty(n, device="cuda"), 11, r) for r in range(ranks)]
    grads = [torch.empty(n, device="cuda") for _ in range(ranks)]
    ono_amd.plan.run_local(algo, wire, res, grads)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(steps):
        ono_amd.plan.run_local(algo, wire, res, grads)
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / steps * 1e3, 2)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    runs = []
    for _ in range(rounds):
        res = {"scale_zero_256mib": scale_zero(steps)["frac_of_hbm_peak"]}
        lr = bench.local_reduce(torch, ono_amd, steps, 3)
        res.update({f"sum_{k}": lr[k]["frac_of_hbm_peak"] for k in ("k2", "k4", "k8")})
        pk = bench.path_kernels(torch, ono_amd, steps, 3)
        res.update({k: v["frac_of_hbm_peak"] for k, v in pk.items() if isinstance(v, dict)})
        res["hops_f16_n4_us"] = ring_local("hops", "f16", steps)
        runs.append(res)
    out = {"occ": os.environ.get("ONO_EW_OCC", "default"), "rounds": rounds}
    out.update({k: statistics.median(r[k] for r in runs) for k in runs[0]})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
