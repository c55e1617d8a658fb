"""The pageable host-fed round's spread: 30 rounds of
ono_ring_pull_grads_host on a 256 MiB bucket (n = 1), per ONO_HOST_THREADS
setting, min / median / worst GiB/s, plus the CPU share the process sees
(affinity, cgroup cpu.max).  usage: python tools/host_fed_spread.py [out.json]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, time, json
sys.path[:0] = [{root!r}, {pkg!r}]
import numpy as np, ono_amd
n = 1 << 26
ring = ono_amd.WorkerRingManager(0, 1, n)
res, grad = np.empty(n, np.float32), np.empty(n, np.float32)
src = np.random.default_rng(1).standard_normal(n, dtype=np.float32) * np.float32(0.01)
ts = []
for r in range(31):
    res[:] = src
    t0 = time.perf_counter()
    ring.pull_grads_host(res, grad)
    if r:
        ts.append(time.perf_counter() - t0)
ts.sort()
g = lambda t: round(n * 4 / t / 2**30, 2)
print(json.dumps({{"best": g(ts[0]), "median": g(ts[len(ts) // 2]), "worst": g(ts[-1]),
                  "below_80pct_of_median": sum(t > ts[len(ts) // 2] / 0.8 for t in ts), "rounds": len(ts)}}))
"""


def main():
    out = {"affinity_cpus": len(os.sched_getaffinity(0)), "nproc": os.cpu_count()}
    try:
        out["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        out["cgroup_cpu_max"] = None
    for t in ("default", "16", "8"):
        env = dict(os.environ)
        if t != "default":
            env["ONO_HOST_THREADS"] = t
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, pkg=os.path.join(ROOT, "oxidized-neural-orchestra_amd"))],
                           capture_output=True, text=True, timeout=300, env=env)
        out[f"threads_{t}"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-300:]
        print(t, out[f"threads_{t}"], flush=True)
    line = json.dumps(out)
    print(line)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(line + "\n")


if __name__ == "__main__":
    main()
