"""Measurement tool (not part of the product): bench.py's path_kernels and
copy_ceiling legs in child processes under environment variants, alternating,
so that a library knob (e.g. ONO_EW_WIDE=0: the 256-thread fill / decode back on
64-thread workgroups) is compared on the same box with the bench's own data.

usage: python tools/pk_ab.py [rounds=2] [VAR=value ...]   (each VAR=value is one variant; "-" = default)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "oxidized-neural-orchestra_amd")]
import torch, ono_amd, bench
pk = bench.path_kernels(torch, ono_amd, 20, 2)
cc = bench.copy_ceiling(torch, ono_amd, 20, 2)
print(json.dumps({{"pk": {{k: v.get("us_per_launch") for k, v in pk.items() if isinstance(v, dict)}},
                   "cc": {{k: v.get("us_per_launch") for k, v in cc.items() if isinstance(v, dict)}}}}))
"""


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    variants = sys.argv[2:] or ["-", "ONO_EW_WIDE=0"]
    res = {}
    for r in range(rounds):
        for v in variants:
            env = dict(os.environ)
            if v != "-":
                k, val = v.split("=", 1)
                env[k] = val
            p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True,
                               text=True, timeout=240)
            if p.returncode:
                print(v, "failed", p.stderr[-2000:])
                return 1
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
            print(f"round {r} {v}: decode {d['pk'].get('f16_decode_scale')} fill64 {d['cc'].get('fill_64MiB')} "
                  f"fill256 {d['cc'].get('fill_256MiB')} copy64 {d['cc'].get('copy_64MiB')}", flush=True)
    for v, ds in res.items():
        keys = sorted(ds[0]["pk"]) + sorted("cc." + k for k in ds[0]["cc"])
        row = {}
        for k in keys:
            src = "cc" if k.startswith("cc.") else "pk"
            kk = k[3:] if src == "cc" else k
            vals = sorted(d[src][kk] for d in ds if d[src].get(kk) is not None)
            if vals:
                row[k] = vals[len(vals) // 2]
        print(v, json.dumps(row))
    return 0


if __name__ == "__main__":
    sys.exit(main())
