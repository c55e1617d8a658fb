"""The drop's A/B (round 5): bench.py's sparse_codec leg (64 MiB gradient, 10 % kept, stream-ordered and
blocking drop / lift) and the config-1 chunk's drop cost, once with the one-launch encoder (default) and
once with ONO_DROP_FUSED=0 (sp_image + sp_move), each in its own process.
usage: python tools/drop_ab.py [out.json]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, json
sys.path[:0] = [{root!r}, {pkg!r}]
import torch, ono_amd, bench
sys.path.insert(0, {tools!r})
import sparse_call_costs as S
torch.cuda.set_device(0)
sc = bench.sparse_codec(torch, ono_amd)
c1 = S.costs(54693, 0.1, 200)
print(json.dumps({{"drop": sc["drop"], "lift": sc.get("lift"), "config1_drop_blocking_us": c1["drop_blocking"],
                  "config1_drop_async_then_sync_us": c1["drop_async_then_sync"]}}))
"""


def main():
    out = {}
    for name, env in (("one_launch", {}), ("two_launches", {"ONO_DROP_FUSED": "0"})):
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, pkg=os.path.join(ROOT, "oxidized-neural-orchestra_amd"),
                                                               tools=os.path.join(ROOT, "tools"))],
                           capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
        out[name] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-600:]
        print(name, json.dumps(out[name])[:800], flush=True)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(json.dumps(out) + "\n")


if __name__ == "__main__":
    main()
