# Round 4 session 20: the default bench line with the same-pool config-2 ceiling (bench.py only).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/bench_s20.log 2>&1 || { tail -30 gpurun_out/bench_s20.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_s20.log") if l.startswith("{")][0])
r = d["roofline"]
print({k: v for k, v in r.items() if not isinstance(v, (dict, list))})
print({k: d["local_reduce"][k] for k in ("k2", "k4", "k8", "copy_zero_same_pool")})
PY
