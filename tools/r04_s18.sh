# Round 4 session 18: config 2 against the 1R2W copy timed over the same buffers in the same passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do timeout -k 10 300 python -u tools/lr_leg.py > gpurun_out/lr_leg_$i.json 2> gpurun_out/lr_leg_$i.err || { tail -20 gpurun_out/lr_leg_$i.err; exit 1; }; done
python3 - <<'PY'
import json
for i in (1, 2):
    d = json.load(open(f"gpurun_out/lr_leg_{i}.json"))
    print(i, {k: (d[k]["us_per_launch"], d[k]["frac_of_hbm_peak"], d[k].get("frac_of_same_pool_copy_zero")) for k in ("k2", "k4", "k8", "copy_zero_same_pool")})
PY
