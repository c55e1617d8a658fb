# Round 4 session 5: sparse parity + codec timing (pl_index one tile per workgroup by
# default, ONO_PL_TPB=2 as a variant; vectorised tile sums in pl_place), launch_phases
# decode / fill rows at 64 MiB, and the bench line with the pooled local_reduce.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
SP_VARIANTS="ONO_PL_TPB=2" bash tools/sp_gpu.sh || exit 1
timeout -k 10 200 ./tools/launch_phases 64 24 > gpurun_out/lp5.txt 2>&1 || { cat gpurun_out/lp5.txt; exit 1; }
grep -E "^(fill|f16 decode|decode|copy)" gpurun_out/lp5.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-tcp-edge --xgmi-coresident 0 > gpurun_out/bench_s5.log 2>&1 || { tail -20 gpurun_out/bench_s5.log; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_s5.log").read().strip().splitlines()[-1])
print("value", d["value"], "roofline", {k: v for k, v in d["roofline"].items() if not isinstance(v, dict)})
for k in ("local_reduce", "copy_ceiling"):
    print(k, {a: (b.get("us_per_launch"), b.get("frac_of_hbm_peak"), b.get("us_per_launch_min"), b.get("us_per_launch_max")) if isinstance(b, dict) else b for a, b in d[k].items() if a not in ("workload", "timing", "hbm_peak_gbs")})
print("path_kernels", {a: b.get("frac_of_hbm_peak") for a, b in d["path_kernels"].items() if isinstance(b, dict)})
sc = d["sparse_codec"]
print("sparse drop", sc["drop"].get("stream_ms"), sc["drop"].get("stream_frac_of_hbm_peak"), "lift", sc["lift_dev"].get("stream_ms"), sc["lift_dev"].get("stream_frac_of_hbm_peak"))
print("host_fed", d.get("host_fed"))
PY
