# Round 6 session 26: the config-1 push's threshold (tools/thr_bench): gather + select back to back and one at a
# time, the select's phases (stamped copy), and two select variants (early exit at one candidate; four waves)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/thr_bench 200 > gpurun_out/r06_s26_thr_bench.json 2>&1 || { cat gpurun_out/r06_s26_thr_bench.json; exit 1; }
timeout -k 10 60 tools/thr_bench 200 >> gpurun_out/r06_s26_thr_bench.json 2>&1 || exit 1
cat gpurun_out/r06_s26_thr_bench.json
