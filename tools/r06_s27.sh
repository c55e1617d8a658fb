# Round 6 session 27: thr_bench again with two more variants (four bits a step with early exit; gather + select
# in one launch, the last workgroup to arrive selecting)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/thr_bench 200 > gpurun_out/r06_s27_thr_bench.json 2>&1 || { cat gpurun_out/r06_s27_thr_bench.json; exit 1; }
timeout -k 10 60 tools/thr_bench 200 >> gpurun_out/r06_s27_thr_bench.json 2>&1 || exit 1
cat gpurun_out/r06_s27_thr_bench.json
