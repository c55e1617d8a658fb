# Round 4 session 40: the whole GPU suite without stopping at a failure (session 39 stopped at one
# wrong cycle of test_xgmi_pool_release_then_fresh_rings[3]), then the stamped lift timings.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/s40_pytest_gpu.log 2>&1; r=$?
tail -6 gpurun_out/s40_pytest_gpu.log
[ $r -le 1 ] || exit $r
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s40_fused.txt 2>&1 || { cat gpurun_out/s40_fused.txt; exit 1; }
grep -E "# lift|^pl_" gpurun_out/s40_fused.txt | grep -v per-XCD
ONO_LIFT_FUSED=0 timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s40_two.txt 2>&1 || { cat gpurun_out/s40_two.txt; exit 1; }
grep -E "# lift|^pl_" gpurun_out/s40_two.txt | grep -v per-XCD
