# Round 4 session 44: the default of two chunk-line replicas under the sparse, pattern and TCP GPU
# tests, and its stamped timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s44_pytest.log 2>&1 || { tail -30 gpurun_out/s44_pytest.log; exit 1; }
tail -2 gpurun_out/s44_pytest.log
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s44_fused.txt 2>&1 || { cat gpurun_out/s44_fused.txt; exit 1; }
grep -E "# lift|^pl_|look-back done" gpurun_out/s44_fused.txt | grep -v per-XCD
