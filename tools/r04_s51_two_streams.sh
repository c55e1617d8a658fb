# Round 4 session 51: two large stream-ordered lifts on two streams at once with the one-in-flight guard
# (events recorded only once a second stream used the form), the sparse and TCP GPU tests, the timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s51_pytest.log 2>&1 || { tail -30 gpurun_out/s51_pytest.log; exit 1; }
tail -2 gpurun_out/s51_pytest.log
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s51_fused.txt 2>&1 || { cat gpurun_out/s51_fused.txt; exit 1; }
grep -E "# lift" gpurun_out/s51_fused.txt
