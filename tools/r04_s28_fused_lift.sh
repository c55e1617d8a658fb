# Round 4 session 28: the stream-ordered lift in one launch (pl_fused) against pl_index + pl_place
# (ONO_LIFT_FUSED=0), stamped, then the sparse and TCP GPU tests on the fused path.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s28_fused.txt 2>&1 || { cat gpurun_out/s28_fused.txt; exit 1; }
grep -E "^#|^pl_" gpurun_out/s28_fused.txt | grep -v per-XCD
ONO_LIFT_FUSED=0 timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s28_two.txt 2>&1 || { cat gpurun_out/s28_two.txt; exit 1; }
grep -E "# lift|^pl_" gpurun_out/s28_two.txt | grep -v per-XCD
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s28_fused2.txt 2>&1 || { cat gpurun_out/s28_fused2.txt; exit 1; }
grep -E "# lift|^pl_" gpurun_out/s28_fused2.txt | grep -v per-XCD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s28_pytest.log 2>&1; r=$?
tail -5 gpurun_out/s28_pytest.log
exit $r
