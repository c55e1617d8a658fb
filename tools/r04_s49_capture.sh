# Round 4 session 49: the stream-ordered lift under graph capture (two launches, replays over new
# stream contents) and the rest of the sparse pattern, sparse and TCP GPU tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s49_pytest.log 2>&1; r=$?
tail -25 gpurun_out/s49_pytest.log
exit $r
