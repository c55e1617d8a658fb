# Round 4 session 50: the graph-capture test with the capture guard (expected to pass) and without it
# (ONO_LIFT_FUSED=2: the one launch captured; expected to fail — the replays' granules pass for each
# other's), then the sparse pattern, sparse and TCP GPU tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=tests/test_gpu_sparse_pattern.py::test_async_lift_under_graph_capture_replays_new_streams
ONO_LIFT_FUSED=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $T > gpurun_out/s50_unguarded.log 2>&1; echo "unguarded rc=$? (1 = the test failed, as expected)"; grep -E "differ|assert|passed|failed" gpurun_out/s50_unguarded.log | head -5
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s50_pytest.log 2>&1; r=$?
tail -2 gpurun_out/s50_pytest.log
exit $r
