# Round 4 session 45: the xGMI tests with the recreate worker's failure description (runs, sub-rounds,
# owner chunks, what the wrong values equal), run once.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_xgmi.py > gpurun_out/s45_pytest_xgmi.log 2>&1; r=$?
tail -8 gpurun_out/s45_pytest_xgmi.log
exit $r
