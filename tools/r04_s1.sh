# Round 4 session 1: the launch-phase decomposition (tools/launch_phases), the
# TCP zip / sparse tests, the xGMI pool tests, then the sparse parity tests +
# codec timing + kernel stats (tools/sp_gpu.sh) for the f16-image pl_place and
# the two-tile pl_index.  Every GPU step under its own limit; the script stops
# at the first failure.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 ./tools/launch_phases 64,256 24 > gpurun_out/lp1.txt 2>&1 || { echo "launch_phases failed"; cat gpurun_out/lp1.txt; exit 1; }
cat gpurun_out/lp1.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "zip or sparse" > gpurun_out/tcp_pytest.log 2>&1 || { tail -30 gpurun_out/tcp_pytest.log; exit 1; }
tail -2 gpurun_out/tcp_pytest.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_xgmi.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "recreate or release" > gpurun_out/xgmi_pytest.log 2>&1 || { tail -30 gpurun_out/xgmi_pytest.log; exit 1; }
tail -2 gpurun_out/xgmi_pytest.log
bash tools/sp_gpu.sh
