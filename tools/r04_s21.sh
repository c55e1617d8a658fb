# Round 4 session 21: the sparse codec with the measured-and-dropped variants removed (one path per
# kernel): sparse / pattern / TCP parity, stamped phases, codec timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1 || { tail -30 gpurun_out/sp_pytest.log; exit 1; }
tail -1 gpurun_out/sp_pytest.log
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/spp21.txt 2>&1 || { cat gpurun_out/spp21.txt; exit 1; }
grep -E "^#" gpurun_out/spp21.txt
SKIP_TESTS=1 bash tools/sp_gpu.sh
