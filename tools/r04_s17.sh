# Round 4 session 17: pattern-path lift with per-chunk sums (pl_index atomics on padded lines,
# pl_place one load per thread for its range): sparse parity, stamped phases, codec timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1 || { tail -30 gpurun_out/sp_pytest.log; exit 1; }
tail -1 gpurun_out/sp_pytest.log
for v in "ONO_PL_PER=16" "ONO_PL_PER=8"; do env $v timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/spp17_$v.txt 2>&1 || { cat gpurun_out/spp17_$v.txt; exit 1; }; echo "== $v"; cat gpurun_out/spp17_$v.txt; done
SKIP_TESTS=1 SP_VARIANTS="ONO_PL_PER=8" bash tools/sp_gpu.sh
