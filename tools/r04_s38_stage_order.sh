# Round 4 session 38: pl_fused striped; the first tile's loads first, the total from a vector load, no wait for the later tiles before the first is published (stamp build: polls per tile, first round's loads
# back, publish time, look-back done by tile index).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s38_fused.txt 2>&1 || { cat gpurun_out/s38_fused.txt; exit 1; }
grep -E "# lift|^pl_" gpurun_out/s38_fused.txt | grep -v per-XCD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s38_pytest.log 2>&1; r=$?
tail -3 gpurun_out/s38_pytest.log
exit $r
