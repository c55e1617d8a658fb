# Round 4 session 41: pl_fused with the first tile's look-back straight after its publication (default)
# against the look-back after every tile is published (tools/sp_phases_bo_late: an ad-hoc
# -DONO_FUSED_FIRST_EARLY=0 build), alternating; then the sparse and TCP GPU tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases_bo_late sp_phases sp_phases_bo_late; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/s41_$b.txt 2>&1 || { cat gpurun_out/s41_$b.txt; exit 1; }; echo "== $b"; grep -E "# lift|^pl_" gpurun_out/s41_$b.txt | grep -v per-XCD; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s41_pytest.log 2>&1; r=$?
tail -3 gpurun_out/s41_pytest.log
exit $r
