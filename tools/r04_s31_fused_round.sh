# Round 4 session 31: pl_fused polling its chunk lines and granules in one round of loads (mid stamp:
# after the look-back), against pl_index + pl_place (ONO_LIFT_FUSED=0); then the sparse and
# TCP GPU tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/s31_$b.txt 2>&1 || { cat gpurun_out/s31_$b.txt; exit 1; }; echo "== $b"; grep -E "# lift|^pl_" gpurun_out/s31_$b.txt | grep -v per-XCD; done
ONO_LIFT_FUSED=0 timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s31_two.txt 2>&1 || { cat gpurun_out/s31_two.txt; exit 1; }
echo "== two launches"; grep -E "# lift|^pl_" gpurun_out/s31_two.txt | grep -v per-XCD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s31_pytest.log 2>&1; r=$?
tail -3 gpurun_out/s31_pytest.log
exit $r
