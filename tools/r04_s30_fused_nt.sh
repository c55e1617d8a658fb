# Round 4 session 30: pl_fused with tile = blockIdx.x (no ticket counter), poll interval s_sleep
# 4 / 16 (default) / 48 (tools/sp_phases_z*: ad-hoc -DONO_POLL_SLEEP builds), against pl_index +
# pl_place (ONO_LIFT_FUSED=0); then the sparse and TCP GPU tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases_z4 sp_phases_z48 sp_phases; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/s30_$b.txt 2>&1 || { cat gpurun_out/s30_$b.txt; exit 1; }; echo "== $b"; grep -E "# lift|^pl_" gpurun_out/s30_$b.txt | grep -v per-XCD; done
ONO_LIFT_FUSED=0 timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s30_two.txt 2>&1 || { cat gpurun_out/s30_two.txt; exit 1; }
echo "== two launches"; grep -E "# lift|^pl_" gpurun_out/s30_two.txt | grep -v per-XCD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse_pattern.py tests/test_gpu_sparse.py tests/test_gpu_tcp.py > gpurun_out/s30_pytest.log 2>&1; r=$?
tail -3 gpurun_out/s30_pytest.log
exit $r
