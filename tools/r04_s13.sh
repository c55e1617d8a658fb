# Round 4 session 13: the two-launch drop (per-workgroup chunk aggregates by atomics in sp_image,
# the record scan folded into sp_move, sp_image over several tiles per workgroup with the next
# tile's values in flight): sparse parity, stamped phases per tiles-per-workgroup, codec timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1 || { tail -30 gpurun_out/sp_pytest.log; exit 1; }
tail -1 gpurun_out/sp_pytest.log
for v in 1 2 4 8 16; do
  ONO_SP_TPW=$v timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/spp_$v.txt 2>&1 || { cat gpurun_out/spp_$v.txt; exit 1; }
  cat gpurun_out/spp_$v.txt
done
SKIP_TESTS=1 SP_VARIANTS="ONO_SP_TPW=2 ONO_SP_TPW=8" bash tools/sp_gpu.sh
