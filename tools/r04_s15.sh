# Round 4 session 15: write-through slot and wire stores, header fields by one lane after the move,
# sp_image's kept-value loop (ONO_SP_VM=1) vs the per-element pass (0): sparse parity, stamped
# phases (and sp_move over 2 / 4 tiles per wave), instruction counts (PMC), codec timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1 || { tail -30 gpurun_out/sp_pytest.log; exit 1; }
tail -1 gpurun_out/sp_pytest.log
for v in "ONO_SP_VM=1" "ONO_SP_VM=0" "ONO_SP_MTPW=2" "ONO_SP_MTPW=4"; do
  env $v timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/spp_$v.txt 2>&1 || { cat gpurun_out/spp_$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/spp_$v.txt
done
bash tools/r04_s14.sh || exit 1
SKIP_TESTS=1 SP_VARIANTS="ONO_SP_VM=0" bash tools/sp_gpu.sh
