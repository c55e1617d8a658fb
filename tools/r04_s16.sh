# Round 4 session 16: wire (sp_move) and g (pl_place) back to nt stores, slots write-through;
# sparse parity, stamped phases for sp_move tiles-per-wave 1 / 2 / 4, codec timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1 || { tail -30 gpurun_out/sp_pytest.log; exit 1; }
tail -1 gpurun_out/sp_pytest.log
for v in "ONO_SP_MTPW=1" "ONO_SP_MTPW=2" "ONO_SP_MTPW=4" "ONO_SP_VM=0"; do
  env $v timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/spp_$v.txt 2>&1 || { cat gpurun_out/spp_$v.txt; exit 1; }
  echo "== $v"; cat gpurun_out/spp_$v.txt
done
SKIP_TESTS=1 SP_VARIANTS="ONO_SP_MTPW=2" bash tools/sp_gpu.sh
