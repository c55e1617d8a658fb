# Round 4 session 19: pl_place over three consecutive tiles per workgroup (one round; the later
# tiles' ranges and links from the tile before; every tile staged by LDS-DMA in the prologue):
# sparse parity (pattern path incl. wide tiles, TCP sparse mode), stamped phases, codec timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1 || { tail -30 gpurun_out/sp_pytest.log; exit 1; }
tail -1 gpurun_out/sp_pytest.log
for v in "ONO_PL_TPW=3" "ONO_PL_TPW=1"; do env $v timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/spp19_$v.txt 2>&1 || { cat gpurun_out/spp19_$v.txt; exit 1; }; echo "== $v"; grep -E "lift|pl_" gpurun_out/spp19_$v.txt; done
SKIP_TESTS=1 SP_VARIANTS="ONO_PL_TPW=1" bash tools/sp_gpu.sh
