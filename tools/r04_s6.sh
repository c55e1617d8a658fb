# Round 4 session 6: sparse parity + codec timing with 128-tile one-wave record-scan
# chunks; the path_kernels / copy_ceiling A/B of the 256-thread fill / decode (ONO_EW_WIDE).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/sp_gpu.sh || exit 1
timeout -k 10 600 python -u tools/pk_ab.py 2 - ONO_EW_WIDE=0 > gpurun_out/pk_ab.txt 2>&1 || { cat gpurun_out/pk_ab.txt; exit 1; }
cat gpurun_out/pk_ab.txt
