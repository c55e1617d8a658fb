# Round 5 final session, part B: the sparse codec's PMC passes (LDS instructions and bank conflicts,
# HBM traffic), the sparse TCP ring end to end (tools/r05_tcp_sparse.sh), the drop's size sweep.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
EXTRA_SETS="SQ_INSTS_LDS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_WAVES" bash tools/sp_pmc.sh > gpurun_out/sp_pmc_final.txt 2>&1 || { tail -20 gpurun_out/sp_pmc_final.txt; exit 1; }
bash tools/r05_tcp_sparse.sh gpurun_out/tcp_sparse_final.jsonl > /dev/null || exit 1
timeout -k 10 400 python3 tools/drop_sizes.py gpurun_out/drop_sizes_final.json > /dev/null 2>&1 || exit 1
grep -E "^[a-z]|LDS" gpurun_out/sp_pmc_final.txt | head -40
cut -c1-200 gpurun_out/tcp_sparse_final.jsonl
