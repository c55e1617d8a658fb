# Round 4 session 3: fewer-workgroup fill / decode / copy rows of launch_phases,
# the bench-vs-tool local_reduce A/B (tools/lr_ab.py, tools/sum_alloc_ab.py) and
# the sparse codec PMC passes (tools/sp_pmc.sh).  Each GPU step has its own limit.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/launch_phases 64,256 24 > gpurun_out/lp3.txt 2>&1 || { echo "launch_phases failed"; cat gpurun_out/lp3.txt; exit 1; }
grep -v "^#     xcd" gpurun_out/lp3.txt
timeout -k 10 300 python -u tools/lr_ab.py 3 40 > gpurun_out/lr_ab.txt 2>&1 || { cat gpurun_out/lr_ab.txt; exit 1; }
cat gpurun_out/lr_ab.txt
timeout -k 10 300 python -u tools/sum_alloc_ab.py 3 > gpurun_out/sum_alloc_ab.txt 2>&1 || { cat gpurun_out/sum_alloc_ab.txt; exit 1; }
cat gpurun_out/sum_alloc_ab.txt
bash tools/sp_pmc.sh > gpurun_out/sp_pmc_table.txt 2>&1 || { tail -20 gpurun_out/sp_pmc_table.txt; exit 1; }
cat gpurun_out/sp_pmc_table.txt
