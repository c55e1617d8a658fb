# Round 4 session 10: the serialized k >= 4 sum with its head or tail workgroups in the parallel form
# (launch_phases at 64 and 256 MiB).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/launch_phases 64,256 24 > gpurun_out/lp10.txt 2>&1 || { cat gpurun_out/lp10.txt; exit 1; }
grep -E "^(sum|copy 1R1W|# [0-9])" gpurun_out/lp10.txt
