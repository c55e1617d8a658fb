# Round 4 session 7: buffer-placement A/B of the config-2 kernel (tools/lr_ab.py).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/lr_ab.py 3 40 > gpurun_out/lr_ab7.txt 2>&1 || { cat gpurun_out/lr_ab7.txt; exit 1; }
cat gpurun_out/lr_ab7.txt
