# Round 4 session 12: launch_phases at 64 MiB with the tool's pattern data and with the
# bench's synthetic gradients (data dependence of the stream rates).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 ./tools/launch_phases 64 24 > gpurun_out/lp12a.txt 2>&1 || { cat gpurun_out/lp12a.txt; exit 1; }
timeout -k 10 200 ./tools/launch_phases 64 24 synth > gpurun_out/lp12b.txt 2>&1 || { cat gpurun_out/lp12b.txt; exit 1; }
timeout -k 10 200 ./tools/launch_phases 64 24 > gpurun_out/lp12c.txt 2>&1 || { cat gpurun_out/lp12c.txt; exit 1; }
for f in lp12a lp12b lp12c; do echo "== $f"; head -1 gpurun_out/$f.txt; grep -E "^(copy 1R1W|copy\+zero 1R2W|fill 0R1W|sum2 2R1W|sum4 4R1W|sum8 8R1W|f16 decode)" gpurun_out/$f.txt; done
