# Round 4 session 8: scale_zero-shape variants at 256 MiB (launch_phases), then the
# measurement half of tools/gpu_session.sh: smoke, the default bench line, its
# rocprofv3 kernel-trace summary, and the two PMC passes for HBM traffic.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 ./tools/launch_phases 256 24 > gpurun_out/lp8.txt 2>&1 || { cat gpurun_out/lp8.txt; exit 1; }
grep -E "^(copy|fill)" gpurun_out/lp8.txt
ONO_SESSION="round-4 session 8 (tools/r04_s8.sh)" ONO_COMMIT="$(cat gpurun_out/commit.txt 2>/dev/null || echo unknown)" SKIP_TESTS=1 bash tools/gpu_session.sh || exit $?
tail -c 1500 gpurun_out/bench.log
cat gpurun_out/pmc_summary.log | tail -20
