# Round 6 final session, sixth pass (after the store and optimizer creation sync): the full GPU parity suite, smoke, the default bench line, its rocprofv3
# kernel trace (and the per-size split), the two PMC passes for HBM traffic (tools/gpu_session.sh),
# then the stamped sparse phases.  ONO_COMMIT names the commit measured.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
ONO_SESSION="round-6 final6 (tools/r06_final6.sh)" bash tools/gpu_session.sh; rc=$?
tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
[ $rc -ne 0 ] && { echo "gpu_session rc=$rc"; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -c 3000 gpurun_out/bench.log 2>/dev/null; exit $rc; }
python3 tools/prof_by_size.py gpurun_out/prof > gpurun_out/kernels_by_size.txt 2>&1
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/sp_phases_final.txt 2>&1 || { cat gpurun_out/sp_phases_final.txt; exit 1; }
tail -c 2500 gpurun_out/bench.log
tail -12 gpurun_out/pmc_summary.log
