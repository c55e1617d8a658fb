# Round 5 final session, part E (the round's last binary: count + emit, one barrier per count round):
# the full GPU parity suite, smoke and the default bench line again, plus the stamped sparse phases.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_e.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_e.log; tail -2 gpurun_out/pytest_gpu_e.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_e.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_e.log 2>&1 || exit $?
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/sp_phases_e.txt 2>&1 || exit 1
tail -c 600 gpurun_out/bench_e.log
tools/emit_ab.sh r05_final_e_ab > gpurun_out/r05_final_e_ab.txt 2>&1 || exit 1
