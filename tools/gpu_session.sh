# One GPU session (run through gpurun from the repo root): parity tests, smoke,
# the default bench line, rocprofv3 kernel-trace summaries of the same bench
# (parent, and the co-resident xGMI children per pid), and the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) that give HBM traffic.  Every GPU step has its own
# time limit; the script stops at the first step that faults, aborts or times
# out.  Outputs land in gpurun_out/ (copied to profiles/ afterwards).
# SKIP_TESTS=1 skips the parity tests (a measurement-only session).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rc=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench_%pid% -- python3 bench.py --no-cpu-baseline --no-host-fed --no-tcp-edge --sweep-mib "" > gpurun_out/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-fed --no-tcp-edge --xgmi-coresident 0 > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-fed --no-tcp-edge --xgmi-coresident 0 > gpurun_out/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_summary.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --elems 67108864 --commit "${ONO_COMMIT:-unknown}" --session "${ONO_SESSION:-gpu_session.sh}" --out gpurun_out/pmc_n1.json > gpurun_out/pmc_summary.log 2>&1
exit $rc
