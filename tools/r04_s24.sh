# Round 4 session 24: the full GPU parity suite and smoke on the final product code.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_s24.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_s24.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s24.log 2>&1 || { cat gpurun_out/smoke_s24.log; exit 1; }
tail -2 gpurun_out/smoke_s24.log
