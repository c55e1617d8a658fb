cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --alt-at-n1 --no-cpu-baseline --no-local-reduce --no-host-fed > gpurun_out/bench_alt.log 2>&1 || exit $?
