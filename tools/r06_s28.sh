# Round 6 session 28: the select with its early exit in the library — the sparse + TCP GPU files once, thr_bench
# (the library's select now the early-exit one), config 1 sparse untimed three times with the hop trace
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sparse.py tests/test_gpu_tcp.py tests/test_gpu_sparse_capture.py tests/test_gpu_sparse_pattern.py tests/test_gpu_consumer.py > gpurun_out/r06_s28_pytest.log 2>&1 || { tail -40 gpurun_out/r06_s28_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s28_pytest.log
timeout -k 10 60 tools/thr_bench 200 > gpurun_out/r06_s28_thr_bench.json 2>&1 || { cat gpurun_out/r06_s28_thr_bench.json; exit 1; }
o=gpurun_out/r06_s28_config1.txt; : > $o
for pass in 1 2 3; do
  echo "== pass $pass" >> $o
  ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
grep -E "==|hops,|s_per_round" $o | cut -c1-150
