# Round 6 session 33: small one-launch lifts (<= 1/64 of the slots) neither query nor record events —
# against ONO_LIFT_SMALL_TRACKED=1, config 1 sparse untimed with the trace, interleaved, three passes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py tests/test_gpu_sparse_pattern.py > gpurun_out/r06_s33_pytest.log 2>&1 || { tail -40 gpurun_out/r06_s33_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s33_pytest.log
o=gpurun_out/r06_s33_trace.txt; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_LIFT_SMALL_TRACKED=1"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
done
for v in "X=1" "ONO_LIFT_SMALL_TRACKED=1"; do
  echo "== 4 ranks $v" >> $o
  env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
cat $o | cut -c1-200
