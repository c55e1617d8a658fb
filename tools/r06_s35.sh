# Round 6 session 35: a sparse push's mask in one launch with the hop's add / copy after the exchange
# (ONO_TCP_MASK=fused, default) against before the exchange (early) — sparse + TCP GPU files once, then config 1
# sparse untimed with the trace, interleaved, three passes; 4 workers
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py tests/test_gpu_sparse.py > gpurun_out/r06_s35_pytest.log 2>&1 || { tail -40 gpurun_out/r06_s35_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s35_pytest.log
o=gpurun_out/r06_s35_trace.txt; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_TCP_MASK=early"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
done
for v in "X=1" "ONO_TCP_MASK=early"; do
  echo "== 4 ranks $v" >> $o
  env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
cat $o | cut -c1-200
