# Round 6 session 34: the drop and the lift hold the scratch lock only to find or make their scratch (not
# through their launches) — sparse + TCP GPU files once, then config 1 sparse untimed with the trace three
# times, 4 workers, 256 MiB sparse
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sparse.py tests/test_gpu_tcp.py tests/test_gpu_sparse_capture.py tests/test_gpu_sparse_pattern.py > gpurun_out/r06_s34_pytest.log 2>&1 || { tail -40 gpurun_out/r06_s34_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s34_pytest.log
o=gpurun_out/r06_s34_trace.txt; : > $o
for pass in 1 2 3; do
  echo "== pass $pass" >> $o
  ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
echo "== 4 ranks" >> $o
timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
echo "== dense" >> $o
timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --phases 0 >> $o 2>&1 || exit 1
echo "== 256MiB sparse" >> $o
timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 67108864 --rounds 10 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
cat $o | cut -c1-200
