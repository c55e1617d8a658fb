# Round 6 session 24: the TCP + sparse GPU files once after the pipelined hop was taken out again (no gain:
# r06_s20, r06_s22, r06_s23), then config 1 sparse untimed three times (the shipped hop)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py tests/test_gpu_sparse.py tests/test_gpu_sparse_capture.py tests/test_gpu_sparse_pattern.py > gpurun_out/r06_s24_pytest.log 2>&1 || { tail -40 gpurun_out/r06_s24_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s24_pytest.log
o=gpurun_out/r06_s24_config1.txt; : > $o
for pass in 1 2 3; do
  echo "== pass $pass" >> $o
  ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
grep -E "==|hops,|s_per_round" $o | cut -c1-150
