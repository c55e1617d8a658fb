# Round 6 session 18: the TCP tests and sparse files once after (a) the inline exchange's non-blocking spin
# (ONO_TCP_SPIN_US), (b) the one-launch lift's in-kernel completion (ONO_LIFT_SIGNAL), (c) one-launch lifts
# shared by the streams of one device (ONO_LIFT_FUSED_SHARE); then each change against its off switch,
# config 1 untimed with the hop trace, interleaved, twice
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py tests/test_gpu_sparse.py tests/test_gpu_sparse_capture.py > gpurun_out/r06_s18_pytest.log 2>&1 || { tail -30 gpurun_out/r06_s18_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s18_pytest.log
o=gpurun_out/r06_s18_variants.txt; : > $o
for pass in 1 2; do
  for v in "X=1" "ONO_TCP_SPIN_US=0" "ONO_LIFT_SIGNAL=0" "ONO_LIFT_FUSED_SHARE=0"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
  echo "== dense pass $pass" >> $o
  timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --phases 0 >> $o 2>&1 || exit 1
  echo "== dense spin0 pass $pass" >> $o
  ONO_TCP_SPIN_US=0 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --phases 0 >> $o 2>&1 || exit 1
  echo "== 4 ranks pass $pass" >> $o
  timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  echo "== 256MiB sparse pass $pass" >> $o
  timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 67108864 --rounds 10 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
grep -E "==|hops,|s_per_round" $o | cut -c1-150
