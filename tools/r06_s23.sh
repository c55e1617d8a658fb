# Round 6 session 23: the pipelined hop, the add gated on a device refusal word the one-launch lift writes (its last
# workgroup copies a refusal to the host status word; r06_s22 read the host word per wave: slower) — TCP + sparse GPU
# files once, then config 1 untimed with the hop trace against ONO_TCP_PIPE=0, interleaved, three passes; 4 workers; 256 MiB
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py tests/test_gpu_sparse.py tests/test_gpu_sparse_capture.py tests/test_gpu_sparse_pattern.py > gpurun_out/r06_s23_pytest.log 2>&1 || { tail -40 gpurun_out/r06_s23_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s23_pytest.log
o=gpurun_out/r06_s23_variants.txt; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_TCP_PIPE=0"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
    echo "== 4 ranks $v pass $pass" >> $o
    env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
    echo "== r0.01 $v pass $pass" >> $o
    env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.01 --phases 0 >> $o 2>&1 || exit 1
  done
done
for v in "X=1" "ONO_TCP_PIPE=0"; do
  echo "== 256MiB $v" >> $o
  env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 67108864 --rounds 10 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
grep -E "==|hops,|s_per_round" $o | cut -c1-150
