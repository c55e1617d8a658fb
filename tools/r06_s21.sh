# Round 6 session 21: the pipelined hop's GPU timeline (kernel trace, config 1 sparse, 2 workers, untimed), and
# the sample's indices gathered from HBM (ONO_THR_HBM=1) now that the hop waits on the GPU chain, three passes
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_s21
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_s21/prof -o run -- tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --sparse 0.1 --phases 0 > gpurun_out/r06_s21/bench.json 2> gpurun_out/r06_s21/bench.err || exit 1
o=gpurun_out/r06_s21_thr_hbm.txt; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_THR_HBM=1"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
done
grep -E "==|hops,|s_per_round" $o | cut -c1-150
