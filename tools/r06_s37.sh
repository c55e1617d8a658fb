# Round 6 session 37: the fused keys read the sample indices from HBM (ONO_THR_HBM=1: the helper uploads each
# bucketed draw) or in place from pinned memory (default) — config 1 sparse untimed with the trace, interleaved,
# three passes (no test run: no code change)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s37_trace.txt; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_THR_HBM=1"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
done
for v in "X=1" "ONO_THR_HBM=1"; do
  echo "== 4 ranks $v" >> $o
  env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
echo "== 256MiB sparse" >> $o
timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 67108864 --rounds 10 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
cat $o | cut -c1-200

