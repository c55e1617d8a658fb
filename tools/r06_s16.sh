# Round 6 session 16: the sample's indices gathered from HBM (ONO_THR_HBM=1: the sampler queue uploads each
# draw) vs from pinned memory (default), untimed config-1 sparse rings with the hop trace, interleaved, twice
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s16_thr_hbm.txt; : > $o
for pass in 1 2; do
  for v in "X=1" "ONO_THR_HBM=1"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
done
grep -E "==|hops|s_per_round" $o | cut -c1-170
