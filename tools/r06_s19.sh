# Round 6 session 19: the lift's in-kernel completion (ONO_LIFT_SIGNAL) and one-launch lifts shared by the
# streams of one device (ONO_LIFT_FUSED_SHARE), each against its off switch and both off (round 5's form),
# config 1 untimed with the hop trace, interleaved, three passes; the exchange's spin is off (r06_s18)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s19_variants.txt; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_LIFT_SIGNAL=0" "ONO_LIFT_FUSED_SHARE=0" "ONO_LIFT_SIGNAL=0 ONO_LIFT_FUSED_SHARE=0"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
  for v in "X=1" "ONO_LIFT_SIGNAL=0 ONO_LIFT_FUSED_SHARE=0"; do
    echo "== 4 ranks $v pass $pass" >> $o
    env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
done
grep -E "==|hops,|s_per_round" $o | cut -c1-150
