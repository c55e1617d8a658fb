# Round 6 session 31: where the config-1 sparse hop's host time goes inside its two waited calls (ONO_TCP_TRACE:
# the one-launch drop's host time before / in / after its launch; the lift's call and its wait), untimed, twice
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
o=gpurun_out/r06_s31_trace.txt; : > $o
for pass in 1 2; do
  echo "== pass $pass" >> $o
  ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
cat $o | cut -c1-200
