# Round 6 session 8: where a config-1 SparseCapable hop's host time goes (ONO_TCP_TRACE=1: per-step host
# time, both ranks' hops), 2 and 4 ranks, r = 0.1
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s8_trace.txt; : > $o
for args in "--ranks 2 --len 109386 --rounds 300 --sparse 0.1" "--ranks 2 --len 109386 --rounds 300 --sparse 0.1" "--ranks 4 --len 109386 --rounds 200 --sparse 0.1"; do
  echo "== $args" >> $o
  ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench $args >> $o 2>&1 || exit 1
done
cut -c1-250 $o
