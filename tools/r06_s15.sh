# Round 6 session 15: session 14 with the sampler queue's waits counted — where an untimed config-1 SparseCapable hop's host time goes (ONO_TCP_TRACE=1,
# --phases 0), 2 ranks r = 0.1 and 0.01, 4 ranks r = 0.1
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s15_trace.txt; : > $o
for args in "--ranks 2 --len 109386 --rounds 300 --sparse 0.1" "--ranks 2 --len 109386 --rounds 300 --sparse 0.01" "--ranks 4 --len 109386 --rounds 200 --sparse 0.1"; do
  echo "== $args" >> $o
  ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench $args --phases 0 >> $o 2>&1 || exit 1
done
cut -c1-250 $o
