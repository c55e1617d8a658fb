# Round 6 session 9: the default sampler drawn several pushes ahead (a queue of 4 slots) — config-1 sparse
# TCP ring traced (ONO_TCP_TRACE) and timed, 2 and 4 ranks; the TCP GPU file (sparse rings bit-exact against
# the oracle, whose stand-in sampler draws the same sequence)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s10_trace.txt; : > $o
for args in "--ranks 2 --len 109386 --rounds 300 --sparse 0.1" "--ranks 2 --len 109386 --rounds 300 --sparse 0.1" "--ranks 4 --len 109386 --rounds 200 --sparse 0.1"; do
  echo "== $args" >> $o
  ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench $args >> $o 2>&1 || exit 1
done
cut -c1-250 $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06_s10_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06_s10_pytest.log; tail -3 gpurun_out/r06_s10_pytest.log
exit $rc
