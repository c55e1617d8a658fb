# Round 6 session 7: the config-1 sparse TCP ring with each push's mask enqueued before the socket exchange
# (default) vs after it (ONO_TCP_MASK_EARLY=0, round 5), interleaved, 3 passes at 2 ranks and 1 at 4; the
# TCP GPU file.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s7_tcp_variants.jsonl; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_TCP_MASK_EARLY=0"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $o
    env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --sparse 0.1 >> $o || exit 1
  done
done
for v in "X=1" "ONO_TCP_MASK_EARLY=0"; do
  echo "{\"variant\": \"$v\", \"pass\": 1}" >> $o
  env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 >> $o || exit 1
done
cut -c1-200 $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06_s7_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06_s7_pytest.log; tail -3 gpurun_out/r06_s7_pytest.log
exit $rc
