# Round 6 session 5: the config-1 sparse TCP ring with the sample's indices gathered from HBM (the helper
# thread's upload) vs from pinned memory (ONO_THR_HBM=0), interleaved, twice; the TCP edge's rings incl. the
# 256 MiB sparse hops whose SparseGrad frames now go up to HBM while on the socket; the TCP GPU file.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s5_tcp_variants.jsonl; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_THR_HBM=0"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $o
    env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --sparse 0.1 >> $o || exit 1
  done
done
cut -c1-200 $o
bash tools/r05_tcp_sparse.sh gpurun_out/r06_s5_tcp_sparse.jsonl > /dev/null || exit 1
cut -c1-330 gpurun_out/r06_s5_tcp_sparse.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06_s5_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06_s5_pytest.log; tail -3 gpurun_out/r06_s5_pytest.log
exit $rc
