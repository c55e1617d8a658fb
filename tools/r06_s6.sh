# Round 6 session 6: the TCP edge's rings (tools/r05_tcp_sparse.sh) twice after the frame buffers got
# headroom (a SparseGrad receive frame pinned once at ono_ring_set_sparse, pinned buffers grown by +25 %)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 2; do bash tools/r05_tcp_sparse.sh gpurun_out/r06_s6_tcp_sparse_$k.jsonl > /dev/null || exit 1; done
cut -c1-330 gpurun_out/r06_s6_tcp_sparse_1.jsonl gpurun_out/r06_s6_tcp_sparse_2.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06_s6_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06_s6_pytest.log; tail -3 gpurun_out/r06_s6_pytest.log
exit $rc
