# Round 6 session 3: the 64 MiB drop A/B after interleaving the two aggregate arrays in each chunk's line
# (round-5 library vs this round's); the sparse and TCP GPU files (the layout, the one launch's in-kernel
# completion, the fused sample gather and the lift from the pinned frame changed); the TCP sparse rings.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/drop_lib_ab.py tools/ab/libono_r05.so tools/ab/libono_r06.so 9 > gpurun_out/r06_s3_drop_ab.json 2> gpurun_out/r06_s3_drop_ab.err || { tail -20 gpurun_out/r06_s3_drop_ab.err; exit 1; }
cat gpurun_out/r06_s3_drop_ab.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse_capture.py tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py \
  tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06_s3_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06_s3_pytest.log; tail -4 gpurun_out/r06_s3_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/r06_s3_pytest.log; exit $rc; fi
for k in 1 2; do bash tools/r05_tcp_sparse.sh gpurun_out/r06_s3_tcp_sparse_$k.jsonl > /dev/null || exit 1; done
cat gpurun_out/r06_s3_tcp_sparse_1.jsonl gpurun_out/r06_s3_tcp_sparse_2.jsonl | cut -c1-260
