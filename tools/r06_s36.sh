# Round 6 session 36: the next push's sample keys gathered by the hop's add / copy launch (the sampler's helper
# buckets each draw by 256-value block; ONO_TCP_FUSE_KEYS=0 keeps the gather launch) — TCP + sparse GPU files
# once, then config 1 sparse untimed with the trace, interleaved, three passes; 4 workers; 256 MiB sparse
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py tests/test_gpu_sparse.py > gpurun_out/r06_s36_pytest.log 2>&1 || { tail -40 gpurun_out/r06_s36_pytest.log; exit 1; }
tail -2 gpurun_out/r06_s36_pytest.log
o=gpurun_out/r06_s36_trace.txt; : > $o
for pass in 1 2 3; do
  for v in "X=1" "ONO_TCP_FUSE_KEYS=0"; do
    echo "== $v pass $pass" >> $o
    env $v ONO_TCP_TRACE=1 timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 400 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
  done
done
for v in "X=1" "ONO_TCP_FUSE_KEYS=0"; do
  echo "== 4 ranks $v" >> $o
  env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 4 --len 109386 --rounds 200 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
done
echo "== 256MiB sparse" >> $o
timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 67108864 --rounds 10 --sparse 0.1 --phases 0 >> $o 2>&1 || exit 1
cat $o | cut -c1-200
