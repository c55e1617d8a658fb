# Round 6 session 4: (1) the 64 MiB drop A/B with sp_emit's totals in an extra workgroup (round-5 library vs
# this round's) and both libraries' stamped phases; (2) the config-1 sparse TCP ring (2 ranks, r = 0.1) per
# change, each variant twice, interleaved: default / lift via an HBM copy (ONO_TCP_LIFT_PINNED=0) / separate
# key gather (ONO_THR_FUSED=0) / signal-kernel wait (ONO_DROP1_SIGNAL=0) / all three (round 5's form);
# (3) the sparse and TCP GPU files.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/drop_lib_ab.py tools/ab/libono_r05.so tools/ab/libono_r06.so 9 > gpurun_out/r06_s4_drop_ab.json 2> gpurun_out/r06_s4_drop_ab.err || { tail -20 gpurun_out/r06_s4_drop_ab.err; exit 1; }
cat gpurun_out/r06_s4_drop_ab.json
timeout -k 10 60 tools/ab/sp_phases_r05 64 24 > gpurun_out/r06_s4_phases_r05.txt 2>&1 || exit 1
timeout -k 10 60 tools/sp_phases 64 24 > gpurun_out/r06_s4_phases_r06.txt 2>&1 || exit 1
grep -E "^sp_count|^sp_emit|drop" gpurun_out/r06_s4_phases_r05.txt | head -8
grep -E "^sp_count|^sp_emit|drop" gpurun_out/r06_s4_phases_r06.txt | head -8
o=gpurun_out/r06_s4_tcp_variants.jsonl; : > $o
for pass in 1 2; do
  for v in "X=1" "ONO_TCP_LIFT_PINNED=0" "ONO_THR_FUSED=0" "ONO_DROP1_SIGNAL=0" "ONO_TCP_LIFT_PINNED=0 ONO_THR_FUSED=0 ONO_DROP1_SIGNAL=0"; do
    echo "{\"variant\": \"$v\", \"pass\": $pass}" >> $o
    env $v timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --sparse 0.1 >> $o || exit 1
  done
done
cut -c1-230 $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_sparse_capture.py tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py \
  tests/test_gpu_tcp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r06_s4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06_s4_pytest.log; tail -3 gpurun_out/r06_s4_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/r06_s4_pytest.log; fi
exit $rc
