# Round 6 session 1: the sparse GPU files once after the bounded writers / device parity / capture change
# (VERDICT r5 item 1), the config-2 full-size k = 2 / 4 / 8 checks, then the drop's timing.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sparse_capture.py tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py \
  tests/test_gpu_tcp.py "tests/test_gpu_kernels.py::test_full_size_sum_scale_property" -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/r06_s1_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r06_s1_pytest.log; tail -15 gpurun_out/r06_s1_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u -c "import sys, json; sys.path[:0] = ['.', 'oxidized-neural-orchestra_amd']; import torch, ono_amd, bench; torch.cuda.set_device(0); print(json.dumps(bench.sparse_codec(torch, ono_amd)))" > gpurun_out/r06_s1_codec.json 2> gpurun_out/r06_s1_codec.err || { tail -20 gpurun_out/r06_s1_codec.err; exit 1; }
cat gpurun_out/r06_s1_codec.json
exit $rc
