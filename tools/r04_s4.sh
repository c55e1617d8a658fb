# Round 4 session 4: the whole GPU parity suite on the new library (256-thread
# fill / decode, nt sc1 copy, plan copies and zero fills on the library's own
# kernels), launch_phases at 64 MiB (lib rows), the local_reduce A/B, the bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 ./tools/launch_phases 64 24 > gpurun_out/lp4.txt 2>&1 || { cat gpurun_out/lp4.txt; exit 1; }
grep -v "^#     xcd" gpurun_out/lp4.txt | head -16
timeout -k 10 600 python -u tools/lr_ab.py 3 40 > gpurun_out/lr_ab4.txt 2>&1 || { cat gpurun_out/lr_ab4.txt; exit 1; }
cat gpurun_out/lr_ab4.txt
