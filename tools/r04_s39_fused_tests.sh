# Round 4 session 39: the one-launch stream-ordered lift under the whole GPU suite (with the new
# one-launch tests: tile counts at its edges, late faults, an unaligned stream, back-to-back sizes),
# then the stamped timing and the two-launch form (ONO_LIFT_FUSED=0) beside it.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/s39_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/s39_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/s39_pytest_gpu.log
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s39_fused.txt 2>&1 || { cat gpurun_out/s39_fused.txt; exit 1; }
grep -E "# lift|^pl_" gpurun_out/s39_fused.txt | grep -v per-XCD
ONO_LIFT_FUSED=0 timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s39_two.txt 2>&1 || { cat gpurun_out/s39_two.txt; exit 1; }
grep -E "# lift|^pl_" gpurun_out/s39_two.txt | grep -v per-XCD
