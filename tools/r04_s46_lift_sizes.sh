# Round 4 session 46: the stream-ordered lift at 8 / 16 / 32 / 48 MiB gradients (one tile per workgroup up
# to 2048 tiles, three above) against the two launches (ONO_LIFT_FUSED=0), stamped build.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in 8 16 32 48; do
  timeout -k 10 60 ./tools/sp_phases $m 24 > gpurun_out/s46_fused_$m.txt 2>&1 || { cat gpurun_out/s46_fused_$m.txt; exit 1; }
  ONO_LIFT_FUSED=0 timeout -k 10 60 ./tools/sp_phases $m 24 > gpurun_out/s46_two_$m.txt 2>&1 || { cat gpurun_out/s46_two_$m.txt; exit 1; }
  echo "== $m MiB"; grep -h "# lift" gpurun_out/s46_fused_$m.txt gpurun_out/s46_two_$m.txt
done
