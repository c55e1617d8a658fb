# Round 4 session 47: where pl_fused should switch from one tile per workgroup to three: the default
# (one up to the device's 2048 slots) against always three (tools/sp_phases_bo_one0) and a switch at
# 512 / 1024 tiles (bo_one512, bo_one1024; ad-hoc -DONO_FUSED_ONE_MAX builds), at 8 / 16 / 32 MiB.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in 8 16 32; do
  for b in sp_phases sp_phases_bo_one0 sp_phases_bo_one512 sp_phases_bo_one1024 sp_phases; do
    timeout -k 10 60 ./tools/$b $m 24 > gpurun_out/s47_${b}_$m.txt 2>&1 || { cat gpurun_out/s47_${b}_$m.txt; exit 1; }
    echo "== $m MiB $b: $(grep -h '# lift' gpurun_out/s47_${b}_$m.txt)"
  done
done
