# Round 4 session 29: pl_fused's poll interval (s_sleep 4 / 16 / 48; tools/sp_phases_z* are ad-hoc
# builds with -DONO_POLL_SLEEP) and a build-out without the look-back (tools/sp_phases_bo_nolook:
# wrong output, timing only), against pl_index + pl_place (ONO_LIFT_FUSED=0).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases_z4 sp_phases_z16 sp_phases_z48 sp_phases_bo_nolook sp_phases_z16; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/s29_$b.txt 2>&1 || { cat gpurun_out/s29_$b.txt; exit 1; }; echo "== $b"; grep -E "# lift|^pl_" gpurun_out/s29_$b.txt | grep -v per-XCD; done
ONO_LIFT_FUSED=0 timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s29_two.txt 2>&1 || { cat gpurun_out/s29_two.txt; exit 1; }
echo "== two launches"; grep -E "# lift|^pl_" gpurun_out/s29_two.txt | grep -v per-XCD
