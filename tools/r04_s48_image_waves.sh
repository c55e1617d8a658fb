# Round 4 session 48: sp_image bounded to 96 VGPRs (five waves per SIMD; tools/sp_phases_bo_w5, an ad-hoc
# -DONO_IMAGE_WAVES=5 build) against the default 102 (four), interleaved.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases_bo_w5 sp_phases sp_phases_bo_w5; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/s48_$b.txt 2>&1 || { cat gpurun_out/s48_$b.txt; exit 1; }; echo "== $b"; grep -E "# sp_phases|^sp_image|^sp_move" gpurun_out/s48_$b.txt | grep -v per-XCD; done
