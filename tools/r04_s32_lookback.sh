# Round 4 session 32: pl_fused's look-back counted (stamp build: polls per tile, first round's loads
# back, publish time, look-back done by tile index).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 ./tools/sp_phases 64 24 > gpurun_out/s32_fused.txt 2>&1 || { cat gpurun_out/s32_fused.txt; exit 1; }
grep -E "# lift|^pl_|^  tiles" gpurun_out/s32_fused.txt | grep -v per-XCD
