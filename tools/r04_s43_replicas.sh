# Round 4 session 43: pl_fused's chunk-line replicas, 2 / 4 / 8 (default) / 16 (tools/sp_phases_bo_rep*:
# ad-hoc -DONO_FUSED_REP builds), each timed twice, interleaved.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases_bo_rep2 sp_phases_bo_rep4 sp_phases_bo_rep16 sp_phases sp_phases_bo_rep2 sp_phases_bo_rep4 sp_phases_bo_rep16; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/s43_$b.txt 2>&1 || { cat gpurun_out/s43_$b.txt; exit 1; }; echo "== $b"; grep -E "# lift|look-back done" gpurun_out/s43_$b.txt; done
