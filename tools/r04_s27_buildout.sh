# Round 4 session 27: build-outs of pl_place (tools/sp_phases_bo_* are ad-hoc builds, not kept:
# sp_phases.hip against copies of ono_sparse.hip with pl_place's output loop (noout), its record
# placement loop (nocand) or both (none) removed; wrong output, timing only).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases_bo_noout sp_phases_bo_nocand sp_phases_bo_none sp_phases; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/bo_$b.txt 2>&1 || { cat gpurun_out/bo_$b.txt; exit 1; }; echo "== $b"; grep -E "# lift|^pl_" gpurun_out/bo_$b.txt | grep -v per-XCD; done
