cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases_buildout sp_phases sp_phases_buildout; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/bo_$b.txt 2>&1 || { cat gpurun_out/bo_$b.txt; exit 1; }; echo "== $b"; head -4 gpurun_out/bo_$b.txt | grep -E "sp_phases:|^sp_image "; done
