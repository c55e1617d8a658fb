# Round 4 session 26: build-out of sp_image's kept-value loop.  tools/sp_phases_buildout is an ad-hoc
# build (not kept): tools/sp_phases.hip compiled against a copy of ono_sparse.hip whose kept loop reads
# `b.keep & 0u` (values and headers never written; the wire is wrong, only the timing is read).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in sp_phases sp_phases_buildout sp_phases sp_phases_buildout; do timeout -k 10 60 ./tools/$b 64 24 > gpurun_out/bo_$b.txt 2>&1 || { cat gpurun_out/bo_$b.txt; exit 1; }; echo "== $b"; head -4 gpurun_out/bo_$b.txt | grep -E "sp_phases:|^sp_image "; done
