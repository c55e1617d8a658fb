# Round 4 session 22: PMC of the current sparse kernels (sp_image, sp_move, pl_index, pl_place):
# wave cycles, waits, instruction counts, HBM bytes (tools/sp_pmc.sh passes).
cd "$GRAFT_REPO_ROOT"
EXTRA_SETS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" bash tools/sp_pmc.sh
