# Round 4 session 42: PMC of the sparse kernels with the one-launch lift (pl_fused<3>): wave cycles,
# waits, instruction counts, HBM bytes (tools/sp_pmc.sh passes, one rocprofv3 --pmc run per set).
cd "$GRAFT_REPO_ROOT"
EXTRA_SETS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" bash tools/sp_pmc.sh
