# Round 4 session 14: instruction counts of the drop kernels (one PMC pass over sp_phases).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/spi_pmc1 -o run -- ./tools/sp_phases 64 8 > gpurun_out/spi_pmc1.log 2>&1 || { echo "pass 1 failed"; tail -5 gpurun_out/spi_pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/spi_pmc2 -o run -- ./tools/sp_phases 64 8 > gpurun_out/spi_pmc2.log 2>&1 || { echo "pass 2 failed"; tail -5 gpurun_out/spi_pmc2.log; exit 1; }
python3 tools/pmc_table.py gpurun_out/spi_pmc1 gpurun_out/spi_pmc2 --match sp_
