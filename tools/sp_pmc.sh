# PMC passes over the sparse codec run (one rocprofv3 --pmc run per counter set,
# each under its own time limit); tools/pmc_table.py summarises per kernel.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_SETS}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/sp_pmc$i -o run -- python3 tools/sparse_codec_run.py 5 > gpurun_out/sp_pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sp_pmc$i.log; exit 1; }
done
python3 tools/pmc_table.py gpurun_out/sp_pmc* --match sp_ sl_ pl_
