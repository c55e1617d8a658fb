# Phase timing of the lift's pattern kernels: ONO_PL_DBG = 16 x (pl_index exit: 1 after staging, 2 after
# the mask scan) + (pl_place exit: 1 after staging and zeroing, 2 before the store); rocprofv3 stats each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${PL_DBG_SET:-0 16 32 1 2}; do
  ONO_PL_DBG=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pl_dbg_$v -o run -- python3 tools/sparse_codec_run.py 20 > gpurun_out/pl_dbg_$v.log 2>&1 || { tail -5 gpurun_out/pl_dbg_$v.log; exit 1; }
  echo "== ONO_PL_DBG=$v"; grep "lift_dev" gpurun_out/pl_dbg_$v.log | head -1
  python3 - "$v" <<'PY'
import csv, glob, sys
for f in glob.glob(f'gpurun_out/pl_dbg_{sys.argv[1]}/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if 'pl_' in r['Name'] or 'sl_' in r['Name']:
            print('  ', r['Name'].replace('(anonymous namespace)::', '').split('(')[0], r['Calls'], round(float(r['AverageNs'])/1000, 2))
PY
done
