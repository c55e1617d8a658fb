# Sparse codec GPU check: the sparse parity tests, then the codec timing
# (tools/sparse_codec_run.py) and its rocprofv3 kernel stats; SP_VARIANTS
# (space-separated env assignments) repeats the timing per variant.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_sparse.py tests/test_gpu_sparse_pattern.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sp_pytest.log 2>&1 || { tail -30 gpurun_out/sp_pytest.log; exit 1; }
tail -3 gpurun_out/sp_pytest.log
fi
for v in default $SP_VARIANTS; do
  echo "== variant $v"
  if [ "$v" = default ]; then
    timeout -k 10 120 python -u tools/sparse_codec_run.py 20 > gpurun_out/sp_run_$v.log 2>&1 || { cat gpurun_out/sp_run_$v.log; exit 1; }
  else
    env $v timeout -k 10 120 python -u tools/sparse_codec_run.py 20 > gpurun_out/sp_run_$v.log 2>&1 || { cat gpurun_out/sp_run_$v.log; exit 1; }
  fi
  grep -E "drop|lift" gpurun_out/sp_run_$v.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp_prof -o sp -- python3 tools/sparse_codec_run.py 20 > gpurun_out/sp_prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob('gpurun_out/sp_prof/*kernel_stats.csv'):
    for r in csv.DictReader(open(f)):
        if any(k in r['Name'] for k in ('sp_', 'sl_', 'pl_')):
            print(r['Name'].replace('(anonymous namespace)::', '').split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2), round(float(r['MaxNs'])/1000, 2))
PY
