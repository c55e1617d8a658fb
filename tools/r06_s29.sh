# Round 6 session 29: the stream-ordered 64 MiB lift regressed in the late session (bench sparse_codec.lift_dev
# stream_ms 1.07 vs 0.023 ms): the shared one-launch rule counted other streams' unrecorded launches as running
# for good; they now age out after 50 ms.  The default bench line once, then its sparse codec figures
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r06_s29_bench.log 2>&1 || { tail -c 3000 gpurun_out/r06_s29_bench.log; exit 1; }
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r06_s29_bench.log") if x.startswith("{")][-1]
d = json.loads(l)
sc = d["sparse_codec"]
print("value", d["value"], "frac", d["roofline"]["frac"])
print("lift_dev", {k: sc["lift_dev"][k] for k in ("ms", "stream_ms", "stream_frac_of_hbm_peak", "stream_refused")})
print("drop", {k: sc["drop"][k] for k in ("ms", "stream_ms", "stream_frac_of_hbm_peak")})
print("tcp sparse c1", d["tcp_edge"]["sparse"]["config1_2_ranks_r0.1"])
PY
