# Round 6 session 17: kernel trace of the config-1 sparse ring (2 workers, r = 0.1, untimed), for the per-hop
# GPU timeline (kernel durations and the idle gaps between them on each worker's stream)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06_s17
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/r06_s17/prof -o run -- tools/ono_tcp_bench --ranks 2 --len 109386 --rounds 300 --sparse 0.1 --phases 0 > gpurun_out/r06_s17/bench.json 2> gpurun_out/r06_s17/bench.err || exit 1
find gpurun_out/r06_s17 -name "*.csv" | head
cat gpurun_out/r06_s17/bench.json
