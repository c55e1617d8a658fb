# Round 6 session 2: the 64 MiB drop A/B, round-5 library vs this round's (device parity, the record check,
# bounded writers), alternating passes in one process; then the TCP edge's sparse rings (tools/ono_tcp_bench)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/drop_lib_ab.py tools/ab/libono_r05.so tools/ab/libono_r06.so 9 > gpurun_out/r06_s2_drop_ab.json 2> gpurun_out/r06_s2_drop_ab.err || { tail -20 gpurun_out/r06_s2_drop_ab.err; exit 1; }
cat gpurun_out/r06_s2_drop_ab.json
bash tools/r05_tcp_sparse.sh gpurun_out/r06_s2_tcp_sparse.jsonl
