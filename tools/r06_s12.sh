# Round 6 session 12: the TCP edge's config-1 rings with and without rank 0's phase timing (--phases 0/1),
# interleaved, twice: dense and sparse r = 0.1 at 2 ranks, sparse at 4 ranks
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s12_phases_ab.jsonl; : > $o
for pass in 1 2; do
  for args in "--ranks 2 --len 109386 --rounds 300" "--ranks 2 --len 109386 --rounds 300 --sparse 0.1" "--ranks 4 --len 109386 --rounds 200 --sparse 0.1"; do
    for ph in 1 0; do
      timeout -k 10 120 tools/ono_tcp_bench $args --phases $ph >> $o || exit 1
    done
  done
done
cut -c1-120 $o
