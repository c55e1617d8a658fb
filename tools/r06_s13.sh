# Round 6 session 13: the TCP edge, round 5's library (tools/ab/ono_tcp_bench_r05: the round-5 commit built
# whole) vs this round's, untimed (--phases 0), interleaved, 3 passes: config 1 dense and sparse r = 0.1 at 2
# ranks, sparse at 4 ranks, 256 MiB sparse r = 0.1 at 2 ranks
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s13_r05_vs_r06.jsonl; : > $o
for pass in 1 2 3; do
  for args in "--ranks 2 --len 109386 --rounds 300" "--ranks 2 --len 109386 --rounds 300 --sparse 0.1" "--ranks 4 --len 109386 --rounds 200 --sparse 0.1" "--ranks 2 --len 67108864 --rounds 10 --sparse 0.1"; do
    for exe in tools/ab/ono_tcp_bench_r05 tools/ono_tcp_bench; do
      echo "{\"exe\": \"$exe\", \"pass\": $pass}" >> $o
      timeout -k 10 120 $exe $args --phases 0 >> $o || exit 1
    done
  done
done
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r06_s13_r05_vs_r06.jsonl")]
agg = collections.defaultdict(list)
for a, b in zip(rows[::2], rows[1::2]):
    agg[(a["exe"].split("/")[-1], b["ranks"], b["len"], b["sparse_r"])].append(round(b["s_per_round"] * 1e3, 4))
for k, v in sorted(agg.items()):
    print(k, v)
PY
