set -e
o=${1:-gpurun_out/r05_s3_tcp_sparse.jsonl}
: > $o
for args in "--ranks 2 --len 109386 --rounds 200" "--ranks 2 --len 109386 --rounds 200 --sparse 0.1" "--ranks 2 --len 109386 --rounds 200 --sparse 0.01" "--ranks 4 --len 109386 --rounds 200 --sparse 0.1" "--ranks 2 --len 67108864 --rounds 10" "--ranks 2 --len 67108864 --rounds 10 --sparse 0.1" "--ranks 2 --len 67108864 --rounds 10 --sparse 0.01"; do
  timeout -k 10 120 tools/ono_tcp_bench $args >> $o
done
cat $o
