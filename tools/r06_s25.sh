# Round 6 session 25: loopback TCP socket buffers (tools/ono_tcp_bench --sockbuf KiB: SO_SNDBUF / SO_RCVBUF on
# every ring socket) against the system's autotuning, 256 MiB dense and sparse r = 0.1 rings, untimed, twice
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r06_s25_sockbuf.txt; : > $o
cat /proc/sys/net/ipv4/tcp_wmem /proc/sys/net/ipv4/tcp_rmem /proc/sys/net/core/wmem_max /proc/sys/net/core/rmem_max >> $o 2>&1
for pass in 1 2; do
  for b in 0 4096 16384 65536; do
    echo "== dense sockbuf $b pass $pass" >> $o
    timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 67108864 --rounds 10 --phases 0 --sockbuf $b >> $o 2>&1 || exit 1
    echo "== sparse sockbuf $b pass $pass" >> $o
    timeout -k 10 120 tools/ono_tcp_bench --ranks 2 --len 67108864 --rounds 10 --sparse 0.1 --phases 0 --sockbuf $b >> $o 2>&1 || exit 1
  done
done
grep -E "==|s_per_round|^[0-9]" $o | cut -c1-150
