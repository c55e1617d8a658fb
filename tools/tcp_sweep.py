"""Sweep the TCP edge's pipelining piece (ONO_TCP_BLOCK_KIB) and the socket
buffer sizes for 2 MI355X workers on one GPU over loopback TCP (bench.py's
tcp_edge leg).  One child process per setting (the piece size is read at ring
creation).  Usage: python tools/tcp_sweep.py [bucket_mib]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, socket, sys, threading, time
sys.path[:0] = [{root!r}, os.path.join({root!r}, "oxidized-neural-orchestra_amd")]
import torch, ono_amd, bench
bufs = int(sys.argv[2])
orig = socket.create_connection
def cc(*a, **k):
    s = orig(*a, **k)
    if bufs:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, bufs)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, bufs)
    return s
socket.create_connection = cc
print(json.dumps(bench.tcp_edge(ono_amd, int(sys.argv[1]) << 18, 5)))
"""


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    code = CHILD.format(root=ROOT)
    for kib in (1024, 2048, 4096, 8192, 16384):
        for bufs in (0, 4 << 20):
            env = dict(os.environ, ONO_TCP_BLOCK_KIB=str(kib))
            out = subprocess.run([sys.executable, "-c", code, str(mib), str(bufs)], env=env,
                                 capture_output=True, text=True, timeout=300)
            line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-300:]
            try:
                d = json.loads(line)
                print(f"piece {kib:6d} KiB  sockbuf {bufs >> 10:6d} KiB  {d.get('ms')} ms  {d.get('gib_s')} GiB/s",
                      flush=True)
            except ValueError:
                print(f"piece {kib} KiB sockbuf {bufs}: {line}", flush=True)


if __name__ == "__main__":
    main()
