#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch
HBM bytes of each kernel (profiles/<round>_pmc_*.json, read by bench.py).

Collection (two separate passes, counters only — MI355X_MICROARCH.md §HBM,
§rocprofv3 PMC slots: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o run -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o run -- python3 bench.py ...

gfx950 corrections applied (same guide): counters are in KiB; FETCH_SIZE
reports exactly half of the bytes of a wide (16 B/lane) coalesced streaming
read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B
streaming stores.

usage: pmc_summary.py --fetch DIR --write DIR --elems N --out FILE [--match SUBSTR ...]
"""
from __future__ import annotations

import argparse
import csv
import glob
import datetime
import json
import os
import re
import statistics


def load(d: str, counter: str) -> dict[str, list[float]]:
    out: dict[str, list[float]] = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                out.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--elems", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--match", nargs="*", default=["ScaleZeroOp", "SumScaleOp", "AccOp", "AddEncodeZeroOp",
                                                  "DecodeScaleOp", "OptOp", "DirectOp<8,"])
    ap.add_argument("--algo-bytes-per-elem", type=float, default=12.0)
    ap.add_argument("--commit", default="unknown", help="git commit of the code the passes ran")
    ap.add_argument("--session", default="", help="which session / box recorded the passes")
    ap.add_argument("--local-elems", type=int, default=16 << 20,
                    help="bucket length of bench.py's local_reduce (SumScaleOp<k> kernels: (k+1) x 4 B/elem)")
    a = ap.parse_args()
    fetch, write = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    kernels = []
    for name in sorted(set(fetch) & set(write)):
        if not any(m in name for m in a.match):
            continue
        if "ScaleZeroOp" in name and not re.search(r"SumScaleOp", name):
            # the headline's launches (a.elems) and local_reduce's same-pool copy+zero ceiling
            # (a.local_elems) are one kernel: split the launches by size (write = 8 B/elem), one entry each
            for elems in (a.elems, a.local_elems):
                ef, ew = 2.0 * elems / 1024, 8.0 * elems / 1024  # expected KiB: read 4 B/elem half-counted, write 8
                fk = [v for v in fetch[name] if 0.7 * ef <= v <= 1.4 * ef]
                wk = [v for v in write[name] if 0.7 * ew <= v <= 1.4 * ew]
                if not fk or not wk:
                    continue
                f_kb, w_kb = statistics.median(fk), statistics.median(wk)
                rd, wr = 2.0 * f_kb * 1024, w_kb * 1024
                algo = 12.0 * elems
                kernels.append({
                    "name": name, "elems": elems, "launches_fetch": len(fk), "launches_write": len(wk),
                    "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
                    "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                    "hbm_bytes_per_launch": rd + wr,
                    "algorithmic_bytes_per_launch": algo,
                    "traffic_over_algorithmic": (rd + wr) / algo,
                })
            continue
        f_kb, w_kb = statistics.median(fetch[name]), statistics.median(write[name])
        rd, wr = 2.0 * f_kb * 1024, w_kb * 1024
        m = re.search(r"SumScaleOp<(\d+),", name)
        o = re.search(r"OptOp<(\d+),", name)
        if m:  # config 2: k inputs read, one output written
            elems, algo = a.local_elems, (int(m.group(1)) + 1) * 4.0 * a.local_elems
        elif o:  # bench.py path_kernels consumer: GD / momentum / Adam, params copy written too
            elems, algo = a.local_elems, {0: 20.0, 1: 28.0, 2: 36.0}.get(int(o.group(1)), 0.0) * a.local_elems
        elif "AccOp" in name or "AddEncodeZeroOp" in name:  # path_kernels: 12 B/elem each
            elems, algo = a.local_elems, 12.0 * a.local_elems
        elif "DecodeScaleOp" in name:  # path_kernels: f16 in, f32 out
            elems, algo = a.local_elems, 6.0 * a.local_elems
        elif "DirectOp<8," in name:  # path_kernels owner chain, 8 M-element chunks: 44 B (f32) / 42 B (f16)
            elems = 8 << 20
            algo = (42.0 if "unsigned short" in name else 44.0) * elems
        else:
            elems, algo = a.elems, a.algo_bytes_per_elem * a.elems
        if not algo:
            continue
        kernels.append({
            "name": name, "elems": elems, "launches_fetch": len(fetch[name]), "launches_write": len(write[name]),
            "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
            "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
            "hbm_bytes_per_launch": rd + wr,
            "algorithmic_bytes_per_launch": algo,
            "traffic_over_algorithmic": (rd + wr) / algo,
        })
    doc = {"note": "median over launches; read = 2 x FETCH_SIZE x 1 KiB (gfx950 half-count), write = WRITE_SIZE x 1 KiB",
           "commit": a.commit, "session": a.session,
           "recorded_utc": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
           "kernels": kernels}
    with open(a.out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
