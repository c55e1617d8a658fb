"""Measurement tool (not part of the product): rocprofv3 kernel-trace CSVs split
by (kernel, grid size) — the --stats summary averages every launch of a kernel
whatever its bucket size, so a 256 MiB and a 64 MiB launch of the same
instantiation land in one row.  Prints calls / average / median / min / max in
microseconds per (kernel, workgroup size, grid threads), with the HBM fraction
when the per-element bytes of the kernel are known.

usage: python tools/prof_by_size.py <dir with *kernel_trace.csv> [substr ...]
"""
import csv
import glob
import os
import statistics
import sys

# algorithmic bytes per element of the path's stream kernels
PER_ELEM = {"ScaleZeroOp<0>": 12, "SumScaleOp<2,": 12, "SumScaleOp<4,": 20, "SumScaleOp<8,": 36, "CopyOp<float>": 8,
            "FillOp<float>": 4, "DecodeScaleOp<unsigned short": 6, "AccOp": 12, "AddEncodeZeroOp<unsigned short": 12}


def main():
    d = sys.argv[1]
    subs = sys.argv[2:]
    rows = {}
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("ono::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
            if subs and not any(s in name for s in subs):
                continue
            key = (name.split("(")[0][:110], int(r["Workgroup_Size_X"]), int(r["Grid_Size_X"]))
            rows.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"# {d}: rocprofv3 kernel-trace durations by (kernel, workgroup, grid threads), microseconds")
    for (name, wg, grid), v in sorted(rows.items()):
        line = (f"{name:110s} wg {wg:4d} grid {grid:10d} calls {len(v):4d} avg {statistics.mean(v):9.2f} "
                f"median {statistics.median(v):9.2f} min {min(v):9.2f} max {max(v):9.2f}")
        for k, per in PER_ELEM.items():
            if k in name:
                # one 16-B vector (4 elements) per thread of the one-shot grid
                elems = grid * 4
                line += f"  ~{elems / (1 << 18):.0f} MiB  avg {per * elems / (statistics.mean(v) * 1e3) / 8000:.4f} of 8 TB/s"
                break
        print(line)


if __name__ == "__main__":
    main()
