"""Per-kernel medians of rocprofv3 --pmc counter_collection CSVs.
usage: pmc_table.py DIR... [--match SUBSTR...]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

args = sys.argv[1:]
match = []
if "--match" in args:
    k = args.index("--match")
    match, args = args[k + 1:], args[:k]
vals = defaultdict(lambda: defaultdict(list))
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = defaultdict(float)  # (dispatch, kernel, counter) -> summed over dimensions
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if match and not any(m in name for m in match):
                continue
            per[(r.get("Dispatch_Id"), name.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, name, ctr), v in per.items():
            vals[name][ctr].append(v)
for name in sorted(vals):
    print(name)
    for ctr in sorted(vals[name]):
        xs = vals[name][ctr]
        print(f"   {ctr:24s} median {statistics.median(xs):16.1f}  n={len(xs)}")
