"""Per-kernel average durations from a rocprofv3 output directory (kernel_stats.csv, or the rocpd .db)."""
import csv, glob, sqlite3, sys
from collections import defaultdict

d = sys.argv[1]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
if f:
    for r in csv.DictReader(open(f[0])):
        n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
        print(f"{n:40s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1000:8.2f} us min {float(r['MinNs'])/1000:8.2f}")
else:
    c = sqlite3.connect(glob.glob(d + "/**/*.db", recursive=True)[0])
    acc = defaultdict(list)
    q = ("select s.kernel_name, k.end - k.start from rocpd_kernel_dispatch k "
         "join rocpd_info_kernel_symbol s on k.kernel_id = s.id")
    for name, dur in c.execute(q):
        acc[name].append(dur)
    for name, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        n = name.replace("(anonymous namespace)::", "").split("(")[0][:40]
        print(f"{n:40s} calls {len(v):5d} avg {sum(v)/len(v)/1000:8.2f} us min {min(v)/1000:8.2f}")
