import csv,glob,sys
f=glob.glob(sys.argv[1]+"/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r["Name"].replace("(anonymous namespace)::","").split("(")[0][:40]
    print(f"{n:40s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1000:8.2f} us min {float(r['MinNs'])/1000:8.2f}")
