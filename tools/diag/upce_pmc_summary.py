"""Per-launch SQ counters of upce_fwd_kernel from tools/pmc_upce2.sh output dirs."""
import csv, glob, sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(list)
for f in glob.glob(f"{d}/sq*/**/*counter_collection.csv", recursive=True):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "upce_fwd" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, c), v in per.items():
        agg[c].append(v)
for c in sorted(agg):
    v = agg[c]
    print(f"{c:28s} {sum(v) / len(v):16.4g}  (launches {len(v)})")
