"""Average rocprofv3 counter values per kernel: pmc_summary.py counter_collection.csv [filter]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if flt in r["Kernel_Name"]:
        agg[(r["Kernel_Name"][:60], r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    print("   ", {c: "%.3g" % (sum(v) / len(v)) for c, v in sorted(d.items())})
