"""Which kernels neighbour the __amd_rocclr_copyBuffer dispatches in a rocprofv3 kernel trace?
usage: copy_sites.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
pairs = collections.Counter()
for i, n in enumerate(names):
    if "copyBuffer" in n:
        prev = names[i - 1][:70] if i else "-"
        nxt = names[i + 1][:70] if i + 1 < len(names) else "-"
        pairs[(prev, nxt)] += 1
print(sum(pairs.values()), "copyBuffer dispatches")
for (p, n), c in pairs.most_common(40):
    print(f"{c:5d}  after {p}\n       before {n}")
