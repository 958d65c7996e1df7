"""Same-box A/B of bench.py --conv-report tables: conv_report_ab.py PREFIX_A PREFIX_B
(glob prefixes of the report files, e.g. gpurun_out/r5h_report_base_ gpurun_out/r5h_report_old2_).
Sums the event-timed us of every (op, geometry) row per report (both tables: train step and eval
forward), averages over the repeated reports of a variant, prints the rows that moved by >= 2 %
and the totals."""
import collections
import glob
import re
import sys

row = re.compile(r"^\s*([0-9.]+) us\s+(fwd|dgrad|wgrad|eval)\s+(.*?)\s+[0-9.]+ GF")


def load(prefix):
    files = sorted(glob.glob(prefix + "*"))
    acc = collections.defaultdict(float)
    for f in files:
        for ln in open(f):
            m = row.match(ln)
            if m:
                acc[(m.group(2), m.group(3).strip())] += float(m.group(1)) / len(files)
    return acc, len(files)


a, na = load(sys.argv[1])
b, nb = load(sys.argv[2])
print(f"# A = {sys.argv[1]}* ({na} reports), B = {sys.argv[2]}* ({nb} reports); us summed over all calls of a row")
print(f"{'op':6s} {'geometry':52s} {'A us':>9s} {'B us':>9s} {'A/B-1':>7s}")
for k in sorted(set(a) | set(b), key=lambda k: -max(a.get(k, 0), b.get(k, 0))):
    x, y = a.get(k, 0.0), b.get(k, 0.0)
    if y > 0 and abs(x / y - 1) >= 0.02:
        print(f"{k[0]:6s} {k[1]:52s} {x:9.1f} {y:9.1f} {100 * (x / y - 1):+6.1f}%")
ta, tb = sum(a.values()), sum(b.values())
print(f"{'total':59s} {ta:9.1f} {tb:9.1f} {100 * (ta / tb - 1):+6.1f}%")
