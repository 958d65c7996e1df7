"""Summarise a rocprofv3 kernel_stats.csv: group template instantiations, per-step ms."""
import csv, collections, subprocess, sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
names = [r["Name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
tot = sum(float(r["TotalDurationNs"]) for r in rows)
agg = collections.defaultdict(lambda: [0, 0.0])
for r, d in zip(rows, dem):
    key = (d if r["Name"].startswith("_Z") else r["Name"]).split("(")[0].replace("void ", "")
    if "conv_gemm_kernel" not in key or "--all" not in sys.argv:
        key = key.split("<")[0]
    if key.startswith("Cijk_"):  # bench.py's torch.mm spacer ahead of the conv-profile step
        key = "hipBLASLt GEMM (bench spacer, not in step)"
    agg[key][0] += int(r["Calls"])
    agg[key][1] += float(r["TotalDurationNs"])
print(f"{'kernel':50s} {'calls':>7s} {'ms/step':>9s} {'avg us':>9s} {'%':>6s}")
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:50s} {c:7d} {t / 1e6 / steps:9.3f} {t / c / 1e3:9.1f} {100 * t / tot:6.1f}")
spacer = sum(t for k, (c, t) in agg.items() if k.startswith("hipBLASLt GEMM (bench spacer"))
print(f"total kernel ms/step: {tot / 1e6 / steps:.3f}  (without the spacer GEMM: {(tot - spacer) / 1e6 / steps:.3f})")
