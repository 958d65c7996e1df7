"""Where do the __amd_rocclr_copyBuffer dispatches of a rocprofv3 kernel trace fall?
Counts them per training iteration (iterations delimited by the Adam update kernel) and names
the neighbouring kernels, so one-time setup copies (parameter uploads, arena initialisation)
are told apart from per-step ones.
usage: copy_sites.py <run_kernel_trace.csv> [step-marker-substring] [kernel-substring (default copyBuffer)]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_dev_kernel"
pat = sys.argv[3] if len(sys.argv) > 3 else "copyBuffer"
grid = [r.get("Grid_Size", r.get("Grid_Size_X", "?")) for r in rows]
names = [r["Kernel_Name"] for r in rows]
step = 0
per_step = collections.Counter()
kernels_per_step = collections.Counter()
pairs = collections.Counter()
last_marker = -10
for i, n in enumerate(names):
    if marker in n:
        if i - last_marker > 1:  # consecutive marker launches (one per arena run) = one step
            step += 1
        last_marker = i
    kernels_per_step[step] += 1
    if pat in n:
        per_step[step] += 1
        prev = names[i - 1][:70] if i else "-"
        nxt = names[i + 1][:70] if i + 1 < len(names) else "-"
        pairs[(step > 0, prev + f" | grid {grid[i]}", nxt)] += 1
print(sum(per_step.values()), pat, "dispatches;", step, "steps (marker", marker + ")")
print("per step (0 = before the first update):", dict(sorted(per_step.items())))
print("dispatches per step:", dict(sorted(kernels_per_step.items())))
for (after_first, p, n), c in pairs.most_common(40):
    print(f"{c:5d}  {'steady' if after_first else 'setup '} after {p}\n             before {n}")
