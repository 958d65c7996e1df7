"""Timeline of the last training step in a rocprofv3 kernel_trace.csv (graph replay): span,
per-queue busy time, time with >= 1 kernel running (union), and the longest idle gaps of the
union with their neighbouring kernels.  A step = the kernels after the previous step's last
Adam launch up to and including this step's.
usage: step_timeline.py run_kernel_trace.csv [top_gaps]"""
import csv
import subprocess
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
# steps end with a run of Adam launches; split runs at gaps in the index sequence
ends = [adam[i] for i in range(len(adam)) if i + 1 == len(adam) or adam[i + 1] != adam[i] + 1]
lo, hi = ends[-2] + 1, ends[-1] + 1
step = rows[lo:hi]
dem = subprocess.run(["c++filt"], input="\n".join(r["Kernel_Name"] for r in step), capture_output=True, text=True).stdout.split("\n")
short = []
for d in dem:
    s = d.split("(")[0].replace("void ", "")
    short.append(s if "conv_gemm_kernel" in s else s.split("<")[0])
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), n) for r, n in zip(step, short)]
t0, t1 = min(a for a, _, _, _ in iv), max(b for _, b, _, _ in iv)
print(f"step: {len(iv)} kernels, span {(t1 - t0) / 1e3:.1f} us")
qs = {}
for a, b, q, _ in iv:
    qs[q] = qs.get(q, 0) + (b - a)
for q, t in sorted(qs.items()):
    print(f"  queue {q}: busy {t / 1e3:.1f} us")
ev = sorted([(a, 1) for a, _, _, _ in iv] + [(b, -1) for _, b, _, _ in iv])
cur, last, busy, conc = 0, t0, 0, {}
gaps = []
for t, d in ev:
    if cur > 0:
        busy += t - last
    conc[cur] = conc.get(cur, 0) + (t - last)
    if cur == 0 and t > last:
        gaps.append((t - last, last, t))
    cur += d
    last = t
print(f"  >= 1 kernel running: {busy / 1e3:.1f} us ({100 * busy / (t1 - t0):.1f} %)")
print("  concurrency (kernels running: us): " + ", ".join(f"{k}: {v / 1e3:.1f}" for k, v in sorted(conc.items())))
print(f"  idle gaps: {len(gaps)}, total {sum(g for g, _, _ in gaps) / 1e3:.1f} us; longest:")
for g, a, b in sorted(gaps, reverse=True)[:top]:
    before = max((x for x in iv if x[1] <= a), key=lambda x: x[1])
    after = min((x for x in iv if x[0] >= b), key=lambda x: x[0])
    print(f"    {g / 1e3:7.2f} us at {(a - t0) / 1e3:8.1f}: after {before[3][:60]} (q{before[2]}) -> {after[3][:60]} (q{after[2]})")
# main-queue waits: intervals where the busiest queue is idle while another queue runs
main = max(qs, key=qs.get)
mi = sorted((a, b) for a, b, q, _ in iv if q == main)
waits, last = [], mi[0][1]
for a, b in mi[1:]:
    if a - last > 3000:  # > 3 us
        waits.append((a - last, last, a))
    last = max(last, b)
print(f"  queue {main} waits > 3 us: {len(waits)}, total {sum(w for w, _, _ in waits) / 1e3:.1f} us")
for w, a, b in sorted(waits, reverse=True)[:top]:
    other = [x for x in iv if x[2] != main and x[0] < b and x[1] > a]
    names = ", ".join(sorted({x[3][:40] for x in other}))[:150]
    print(f"    {w / 1e3:7.1f} us at {(a - t0) / 1e3:8.1f}: other queues run {names}")
