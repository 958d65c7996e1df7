"""Ordered kernel sequence of the last replayed step from a rocprofv3 kernel_trace.csv.

usage: python tools/diag/ktrace_seq.py run_kernel_trace.csv LAST_N > seq.txt
Prints start offset (us), duration (us) and the demangled short kernel name of the last LAST_N
kernels in dispatch-start order, so that stray launches (blit copies, torch elementwise kernels)
can be attributed to their neighbours."""
import csv
import subprocess
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
names = [r["Kernel_Name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
t0 = int(rows[0]["Start_Timestamp"])
for r, d in zip(rows, dem):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    short = d.split("(")[0].replace("void ", "")
    if "conv_gemm_kernel" not in short:
        short = short.split("<")[0]
    print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}  q{r.get('Queue_Id', '?'):>3s}  {short[:110]}")
