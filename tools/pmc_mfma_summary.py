"""MFMA utilisation per kernel from a tools/pmc_mfma.sh pass.

util_clk  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)   (per-XCD busy cycles)
util_2.4  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x 2.4 GHz)     (vs the peak clock)
usage: pmc_mfma_summary.py DIR/run_counter_collection.csv [steps]"""
import collections
import csv
import subprocess
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
disp = collections.defaultdict(dict)
for r in rows:
    d = disp[r["Dispatch_Id"]]
    d["name"] = r["Kernel_Name"]
    d["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    d[r["Counter_Name"]] = float(r["Counter_Value"])
names = sorted({d["name"] for d in disp.values()})
dem = dict(zip(names, subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")))
agg = collections.defaultdict(lambda: collections.Counter())
for d in disp.values():
    key = dem.get(d["name"], d["name"]).split("(")[0].replace("void ", "")
    a = agg[key]
    a["n"] += 1
    a["dur"] += d["dur"]
    for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
              "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES", "SQ_WAVES"):
        a[c] += d.get(c, 0.0)
tot_dur = sum(a["dur"] for a in agg.values())
print(f"{'kernel':72s} {'n':>5s} {'us/step':>9s} {'%time':>6s} {'mfma%clk':>9s} {'mfma%2.4':>9s} {'wait%':>6s} {'instw%':>6s}")
for k, a in sorted(agg.items(), key=lambda x: -x[1]["dur"])[:40]:
    busy = a["SQ_VALU_MFMA_BUSY_CYCLES"]
    u1 = busy / (1024 * a["GRBM_GUI_ACTIVE"] / 8) if a["GRBM_GUI_ACTIVE"] else 0
    u2 = busy / (1024 * a["dur"] * 2.4) if a["dur"] else 0
    wc = a["SQ_WAVE_CYCLES"] or 1
    print(f"{k[:72]:72s} {a['n']:5d} {a['dur'] / 1e3 / steps:9.1f} {100 * a['dur'] / tot_dur:6.1f} {100 * u1:9.1f} "
          f"{100 * u2:9.1f} {100 * a['SQ_WAIT_ANY'] / wc:6.1f} {100 * a['SQ_WAIT_INST_ANY'] / wc:6.1f}")
for label, fams in (("conv family", ("conv_gemm", "hconv")),
                    ("conv family incl. tapconv / imgconv / nwgrad", ("conv_gemm", "hconv", "nwgrad", "tapconv", "imgconv"))):
    conv = [a for k, a in agg.items() if any(f in k for f in fams)]
    busy = sum(a["SQ_VALU_MFMA_BUSY_CYCLES"] for a in conv)
    dur = sum(a["dur"] for a in conv)
    gui = sum(a["GRBM_GUI_ACTIVE"] for a in conv)
    print(f"{label}: {dur / 1e3 / steps:.1f} us/step, MFMA busy {100 * busy / (1024 * gui / 8):.1f} % of busy clocks, "
          f"{100 * busy / (1024 * dur * 2.4):.1f} % at 2.4 GHz; MFMA busy cycles/step {busy / steps:.3g}")
