"""Per-step HBM traffic by kernel from tools/pmc_bench.sh's two --pmc passes.

Usage: pmc_traffic.py DIR STEPS|auto [OUT.json]
(auto: steps = dispatches of upce_fwd_kernel, which runs once per training step -- the
bench's eager warm-up and GraphedStep warm-up iterations are profiled too)
FETCH_SIZE and WRITE_SIZE are in KB per dispatch (rocprofv3); on gfx950 FETCH_SIZE reports
half the bytes of wide (16 B/lane) streaming reads (MI355X_MICROARCH.md, HBM section), so
fetch bytes = 2 x FETCH_SIZE x 1024.  WRITE_SIZE is exact for 16-B stores."""
import collections
import csv
import glob
import json
import re
import sys


def load(d, counter):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]] += float(r["Counter_Value"])
    return agg


def short(names):
    """Base kernel name: Itanium length-prefixed identifier for mangled names (c++filt does
    not know every gfx type code, e.g. DF16b), else the text before '(' / '<'."""
    out = []
    for n in names:
        m = re.match(r"_Z(\d+)", n)
        out.append(n[m.end():m.end() + int(m.group(1))] if m else n.split("(")[0].replace("void ", "").split("<")[0])
    return out


def main():
    d = sys.argv[1]
    if sys.argv[2] == "auto":
        path = glob.glob(f"{d}/fetch/**/*counter_collection.csv", recursive=True)[0]
        steps = float(len({r["Dispatch_Id"] for r in csv.DictReader(open(path))
                           if "upce_fwd_kernel" in r["Kernel_Name"]}))
    else:
        steps = float(sys.argv[2])
    fetch, write = load(d + "/fetch", "FETCH_SIZE"), load(d + "/write", "WRITE_SIZE")
    names = sorted(set(fetch) | set(write))
    if "--variants" in sys.argv:  # per instantiation (full kernel name) instead of per base name
        sys.argv.remove("--variants")
        rows = sorted(((2 * 1024 * fetch.get(n, 0.0) / steps, 1024 * write.get(n, 0.0) / steps, n) for n in names),
                      key=lambda x: -(x[0] + x[1]))
        print(f"{'kernel (instantiation)':90s} {'read MB/step':>13s} {'write MB/step':>14s}")
        for r, w, n in rows[:40]:
            print(f"{n[:90]:90s} {r / 1e6:13.1f} {w / 1e6:14.1f}")
        return
    per = collections.defaultdict(lambda: [0.0, 0.0])
    for n, s in zip(names, short(names)):
        per[s][0] += 2 * 1024 * fetch.get(n, 0.0) / steps
        per[s][1] += 1024 * write.get(n, 0.0) / steps
    tot = [sum(v[0] for v in per.values()), sum(v[1] for v in per.values())]
    print(f"{'kernel':40s} {'read MB/step':>13s} {'write MB/step':>14s}")
    for k, (r, w) in sorted(per.items(), key=lambda x: -(x[1][0] + x[1][1])):
        print(f"{k:40s} {r / 1e6:13.1f} {w / 1e6:14.1f}")
    print(f"{'total':40s} {tot[0] / 1e6:13.1f} {tot[1] / 1e6:14.1f}")
    if len(sys.argv) > 3:
        # every conv-family launch (implicit GEMM, direct convs and their helpers), as the
        # live roofline's event-timed conv calls include them
        fams = ("conv_gemm_kernel", "hconv_fwd_kernel", "hconv_dgrad_nt_kernel", "nwgrad_kernel", "tapconv_kernel", "tapwgrad_kernel", "imgconv_fwd_kernel", "imgconv_pool_kernel",
                "pw_dgrad_kernel", "pooled_fwd_vec_kernel", "pooled_dgrad_vec_kernel", "pooled_wgrad_kernel",
                "split_reduce_many_kernel", "split_reduce_kernel", "dgrad_pack_kernel", "repack_wt_kernel",
                "pad_channels_kernel", "dgrad_split_reduce_kernel", "fwd_split_reduce_kernel", "sp_repack_w_kernel",
                "sp_unpack_dw_kernel")
        conv = [sum(per[k][0] for k in fams if k in per), sum(per[k][1] for k in fams if k in per)]
        json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py (tools/pmc_bench.sh); "
                             "fetch x2 gfx950 correction", "steps_profiled": steps,
                   "conv_gemm_kernel_bytes_per_step": conv[0] + conv[1],
                   "conv_gemm_kernel_read_bytes_per_step": conv[0], "conv_gemm_kernel_write_bytes_per_step": conv[1],
                   "all_kernels_bytes_per_step": tot[0] + tot[1],
                   "per_kernel_bytes_per_step": {k: v[0] + v[1] for k, v in per.items()}},
                  open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
