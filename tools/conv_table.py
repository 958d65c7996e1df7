"""Per-layer conv table (markdown) from a `bench.py --conv-report` stderr capture: one row per
conv geometry, fwd / dgrad / wgrad microseconds and TF/s, summed over the layers sharing it.
usage: python tools/conv_table.py REPORT.txt [rows]"""
import collections
import re
import sys

LINE = re.compile(r"^\s*([\d.]+) us\s+(fwd|dgrad|wgrad)\s+(n\d+ \S+ -> \S+ k\d+ s\d+ d\d+)\s+([\d.]+) GF")


def main():
    path = sys.argv[1]
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    agg = collections.defaultdict(lambda: {"n": collections.Counter(), "us": collections.Counter(), "gf": collections.Counter()})
    for ln in open(path):
        m = LINE.match(ln)
        if not m:
            continue
        us, tag, geo, gf = float(m.group(1)), m.group(2), m.group(3), float(m.group(4))
        a = agg[geo]
        a["n"][tag] += 1
        a["us"][tag] += us
        a["gf"][tag] += gf
    total = sum(sum(a["us"].values()) for a in agg.values())
    order = sorted(agg.items(), key=lambda kv: -sum(kv[1]["us"].values()))
    print("| conv geometry (batch, in HxWxC -> out HxWxC, kernel, stride, dilation) | layers | fwd us (TF/s) | dgrad us (TF/s) | wgrad us (TF/s) | share of conv time |")
    print("|---|---|---|---|---|---|")
    for geo, a in order[:rows]:
        cells = []
        for tag in ("fwd", "dgrad", "wgrad"):
            if a["n"][tag]:
                us = a["us"][tag]
                cells.append(f"{us:.0f} ({a['gf'][tag] / (us * 1e-6) / 1e3:.0f})")
            else:
                cells.append("-")
        share = sum(a["us"].values()) / total
        print(f"| {geo} | {max(a['n'].values())} | {' | '.join(cells)} | {100 * share:.1f} % |")
    print(f"\n(total conv {total / 1000:.2f} ms over {len(agg)} geometries; TF/s = algorithmic flop / event time)")


if __name__ == "__main__":
    main()
