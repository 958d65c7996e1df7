"""A/B variant: the round-5 serial-load loops of pooled_wgrad_kernel, colsum_part_kernel and
colsum_final_kernel (one load per iteration), taken from git REV's conv.hip: oldsmall.py [REV]."""
import os
import subprocess
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import ROOT, build  # noqa: E402

rev = sys.argv[1] if len(sys.argv) > 1 else "c160d4a"
old = subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:rtsds_amd/csrc/conv.hip"], text=True)
cur = open(os.path.join(ROOT, "rtsds_amd", "csrc", "conv.hip")).read()


def region(text, start, end):
    i = text.index(start)
    return text[i:text.index(end, i)]


edits = []
for a, b in (("__global__ void __launch_bounds__(256) pooled_wgrad_kernel", "// Vector forms (C % V == 0)"),
             ("__global__ void __launch_bounds__(256) colsum_part_kernel", "static const int kColsumRB")):
    edits.append((region(cur, a, b), region(old, a, b)))
build("oldsmall", {"conv.hip": edits}, ["conv"])
