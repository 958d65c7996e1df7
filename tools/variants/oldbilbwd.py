"""A/B variant: the fused bilinear backward as of round 5 (one load per tap over the whole
table row, margins included), taken from git HEAD~N's ew.hip: oldbilbwd.py [REV]."""
import os
import subprocess
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import ROOT, build  # noqa: E402

rev = sys.argv[1] if len(sys.argv) > 1 else "1bc3f56"
old_src = subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:rtsds_amd/csrc/ew.hip"], text=True)
cur_src = open(os.path.join(ROOT, "rtsds_amd", "csrc", "ew.hip")).read()
A, B = "// Both passes in one kernel for 16-B channel vectors", "extern \"C\" int rtsds_bilinear_fwd("


def region(text, a=A):
    i, j = text.index(a), text.index(B)
    return text[i:j]


build("oldbilbwd", {"ew.hip": [(region(cur_src, "// [first, last] nonzero entry"), region(old_src))]}, ["ew"])
