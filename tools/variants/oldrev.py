"""A/B variant: one csrc unit as of a git revision (the tree's other objects):
oldrev.py NAME UNIT REV  ->  rtsds_amd/var_NAME.so with csrc/UNIT.hip taken from REV."""
import os
import subprocess
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import ROOT, build  # noqa: E402

name, unit, rev = sys.argv[1:4]
old = subprocess.check_output(["git", "-C", ROOT, "show", f"{rev}:rtsds_amd/csrc/{unit}.hip"], text=True)
cur = open(os.path.join(ROOT, "rtsds_amd", "csrc", unit + ".hip")).read()
build(name, {unit + ".hip": [(cur, old)]}, [unit])
