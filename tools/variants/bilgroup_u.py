"""Variants of bilinear_fwd_group_vec_kernel's column vectors per thread (kBilGroupU)."""
import sys
sys.path.insert(0, __import__("os").path.dirname(__file__))
from textvariant import build  # noqa: E402

for u in sys.argv[1:]:
    build(f"bilu{u}", {"ew.hip": [("static constexpr auto kBilGroupU = 2;", f"static constexpr auto kBilGroupU = {u};")]}, ["ew"])
