"""A/B variant: the stem maxpool backward on the per-pixel gather kernel (maxpool_bwd_k3s2) instead of the quad kernel."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import build  # noqa: E402

build("oldpool", {"ew.hip": [("if (c % VecT<T>::N == 0 && k == 3 && s == 2 && (p == 0 || p == 1) && total < (1L << 31)) {",
                              "if (false) {")]}, ["ew"])
