"""A/B variants of the BatchNorm backward statistics pass's row blocks: bnrb.py -> var_bnrb1k (up
to 1024 row blocks: 4 workgroups per CU), var_bnrb1ku4 (1024 and 4 rows in flight per thread)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import build  # noqa: E402

RB = "static constexpr auto kBnBwdRBMax = 512;"
U = "    constexpr int U = 2;  // rows in flight per thread (loads issued before any use)"
build("bnrb1k", {"bn.hip": [(RB, "static constexpr auto kBnBwdRBMax = 1024;")]}, ["bn"])
build("bnrb1ku4", {"bn.hip": [(RB, "static constexpr auto kBnBwdRBMax = 1024;"), (U, "    constexpr int U = 4;")]}, ["bn"])
