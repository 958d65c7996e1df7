"""A/B variants of the narrow 1x1 data gradient's small-map tiling: pwtile.py -> var_pw64 (one
64-pixel tile size, round-5 launch), var_pwr4 (4 rows per pass), var_pw8 (8-pixel small tiles)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import build  # noqa: E402

T = "constexpr int kPwTileSmall = 16;"
R = "constexpr int kPwRows = 1; "
build("pw64", {"pw.hip": [(T, "constexpr int kPwTileSmall = 64;")]}, ["pw"])
build("pwr4", {"pw.hip": [(R, "constexpr int kPwRows = 4; ")]}, ["pw"])
build("pw8", {"pw.hip": [(T, "constexpr int kPwTileSmall = 8;")]}, ["pw"])
