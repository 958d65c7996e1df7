"""A/B variant: the DGRAD weight repack with a guarded load per element (before round 6)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import build  # noqa: E402

NEW = """  // clamped, unconditional loads, all 16 in flight (a guarded load per element serialised them:
  // one memory round trip each), then the zero fill of the padding selected
  T v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int co = min(ot * 64 + ly + 4 * k, g.co_n - 1), ci = min(ct * 64 + lx, g.ci_n - 1);
    v[k] = w[((co * g.kh + r) * g.kw + sc) * g.ci_n + ci];
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int co = ot * 64 + ly + 4 * k, ci = ct * 64 + lx;
    tile[ly + 4 * k][lx] = (co < g.co_n && ci < g.ci_n) ? to_f(v[k]) : 0.f;
  }"""
OLD = """#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int co = ot * 64 + ly + 4 * k, ci = ct * 64 + lx;
    tile[ly + 4 * k][lx] = (co < g.co_n && ci < g.ci_n) ? to_f(w[((co * g.kh + r) * g.kw + sc) * g.ci_n + ci]) : 0.f;
  }"""
build("oldpack", {"conv.hip": [(NEW, OLD)]}, ["conv"])
