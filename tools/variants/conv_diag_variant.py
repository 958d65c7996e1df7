"""Diagnostic variants of the implicit-GEMM conv kernels (out of tree, tools/variants/textvariant.py):

  nogather  every LDS-DMA of the buffer-resource paths (FWD / DGRAD tap-aligned tiles, WGRAD
            whole-row tiles) reads the same 8 KB at the start of its operand instead of the
            im2col gather: the K loop's issue / barrier / MFMA structure is unchanged, only the
            memory side becomes L2 / L1-resident.
  noepi     the workgroup returns after the K loop (no epilogue, no BatchNorm statistics);
            the accumulators are kept alive by a data-dependent test that never passes.
  both      nogather + noepi.

usage: python3 tools/variants/conv_diag_variant.py NAME [NAME ...]  ->  rtsds_amd/var_diag_NAME.so
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from textvariant import build  # noqa: E402

SMALL = "((((i) * (8 * NW) + wave * 8 + (lane >> 3)) & 63) * 128 + (lane & 7) * 16)"
EDITS = {
    "nogather": [
        ("const int voff = ok ? gba_base[i] + toff2 : (int)0x80000000;",
         "const int voff = ok ? " + SMALL + " : " + SMALL + ";"),
        ("buf_lds16(rs_b, sb + (i * (8 * NW) + wave * 8) * BK, gbb_off[i], kb * 2);",
         "buf_lds16(rs_b, sb + (i * (8 * NW) + wave * 8) * BK, " + SMALL + ", 0);"),
        ("buf_lds16(rs_a, sa + (i * NW + wave) * RPA * BM, wga_off[i], k0 * P.k * 2);",
         "buf_lds16(rs_a, sa + (i * NW + wave) * RPA * BM, " + SMALL + ", 0);"),
        ("buf_lds16(rs_b, sb + (i * NW + wave) * RPB * BN, ok ? ub + wgb_cb[i] : (int)0x80000000, 0);",
         "buf_lds16(rs_b, sb + (i * NW + wave) * RPB * BN, ok ? " + SMALL + " : " + SMALL + ", 0);"),
    ],
    "noepi": [
        ("  // ---- epilogue: C[row][col], row = (lane>>4)*4 + e, col = lane&15 within each 16x16 block\n",
         "  if (acc[0][0][0] != 1234.5f) return;\n"
         "  // ---- epilogue: C[row][col], row = (lane>>4)*4 + e, col = lane&15 within each 16x16 block\n"),
    ],
}
EDITS["both"] = EDITS["nogather"] + EDITS["noepi"]

if __name__ == "__main__":
    for n in sys.argv[1:]:
        build("diag_" + n, {"conv_gemm_kernel.h": EDITS[n]}, ["conv_gemm_fwd", "conv_gemm_dgrad", "conv_gemm_wgrad"])
