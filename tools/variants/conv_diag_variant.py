"""Build diagnostic variants of the implicit-GEMM conv kernels (out of tree; csrc/ keeps no
diagnostic macros).  Each variant rewrites a temporary copy of csrc/conv_gemm_kernel.h:

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
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "rtsds_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function", "-Wno-unused-variable"]

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


def build(name):
    tmp = os.path.join(CSRC, "build", "diag_" + name)
    shutil.rmtree(tmp, ignore_errors=True)
    src = os.path.join(tmp, "x", "src")  # common.h includes ../../include/rtsds_hip.h
    os.makedirs(src)
    os.makedirs(os.path.join(tmp, "include"))
    shutil.copy(os.path.join(ROOT, "include", "rtsds_hip.h"), os.path.join(tmp, "include"))
    for f in os.listdir(CSRC):
        if f.endswith((".h", ".hip")):
            shutil.copy(os.path.join(CSRC, f), os.path.join(src, f))
    hdr = os.path.join(src, "conv_gemm_kernel.h")
    text = open(hdr).read()
    for old, new in EDITS[name]:
        n = text.count(old)
        if n != 1:
            raise SystemExit(f"{name}: pattern found {n} times: {old[:60]}")
        text = text.replace(old, new)
    open(hdr, "w").write(text)
    objs = []
    procs = []
    for unit in ("conv_gemm_fwd", "conv_gemm_dgrad", "conv_gemm_wgrad"):
        o = os.path.join(tmp, unit + ".o")
        procs.append(subprocess.Popen([HIPCC, *FLAGS, "-c", os.path.join(src, unit + ".hip"), "-o", o]))
        objs.append(o)
    for p in procs:
        if p.wait() != 0:
            raise SystemExit(f"{name}: compile failed")
    for f in os.listdir(os.path.join(CSRC, "build")):
        if f.endswith(".o") and not f.startswith("conv_gemm_"):
            objs.append(os.path.join(CSRC, "build", f))
    out = os.path.join(ROOT, "rtsds_amd", f"var_diag_{name}.so")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs])
    print("built", out)


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
