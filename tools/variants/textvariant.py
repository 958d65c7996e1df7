"""Out-of-tree kernel variants by text edits (csrc/ keeps no A/B macros): copy csrc/ to a
scratch directory, apply exact-match edits, recompile the named units and link them with the
main build's other objects into rtsds_amd/var_NAME.so (same ABI revision as the tree).

    from textvariant import build
    build("u2", {"ew.hip": [(old, new), ...]}, units=["ew"])
"""
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "rtsds_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-function", "-Wno-unused-variable"]


def build(name, edits, units):
    tmp = os.path.join(CSRC, "build", "var_" + name)
    shutil.rmtree(tmp, ignore_errors=True)
    src = os.path.join(tmp, "x", "src")  # common.h includes ../../include/rtsds_hip.h
    os.makedirs(src)
    os.makedirs(os.path.join(tmp, "include"))
    shutil.copy(os.path.join(ROOT, "include", "rtsds_hip.h"), os.path.join(tmp, "include"))
    for f in os.listdir(CSRC):
        if f.endswith((".h", ".hip")):
            shutil.copy(os.path.join(CSRC, f), os.path.join(src, f))
    for f, pairs in edits.items():
        path = os.path.join(src, f)
        text = open(path).read()
        for old, new in pairs:
            n = text.count(old)
            if n != 1:
                raise SystemExit(f"{name}: {f}: pattern found {n} times: {old[:70]!r}")
            text = text.replace(old, new)
        open(path, "w").write(text)
    procs, objs = [], []
    for unit in units:
        o = os.path.join(tmp, unit + ".o")
        procs.append(subprocess.Popen([HIPCC, *FLAGS, "-c", os.path.join(src, unit + ".hip"), "-o", o]))
        objs.append(o)
    for p in procs:
        if p.wait() != 0:
            raise SystemExit(f"{name}: compile failed")
    for f in sorted(os.listdir(os.path.join(CSRC, "build"))):
        if f.endswith(".o") and f[:-2] not in units:
            objs.append(os.path.join(CSRC, "build", f))
    out = os.path.join(ROOT, "rtsds_amd", f"var_{name}.so")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs])
    print("built", out)
    return out
