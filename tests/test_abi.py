"""C-ABI boundary checks (CPU): the library builds/loads without a GPU, exports every
function include/rtsds_hip.h declares, and the ctypes signatures agree with the header."""
import os
import re

import pytest

from rtsds_amd import _lib

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "rtsds_hip.h")


def _declarations():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(int|size_t)\s+(rtsds_\w+)\s*\(([^)]*)\)\s*;", text):
        args = m.group(3).strip()
        n = 0 if args in ("", "void") else len(args.split(","))
        decls[m.group(2)] = (m.group(1), n)
    return decls


def test_header_parses():
    d = _declarations()
    assert "rtsds_conv2d_fwd" in d and len(d) >= 30


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in _declarations():
        assert hasattr(lib, name), name


@pytest.mark.parametrize("name", sorted(_declarations()))
def test_ctypes_signature_matches_header(name):
    ret, nargs = _declarations()[name]
    assert name in _lib.SIGNATURES, f"{name} not bound in rtsds_amd/_lib.py"
    res, args = _lib.SIGNATURES[name]
    assert len(args) == nargs, (name, len(args), nargs)
    assert (res is _lib.c_size_t) == (ret == "size_t"), name


def test_abi_version_matches_header():
    """The loader refuses a library of another ABI revision (stale A/B variant builds)."""
    m = re.search(r"#define RTSDS_ABI_VERSION (\d+)", open(HDR).read())
    assert m and int(m.group(1)) == _lib.ABI_VERSION
    assert _lib.load().rtsds_abi_version() == _lib.ABI_VERSION


def test_errors_raise_without_fallback():
    # the product path refuses CPU tensors instead of silently computing elsewhere
    import torch
    from rtsds_amd import functional as F
    x = torch.zeros(1, 3, 8, 8)
    with pytest.raises(RuntimeError, match="HIP"):
        F.pack_input(x, torch.float32)


def test_upce_workspace_aux_wave_never_shrinks_support():
    """Host planning of the fused upsample + CE (no GPU call): the auxiliary wave's LDS fold rows
    are used only where they fit, so 3 heads at a x2 resize (over the LDS cap with them) still
    take the fused path -- without the auxiliary wave -- and the x8 bench geometry keeps it."""
    lib = _lib.load()
    x2 = [lib.rtsds_upce_workspace(h, 2, 8, 16, 19, 16, 32, 0.5, 0.5) for h in (1, 2, 3)]
    assert all(w > 0 for w in x2), x2
    x8 = [lib.rtsds_upce_workspace(h, 8, 64, 128, 19, 512, 1024, 0.125, 0.125) for h in (3, 4)]
    assert x8[0] > 0 and x8[1] > 0
