"""ctypes binding of librtsds_hip.so (the C ABI declared in include/rtsds_hip.h).

The HIP library is the only compute path: if it is missing, cannot be loaded, or no HIP
device is present, every op raises -- there is no CPU / eager-PyTorch fallback.
``torch`` is imported first so that the process-wide HIP runtime is torch's own
``libamdhip64.so.7`` (same SONAME as the one the library links against).
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below)

_HERE = os.path.dirname(os.path.abspath(__file__))
# RTSDS_LIB: alternative in-tree build of the same ABI (kernel-variant A/B measurements)
DEFAULT_LIB_PATH = os.path.join(_HERE, "librtsds_hip.so")
ABI_VERSION = 10  # include/rtsds_hip.h RTSDS_ABI_VERSION
LIB_PATH = os.environ.get("RTSDS_LIB") or DEFAULT_LIB_PATH

F32, BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_LEAKY, ACT_SIGMOID = 0, 1, 2, 3
ACCUMULATE = 0x100
INPUT_PADDED = 0x400
WEIGHT_PACKED = 0x800
UPCE_SET_CORRECT = 2  # rtsds_upce_fwd want_grad flag
ERRORS = {1: "bad shape", 2: "unsupported configuration", 3: "HIP launch failure", 4: "workspace too small"}

c_int, c_long, c_float, c_size_t, c_void_p = (ctypes.c_int, ctypes.c_long, ctypes.c_float,
                                              ctypes.c_size_t, ctypes.c_void_p)


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("n", "h", "w", "c", "ho", "wo", "k", "kh", "kw", "sh", "sw",
                                     "ph", "pw", "dh", "dw", "dtype")]


class SplitReduceDesc(ctypes.Structure):
    """rtsds_split_reduce_desc (include/rtsds_hip.h)."""
    _fields_ = [("slab", c_void_p), ("dw", c_void_p), ("slab_stride", c_long), ("nv", c_int), ("cv", c_int),
                ("cp", c_int), ("splits", c_int), ("accumulate", c_int)]


P = c_void_p
# name -> (restype, argtypes)
SIGNATURES = {
    "rtsds_conv2d_fwd_workspace": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rtsds_conv2d_input_pitch": (c_int, [ctypes.POINTER(ConvDesc)]),
    "rtsds_conv2d_fwd_stats_tiles": (c_int, [ctypes.POINTER(ConvDesc)]),
    "rtsds_conv2d_fwd": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, c_int, P, P, c_size_t, P]),
    "rtsds_conv2d_fwd_bn": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, P, P, c_int, P, c_size_t, P]),
    "rtsds_conv2d_fwd_bn_ld": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, P, c_long, c_int, P, c_size_t, P]),
    "rtsds_conv2d_fwd_bn_maxpool": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, P, c_int, c_int, c_int, c_int, P,
                                            c_size_t, P]),
    "rtsds_conv2d_dgrad_workspace": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rtsds_conv2d_dgrad_pack_bytes": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rtsds_conv2d_dgrad_pack_many": (c_int, [c_int, ctypes.POINTER(ConvDesc), P, P, P]),
    "rtsds_conv2d_dgrad": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, c_int, P, c_size_t, P]),
    "rtsds_conv2d_dgrad_act": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, c_int, P, c_size_t, P]),
    "rtsds_conv2d_dgrad_bnstats_tiles": (c_int, [ctypes.POINTER(ConvDesc)]),
    "rtsds_conv2d_dgrad_bnstats": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, P, P, P, P, c_int, P, P, c_size_t, P]),
    "rtsds_conv2d_wgrad_workspace": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "rtsds_conv2d_wgrad": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, c_int, P, c_size_t, P]),
    "rtsds_conv2d_wgrad_deferred": (c_int, [ctypes.POINTER(ConvDesc), P, P, P, P, c_int, P, c_size_t,
                                            ctypes.POINTER(SplitReduceDesc), P]),
    "rtsds_split_reduce_many": (c_int, [c_int, ctypes.POINTER(SplitReduceDesc), P]),
    "rtsds_bn_workspace": (c_size_t, [c_long, c_int]),
    "rtsds_bn_fwd": (c_int, [P, P, P, c_long, c_int, P, P, P, P, P, P, P, c_float, c_float, c_int,
                             c_int, P, c_int, c_int, P, c_size_t, P]),
    "rtsds_bn_fwd_ld": (c_int, [P, P, P, c_long, c_long, c_int, P, P, P, P, P, P, P, c_float, c_float, c_int,
                                c_int, P, c_int, c_int, P, c_size_t, P]),
    "rtsds_bn_fold": (c_int, [P, P, P, P, P, c_float, c_int, P, P, P]),
    "rtsds_pooled_mlp_fwd": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "rtsds_pooled_mlp_bwd": (c_int, [P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "rtsds_bn_bwd_part": (c_int, [P, P, P, P, P, c_long, c_int, P, P, P, P, c_int, c_int, c_int, P, c_int, c_int, P,
                                  c_size_t, P]),
    "rtsds_bn_bwd": (c_int, [P, P, P, P, P, P, P, c_long, c_int, P, P, P, P, c_int, c_int, c_int, c_int,
                             P, c_size_t, P]),
    "rtsds_bn_bwd_ld": (c_int, [P, c_long, P, P, P, P, P, P, c_long, c_int, P, P, P, P, c_int, c_int, c_int, c_int,
                                P, c_size_t, P]),
    "rtsds_bn_relu_maxpool_fwd": (c_int, [P, P, P] + [c_int] * 7 + [P, P, P, P, P, P, P, c_float, c_float, c_int, P,
                                                                   c_int, c_int, P, c_size_t, P]),
    "rtsds_bn_relu_maxpool_bwd": (c_int, [P, P, P, P, P, P] + [c_int] * 7 + [P, P, P, P, c_int, c_int, c_int, P,
                                                                            c_size_t, P]),
    "rtsds_nchw_to_nhwc": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P]),
    "rtsds_nchw_to_nhwc_pad": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "rtsds_cast": (c_int, [P, c_int, P, c_int, c_long, P]),
    "rtsds_ffm_head_eval_workspace": (c_size_t, [c_int, c_long, c_int]),
    "rtsds_ffm_head_eval": (c_int, [P, P, P, P, P, P, P, P, c_int, c_long, c_int, c_int, P, c_size_t, P]),
    "rtsds_graph_split": (c_int, [P, c_int, P, P, P]),
    "rtsds_graph_split_launch": (c_int, [P, P]),
    "rtsds_graph_lanes": (c_int, [P, c_int]),
    "rtsds_graph_nodes": (c_int, [P]),
    "rtsds_abi_version": (c_int, []),
    "rtsds_capture_nodes": (c_int, [P]),
    "rtsds_graph_split_destroy": (c_int, [P]),
    "rtsds_copy_channels": (c_int, [P, c_int, c_int, P, c_int, c_int, c_long, c_int, c_int, c_int, P]),
    "rtsds_act_fwd": (c_int, [P, P, c_long, c_int, c_int, P]),
    "rtsds_act_bwd": (c_int, [P, P, P, c_long, c_int, c_float, c_int, P]),
    "rtsds_maxpool_fwd": (c_int, [P, P, P] + [c_int] * 10 + [P]),
    "rtsds_maxpool_bwd": (c_int, [P, P, P] + [c_int] * 10 + [P]),
    "rtsds_gap_workspace": (c_size_t, [c_int, c_long, c_int]),
    "rtsds_gap_fwd": (c_int, [P, P, c_int, c_long, c_int, c_int, P, c_size_t, P]),
    "rtsds_gap_bwd": (c_int, [P, P, c_int, c_long, c_int, c_int, c_int, P]),
    "rtsds_chscale_fwd": (c_int, [P, P, P, c_int, c_long, c_int, c_int, c_int, P]),
    "rtsds_chscale_bwd": (c_int, [P, P, P, P, P, c_int, c_long, c_int, c_int, c_int, P, c_size_t, P]),
    "rtsds_bilinear_fwd": (c_int, [P, P] + [c_int] * 6 + [c_float, c_float, c_int, c_int, c_int, P]),
    "rtsds_bilinear_fwd_scaled": (c_int, [P, P, P, P] + [c_int] * 6 + [c_float, c_float, c_int, c_int, c_int, P]),
    "rtsds_bilinear_bwd_workspace": (c_size_t, [c_int] * 6),
    "rtsds_bilinear_bwd": (c_int, [P, P] + [c_int] * 6 + [c_float, c_float, c_int, c_int, c_int, P, c_size_t, P]),
    "rtsds_softmax_fwd": (c_int, [P, c_long, c_long, c_long, P, c_int, c_int, c_long, c_int, c_int, P]),
    "rtsds_softmax_bwd": (c_int, [P, P, c_int, P, c_long, c_long, c_long, c_int, c_long, c_int, c_int,
                                  P]),
    "rtsds_ce_workspace": (c_size_t, []),
    "rtsds_ce_fwd": (c_int, [P, c_long, c_long, c_long, P, P, c_int, c_long, c_int, c_int, c_int, P,
                             c_size_t, P]),
    "rtsds_ce_bwd": (c_int, [P, c_long, c_long, c_long, P, P, P, P, c_int, c_long, c_int, c_int, c_int,
                             P]),
    "rtsds_bce_fwd": (c_int, [P, P, P, c_int, P]),
    "rtsds_bce_bwd": (c_int, [P, P, P, P, c_int, P]),
    "rtsds_adam_step_dev": (c_int, [P, P, P, P, P, c_long, P, c_float, c_float, c_float, c_float, c_float, c_int, P]),
    "rtsds_upsoftmax_fwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_int, c_int, P]),
    "rtsds_upsoftmax_bwd_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "rtsds_upsoftmax_bwd": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                                    c_int, P, c_size_t, P]),
    "rtsds_resize_aa_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "rtsds_resize_aa": (c_int, [P, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int, P, P, c_int, c_int,
                                P, c_size_t, P]),
    "rtsds_gaussian_blur": (c_int, [P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_float, c_float, P]),
    "rtsds_gta5_decode": (c_int, [P, P, c_int, c_int, P]),
    "rtsds_sgd_step": (c_int, [P, P, P, P, c_long, P, c_float, c_float, c_float, c_float, c_int, c_int,
                               c_float, c_int, P]),
    "rtsds_adam_step": (c_int, [P, P, P, P, P, c_long, c_float, c_float, c_float, c_float, c_float,
                                c_int, c_float, c_int, P]),
    "rtsds_argmax": (c_int, [P, c_long, c_long, c_long, P, P, P, c_int, c_long, c_int, c_int, P]),
    "rtsds_confusion": (c_int, [P, P, P, c_long, c_int, P]),
    "rtsds_adaptive_avgpool_fwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "rtsds_adaptive_avgpool_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "rtsds_upce_finish": (c_int, [c_int, P, P, P, P]),
    "rtsds_ce_finish": (c_int, [P, P, P]),
    "rtsds_upce_workspace": (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float]),
    "rtsds_upce_fwd": (c_int, [c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                               c_int, P, P, P, c_int, c_int, P, c_size_t, P]),
    "rtsds_upce_bwd": (c_int, [c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_float,
                               c_int, P, c_size_t, P]),
}

_lib = None


def load(path=LIB_PATH):
    """dlopen the library and attach signatures (no GPU needed).  Raises if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise RuntimeError(f"rtsds_amd: HIP library not built ({path}); run __graft_entry__.build()")
        lib = ctypes.CDLL(path)
        # the library must be built from this ABI revision (include/rtsds_hip.h RTSDS_ABI_VERSION):
        # an A/B variant built from older sources (tools/build_rev_variant.sh) with a changed
        # signature would otherwise be called with the wrong arguments
        ver = getattr(lib, "rtsds_abi_version", None)
        if ver is None:
            raise RuntimeError(f"rtsds_amd: {path} predates the ABI version check; rebuild it")
        ver.restype, ver.argtypes = ctypes.c_int, []
        if ver() != ABI_VERSION:
            raise RuntimeError(f"rtsds_amd: {path} has ABI revision {ver()}, this package needs {ABI_VERSION}")
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib = lib
    return _lib


class _Lib:
    def __getattr__(self, name):
        fn = getattr(load(), name)

        def call(*args):
            rc = fn(*args)
            if name.endswith(("_workspace", "_tiles", "_pitch", "_bytes")):  # queries: the value itself
                return rc
            if rc != 0:
                raise RuntimeError(f"rtsds_amd: {name} failed: {ERRORS.get(rc, rc)}")
            return rc
        return call


lib = _Lib()
