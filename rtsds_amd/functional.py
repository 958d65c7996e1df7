"""Autograd functions over the C ABI (include/rtsds_hip.h).

Every forward and backward here is a call into librtsds_hip.so on the current HIP stream;
PyTorch supplies only memory (caching allocator), the stream and the autograd graph.
Activations are NHWC tensors of logical shape [N, C, H, W] (``torch.channels_last``) in the
runtime compute dtype; parameters, statistics and losses are fp32.
"""
import ctypes

import numpy as np
import torch

from ._lib import ACT_RELU, ACT_SIGMOID, INPUT_PADDED, UPCE_SET_CORRECT, WEIGHT_PACKED, ConvDesc, SplitReduceDesc, lib
from .runtime import (CL, bump_params_epoch, collective, dcode, dp_world, empty_nhwc, nhwc, params_epoch,
                      register_fold, require_hip, side_enabled, side_fork, stream, workspace)

_P = lambda t: None if t is None else t.data_ptr()  # noqa: E731

# Optional conv-kernel timing (bench.py's live roofline): when ``CONV_PROFILE`` is a list,
# every implicit-GEMM launch is bracketed by HIP events on the launch stream and
# (start, end, algorithmic_flops) is appended.
CONV_PROFILE = None


def _conv_flops(d):
    return 2.0 * d.n * d.ho * d.wo * d.k * d.c * d.kh * d.kw


class _Timed:
    def __init__(self, d, tag="fwd"):
        self.d, self.tag = d, tag

    def __enter__(self):
        if CONV_PROFILE is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if CONV_PROFILE is not None:
            self.e1.record()
            CONV_PROFILE.append((self.e0, self.e1, _conv_flops(self.d), self.tag, self.d))


# ----------------------------------------------------------------------------- grad sinks
def _sink(p):
    """The flat-arena gradient view of parameter ``p`` if an rtsds optimizer owns it.
    Backward kernels then accumulate straight into it (accumulate flag) and the Function
    returns None for ``p``, so autograd's per-parameter AccumulateGrad add never runs."""
    ref = getattr(p, "_rt_arena", None) if p is not None else None
    if ref is None:
        return None
    arena, i = ref
    return arena.sink(i)


def _sinks(*params):
    """All-or-nothing: the sinks of every given (non-None) parameter, or None."""
    out = []
    for p in params:
        if p is None:
            out.append(None)
            continue
        s = _sink(p)
        if s is None:
            return None
        out.append(s)
    return out


# ----------------------------------------------------------------------------- conv
def _conv_desc(x, k, kh, kw, stride, padding, dilation):
    n, c, h, w = x.shape
    ho = (h + 2 * padding[0] - dilation[0] * (kh - 1) - 1) // stride[0] + 1
    wo = (w + 2 * padding[1] - dilation[1] * (kw - 1) - 1) // stride[1] + 1
    d = ConvDesc(n, h, w, c, ho, wo, k, kh, kw, stride[0], stride[1], padding[0], padding[1],
                 dilation[0], dilation[1], dcode(x))
    return d


def is_padded_input(x, d=None):
    """A tensor written with the padded channel pitch a conv gathers (upsample_softmax's class
    probabilities, pitch 32; pack_input's 3-channel images, pitch 4): [N, C, H, W] view of an
    NHWC [N, H, W, Cp] buffer, zero in C..Cp-1.  With a conv descriptor ``d``: and Cp is the
    pitch that conv reads (rtsds_conv2d_input_pitch)."""
    cp = getattr(x, "_rt_cpad", None)
    ok = cp is not None and x.dim() == 4 and x.stride(1) == 1 and x.stride(3) == cp and \
        x.stride(2) == cp * x.shape[3] and x.stride(0) == cp * x.shape[2] * x.shape[3]
    return ok and (d is None or lib.rtsds_conv2d_input_pitch(ctypes.byref(d)) == cp)


def detach_padded(x):
    """x.detach() keeping the padded-input marker (tensor attributes do not survive detach)."""
    y = x.detach()
    if getattr(x, "_rt_cpad", None) is not None:
        y._rt_cpad = x._rt_cpad
    return y


# ----------------------------------------------------------------------------- packed dgrad weights
# The data-gradient GEMMs read each conv weight transposed ([ci][tap][co], flipped / split per
# stride-2 phase by route).  For weights owned by an rtsds optimizer the transposed copy is
# refreshed by the optimizer right after its update -- every registered conv in one launch
# (optim._Arena.repack -> rtsds_conv2d_dgrad_pack_many) -- and the backward passes it with
# RTSDS_WEIGHT_PACKED instead of repacking per call.  A conv registers on its first backward;
# the copy is used once the optimizer has packed it from the current bf16 shadow.
_DPACK = {"on": True}


def set_dgrad_packs(on):
    """Use optimizer-maintained packed dgrad weights (default on; off: repack per call)."""
    _DPACK["on"] = bool(on)


class _DPack:
    __slots__ = ("arena", "key", "desc", "buf", "valid")


def _desc_key(d):
    return tuple(getattr(d, f) for f, _ in ConvDesc._fields_)


def _dgrad_weight(weight, wq, d):
    """(weight operand, flag) for a data-gradient launch of ``weight`` with descriptor ``d``."""
    if not _DPACK["on"] or wq.dtype != torch.bfloat16 or weight is None:
        return wq, 0
    ref = getattr(weight, "_rt_arena", None)
    if ref is None:
        return wq, 0
    pk = getattr(weight, "_rt_dpack", None)
    if pk is not None and pk.arena is ref[0]:
        if pk.key == _desc_key(d) and pk.buf is not None and pk.valid is not None and \
                pk.valid == getattr(weight, "_rt_shadow_key", None) and wq is getattr(weight, "_rt_shadow", None):
            return pk.buf, WEIGHT_PACKED
        return wq, 0
    pk = _DPack()
    pk.arena, pk.key, pk.valid = ref[0], _desc_key(d), None
    pk.desc = ConvDesc(*pk.key)
    nb = lib.rtsds_conv2d_dgrad_pack_bytes(ctypes.byref(d))
    pk.buf = torch.empty(nb // 2, dtype=torch.bfloat16, device=wq.device) if nb else None
    weight._rt_dpack = pk
    if nb:
        ref[0].dpacks.append(weight)
    return wq, 0


class GradJoin:
    """Gradient of a tensor read by ``n`` rtsds Functions -- a residual block's input, read by
    conv1 and by the identity (BatchNorm residual) or downsample branch
    (build_contextpath.py BasicBlock / Bottleneck; torchvision resnet.py semantics).

    Autograd would sum the ``n`` contributions with its own elementwise add over the whole
    activation.  Instead the first contribution's buffer is kept here and handed to the next
    producer, whose kernel accumulates into it (conv dgrad ``accumulate`` flag); the first
    ``n - 1`` backward calls return None for the tensor and the last returns the sum, so the
    engine sees one gradient.  Order-independent: whichever producer runs last returns.

    ``first_returns``: for a tensor whose readers need not all be reached by the backward (a
    model output the caller may leave out of the loss): the first contribution returns its
    buffer and later ones accumulate into it in place and return None -- the engine runs the
    tensor's producer only after every reached reader, so it sees the full sum either way."""

    __slots__ = ("left", "buf", "first")

    def __init__(self, n, first_returns=False):
        self.left = n
        self.buf = None
        self.first = first_returns

    def put(self, g):
        """Record this producer's finished contribution (``g`` already includes ``buf``)."""
        if self.first:
            if self.buf is None:
                self.buf = g
                return g
            return None  # accumulated into the returned buffer
        self.buf = g
        self.left -= 1
        return g if self.left == 0 else None


def _join_add(join, g):
    """Contribution ``g`` computed into its own buffer: fold any earlier one in, then put."""
    if join is None:
        return g
    if join.buf is not None:  # not reached in the residual blocks (the BN runs first)
        if join.first:
            join.buf.add_(g)
            return join.put(join.buf)
        g.add_(join.buf)
    return join.put(g)


# ----------------------------------------------------------------------------- deferred wgrad reduce
# The split-K weight gradients of one backward pass leave their fp32 partial slabs in workspace
# and are reduced into the optimizer's gradient arena together, by one rtsds_split_reduce_many
# launch at the end of the backward (an autograd engine callback, so .grad is complete when
# backward() returns) instead of one small launch per conv (~27 per BiSeNet step).  Same sums,
# same order.  Off while bench.py event-times each conv (CONV_PROFILE).
DEFER_WGRAD_REDUCE = True
_deferred = []  # [(SplitReduceDesc, workspace tensor holding the slabs, stream of the wgrad)]


def flush_wgrad_reduce():
    """Run the pending split-K reductions (every deferral also queues this as an end-of-backward
    callback; the first one of a backward pass does the work, optim.step() calls it too)."""
    global _deferred
    items, _deferred = _deferred, []
    if not items:
        return
    cur = torch.cuda.current_stream(items[0][1].device)
    for st in {it[2] for it in items}:  # wgrads issued on branch streams
        if st != cur:
            cur.wait_stream(st)
    # one launch per run of distinct targets (a parameter reduced twice keeps its order)
    batch, seen = [], set()
    for desc, _ws, _st in items + [(None, None, None)]:
        if desc is None or desc.dw in seen or len(batch) == 16:
            if batch:
                arr = (SplitReduceDesc * len(batch))(*batch)
                lib.rtsds_split_reduce_many(len(batch), arr, cur.cuda_stream)
            batch, seen = [], set()
        if desc is not None:
            batch.append(desc)
            seen.add(desc.dw)
    for _desc, ws, st in items:
        if st != cur:
            ws.record_stream(cur)


def _wgrad_into_arena(d, x, g, sinks, xflag, ws):
    """Weight gradient accumulated into the optimizer arena; its split-K reduction deferred to
    the end of the backward pass when allowed."""
    if DEFER_WGRAD_REDUCE and CONV_PROFILE is None and x.dtype == torch.bfloat16:
        pend = SplitReduceDesc()
        lib.rtsds_conv2d_wgrad_deferred(ctypes.byref(d), _P(x), _P(g), _P(sinks[0]), _P(sinks[1]), 1 | xflag,
                                        _P(ws), ws.numel(), ctypes.byref(pend), stream())
        if pend.nv > 0:
            _deferred.append((pend, ws, torch.cuda.current_stream(ws.device)))
            torch.autograd.Variable._execution_engine.queue_callback(flush_wgrad_reduce)
        return
    with _Timed(d, "wgrad"):
        lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(x), _P(g), _P(sinks[0]), _P(sinks[1]), 1 | xflag,
                               _P(ws), ws.numel(), stream())


class ConvFn(torch.autograd.Function):
    """nn.Conv2d forward / backward (bias and LeakyReLU/ReLU epilogue optionally fused).

    ``wq`` is the weight in compute dtype and kernel layout [Cout][KH][KW][Cin] (the fp32
    parameter itself or its bf16 shadow); gradients are returned for ``weight``."""

    @staticmethod
    def forward(ctx, x, weight, bias, wq, stride, padding, dilation, act, stats, join=None, fold=(0, False),
                bn_link=None):
        """``fold = (in_act, out_folded)``: ``in_act`` -- x is the output of a ReLU / LeakyReLU
        whose backward this conv's data gradient applies in its epilogue
        (rtsds_conv2d_dgrad_act); ``out_folded`` -- the single consumer of y does that for this
        conv's own ``act``, so the backward takes dy as the pre-activation gradient.  Set only
        by modules whose intermediate activations have exactly one reader (discriminators)."""
        require_hip(x, weight)
        k, _, kh, kw = weight.shape
        padded = hasattr(x, "_rt_cpad") and is_padded_input(x, _conv_desc(x, k, kh, kw, stride, padding, dilation))
        if not padded:
            x = nhwc(x)
        d = _conv_desc(x, k, kh, kw, stride, padding, dilation)
        y = empty_nhwc(d.n, k, d.ho, d.wo, x.dtype, x.device)
        ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
        flag = INPUT_PADDED if padded else 0
        with _Timed(d, "fwd"):
            lib.rtsds_conv2d_fwd(ctypes.byref(d), _P(x), _P(wq), _P(bias), _P(y), act | flag, _P(stats), _P(ws),
                                        ws.numel(), stream())
        ctx.xflag = flag
        ctx.in_act, ctx.out_folded = fold
        ctx.bn_link = bn_link if join is None and not fold[0] else None
        if ctx.in_act and join is not None:
            raise RuntimeError("rtsds_amd: a conv whose input gradient is masked cannot join other readers")
        ctx.d, ctx.act, ctx.has_bias = d, act, bias is not None
        ctx.params = (weight, bias)
        ctx.join = join
        ctx.save_for_backward(x, wq, y if act else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wq, y = ctx.saved_tensors
        d = ctx.d
        dy = nhwc(dy)
        if dy.dtype != x.dtype:
            dy = cast(dy, x.dtype)
        if ctx.act and not ctx.out_folded:
            g = torch.empty_like(dy)
            lib.rtsds_act_bwd(_P(dy), _P(y), _P(g), dy.numel(), ctx.act, 1.0, dcode(dy), stream())
        else:
            g = dy  # (out_folded: the consumer's dgrad already applied act')
        dx = dw = db = None
        # weight gradient into the optimizer's arena: on the side stream, overlapping the
        # data-gradient chain (runtime.side_fork); forked before the dgrad launch
        wg_side = None
        if ctx.needs_input_grad[1] and side_enabled(d.n * d.ho * d.wo) and CONV_PROFILE is None:
            weight, bias = ctx.params
            sinks = _sinks(weight, bias if ctx.needs_input_grad[2] else None)
            if sinks is not None:
                ws = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), x.device)
                side = side_fork(x, g, ws)
                lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(x), _P(g), _P(sinks[0]), _P(sinks[1]), 1 | ctx.xflag,
                                       _P(ws), ws.numel(), side.cuda_stream)
                wg_side = True
        if ctx.needs_input_grad[0]:
            join = ctx.join
            acc = join is not None and join.buf is not None  # accumulate onto the earlier contribution
            dx = join.buf if acc else empty_nhwc(d.n, d.c, d.h, d.w, x.dtype, x.device)
            ws = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
            link = ctx.bn_link
            wd, wpk = _dgrad_weight(ctx.params[0], wq, d)
            tiles = 0
            if link is not None and link.src is not None and not acc and g.dtype == torch.bfloat16:
                tiles = lib.rtsds_conv2d_dgrad_bnstats_tiles(ctypes.byref(d))
            with _Timed(d, "dgrad"):
                if tiles:
                    bx, bsm, bsi, bg, bb, bact = link.src
                    part = torch.empty(d.c * tiles * 2, dtype=torch.float32, device=x.device)
                    lib.rtsds_conv2d_dgrad_bnstats(ctypes.byref(d), _P(g), _P(wd), _P(dx), _P(bx), _P(bg), _P(bb),
                                                   _P(bsm), _P(bsi), bact | wpk, _P(part), _P(ws), ws.numel(), stream())
                    link.part, link.nrb = part, tiles
                elif ctx.in_act:
                    lib.rtsds_conv2d_dgrad_act(ctypes.byref(d), _P(g), _P(wd), _P(dx), _P(x), ctx.in_act | wpk,
                                               _P(ws), ws.numel(), stream())
                else:
                    lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(g), _P(wd), _P(dx), (1 if acc else 0) | wpk, _P(ws),
                                           ws.numel(), stream())
            if join is not None:
                dx = join.put(dx)
        if (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]) and not wg_side:
            weight, bias = ctx.params
            sinks = _sinks(weight, bias if ctx.needs_input_grad[2] else None) if ctx.needs_input_grad[1] else None
            ws = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), x.device)
            if sinks is not None:
                _wgrad_into_arena(d, x, g, sinks, ctx.xflag, ws)
                dw = None
                db = None
            else:
                dw = torch.empty((d.k, d.c, d.kh, d.kw), dtype=torch.float32, device=x.device,
                                 memory_format=CL)
                db = torch.empty(d.k, dtype=torch.float32, device=x.device) if ctx.has_bias else None
                with _Timed(d, "wgrad"):
                    lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(x), _P(g), _P(dw), _P(db), ctx.xflag, _P(ws),
                                                  ws.numel(), stream())
                if not ctx.needs_input_grad[1]:
                    dw = None
        return dx, dw, db, None, None, None, None, None, None, None, None, None


def conv2d(x, weight, bias, wq, stride=(1, 1), padding=(0, 0), dilation=(1, 1), act=0, bn_stats=False,
           join=None, in_act=0, fold_out=False, bn_link=None):
    """bn_stats=True: the conv epilogue also emits the following BatchNorm's per-tile batch
    statistics, attached to the output as ``_rt_bn_stats`` and consumed by batch_norm().
    ``join``: GradJoin shared with the other readers of ``x``."""
    stats = nrb = None
    if bn_stats and act == 0:
        n, _, h, w = x.shape
        k, _, kh, kw = weight.shape
        d = _conv_desc(x, k, kh, kw, stride, padding, dilation)
        nrb = lib.rtsds_conv2d_fwd_stats_tiles(ctypes.byref(d))
        stats = torch.empty(nrb * k * 4, dtype=torch.float32, device=x.device)  # [k][nrb][4]
    y = ConvFn.apply(x, weight, bias, wq, tuple(stride), tuple(padding), tuple(dilation), act, stats, join,
                     (in_act, bool(fold_out and act in (1, 2))), bn_link)
    if stats is not None:
        y._rt_bn_stats = (stats, nrb)
    return y


def _bn_fold(gamma, beta, running_mean, running_var, bias, eps, k):
    """Eval-mode BatchNorm folded with the conv bias into [scale | shift] (rtsds_bn_fold), cached
    on the running-mean tensor: recomputed -- in place, so captured graphs keep reading the
    same buffer -- only when a parameter / statistic changed (tensor versions for torch-side
    writes, runtime.params_epoch for the rtsds optimizer and train-mode BatchNorm, which write
    through raw pointers).  A GraphedForward capture registers the refresh, run before every
    replay."""
    ts = (gamma, beta, running_mean, running_var, bias)

    def key():
        return (params_epoch(), float(eps)) + tuple((t.data_ptr(), t._version) if t is not None else None for t in ts)

    ent = getattr(running_mean, "_rt_fold", None)
    if ent is None or ent[1].numel() != 2 * k or ent[1].device != running_mean.device:
        ent = [None, torch.empty(2 * k, dtype=torch.float32, device=running_mean.device)]
        running_mean._rt_fold = ent
    ss = ent[1]

    def refresh():
        kk = key()
        if ent[0] != kk:
            lib.rtsds_bn_fold(_P(gamma), _P(beta), _P(running_mean), _P(running_var), _P(bias), float(eps), k,
                              _P(ss), ss.data_ptr() + 4 * k, stream())
            ent[0] = kk

    refresh()
    register_fold(refresh)
    return ss


def conv_bn_eval(x, weight, bias, wq, stride, padding, dilation, gamma, beta, running_mean, running_var,
                 eps, act=0, residual=None, out=None):
    """Inference (no autograd) conv -> BatchNorm(running statistics) [-> + residual] [-> act]
    as ONE implicit-GEMM launch: the BN is folded into a per-channel scale / shift of the conv
    epilogue (rtsds_bn_fold + rtsds_conv2d_fwd_bn).  Same function as the unfused
    conv2d -> batch_norm(training=False) chain, with the BN applied to the fp32 accumulators.
    ``out = (buf, off)``: write y straight into channels [off, off + k) of the wider NHWC
    tensor ``buf`` (rtsds_conv2d_fwd_bn_ld) and return that slice as a view; where the kernel
    route does not support it, a plain y is returned (the caller copies)."""
    require_hip(x, weight)
    k, _, kh, kw = weight.shape
    flag = INPUT_PADDED if hasattr(x, "_rt_cpad") and \
        is_padded_input(x, _conv_desc(x, k, kh, kw, stride, padding, dilation)) else 0
    if not flag:
        x = nhwc(x)
    d = _conv_desc(x, k, kh, kw, stride, padding, dilation)
    ss = _bn_fold(gamma, beta, running_mean, running_var, bias, eps, k)
    if residual is not None:
        residual = nhwc(residual)
        if residual.dtype != x.dtype or tuple(residual.shape) != (d.n, k, d.ho, d.wo):
            raise RuntimeError("rtsds_amd.conv_bn_eval: residual must match the conv output")
    ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
    if out is not None and residual is None:
        buf, off = out
        if tuple(buf.shape[2:]) == (d.ho, d.wo) and buf.shape[0] == d.n and buf.dtype == x.dtype and \
                0 <= off and off + k <= buf.shape[1] and buf.stride(1) == 1 and buf.stride(3) == buf.shape[1]:
            try:
                with _Timed(d, "fwd"):
                    lib.rtsds_conv2d_fwd_bn_ld(ctypes.byref(d), _P(x), _P(wq), _P(ss), ss.data_ptr() + 4 * k,
                                               buf.data_ptr() + off * buf.element_size(), buf.shape[1], act | flag,
                                               _P(ws), ws.numel(), stream())
                return buf[:, off:off + k]
            except RuntimeError as e:
                if "unsupported" not in str(e):
                    raise
    y = empty_nhwc(d.n, k, d.ho, d.wo, x.dtype, x.device)
    with _Timed(d, "fwd"):
        lib.rtsds_conv2d_fwd_bn(ctypes.byref(d), _P(x), _P(wq), _P(ss), ss.data_ptr() + 4 * k, _P(residual), _P(y),
                                act | flag, _P(ws), ws.numel(), stream())
    return y


def conv_bn_maxpool_eval(x, weight, bias, wq, stride, padding, dilation, gamma, beta, running_mean, running_var, eps,
                         act, pool_k, pool_s, pool_p, ceil_mode):
    """Inference stem: pool(act(bn(conv(x)))) with the BN folded and the 3x3 stride-2 pool in
    the conv's epilogue (rtsds_conv2d_fwd_bn_maxpool; the full-resolution activation is never
    written).  None where that route does not apply (the caller runs the separate ops)."""
    require_hip(x, weight)
    if pool_k != 3 or pool_s != 2 or x.dtype != torch.bfloat16:
        return None
    k, _, kh, kw = weight.shape
    flag = INPUT_PADDED if hasattr(x, "_rt_cpad") and \
        is_padded_input(x, _conv_desc(x, k, kh, kw, stride, padding, dilation)) else 0
    if not flag:
        x = nhwc(x)
    d = _conv_desc(x, k, kh, kw, stride, padding, dilation)
    hp, wp = pool_out(d.ho, 3, 2, pool_p, ceil_mode), pool_out(d.wo, 3, 2, pool_p, ceil_mode)
    ss = _bn_fold(gamma, beta, running_mean, running_var, bias, eps, k)
    y = empty_nhwc(d.n, k, hp, wp, x.dtype, x.device)
    ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
    try:
        with _Timed(d, "fwd"):
            lib.rtsds_conv2d_fwd_bn_maxpool(ctypes.byref(d), _P(x), _P(wq), _P(ss), ss.data_ptr() + 4 * k, _P(y),
                                            act | flag, hp, wp, pool_p, _P(ws), ws.numel(), stream())
    except RuntimeError as e:
        if "unsupported" in str(e):  # not the stem geometry: the separate ops
            return None
        raise
    return y


class ConvSumFn(torch.autograd.Function):
    """sum_i conv_i(x) + bias_i over convs sharing x and output shape (ASPP,
    deeplabv2.py:62-66): one output buffer accumulated in the GEMM epilogue; the backward
    accumulates all dgrads into one dx."""

    @staticmethod
    def forward(ctx, x, geoms, *wb):
        require_hip(x)
        x = nhwc(x)
        m = len(geoms)
        weights, biases, wqs = wb[:m], wb[m:2 * m], wb[2 * m:]
        descs = []
        y = None
        for i, (stride, padding, dilation) in enumerate(geoms):
            k, _, kh, kw = weights[i].shape
            d = _conv_desc(x, k, kh, kw, stride, padding, dilation)
            if y is None:
                y = empty_nhwc(d.n, k, d.ho, d.wo, x.dtype, x.device)
            ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
            with _Timed(d, "fwd"):
                lib.rtsds_conv2d_fwd(ctypes.byref(d), _P(x), _P(wqs[i]), _P(biases[i]), _P(y),
                                     0x100 if i else 0, None, _P(ws), ws.numel(), stream())
            descs.append(d)
        ctx.descs = descs
        ctx.params = tuple(weights) + tuple(biases)
        ctx.has_bias = [b is not None for b in biases]
        ctx.save_for_backward(x, *wqs)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, *wqs = ctx.saved_tensors
        dy = nhwc(dy)
        m = len(wqs)
        dx = None
        dws, dbs = [None] * m, [None] * m
        for i, d in enumerate(ctx.descs):
            if ctx.needs_input_grad[0]:
                if dx is None:
                    dx = empty_nhwc(d.n, d.c, d.h, d.w, x.dtype, x.device)
                ws = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
                wd, wpk = _dgrad_weight(ctx.params[i], wqs[i], d)
                with _Timed(d, "dgrad"):
                    lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wd), _P(dx), (1 if i else 0) | wpk,
                                           _P(ws), ws.numel(), stream())
            if ctx.needs_input_grad[2 + i] or ctx.needs_input_grad[2 + m + i]:
                w_i, b_i = ctx.params[i], ctx.params[m + i]
                sinks = (_sinks(w_i, b_i if ctx.needs_input_grad[2 + m + i] else None)
                         if ctx.needs_input_grad[2 + i] else None)
                ws = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), x.device)
                if sinks is not None:
                    with _Timed(d, "wgrad"):
                        lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(x), _P(dy), _P(sinks[0]), _P(sinks[1]),
                                               1, _P(ws), ws.numel(), stream())
                    continue
                dw = torch.empty((d.k, d.c, d.kh, d.kw), dtype=torch.float32, device=x.device,
                                 memory_format=CL)
                db = torch.empty(d.k, dtype=torch.float32, device=x.device) if ctx.has_bias[i] else None
                with _Timed(d, "wgrad"):
                    lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(x), _P(dy), _P(dw), _P(db), 0, _P(ws),
                                           ws.numel(), stream())
                dws[i] = dw if ctx.needs_input_grad[2 + i] else None
                dbs[i] = db
        return (dx, None, *dws, *dbs, *([None] * m))


# ----------------------------------------------------------------------------- batch norm
BN_BWD_LINK = True  # False: every BatchNorm backward computes its own statistics (A/B tests)


class BnBwdLink:
    """Hands a train-mode BatchNorm's backward statistics from the data gradient of the conv
    that reads its (activated) output to the BatchNorm's backward, which then skips its own
    statistics pass (rtsds_conv2d_dgrad_bnstats -> rtsds_bn_bwd_part).  Created by a module
    whose BatchNorm output has exactly that one reader (ResNet BasicBlock bn1 -> conv2,
    Bottleneck bn1 -> conv2 -> bn2 -> conv3); ignored wherever a route does not apply."""

    __slots__ = ("src", "part", "nrb")

    def __init__(self):
        self.src = None   # (bn input x, save_mean, save_invstd, gamma, beta, act), set by the BN forward
        self.part = None  # set by the conv backward, consumed by the BN backward
        self.nrb = 0


class BatchNormFn(torch.autograd.Function):
    """BatchNorm2d (+ residual add) (+ ReLU/LeakyReLU) fused, train or eval statistics."""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, running_mean, running_var, training, momentum, eps, act,
                stats, stats_nrb, nbt, res_join=None, link=None, out=None):
        require_hip(x)
        x = nhwc(x)
        if res is not None:
            res = nhwc(res)
        n, c, h, w = x.shape
        rows = n * h * w
        keep_y = res is not None or act == ACT_SIGMOID
        ld = c
        if out is not None and not keep_y and x.dtype == torch.bfloat16 and c % 8 == 0 and out[0].shape[1] % 8 == 0:
            # y written straight into channels [off, off + c) of out's NHWC buffer (a view)
            buf, off = out
            ld = buf.shape[1]
            y = buf[:, off:off + c]
        else:
            y = torch.empty_like(x, memory_format=CL)
        sm = torch.empty(c, dtype=torch.float32, device=x.device)
        si = torch.empty(c, dtype=torch.float32, device=x.device)
        ws = workspace(lib.rtsds_bn_workspace(rows, c), x.device)
        lib.rtsds_bn_fwd_ld(_P(x), _P(res), _P(y), ld, rows, c, _P(gamma), _P(beta), _P(running_mean),
                            _P(running_var), _P(nbt), _P(sm), _P(si), float(momentum), float(eps), int(training),
                            act, _P(stats) if training else None, int(stats_nrb or 0), dcode(x), _P(ws),
                            ws.numel(), stream())
        ctx.meta = (rows, c, int(training), act, res is not None)
        ctx.gamma, ctx.beta = gamma, beta
        ctx.res_join = res_join
        # Without a residual the ReLU/LeakyReLU mask is recomputed from x in the backward
        # (bit-identical pre-activation), so y is neither kept nor re-read.
        ctx.save_for_backward(x, y if keep_y else None, gamma, beta, sm, si)
        ctx.link = None
        if link is not None and BN_BWD_LINK and training and res is None and act in (0, 1, 2) \
                and x.dtype == torch.bfloat16 and c % 8 == 0:
            link.src, link.part = (x, sm, si, gamma, beta, act), None
            ctx.link = link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, beta, sm, si = ctx.saved_tensors
        rows, c, training, act, has_res = ctx.meta
        ldy = _channel_slice_pitch(dy) if ctx.link is None else 0
        if not ldy:
            dy = nhwc(dy)
            ldy = c
        need_dx, need_g, need_b, need_r = (ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                                           ctx.needs_input_grad[2], ctx.needs_input_grad[3])
        dx = torch.empty_like(x, memory_format=CL) if need_dx else None
        dres = torch.empty_like(x, memory_format=CL) if (has_res and need_r) else None
        sinks = _sinks(ctx.gamma if need_g else None, ctx.beta if need_b else None) if (need_g or need_b) else None
        if sinks is not None:
            dg, db, acc = sinks[0], sinks[1], 1
        else:
            dg = torch.empty(c, dtype=torch.float32, device=x.device) if need_g else None
            db = torch.empty(c, dtype=torch.float32, device=x.device) if need_b else None
            acc = 0
        ws = workspace(lib.rtsds_bn_workspace(rows, c), x.device)
        link = ctx.link
        if link is not None and link.part is not None and dy.dtype == x.dtype:
            # statistics from the reading conv's data-gradient epilogue
            lib.rtsds_bn_bwd_part(_P(dy), _P(x), _P(dx), _P(dg), _P(db), rows, c, _P(gamma), _P(beta), _P(sm),
                                  _P(si), training, act, acc, _P(link.part), link.nrb, dcode(x), _P(ws), ws.numel(),
                                  stream())
        else:
            lib.rtsds_bn_bwd_ld(_P(dy), ldy, _P(x), _P(y), _P(dx), _P(dres), _P(dg), _P(db), rows, c,
                                _P(gamma), _P(beta), _P(sm), _P(si), training, act, acc, dcode(x), _P(ws), ws.numel(),
                                stream())
        if link is not None:
            link.src = link.part = None
        if acc:
            dg = db = None
        if dres is not None:
            dres = _join_add(ctx.res_join, dres)
        return dx, dg, db, dres, None, None, None, None, None, None, None, None, None, None, None, None


def _channel_slice_pitch(t):
    """Row pitch of a bf16 [N, C, H, W] view that is a channel slice of a wider NHWC buffer
    (C % 8 == 0, pitch % 8 == 0, pitch > C), else 0."""
    if t.dim() != 4 or t.dtype != torch.bfloat16:
        return 0
    n, c, h, w = t.shape
    ld = t.stride(3)
    if c % 8 or ld % 8 or ld <= c or t.stride(1) != 1 or t.stride(2) != w * ld or (n > 1 and t.stride(0) != h * w * ld) \
            or t.data_ptr() % 16:
        return 0
    return ld


def batch_norm(x, gamma, beta, running_mean, running_var, training, momentum, eps, act=0,
               residual=None, num_batches_tracked=None, res_join=None, link=None, out=None):
    """``num_batches_tracked`` (int64, optional) is incremented by the finalize kernel.
    ``res_join``: GradJoin shared with the other readers of ``residual``.  ``out``: (NHWC
    buffer, channel offset) to write y into (a view of it is returned; bf16 without residual)."""
    st = getattr(x, "_rt_bn_stats", None) if training else None
    stats, nrb = st if st is not None else (None, None)
    if training and running_mean is not None:
        bump_params_epoch()  # running statistics change (raw-pointer write)
    return BatchNormFn.apply(x, gamma, beta, residual, running_mean, running_var, training,
                             momentum, eps, act, stats, nrb, num_batches_tracked, res_join, link, out)


# ----------------------------------------------------------------------------- layout / dtype
def pack_input(x, dtype):
    """NCHW fp32 batch (reference loaders, reference-layout activations) -> NHWC compute dtype.
    Differentiable when ``x`` requires grad (discriminator / UpSampler inputs): the gradient
    goes back as the NHWC tensor cast to x's dtype (same logical NCHW shape)."""
    require_hip(x)
    if x.dtype == dtype and x.dim() == 4 and (x.is_contiguous(memory_format=CL) and x.shape[1] > 1 or is_padded_input(x)):
        return x
    if x.requires_grad and torch.is_grad_enabled():
        return PackInputFn.apply(x, dtype)
    return _pack(x, dtype)


class PackInputFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.xdtype = x.dtype
        return _pack(x, dtype)

    @staticmethod
    def backward(ctx, dy):
        return cast(nhwc(dy), ctx.xdtype), None


def pack_input_into(x, y):
    """pack_input(x, y.dtype) written into the existing packed tensor ``y`` (same shape): a
    captured graph's input buffer refilled with one pass over x."""
    require_hip(x)
    xf = (x if x.dtype == torch.float32 else cast(x, torch.float32)).contiguous()
    n, c, h, w = xf.shape
    if tuple(y.shape) != (n, c, h, w):
        raise RuntimeError("rtsds_amd.pack_input_into: shape mismatch")
    if is_padded_input(y):
        lib.rtsds_nchw_to_nhwc_pad(_P(xf), _P(y), n, c, h, w, y._rt_cpad, 0 if y.dtype == torch.float32 else 1, stream())
    elif y.is_contiguous(memory_format=CL):
        lib.rtsds_nchw_to_nhwc(_P(xf), _P(y), n, c, h, w, 0 if y.dtype == torch.float32 else 1, stream())
    else:
        raise RuntimeError("rtsds_amd.pack_input_into: y is not a packed input")
    return y


def _pack(x, dtype):
    xf = x if x.dtype == torch.float32 else cast(x, torch.float32)
    xf = xf.contiguous()
    n, c, h, w = xf.shape
    if c == 3 and dtype == torch.bfloat16:
        # the image in the 4-channel pitch of its convs' superpixel gathers (stem / spatial
        # path, RTSDS_INPUT_PADDED): they skip their own pad pass; other readers see a
        # [N, 3, H, W] tensor (non-conv readers make an NHWC copy via nhwc())
        buf = torch.empty((n, h, w, 4), dtype=dtype, device=x.device)
        lib.rtsds_nchw_to_nhwc_pad(_P(xf), _P(buf), n, c, h, w, 4, 1, stream())
        y = buf.permute(0, 3, 1, 2)[:, :3]
        y._rt_cpad = 4
        return y
    y = empty_nhwc(n, c, h, w, dtype, x.device)
    lib.rtsds_nchw_to_nhwc(_P(xf), _P(y), n, c, h, w, 0 if dtype == torch.float32 else 1, stream())
    return y


def cast(t, dtype):
    """dtype conversion on device, preserving the memory layout."""
    if t.dtype == dtype:
        return t
    out = torch.empty_like(t, dtype=dtype)
    if not (t.is_contiguous() or t.is_contiguous(memory_format=CL)):
        raise RuntimeError("rtsds_amd.cast: dense tensor required")
    if out.stride() != t.stride():
        raise RuntimeError("rtsds_amd.cast: layout mismatch")
    lib.rtsds_cast(_P(t), dcode(t), _P(out), dcode(out), t.numel(), stream())
    return out


class CatFn(torch.autograd.Function):
    """torch.cat(dim=1) of NHWC tensors (build_bisenet.py:72,153).  ``joins[i]``: GradJoin of
    input i when it has other readers (the split slice is accumulated into their gradient)."""

    @staticmethod
    def forward(ctx, joins, *xs):
        xs = [nhwc(x) for x in xs]
        n, _, h, w = xs[0].shape
        ct = sum(x.shape[1] for x in xs)
        y = empty_nhwc(n, ct, h, w, xs[0].dtype, xs[0].device)
        off = 0
        for x in xs:
            c = x.shape[1]
            lib.rtsds_copy_channels(_P(x), c, 0, _P(y), ct, off, n * h * w, c, 0, dcode(x), stream())
            off += c
        ctx.split = [x.shape[1] for x in xs]
        ctx.joins = joins
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = nhwc(dy)
        n, ct, h, w = dy.shape
        outs, off = [None], 0
        for i, c in enumerate(ctx.split):
            if ctx.needs_input_grad[1 + i]:
                join = ctx.joins[i] if ctx.joins else None
                acc = join is not None and join.buf is not None
                g = join.buf if acc else empty_nhwc(n, c, h, w, dy.dtype, dy.device)
                lib.rtsds_copy_channels(_P(dy), ct, off, _P(g), c, 0, n * h * w, c, 1 if acc else 0, dcode(dy),
                                        stream())
                outs.append(join.put(g) if join is not None else g)
            else:
                outs.append(None)
            off += c
        return tuple(outs)


class CatResizeFn(torch.autograd.Function):
    """cat([x0] + [interpolate_bilinear(x, size) for x in xs], dim=1) (build_bisenet.py:151-153
    and the FFM's cat, :72) with each resize written straight into its channel slice of the
    output (rtsds_bilinear_fwd's output pitch / offset) and, backward, each resize's gradient
    read straight from its slice of dy (rtsds_bilinear_bwd's input pitch / offset): neither the
    resized maps nor their gradients exist on their own; x0 (already at ``size``) is the one
    copy each way.  ``joins[k]``: GradJoin of xs[k]'s readers (BiSeNet's cx1 / cx2 also feed the
    supervision convs, whose data gradients then accumulate into the resize adjoint's buffer)."""

    @staticmethod
    def forward(ctx, size, joins, into, x0, *xs):
        xs = [nhwc(x) for x in xs]
        ct = x0.shape[1] + sum(x.shape[1] for x in xs)
        # x0 already written as channels [0, c0) of ``into`` (its producer's pitched store): no copy
        ctx.x0_in_place = into is not None and tuple(into.shape[1:]) == (ct,) + tuple(x0.shape[2:]) and \
            x0.data_ptr() == into.data_ptr() and _channel_slice_pitch(x0) == ct
        if not ctx.x0_in_place:
            x0 = nhwc(x0)
        n, c0, h, w = x0.shape
        if (h, w) != (int(size[0]), int(size[1])):
            raise RuntimeError("rtsds_amd.concat_resized: x0 must have the target size")
        y = into if ctx.x0_in_place else empty_nhwc(n, ct, h, w, x0.dtype, x0.device)
        if not ctx.x0_in_place:
            lib.rtsds_copy_channels(_P(x0), c0, 0, _P(y), ct, 0, n * h * w, c0, 0, dcode(x0), stream())
        off, geos = c0, []
        for x in xs:
            _, c, hi, wi = x.shape
            ho, wo, sh, sw = upsample_geometry(x, size=size)
            lib.rtsds_bilinear_fwd(_P(x), _P(y), n, hi, wi, c, ho, wo, sh, sw, ct, off, dcode(x), stream())
            geos.append((off, c, hi, wi, ho, wo, sh, sw))
            off += c
        ctx.meta = (n, c0, h, w, ct, geos)
        ctx.joins = joins
        return y

    @staticmethod
    def backward(ctx, dy):
        n, c0, h, w, ct, geos = ctx.meta
        dy = nhwc(dy)
        grads = [None, None, None, None]
        if ctx.needs_input_grad[3]:
            if ctx.x0_in_place:  # x0's producer reads its gradient from the slice in place
                grads[3] = dy[:, :c0]
            else:
                g0 = empty_nhwc(n, c0, h, w, dy.dtype, dy.device)
                lib.rtsds_copy_channels(_P(dy), ct, 0, _P(g0), c0, 0, n * h * w, c0, 0, dcode(dy), stream())
                grads[3] = g0
        for k, (off, c, hi, wi, ho, wo, sh, sw) in enumerate(geos):
            if not ctx.needs_input_grad[4 + k]:
                grads.append(None)
                continue
            dx = empty_nhwc(n, c, hi, wi, dy.dtype, dy.device)
            ws = workspace(lib.rtsds_bilinear_bwd_workspace(n, hi, wi, c, ho, wo), dy.device)
            lib.rtsds_bilinear_bwd(_P(dy), _P(dx), n, hi, wi, c, ho, wo, sh, sw, ct, off, dcode(dy), _P(ws),
                                   ws.numel(), stream())
            # first contribution: the other reader accumulates into dx (otherwise one add)
            grads.append(_join_add(ctx.joins[k], dx) if ctx.joins else dx)
        return tuple(grads)


def concat_resized(x0, xs, size, joins=None, into=None):
    """cat([x0] + [interpolate_bilinear(x, size) for x in xs], dim=1) without materialising the
    resized maps (CatResizeFn).  ``joins``: per-xs GradJoin (or None) for inputs with other readers.
    ``into``: the preallocated NHWC output; when x0 already is its leading channel slice (e.g.
    written there by nn.conv_bn(out=...)), x0 is neither copied in nor its gradient copied out."""
    return CatResizeFn.apply((int(size[0]), int(size[1])), tuple(joins) if joins else None, into, x0, *xs)


def concat_resized_scaled_eval(x0, parts, size, into=None):
    """Inference only: concat_resized(x0, [channel_scale(...channel_scale(x, s1)..., sk) for
    (x, (s1, ...)) in parts], size) with the (at most two) channel scales applied to the resize's
    taps (rtsds_bilinear_fwd_scaled; bit-identical to the separate ops).  None when a part's
    geometry is outside the fused kernel (the caller then runs the separate ops).  ``into``: the
    preallocated output; x0 is not copied when it already is its leading channel slice (the
    spatial path's conv wrote it there, conv_bn_eval(out=...))."""
    in_place = into is not None and x0.data_ptr() == into.data_ptr() and x0.stride() == into.stride()
    if not in_place:
        x0 = nhwc(x0)
    n, c0, h, w = x0.shape
    ps = []
    for x, scales in parts:
        x = nhwc(x)
        if len(scales) > 2 or x.shape[-2] > h or x.shape[-1] > w:
            return None
        ss = [(s if s.dtype == x.dtype else cast(s, x.dtype)).contiguous() for s in scales]
        ps.append((x, ss + [None] * (2 - len(ss))))
    ct = c0 + sum(x.shape[1] for x, _ in ps)
    if into is not None and tuple(into.shape) == (n, ct, h, w) and into.dtype == x0.dtype:
        y = into
    else:
        y, in_place = empty_nhwc(n, ct, h, w, x0.dtype, x0.device), False
    off = c0
    for x, (s1, s2) in ps:
        _, c, hi, wi = x.shape
        ho, wo, sh, sw = upsample_geometry(x, size=size)
        try:
            lib.rtsds_bilinear_fwd_scaled(_P(x), _P(s1), _P(s2), _P(y), n, hi, wi, c, ho, wo, sh, sw, ct, off, dcode(x), stream())
        except RuntimeError as e:
            if "unsupported" in str(e):
                return None
            raise
        off += c
    if not in_place:
        lib.rtsds_copy_channels(_P(x0), c0, 0, _P(y), ct, 0, n * h * w, c0, 0, dcode(x0), stream())
    return y


def ffm_head_eval(feature, w1, b1, w2, b2, w3, b3):
    """Inference only: conv3(f * a + f) + b3 with a = sigmoid(conv2(relu(conv1(GAP(f)) + b1)) + b2)
    -- FeatureFusionModule's attention tail and BiSeNet's final 1x1 conv (build_bisenet.py:75-80,
    167) in one launch (rtsds_ffm_head_eval).  w*: [c, c, 1, 1] weights in the feature's dtype."""
    f = nhwc(feature)
    n, c, h, w = f.shape
    out = empty_nhwc(n, c, h, w, f.dtype, f.device)
    ws = [t.reshape(c, c).contiguous() for t in (w1, w2, w3)]
    bs = [None if b is None else b.float().contiguous() for b in (b1, b2, b3)]
    wk = workspace(lib.rtsds_ffm_head_eval_workspace(n, h * w, c), f.device)
    lib.rtsds_ffm_head_eval(_P(f), _P(ws[0]), _P(bs[0]), _P(ws[1]), _P(bs[1]), _P(ws[2]), _P(bs[2]), _P(out), n, h * w, c,
                            dcode(f), _P(wk), wk.numel(), stream())
    return out


def cat(xs, joins=None):
    """``joins``: per-input GradJoin (or None) for inputs that have other readers."""
    return CatFn.apply(joins, *xs)


# ----------------------------------------------------------------------------- pointwise
class ActFn(torch.autograd.Function):
    """ReLU (1) / LeakyReLU(0.2) (2) / sigmoid (3)."""

    @staticmethod
    def forward(ctx, x, act):
        require_hip(x)
        x = x.contiguous(memory_format=CL) if x.dim() == 4 else x.contiguous()
        y = torch.empty_like(x)
        lib.rtsds_act_fwd(_P(x), _P(y), x.numel(), act, dcode(x), stream())
        ctx.act = act
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous(memory_format=CL) if dy.dim() == 4 else dy.contiguous()
        dx = torch.empty_like(y)
        lib.rtsds_act_bwd(_P(dy), _P(y), _P(dx), y.numel(), ctx.act, 1.0, dcode(y), stream())
        return dx, None


def relu(x):
    return ActFn.apply(x, 1)


def leaky_relu(x):
    return ActFn.apply(x, 2)


def sigmoid(x):
    return ActFn.apply(x, 3)


class GradReverseFn(torch.autograd.Function):
    """GradientReversalFunction (model.py:9-17): identity forward, -alpha * grad backward."""

    @staticmethod
    def forward(ctx, x, alpha):
        ctx.alpha = float(alpha)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous(memory_format=CL) if dy.dim() == 4 else dy.contiguous()
        dx = torch.empty_like(dy)
        lib.rtsds_act_bwd(_P(dy), None, _P(dx), dy.numel(), 0, -ctx.alpha, dcode(dy), stream())
        return dx, None


# ----------------------------------------------------------------------------- pooling
def pool_out(size, k, s, p, ceil_mode):
    """ATen pooling_output_shape (dilation 1)."""
    num = size + 2 * p - (k - 1) - 1 + ((s - 1) if ceil_mode else 0)
    o = num // s + 1
    if ceil_mode and (o - 1) * s >= size + p:
        o -= 1
    return o


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil_mode):
        require_hip(x)
        x = nhwc(x)
        n, c, h, w = x.shape
        ho, wo = pool_out(h, k, s, p, ceil_mode), pool_out(w, k, s, p, ceil_mode)
        y = empty_nhwc(n, c, ho, wo, x.dtype, x.device)
        # inference (no gradient): the argmax bytes are not written where the kernel allows it
        need = ctx.needs_input_grad[0] or not (k == 3 and c % (8 if x.dtype == torch.bfloat16 else 4) == 0)
        idx = torch.empty((n, ho, wo, c), dtype=torch.uint8, device=x.device) if need else None
        lib.rtsds_maxpool_fwd(_P(x), _P(y), _P(idx), n, h, w, c, ho, wo, k, s, p, dcode(x), stream())
        ctx.geo = (n, h, w, c, ho, wo, k, s, p)
        ctx.dtype = x.dtype
        ctx.save_for_backward(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        n, h, w, c, ho, wo, k, s, p = ctx.geo
        dy = nhwc(dy)
        dx = empty_nhwc(n, c, h, w, dy.dtype, dy.device)
        lib.rtsds_maxpool_bwd(_P(dy), _P(idx), _P(dx), n, h, w, c, ho, wo, k, s, p, dcode(dy), stream())
        return dx, None, None, None, None


def max_pool2d(x, k, s, p, ceil_mode=False):
    return MaxPoolFn.apply(x, k, s, p, ceil_mode)


class BnReluMaxPoolFn(torch.autograd.Function):
    """BatchNorm2d + ReLU + MaxPool2d(3, 2, p) (the ResNet stem bn1 -> relu -> maxpool,
    build_contextpath.py:15-18 via torchvision resnet.py; deeplabv2.py:106-110): the forward
    is one pass that never writes the full-resolution activation (bn.hip)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, training, momentum, eps, stats, stats_nrb, nbt,
                p, ceil_mode):
        require_hip(x)
        x = nhwc(x)
        n, c, h, w = x.shape
        ho, wo = pool_out(h, 3, 2, p, ceil_mode), pool_out(w, 3, 2, p, ceil_mode)
        y = empty_nhwc(n, c, ho, wo, x.dtype, x.device)
        idx = torch.empty((n, ho, wo, c), dtype=torch.uint8, device=x.device)
        sm = torch.empty(c, dtype=torch.float32, device=x.device)
        si = torch.empty(c, dtype=torch.float32, device=x.device)
        ws = workspace(lib.rtsds_bn_workspace(n * h * w, c), x.device)
        lib.rtsds_bn_relu_maxpool_fwd(_P(x), _P(y), _P(idx), n, h, w, c, ho, wo, p, _P(gamma), _P(beta),
                                      _P(running_mean), _P(running_var), _P(nbt), _P(sm), _P(si), float(momentum),
                                      float(eps), int(training), _P(stats) if training else None,
                                      int(stats_nrb or 0), dcode(x), _P(ws), ws.numel(), stream())
        ctx.meta = (n, c, h, w, ho, wo, p, int(training))
        ctx.gamma, ctx.beta = gamma, beta
        ctx.save_for_backward(x, idx, gamma, beta, sm, si)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, idx, gamma, beta, sm, si = ctx.saved_tensors
        n, c, h, w, ho, wo, p, training = ctx.meta
        dy = nhwc(dy)
        if dy.dtype != x.dtype:
            dy = cast(dy, x.dtype)
        need_dx, need_g, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        dx = torch.empty_like(x, memory_format=CL) if need_dx else None
        sinks = _sinks(ctx.gamma if need_g else None, ctx.beta if need_b else None) if (need_g or need_b) else None
        if sinks is not None:
            dg, db, acc = sinks[0], sinks[1], 1
        else:
            dg = torch.empty(c, dtype=torch.float32, device=x.device) if need_g else None
            db = torch.empty(c, dtype=torch.float32, device=x.device) if need_b else None
            acc = 0
        # backward unfused: the pool gradient is materialised once (16-B scatter-free gather,
        # rtsds_maxpool_bwd) and the BatchNorm backward reads it directly -- measured faster
        # than gathering it inside both BatchNorm passes (rtsds_bn_relu_maxpool_bwd: 94 + 108
        # vs 66 + 45 + 60 us at the BiSeNet stem, the gather's 4-window compare is VALU-bound)
        g = empty_nhwc(n, c, h, w, dy.dtype, dy.device)
        lib.rtsds_maxpool_bwd(_P(dy), _P(idx), _P(g), n, h, w, c, ho, wo, 3, 2, p, dcode(dy), stream())
        ws = workspace(lib.rtsds_bn_workspace(n * h * w, c), x.device)
        lib.rtsds_bn_bwd(_P(g), _P(x), None, _P(dx), None, _P(dg), _P(db), n * h * w, c, _P(gamma), _P(beta),
                         _P(sm), _P(si), training, ACT_RELU, acc, dcode(x), _P(ws), ws.numel(), stream())
        if acc:
            dg = db = None
        return dx, dg, db, None, None, None, None, None, None, None, None, None, None


def bn_relu_maxpool_ok(x, k, s, p):
    """Shapes the fused stem kernels take: bf16 NHWC, channels % 8, MaxPool2d(3, 2, p <= 1)."""
    return x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0 and k == 3 and s == 2 and p in (0, 1)


def bn_relu_maxpool(x, gamma, beta, running_mean, running_var, training, momentum, eps, p, ceil_mode,
                    num_batches_tracked=None):
    st = getattr(x, "_rt_bn_stats", None) if training else None
    stats, nrb = st if st is not None else (None, None)
    if training and running_mean is not None:
        bump_params_epoch()  # running statistics change (raw-pointer write)
    return BnReluMaxPoolFn.apply(x, gamma, beta, running_mean, running_var, training, momentum, eps, stats, nrb,
                                 num_batches_tracked, p, ceil_mode)


class PooledMlpFn(torch.autograd.Function):
    """sigmoid(conv2(relu(conv1(p)))) on pooled [N, C, 1, 1] vectors -- the FFM attention
    (build_bisenet.py:67-70) -- forward as one launch (rtsds_pooled_mlp_fwd) bit-identical to the
    two pooled conv launches, backward as one launch (rtsds_pooled_mlp_bwd) bit-identical to the
    six of the per-conv chain."""

    @staticmethod
    def forward(ctx, p, w1, b1, wq1, w2, b2, wq2):
        p = nhwc(p)
        n, c0 = p.shape[0], p.shape[1]
        c1, c2 = w1.shape[0], w2.shape[0]
        h = empty_nhwc(n, c1, 1, 1, p.dtype, p.device)
        a = empty_nhwc(n, c2, 1, 1, p.dtype, p.device)
        lib.rtsds_pooled_mlp_fwd(_P(p), _P(wq1), _P(b1), _P(wq2), _P(b2), _P(h), _P(a), n, c0, c1, c2, dcode(p), stream())
        ctx.params = (w1, b1, w2, b2)
        ctx.dims = (n, c0, c1, c2)
        ctx.save_for_backward(p, h, a, wq1, wq2)
        return a

    @staticmethod
    def backward(ctx, da):
        p, h, a, wq1, wq2 = ctx.saved_tensors
        w1, b1, w2, b2 = ctx.params
        n, c0, c1, c2 = ctx.dims
        da = nhwc(da)
        if da.dtype != a.dtype:
            da = cast(da, a.dtype)
        sinks = _sinks(w1, b1, w2, b2)
        if sinks is not None:
            dw1, db1, dw2, db2 = sinks
            acc = 1
        else:
            dw1 = torch.empty(c1, c0, 1, 1, dtype=torch.float32, device=p.device)
            dw2 = torch.empty(c2, c1, 1, 1, dtype=torch.float32, device=p.device)
            db1 = torch.empty(c1, dtype=torch.float32, device=p.device) if b1 is not None else None
            db2 = torch.empty(c2, dtype=torch.float32, device=p.device) if b2 is not None else None
            acc = 0
        dp = empty_nhwc(n, c0, 1, 1, p.dtype, p.device)
        lib.rtsds_pooled_mlp_bwd(_P(da), _P(a), _P(h), _P(p), _P(wq1), _P(wq2), _P(dw1), _P(db1), _P(dw2), _P(db2),
                                 _P(dp), n, c0, c1, c2, acc, dcode(p), stream())
        if acc:
            dw1 = db1 = dw2 = db2 = None
        return dp, dw1, db1, None, dw2, db2, None


def pooled_mlp_ok(p, c1, c2):
    """Shapes rtsds_pooled_mlp_bwd reproduces bit for bit: N <= 8 pooled rows, <= 64 channels,
    channel counts off the vector kernels' multiples."""
    n, c0 = p.shape[0], p.shape[1]
    v = 8 if p.dtype == torch.bfloat16 else 4
    return p.dim() == 4 and p.shape[2] == p.shape[3] == 1 and n <= 8 and max(c0, c1, c2) <= 64 and \
        all(c % v for c in (c0, c1, c2)) and p.dtype in (torch.bfloat16, torch.float32)


def pooled_mlp(p, w1, b1, wq1, w2, b2, wq2):
    return PooledMlpFn.apply(p, w1, b1, wq1, w2, b2, wq2)


class GapFn(torch.autograd.Function):
    """Mean over H, W keeping dims -> [N, C, 1, 1].  ``join``: GradJoin shared with the other
    reader of x (the attention modules' channel scale): the backward adds its broadcast into
    that reader's gradient buffer instead of autograd summing two full-size gradients."""

    @staticmethod
    def forward(ctx, x, join=None):
        require_hip(x)
        x = nhwc(x)
        n, c, h, w = x.shape
        y = empty_nhwc(n, c, 1, 1, x.dtype, x.device)
        ws = workspace(lib.rtsds_gap_workspace(n, h * w, c), x.device)
        lib.rtsds_gap_fwd(_P(x), _P(y), n, h * w, c, dcode(x), _P(ws), ws.numel(), stream())
        ctx.shape = (n, c, h, w)
        ctx.join = join
        return y

    @staticmethod
    def backward(ctx, dy):
        n, c, h, w = ctx.shape
        dy = dy.contiguous()
        join = ctx.join
        acc = join is not None and join.buf is not None
        dx = join.buf if acc else empty_nhwc(n, c, h, w, dy.dtype, dy.device)
        lib.rtsds_gap_bwd(_P(dy), _P(dx), n, h * w, c, 1 if acc else 0, dcode(dy), stream())
        return (join.put(dx) if join is not None else dx), None


def global_avg_pool(x, join=None):
    """``join``: GradJoin shared with x's other reader (see GapFn)."""
    return GapFn.apply(x, join)


class ChScaleFn(torch.autograd.Function):
    """x * a[N,C,1,1] (mode 0) or x * a + x (mode 1).  ``join``: GradJoin shared with x's
    other reader (GapFn); ``join_a``: the same for a's other reader."""

    @staticmethod
    def forward(ctx, x, a, mode, join=None, join_a=None):
        require_hip(x, a)
        x = nhwc(x)
        a = a.contiguous()
        n, c, h, w = x.shape
        if a.dtype != x.dtype:
            a = cast(a, x.dtype)
        y = torch.empty_like(x, memory_format=CL)
        lib.rtsds_chscale_fwd(_P(x), _P(a), _P(y), n, h * w, c, mode, dcode(x), stream())
        ctx.mode = mode
        ctx.join, ctx.join_a = join, join_a
        ctx.save_for_backward(x, a)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, a = ctx.saved_tensors
        n, c, h, w = x.shape
        dy = nhwc(dy)
        dx = torch.empty_like(x, memory_format=CL) if ctx.needs_input_grad[0] else None
        da = torch.empty_like(a) if ctx.needs_input_grad[1] else None
        ws = workspace(lib.rtsds_gap_workspace(n, h * w, c) if da is not None else 0, x.device)
        lib.rtsds_chscale_bwd(_P(dy), _P(x), _P(a), _P(dx), _P(da), n, h * w, c, ctx.mode,
                              dcode(x), _P(ws), ws.numel(), stream())
        if dx is not None and ctx.join is not None:
            dx = _join_add(ctx.join, dx)
        if da is not None and ctx.join_a is not None:
            da = _join_add(ctx.join_a, da)
        return dx, da, None, None, None


def channel_scale(x, a, residual=False, join=None, join_a=None):
    """``join`` / ``join_a``: GradJoin shared with x's / a's other reader (see GapFn)."""
    return ChScaleFn.apply(x, a, 1 if residual else 0, join, join_a)


# ----------------------------------------------------------------------------- bilinear
def _src_scale(in_size, out_size, scale_factor):
    """ATen area_pixel_compute_scale (align_corners=False), fp32."""
    if scale_factor is not None and scale_factor > 0:
        return float(np.float32(1.0 / scale_factor))
    return float(np.float32(in_size) / np.float32(out_size))


class BilinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ho, wo, sh, sw):
        require_hip(x)
        x = nhwc(x)
        n, c, hi, wi = x.shape
        y = empty_nhwc(n, c, ho, wo, x.dtype, x.device)
        lib.rtsds_bilinear_fwd(_P(x), _P(y), n, hi, wi, c, ho, wo, sh, sw, c, 0, dcode(x), stream())
        ctx.geo = (n, hi, wi, c, ho, wo, sh, sw)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, hi, wi, c, ho, wo, sh, sw = ctx.geo
        dy = nhwc(dy)
        dx = empty_nhwc(n, c, hi, wi, dy.dtype, dy.device)
        ws = workspace(lib.rtsds_bilinear_bwd_workspace(n, hi, wi, c, ho, wo), dy.device)
        lib.rtsds_bilinear_bwd(_P(dy), _P(dx), n, hi, wi, c, ho, wo, sh, sw, c, 0, dcode(dy), _P(ws),
                               ws.numel(), stream())
        return dx, None, None, None, None


def interpolate_bilinear(x, size=None, scale_factor=None):
    """F.interpolate(x, size | scale_factor, mode='bilinear', align_corners=False)."""
    hi, wi = x.shape[-2:]
    if size is not None:
        ho, wo = int(size[0]), int(size[1])
        sh, sw = _src_scale(hi, ho, None), _src_scale(wi, wo, None)
    else:
        ho, wo = int(np.floor(hi * scale_factor)), int(np.floor(wi * scale_factor))
        sh = sw = _src_scale(hi, ho, scale_factor)
    return BilinearFn.apply(x, ho, wo, sh, sw)


# ----------------------------------------------------------------------------- softmax / losses
def _pix_strides(x):
    """(sn, sc, shw) element strides of a [N, C, H, W] tensor whose H, W flatten."""
    sn, sc, s_h, s_w = x.stride()
    if x.shape[2] > 1 and s_h != x.shape[3] * s_w:
        raise RuntimeError("rtsds_amd: logits must have flattenable H, W")
    return sn, sc, s_w


class SoftmaxFn(torch.autograd.Function):
    """F.softmax(x, dim=1) (train.py:225,245,256); output NHWC."""

    @staticmethod
    def forward(ctx, x):
        require_hip(x)
        n, c, h, w = x.shape
        sn, sc, shw = _pix_strides(x)
        y = empty_nhwc(n, c, h, w, x.dtype, x.device)
        lib.rtsds_softmax_fwd(_P(x), sn, sc, shw, _P(y), c, n, h * w, c, dcode(x), stream())
        ctx.save_for_backward(y)
        ctx.xlayout = (x.stride(), x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        n, c, h, w = y.shape
        dy = nhwc(dy)
        if dy.dtype != y.dtype:
            dy = cast(dy, y.dtype)
        dx = empty_nhwc(n, c, h, w, y.dtype, y.device)
        sn, sc, shw = _pix_strides(dx)
        lib.rtsds_softmax_bwd(_P(dy), _P(y), c, _P(dx), sn, sc, shw, n, h * w, c, dcode(y), stream())
        return dx


def softmax(x, dim=1):
    if dim != 1:
        raise NotImplementedError("rtsds_amd.softmax: only dim=1 (channels) is on the hot path")
    return SoftmaxFn.apply(x)


class CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target, ignore_index):
        require_hip(x, target)
        if target.dim() == 4:
            target = target.squeeze(1)
        target = target.contiguous()
        if target.dtype != torch.int64:
            target = target.long()
        n, c, h, w = x.shape
        if tuple(target.shape) != (n, h, w):
            raise RuntimeError(f"rtsds_amd: target shape {tuple(target.shape)} != {(n, h, w)}")
        sn, sc, shw = _pix_strides(x)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        ws = workspace(lib.rtsds_ce_workspace(), x.device)
        lib.rtsds_ce_fwd(_P(x), sn, sc, shw, _P(target), _P(loss), n, h * w, c, ignore_index,
                         dcode(x), _P(ws), ws.numel(), stream())
        if dp_world() > 1:  # global-batch mean: local loss sum over the all-reduced count
            import torch.distributed as dist
            cnt = ws.view(torch.float32)[2048:2049]
            collective(lambda: dist.all_reduce(cnt))
            lib.rtsds_ce_finish(_P(ws), _P(loss), stream())
        ctx.ignore = ignore_index
        ctx.save_for_backward(x, target, ws)
        return loss

    @staticmethod
    def backward(ctx, g):
        x, target, ws = ctx.saved_tensors
        n, c, h, w = x.shape
        sn, sc, shw = _pix_strides(x)
        dx = torch.empty_strided(x.shape, x.stride(), dtype=x.dtype, device=x.device)
        g = g.contiguous().float()
        count = ws.view(torch.float32)[2048:2049]
        lib.rtsds_ce_bwd(_P(x), sn, sc, shw, _P(target), _P(g), _P(count), _P(dx), n, h * w, c,
                         ctx.ignore, dcode(x), stream())
        return dx, None, None


def cross_entropy(x, target, ignore_index=-100):
    return CrossEntropyFn.apply(x, target, ignore_index)


class AdaptiveAvgPoolFn(torch.autograd.Function):
    """F.adaptive_avg_pool2d(x, (ho, wo)) (train.py:410,438,445), NHWC."""

    @staticmethod
    def forward(ctx, x, ho, wo):
        require_hip(x)
        x = nhwc(x)
        n, c, hi, wi = x.shape
        y = empty_nhwc(n, c, ho, wo, x.dtype, x.device)
        lib.rtsds_adaptive_avgpool_fwd(_P(x), _P(y), n, hi, wi, c, ho, wo, dcode(x), stream())
        ctx.geo = (n, c, hi, wi, ho, wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, c, hi, wi, ho, wo = ctx.geo
        dy = nhwc(dy)
        dx = empty_nhwc(n, c, hi, wi, dy.dtype, dy.device)
        lib.rtsds_adaptive_avgpool_bwd(_P(dy), _P(dx), n, hi, wi, c, ho, wo, dcode(dy), stream())
        return dx, None, None


def adaptive_avg_pool2d(x, output_size):
    """Identity (same tensor, as ATen's values) when the size already matches."""
    ho, wo = (output_size, output_size) if isinstance(output_size, int) else output_size
    if tuple(x.shape[-2:]) == (int(ho), int(wo)):
        return x
    return AdaptiveAvgPoolFn.apply(x, int(ho), int(wo))


class UpsampleCrossEntropyFn(torch.autograd.Function):
    """sum_h CrossEntropy(interpolate_bilinear(head_h, (H, W)), target) without materialising
    the full-resolution logits (rtsds_upce_*; the chain it replaces is cited in the header).
    Also adds head 0's argmax==target pixel count into ``correct`` when given."""

    @staticmethod
    def forward(ctx, target, geo, ignore_index, correct, set_correct, *heads):
        n, c, hl, wl, H, W, sh, sw = geo
        xs = [nhwc(h) for h in heads]
        k = len(xs)
        dt = dcode(xs[0])
        nbytes = lib.rtsds_upce_workspace(k, n, hl, wl, c, H, W, sh, sw)
        ws = workspace(nbytes, xs[0].device)
        ptrs = (ctypes.c_void_p * k)(*[x.data_ptr() for x in xs])
        per_head = torch.empty(k, dtype=torch.float32, device=xs[0].device)
        total = torch.empty((), dtype=torch.float32, device=xs[0].device)
        want = any(ctx.needs_input_grad[5:])
        flags = int(want) | (UPCE_SET_CORRECT if set_correct else 0)
        lib.rtsds_upce_fwd(k, ptrs, _P(target), n, hl, wl, c, H, W, sh, sw, ignore_index, _P(per_head),
                           _P(total), _P(correct), flags, dt, _P(ws), ws.numel(), stream())
        if dp_world() > 1:
            # global-batch mean: this rank's loss sums over the all-reduced valid-pixel count
            # (its contribution; the ranks' losses and gradients then SUM to the single-device
            # values, see runtime.dp_world)
            import torch.distributed as dist
            cnt = ws.view(torch.float32)[:1]
            collective(lambda: dist.all_reduce(cnt))
            lib.rtsds_upce_finish(k, _P(ws), _P(per_head), _P(total), stream())
        ctx.geo, ctx.k, ctx.dt, ctx.dtype = geo, k, dt, xs[0].dtype
        ctx.ws = ws
        ctx.per_head = per_head
        return total

    @staticmethod
    def backward(ctx, g):
        n, c, hl, wl, H, W, sh, sw = ctx.geo
        ws = ctx.ws
        dxs = [empty_nhwc(n, c, hl, wl, ctx.dtype, ws.device) for _ in range(ctx.k)]
        ptrs = (ctypes.c_void_p * ctx.k)(*[d.data_ptr() for d in dxs])
        g = g.contiguous().float()
        lib.rtsds_upce_bwd(ctx.k, _P(g), 0, ptrs, n, hl, wl, c, H, W, sh, sw, ctx.dt, _P(ws), ws.numel(),
                           stream())
        ctx.ws = None
        return (None, None, None, None, None, *dxs)


def interpolate_geometry(x, geo):
    """interpolate_bilinear with a precomputed upsample_geometry()."""
    ho, wo, sh, sw = geo
    return BilinearFn.apply(x, ho, wo, sh, sw)


def upsample_geometry(x, size=None, scale_factor=None):
    """(H, W, scale_h, scale_w) of interpolate_bilinear(x, size | scale_factor)."""
    hi, wi = x.shape[-2:]
    if size is not None:
        ho, wo = int(size[0]), int(size[1])
        return ho, wo, _src_scale(hi, ho, None), _src_scale(wi, wo, None)
    ho, wo = int(np.floor(hi * scale_factor)), int(np.floor(wi * scale_factor))
    s = _src_scale(hi, ho, scale_factor)
    return ho, wo, s, s


def upsample_cross_entropy_supported(heads, geo, ignore_index):
    h0 = heads[0]
    n, c, hl, wl = h0.shape
    ho, wo, sh, sw = geo
    if len(heads) > 4 or any(tuple(h.shape) != tuple(h0.shape) or h.dtype != h0.dtype for h in heads):
        return False
    return lib.rtsds_upce_workspace(len(heads), n, hl, wl, c, ho, wo, sh, sw) > 0


def upsample_cross_entropy(heads, target, geo, ignore_index=-100, correct=None, set_correct=False):
    """Sum over heads (in order) of cross_entropy(interpolate_bilinear(head, ...), target),
    fused; ``geo`` from upsample_geometry().  ``correct``: optional int64 device counter that
    receives head 0's pixel-accuracy matches (added; ``set_correct``: overwritten, so the
    caller need not zero it).  Returns the total loss."""
    require_hip(target, *heads)
    t = target.squeeze(1) if target.dim() == 4 else target
    t = t.contiguous()
    if t.dtype != torch.int64:
        t = t.long()
    n, c, hl, wl = heads[0].shape
    ho, wo, sh, sw = geo
    if tuple(t.shape) != (n, ho, wo):
        raise RuntimeError(f"rtsds_amd: target shape {tuple(t.shape)} != {(n, ho, wo)}")
    if not upsample_cross_entropy_supported(heads, geo, ignore_index):
        raise RuntimeError("rtsds_amd: fused upsample+CE does not cover this geometry")
    full = (n, c, hl, wl, ho, wo, sh, sw)
    fn = UpsampleCrossEntropyFn
    total = fn.apply(t, full, int(ignore_index), correct, bool(set_correct), *heads)
    return total


class UpsampleSoftmaxFn(torch.autograd.Function):
    """softmax(interpolate_bilinear(x, geo), dim=1) in one pass (rtsds_upsoftmax_fwd), written
    zero-padded to 32 channels so the discriminator's first conv reads it directly
    (RTSDS_INPUT_PADDED); backward = softmax backward + resize adjoint in one pass plus the
    vertical adjoint (rtsds_upsoftmax_bwd).  Bit-identical to interpolate -> softmax."""

    @staticmethod
    def forward(ctx, x, geo):
        require_hip(x)
        x = nhwc(x)
        n, c, hi, wi = x.shape
        ho, wo, sh, sw = geo
        cp = 32
        buf = torch.empty((n, ho, wo, cp), dtype=x.dtype, device=x.device)
        lib.rtsds_upsoftmax_fwd(_P(x), _P(buf), n, hi, wi, c, ho, wo, sh, sw, cp, dcode(x), stream())
        ctx.geo, ctx.shape, ctx.cp = geo, (n, c, hi, wi), cp
        ctx.save_for_backward(buf)
        return buf.permute(0, 3, 1, 2)[:, :c]

    @staticmethod
    def backward(ctx, dy):
        buf, = ctx.saved_tensors
        n, c, hi, wi = ctx.shape
        ho, wo, sh, sw = ctx.geo
        dy = nhwc(dy)
        if dy.dtype != buf.dtype:
            dy = cast(dy, buf.dtype)
        dx = empty_nhwc(n, c, hi, wi, buf.dtype, buf.device)
        ws = workspace(lib.rtsds_upsoftmax_bwd_workspace(n, hi, wi, c, ho, wo), buf.device)
        lib.rtsds_upsoftmax_bwd(_P(dy), c, _P(buf), ctx.cp, _P(dx), n, hi, wi, c, ho, wo, sh, sw, dcode(buf),
                                       _P(ws), ws.numel(), stream())
        return dx, None


def upsample_softmax(x, geo):
    """softmax over classes of the resized head (train.py:225,245,256), as the discriminator's
    zero-padded input (functional.is_padded_input)."""
    y = UpsampleSoftmaxFn.apply(x, geo)
    y._rt_cpad = 32
    return y


class BCEWithLogitsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target):
        require_hip(x, target)
        xf = cast(x.contiguous(), torch.float32)
        tf = cast(target.contiguous(), torch.float32) if target.dtype != torch.float32 else target.contiguous()
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        lib.rtsds_bce_fwd(_P(xf), _P(tf), _P(loss), xf.numel(), stream())
        ctx.xdtype = x.dtype
        ctx.save_for_backward(xf, tf)
        return loss

    @staticmethod
    def backward(ctx, g):
        xf, tf = ctx.saved_tensors
        dx = torch.empty_like(xf)
        lib.rtsds_bce_bwd(_P(xf), _P(tf), _P(g.contiguous().float()), _P(dx), xf.numel(), stream())
        return cast(dx, ctx.xdtype), None


def bce_with_logits(x, target):
    return BCEWithLogitsFn.apply(x, target)


# ----------------------------------------------------------------------------- metrics
def argmax_channels(x, target=None, correct=None, want_map=True):
    """argmax over dim 1 (first max wins) -> int64 [N, H, W]; optionally adds the number of
    pixels equal to ``target`` into the device counter ``correct`` (uint64 view)."""
    require_hip(x)
    n, c, h, w = x.shape
    sn, sc, shw = _pix_strides(x)
    out = torch.empty((n, h, w), dtype=torch.int64, device=x.device) if want_map else None
    t = None
    if target is not None:
        t = target.squeeze(1) if target.dim() == 4 else target
        t = t.contiguous().long()
    lib.rtsds_argmax(_P(x), sn, sc, shw, _P(out), _P(t), _P(correct), n, h * w, c, dcode(x), stream())
    return out


def confusion(label, pred, hist, nc):
    lib.rtsds_confusion(_P(label.contiguous()), _P(pred.contiguous()), _P(hist), label.numel(), nc,
                        stream())
