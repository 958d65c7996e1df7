"""torch.nn-compatible layers whose forward/backward run on librtsds_hip.so.

``Conv2d`` / ``BatchNorm2d`` subclass the torch classes so parameters, buffers,
``state_dict`` keys and ``isinstance`` checks (e.g. build_bisenet.py:130-139) are exactly the
reference's; only ``forward`` differs.  Conv weights are stored channels_last, i.e. in the
kernel's [Cout][KH][KW][Cin] layout, with the logical shape [Cout, Cin, KH, KW] unchanged.
Extra keyword ``act`` fuses a following ReLU / LeakyReLU / sigmoid into the epilogue.
"""
import torch
from torch import nn

from . import functional as F
from ._lib import lib
from .runtime import CL, compute_dtype

ACT = {None: 0, "relu": 1, "leaky": 2, "sigmoid": 3}


def _shadow(w, dtype):
    """Weight in compute dtype and kernel layout.  bf16 shadows are cached on the parameter
    and refreshed when its storage or version changes (or written directly by rtsds Adam)."""
    if dtype == torch.float32:
        return w.detach() if w.is_contiguous(memory_format=CL) else w.detach().contiguous(memory_format=CL)
    sh = getattr(w, "_rt_shadow", None)
    key = (w.data_ptr(), w._version)
    if sh is not None and getattr(w, "_rt_shadow_key", None) == key and sh.device == w.device:
        return sh
    if sh is None or sh.shape != w.shape or sh.device != w.device:
        sh = torch.empty(w.shape, dtype=torch.bfloat16, device=w.device, memory_format=CL)
    src = w.detach()
    if not src.is_contiguous(memory_format=CL):
        src = src.contiguous(memory_format=CL)
    lib.rtsds_cast(src.data_ptr(), 0, sh.data_ptr(), 1, src.numel(), torch.cuda.current_stream().cuda_stream)
    w._rt_shadow, w._rt_shadow_key = sh, key
    return sh


class Conv2d(nn.Conv2d):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.groups != 1 or self.padding_mode != "zeros":
            raise NotImplementedError("rtsds_amd.Conv2d: groups=1, zero padding only")
        self.weight.data = self.weight.data.contiguous(memory_format=CL)

    def _apply(self, fn, *a, **k):
        out = super()._apply(fn, *a, **k)
        if not self.weight.is_contiguous(memory_format=CL):
            self.weight.data = self.weight.data.contiguous(memory_format=CL)
        return out

    def forward(self, x, act=None, bn_stats=False, join=None, in_act=None, fold_out=False, bn_link=None):
        """``bn_stats``: also emit the batch statistics of a directly following train-mode
        BatchNorm from the conv epilogue (see functional.conv2d).  ``join``: a
        functional.GradJoin shared with the other readers of ``x``.  ``in_act`` / ``fold_out``:
        activation-backward folding between chained convs (functional.ConvFn)."""
        wq = _shadow(self.weight, x.dtype)
        return F.conv2d(x, self.weight, self.bias, wq, self.stride, self.padding, self.dilation,
                        ACT[act], bn_stats, join, ACT[in_act], fold_out, bn_link)


class BatchNorm2d(nn.BatchNorm2d):
    def forward(self, x, act=None, residual=None, res_join=None, link=None, out=None):
        training = self.training or not self.track_running_stats
        if training and x.shape[0] * x.shape[2] * x.shape[3] == 1:
            raise ValueError(f"Expected more than 1 value per channel when training, got input size {tuple(x.shape)}")
        if self.momentum is None:
            raise NotImplementedError("rtsds_amd.BatchNorm2d: cumulative moving average (momentum=None)")
        rm = self.running_mean if self.track_running_stats else None
        rv = self.running_var if self.track_running_stats else None
        # num_batches_tracked.add_(1) happens inside the statistics-finalize kernel
        nbt = self.num_batches_tracked if (self.training and self.track_running_stats) else None
        return F.batch_norm(x, self.weight, self.bias, rm, rv, training, self.momentum, self.eps,
                            ACT[act], residual, nbt, res_join, link, out)


class ReLU(nn.Module):
    def __init__(self, inplace=False):
        super().__init__()
        self.inplace = inplace

    def forward(self, x):
        return F.relu(x)


class LeakyReLU(nn.Module):
    def __init__(self, negative_slope=0.2):
        super().__init__()
        if negative_slope != 0.2:
            raise NotImplementedError("rtsds_amd.LeakyReLU: slope 0.2 (model.py:62,73)")
        self.negative_slope = negative_slope

    def forward(self, x):
        return F.leaky_relu(x)


class Sigmoid(nn.Module):
    def forward(self, x):
        return F.sigmoid(x)


class AdaptiveAvgPool2d(nn.Module):
    def __init__(self, output_size=(1, 1)):
        super().__init__()
        osz = (output_size, output_size) if isinstance(output_size, int) else tuple(output_size)
        if osz != (1, 1):
            raise NotImplementedError("rtsds_amd.AdaptiveAvgPool2d: output (1, 1) only")
        self.output_size = output_size

    def forward(self, x):
        return F.global_avg_pool(x)


class MaxPool2d(nn.Module):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False):
        super().__init__()
        self.kernel_size, self.stride = kernel_size, stride or kernel_size
        self.padding, self.ceil_mode = padding, ceil_mode

    def forward(self, x):
        return F.max_pool2d(x, self.kernel_size, self.stride, self.padding, self.ceil_mode)


def _no_grad_needed(conv, bn, x, residual):
    if not torch.is_grad_enabled():
        return True
    ts = [x, residual, conv.weight, conv.bias, bn.weight, bn.bias]
    return not any(t is not None and t.requires_grad for t in ts)


def conv_bn(conv, bn, x, act=None, residual=None, join=None, res_join=None, in_link=None, out_link=None, out=None):
    """bn(conv(x)) with the BatchNorm's batch statistics produced by the conv epilogue
    (train mode) instead of a separate pass over the conv output.  Eval mode without
    autograd (inference, validation): the BN (+ residual + act) folds into the conv's
    epilogue -- one launch per ConvBlock / residual branch.  ``join`` / ``res_join``:
    functional.GradJoin shared by the readers of ``x`` / ``residual`` (residual blocks).
    ``in_link``: functional.BnBwdLink of the BatchNorm that produced ``x`` (its backward
    statistics come from this conv's data gradient); ``out_link``: the link this BatchNorm
    registers with (its output's single reader passes it as ``in_link``).  ``out``: (NHWC buffer,
    channel offset) the result is written into (functional.conv_bn_eval at inference,
    functional.batch_norm in training; a view of the slice is returned)."""
    use_batch = bn.training or not bn.track_running_stats
    if not use_batch and bn.momentum is not None and _no_grad_needed(conv, bn, x, residual):
        wq = _shadow(conv.weight, x.dtype)
        return F.conv_bn_eval(x, conv.weight, conv.bias, wq, conv.stride, conv.padding, conv.dilation,
                              bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, ACT[act], residual, out=out)
    return bn(conv(x, bn_stats=use_batch, join=join, bn_link=in_link), act=act, residual=residual, res_join=res_join,
              link=out_link, out=out)


def conv_bn_relu_maxpool(conv, bn, pool, x):
    """pool(relu(bn(conv(x)))) -- the ResNet stem.  Train-mode (batch statistics) bf16 with a
    3x3 stride-2 pool: the BN apply, ReLU and pool run as one pass (functional.bn_relu_maxpool,
    statistics from the conv epilogue); inference: conv + folded BN + ReLU + pool in one launch
    (bf16 image stem); otherwise the separate ops."""
    use_batch = bn.training or not bn.track_running_stats
    k = pool.kernel_size if isinstance(pool.kernel_size, int) else pool.kernel_size[0]
    s = pool.stride if isinstance(pool.stride, int) else pool.stride[0]
    p = pool.padding if isinstance(pool.padding, int) else pool.padding[0]
    if use_batch and bn.momentum is not None and x.dtype == torch.bfloat16 and conv.out_channels % 8 == 0 \
            and k == 3 and s == 2 and p in (0, 1):
        y = conv(x, bn_stats=True)
        if F.bn_relu_maxpool_ok(y, k, s, p):
            rm = bn.running_mean if bn.track_running_stats else None
            rv = bn.running_var if bn.track_running_stats else None
            nbt = bn.num_batches_tracked if (bn.training and bn.track_running_stats) else None
            return F.bn_relu_maxpool(y, bn.weight, bn.bias, rm, rv, True, bn.momentum, bn.eps, p, pool.ceil_mode, nbt)
        return pool(bn(y, act="relu"))
    if not use_batch and bn.momentum is not None and _no_grad_needed(conv, bn, x, None) and k == 3 and s == 2:
        # inference: the pool runs in the folded conv's epilogue (rtsds_conv2d_fwd_bn_maxpool)
        y = F.conv_bn_maxpool_eval(x, conv.weight, conv.bias, _shadow(conv.weight, x.dtype), conv.stride, conv.padding,
                                   conv.dilation, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps,
                                   ACT["relu"], k, s, p, pool.ceil_mode)
        if y is not None:
            return y
    return pool(conv_bn(conv, bn, x, "relu"))


def grad_join(x, n):
    """A functional.GradJoin for ``x`` read by ``n`` rtsds Functions, or None when no
    gradient flows to ``x``."""
    return F.GradJoin(n) if (torch.is_grad_enabled() and x.requires_grad) else None


def to_input(x):
    """Reference-layout NCHW fp32 batch -> NHWC in the runtime compute dtype."""
    return F.pack_input(x, compute_dtype())
