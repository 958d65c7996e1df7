"""Output-space discriminators on the MI355X kernels -- drop-in for the reference's
models/domain_shift/adversarial/model.py.

k4 s2 p1 convolutions with bias; the LeakyReLU(0.2) is fused into each conv's epilogue, and
its backward into the next conv's data-gradient epilogue (mask from the sign of that conv's
input: rtsds_conv2d_dgrad_act), so the activation gradient is never a separate pass.  The head is conv -> global average
pool -> [N, 1, 1, 1] logit, as in the reference.
"""
import torch
from torch import nn
from torch.autograd import Function

from rtsds_amd import functional as F
from rtsds_amd.nn import AdaptiveAvgPool2d, Conv2d, LeakyReLU, to_input


class GradientReversalFunction(Function):
    """model.py:9-17: identity forward, -alpha * grad backward (HIP scale kernel)."""

    @staticmethod
    def forward(ctx, x, alpha):
        return F.GradReverseFn.forward(ctx, x, alpha)

    @staticmethod
    def backward(ctx, grad_output):
        return F.GradReverseFn.backward(ctx, grad_output)


class UpSampler(nn.Module):
    """model.py:19-28: x8 bilinear -> 1x1 conv, evaluated as 1x1 conv -> x8 bilinear (the two
    commute exactly: see build_bisenet.BiSeNet.forward)."""

    def __init__(self, num_classes) -> None:
        super().__init__()
        self.conv = Conv2d(in_channels=num_classes, out_channels=num_classes, kernel_size=1)

    def forward(self, x):
        return F.interpolate_bilinear(self.conv(_nhwc_input(x)), scale_factor=8)


def _nhwc_input(x):
    """Accept an rtsds NHWC activation, the zero-padded class probabilities of
    functional.upsample_softmax (read in place by conv1), or a reference-layout NCHW fp32
    tensor."""
    if F.is_padded_input(x):
        return x
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] > 1:
        return x
    return to_input(x)


class DomainDiscriminator(nn.Module):
    """model.py:30-64: 19->64->128->256->512->1, k4 s2 p1, LeakyReLU(0.2), GAP, optional GRL."""

    accepts_padded_probs = True  # conv1 reads functional.upsample_softmax's padded output

    def __init__(self, num_classes=19, with_grl=False, lambda_: float = 0.1) -> None:
        super(DomainDiscriminator, self).__init__()
        self.with_grl = with_grl
        self.lambda_ = lambda_
        self.conv1 = Conv2d(19, 64, kernel_size=4, stride=2, padding=1)
        self.conv2 = Conv2d(64, 128, kernel_size=4, stride=2, padding=1)
        self.conv3 = Conv2d(128, 256, kernel_size=4, stride=2, padding=1)
        self.conv4 = Conv2d(256, 512, kernel_size=4, stride=2, padding=1)
        self.classifier = Conv2d(512, 1, kernel_size=4, stride=2, padding=1)
        self.leaky_relu = LeakyReLU(0.2)
        self.avgpool = AdaptiveAvgPool2d((1, 1))

    fold_act = True  # LeakyReLU backward of conv_i applied by conv_{i+1}'s data gradient

    def forward(self, x):
        x = _nhwc_input(x)
        f = self.fold_act
        prev = None
        for conv in (self.conv1, self.conv2, self.conv3, self.conv4):
            x = conv(x, act="leaky", in_act=prev, fold_out=f)
            prev = "leaky" if f else None
        x = self.avgpool(self.classifier(x, in_act=prev))
        if self.with_grl:
            x = F.GradReverseFn.apply(x, self.lambda_)
        return x


class TinyDomainDiscriminator(nn.Module):
    """model.py:67-83: conv 19->64 k4s2p1 + LeakyReLU(0.2) -> conv 64->1 k4s2p1 -> GAP."""

    accepts_padded_probs = True

    def __init__(self, num_classes=19) -> None:
        super(TinyDomainDiscriminator, self).__init__()
        self.conv1 = Conv2d(num_classes, 64, kernel_size=4, stride=2, padding=1)
        self.classifier = Conv2d(64, 1, kernel_size=4, stride=2, padding=1)
        self.leaky_relu = LeakyReLU(0.2)
        self.avgpool = AdaptiveAvgPool2d((1, 1))

    fold_act = True  # conv1's LeakyReLU backward applied by the classifier's data gradient

    def forward(self, x):
        x = _nhwc_input(x)
        f = self.fold_act
        h = self.conv1(x, act="leaky", fold_out=f)
        return self.avgpool(self.classifier(h, in_act="leaky" if f else None))
