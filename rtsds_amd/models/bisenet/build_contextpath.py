"""BiSeNet context path on the HIP kernels (reference: models/bisenet/build_contextpath.py).

The reference wraps ``torchvision.models.resnet18/101(pretrained=True)`` (torchvision 0.18,
requirements.txt:85) and returns (layer3, layer4, global-average tail).  torchvision is
not a dependency here: the ResNet below carries torchvision's sub-module names
(``features.conv1 ... features.fc``) so ``state_dict`` keys -- including the aliased
``context_path.conv1`` / ``context_path.features.conv1`` pairs the reference registers -- are
identical.  ``pretrained`` weights (a network download in the reference,
build_contextpath.py:8,35) are not fetched; load a state_dict instead.  Unlike the reference's
``build_contextpath`` (build_contextpath.py:59-63), only the requested depth is built.
"""
import torch
from torch import nn

from rtsds_amd import functional as F
from rtsds_amd.functional import BnBwdLink
from rtsds_amd.nn import BatchNorm2d, Conv2d, MaxPool2d, ReLU, conv_bn, conv_bn_relu_maxpool, grad_join
from rtsds_amd.runtime import grad_cut


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU(inplace=True)
        self.conv2 = Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # x has two readers (conv1 and the identity / downsample branch): their gradients meet
        # in one buffer (the later producer's kernel accumulates) instead of an autograd add
        join = grad_join(x, 2)
        skip = x
        if self.downsample is not None:
            skip = conv_bn(self.downsample[0], self.downsample[1], x, join=join)
        link = BnBwdLink()  # bn1's output has one reader, conv2: its dgrad yields bn1's backward statistics
        t = conv_bn(self.conv1, self.bn1, x, "relu", join=join, out_link=link)
        # bn2 + residual add + ReLU in one pass
        return conv_bn(self.conv2, self.bn2, t, "relu", skip,
                       res_join=join if self.downsample is None else None, in_link=link)


class Bottleneck(nn.Module):
    """torchvision v1.5 bottleneck (stride on the 3x3)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = BatchNorm2d(planes * 4)
        self.relu = ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        join = grad_join(x, 2)  # as BasicBlock
        skip = x
        if self.downsample is not None:
            skip = conv_bn(self.downsample[0], self.downsample[1], x, join=join)
        l1, l2 = BnBwdLink(), BnBwdLink()  # bn1 -> conv2, bn2 -> conv3 (single readers)
        t = conv_bn(self.conv1, self.bn1, x, "relu", join=join, out_link=l1)
        t = conv_bn(self.conv2, self.bn2, t, "relu", in_link=l1, out_link=l2)
        return conv_bn(self.conv3, self.bn3, t, "relu", skip,
                       res_join=join if self.downsample is None else None, in_link=l2)


class ResNet(nn.Module):
    """torchvision-compatible ResNet trunk (names: conv1, bn1, relu, maxpool, layer1-4,
    avgpool, fc).  ``fc`` is kept only for state_dict parity; it never runs."""

    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.relu = ReLU(inplace=True)
        self.maxpool = MaxPool2d(3, 2, 1)
        self.layer1 = self._stage(block, 64, layers[0], 1)
        self.layer2 = self._stage(block, 128, layers[1], 2)
        self.layer3 = self._stage(block, 256, layers[2], 2)
        self.layer4 = self._stage(block, 512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _stage(self, block, planes, count, stride):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(Conv2d(self.inplanes, planes * block.expansion, 1, stride, bias=False),
                                 BatchNorm2d(planes * block.expansion))
        mods = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        for _ in range(1, count):
            mods.append(block(self.inplanes, planes))
        return nn.Sequential(*mods)


class _ContextPath(nn.Module):
    def __init__(self, trunk):
        super().__init__()
        self.features = trunk
        self.conv1 = trunk.conv1
        self.bn1 = trunk.bn1
        self.relu = trunk.relu
        self.maxpool1 = trunk.maxpool
        self.layer1, self.layer2 = trunk.layer1, trunk.layer2
        self.layer3, self.layer4 = trunk.layer3, trunk.layer4

    # where ``mid`` runs: after the stem (0), layer1 (1) or layer2 (2)
    fork_after = 1  # bs-8 train step: 1 vs 2 +0.5 % (profiles/r5ae_fork_point_ab.txt)

    def forward(self, x, mid=None, tail_join=None):
        """x: NHWC compute-dtype batch -> (1/16 features, 1/32 features, GAP(1/32)).  ``mid``:
        called after stage ``fork_after`` (BiSeNet forks its spatial path there).  ``tail_join``:
        GradJoin of the 1/32 features' readers (the GAP here and the caller's attention scale)."""
        if mid is not None and self.fork_after < 0:
            mid()
        t = conv_bn_relu_maxpool(self.conv1, self.bn1, self.maxpool1, x)
        for i, layer in enumerate((self.layer1, self.layer2)):
            if mid is not None and self.fork_after == i:
                mid()
            t = layer(t)
        if mid is not None and self.fork_after >= 2:
            mid()
        f3 = grad_cut(self.layer3(t))  # data-parallel two-phase backward (runtime.grad_cut)
        f4 = self.layer4(f3)
        return f3, f4, F.global_avg_pool(f4, tail_join)


class resnet18(_ContextPath):
    def __init__(self, pretrained=True):
        super().__init__(ResNet(BasicBlock, [2, 2, 2, 2]))


class resnet101(_ContextPath):
    def __init__(self, pretrained=True):
        super().__init__(ResNet(Bottleneck, [3, 4, 23, 3]))


def build_contextpath(name):
    builders = {"resnet18": resnet18, "resnet101": resnet101}
    if name not in builders:
        raise KeyError(name)
    return builders[name](pretrained=True)
