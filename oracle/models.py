"""Plain-PyTorch fp32 CPU restatement of the reference modules (TEST INFRASTRUCTURE).

Sub-module names and registration order follow the reference exactly so that
``state_dict`` keys (including the aliased ``context_path.conv1`` / ``context_path.features.conv1``
pairs) are identical -- the weight recipe in ``oracle.weights`` and the HIP models both
rely on that.  Each class cites the reference lines it restates.
"""
import torch
import torch.nn.functional as F
from torch import nn

from . import tv_resnet


# --------------------------------------------------------------------------- BiSeNet
class ConvBlock(nn.Module):
    """conv(no bias) -> BN -> ReLU  (reference models/bisenet/build_bisenet.py:8-18)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=2, padding=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding, bias=False)
        self.bn = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU()

    def forward(self, x):
        return F.relu(self.bn(self.conv1(x)))


class Spatial_path(nn.Module):
    """Three stride-2 ConvBlocks 3->64->128->256 (build_bisenet.py:21-32)."""

    def __init__(self):
        super().__init__()
        self.convblock1 = ConvBlock(3, 64)
        self.convblock2 = ConvBlock(64, 128)
        self.convblock3 = ConvBlock(128, 256)

    def forward(self, x):
        return self.convblock3(self.convblock2(self.convblock1(x)))


class AttentionRefinementModule(nn.Module):
    """GAP -> 1x1 conv(bias) -> BN -> sigmoid -> x*a  (build_bisenet.py:35-53)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, 1)
        self.bn = nn.BatchNorm2d(out_channels)
        self.sigmoid = nn.Sigmoid()
        self.in_channels = in_channels
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))

    def forward(self, x):
        a = torch.sigmoid(self.bn(self.conv(x.mean((2, 3), keepdim=True))))
        return x * a


class FeatureFusionModule(nn.Module):
    """cat -> ConvBlock(s1) -> GAP -> 1x1 -> ReLU -> 1x1 -> sigmoid -> f*a + f (build_bisenet.py:56-81)."""

    def __init__(self, num_classes, in_channels):
        super().__init__()
        self.in_channels = in_channels
        self.convblock = ConvBlock(in_channels, num_classes, stride=1)
        self.conv1 = nn.Conv2d(num_classes, num_classes, 1)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2d(num_classes, num_classes, 1)
        self.sigmoid = nn.Sigmoid()
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))

    def forward(self, a, b):
        f = self.convblock(torch.cat((a, b), 1))
        g = torch.sigmoid(self.conv2(F.relu(self.conv1(f.mean((2, 3), keepdim=True)))))
        return f * g + f


class ContextPath(nn.Module):
    """torchvision ResNet wrapper returning (layer3, layer4, GAP(layer4))
    (reference models/bisenet/build_contextpath.py:5-29 / 32-57).  The aliases
    conv1/bn1/relu/maxpool1/layer* are registered after ``features`` exactly as there."""

    def __init__(self, depth):
        super().__init__()
        self.features = tv_resnet.resnet18() if depth == 18 else tv_resnet.resnet101()
        f = self.features
        self.conv1, self.bn1, self.relu, self.maxpool1 = f.conv1, f.bn1, f.relu, f.maxpool
        self.layer1, self.layer2, self.layer3, self.layer4 = f.layer1, f.layer2, f.layer3, f.layer4

    def forward(self, x):
        x = self.maxpool1(F.relu(self.bn1(self.conv1(x))))
        f3 = self.layer3(self.layer2(self.layer1(x)))
        f4 = self.layer4(f3)
        tail = f4.mean(3, keepdim=True).mean(2, keepdim=True)
        return f3, f4, tail


class BiSeNet(nn.Module):
    """reference models/bisenet/build_bisenet.py:84-172."""

    def __init__(self, num_classes, context_path, with_interpolation=True):
        super().__init__()
        self.with_interpolation = with_interpolation
        self.saptial_path = Spatial_path()
        self.context_path = ContextPath(18 if context_path == "resnet18" else 101)
        c3, c4 = (256, 512) if context_path == "resnet18" else (1024, 2048)
        self.attention_refinement_module1 = AttentionRefinementModule(c3, c3)
        self.attention_refinement_module2 = AttentionRefinementModule(c4, c4)
        self.supervision1 = nn.Conv2d(c3, num_classes, 1)
        self.supervision2 = nn.Conv2d(c4, num_classes, 1)
        self.feature_fusion_module = FeatureFusionModule(num_classes, 256 + c3 + c4)
        self.conv = nn.Conv2d(num_classes, num_classes, 1)

    def forward(self, x):
        sx = self.saptial_path(x)
        f3, f4, tail = self.context_path(x)
        cx1 = self.attention_refinement_module1(f3)
        cx2 = self.attention_refinement_module2(f4) * tail
        hw = sx.shape[-2:]
        cx1 = F.interpolate(cx1, size=hw, mode="bilinear")
        cx2 = F.interpolate(cx2, size=hw, mode="bilinear")
        if self.training:
            s1 = F.interpolate(self.supervision1(cx1), size=x.shape[-2:], mode="bilinear")
            s2 = F.interpolate(self.supervision2(cx2), size=x.shape[-2:], mode="bilinear")
        out = self.feature_fusion_module(sx, torch.cat((cx1, cx2), 1))
        if self.with_interpolation:
            out = self.conv(F.interpolate(out, scale_factor=8, mode="bilinear"))
        return (out, s1, s2) if self.training else out


# --------------------------------------------------------------------------- DeepLabV2
class Bottleneck(nn.Module):
    """Caffe-style bottleneck, stride on the first 1x1, frozen BN affine
    (reference models/deeplabv2/deeplabv2.py:7-47)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, dilation=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, dilation, dilation=dilation, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        for bn in (self.bn1, self.bn2, self.bn3):
            bn.weight.requires_grad_(False)
            bn.bias.requires_grad_(False)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        return F.relu(self.bn3(self.conv3(y)) + idt)


class ClassifierModule(nn.Module):
    """ASPP = sum of dilated 3x3 convs with bias (deeplabv2.py:50-66)."""

    def __init__(self, inplanes, dilation_series, padding_series, num_classes):
        super().__init__()
        self.conv2d_list = nn.ModuleList(
            nn.Conv2d(inplanes, num_classes, 3, 1, p, dilation=d, bias=True)
            for d, p in zip(dilation_series, padding_series))

    def forward(self, x):
        out = self.conv2d_list[0](x)
        for conv in self.conv2d_list[1:]:
            out = out + conv(x)
        return out


class ResNetMulti(nn.Module):
    """deeplabv2.py:69-131 (training returns (x, None, None))."""

    def __init__(self, layers=(3, 4, 23, 3), num_classes=19):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.bn1.weight.requires_grad_(False)
        self.bn1.bias.requires_grad_(False)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1, ceil_mode=True)
        self.layer1 = self._stage(64, layers[0], 1, 1)
        self.layer2 = self._stage(128, layers[1], 2, 1)
        self.layer3 = self._stage(256, layers[2], 1, 2)
        self.layer4 = self._stage(512, layers[3], 1, 4)
        self.layer6 = ClassifierModule(2048, [6, 12, 18, 24], [6, 12, 18, 24], num_classes)

    def _stage(self, planes, blocks, stride, dilation):
        ds = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                           nn.BatchNorm2d(planes * 4))
        ds[1].weight.requires_grad_(False)
        ds[1].bias.requires_grad_(False)
        mods = [Bottleneck(self.inplanes, planes, stride, dilation, ds)]
        self.inplanes = planes * 4
        mods += [Bottleneck(self.inplanes, planes, dilation=dilation) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x):
        H, W = x.shape[-2:]
        x = self.maxpool(F.relu(self.bn1(self.conv1(x))))
        x = self.layer6(self.layer4(self.layer3(self.layer2(self.layer1(x)))))
        x = F.interpolate(x, size=(H, W), mode="bilinear")
        return (x, None, None) if self.training else x


# --------------------------------------------------------------------------- discriminators
class TinyDomainDiscriminator(nn.Module):
    """conv 19->64 k4s2p1 -> LeakyReLU(0.2) -> conv 64->1 k4s2p1 -> GAP
    (reference models/domain_shift/adversarial/model.py:67-83)."""

    def __init__(self, num_classes=19):
        super().__init__()
        self.conv1 = nn.Conv2d(num_classes, 64, 4, 2, 1)
        self.classifier = nn.Conv2d(64, 1, 4, 2, 1)
        self.leaky_relu = nn.LeakyReLU(0.2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))

    def forward(self, x):
        return self.classifier(F.leaky_relu(self.conv1(x), 0.2)).mean((2, 3), keepdim=True)


class DomainDiscriminator(nn.Module):
    """5 k4s2p1 convs 19->64->128->256->512->1 + LeakyReLU(0.2) + GAP, optional GRL
    (model.py:30-64)."""

    def __init__(self, num_classes=19, with_grl=False, lambda_=0.1):
        super().__init__()
        self.with_grl = with_grl
        self.lambda_ = lambda_
        self.conv1 = nn.Conv2d(19, 64, 4, 2, 1)
        self.conv2 = nn.Conv2d(64, 128, 4, 2, 1)
        self.conv3 = nn.Conv2d(128, 256, 4, 2, 1)
        self.conv4 = nn.Conv2d(256, 512, 4, 2, 1)
        self.classifier = nn.Conv2d(512, 1, 4, 2, 1)
        self.leaky_relu = nn.LeakyReLU(0.2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))

    def forward(self, x):
        for c in (self.conv1, self.conv2, self.conv3, self.conv4):
            x = F.leaky_relu(c(x), 0.2)
        x = self.classifier(x).mean((2, 3), keepdim=True)
        if self.with_grl:
            x = _GRL.apply(x, self.lambda_)
        return x


class _GRL(torch.autograd.Function):
    """Gradient reversal: identity forward, -alpha * grad backward (model.py:9-17)."""

    @staticmethod
    def forward(ctx, x, alpha):
        ctx.alpha = alpha
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return -ctx.alpha * g, None


class UpSampler(nn.Module):
    """x8 bilinear (align_corners=False) -> 1x1 conv with bias (model.py:19-28)."""

    def __init__(self, num_classes):
        super().__init__()
        self.conv = nn.Conv2d(num_classes, num_classes, kernel_size=1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=8, mode="bilinear"))
