"""DeepLabV2 (ResNet-101 + ASPP) on the MI355X kernels -- drop-in for the reference's
models/deeplabv2/deeplabv2.py.

Caffe-style bottlenecks (stride on the first 1x1, deeplabv2.py:13), BN with frozen affine but
train-mode batch statistics (deeplabv2.py:14-27), ceil-mode max pool (:79), atrous layer3/4
(:82-83), ASPP as the sum of four dilated 3x3 convs (:50-66) computed as ONE accumulating
output buffer, bilinear upsampling to the input size (:126).  Training returns
(x, None, None) (:128-129).
"""
import torch
import torch.nn as nn

from rtsds_amd import functional as F
from rtsds_amd.functional import BnBwdLink
from rtsds_amd.nn import BatchNorm2d, Conv2d, MaxPool2d, ReLU, conv_bn, conv_bn_relu_maxpool, grad_join, to_input
from rtsds_amd.nn import _shadow
from rtsds_amd.runtime import grad_cut

affine_par = True


def _freeze(bn):
    for p in bn.parameters():
        p.requires_grad = False
    return bn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, dilation=1, downsample=None):
        super(Bottleneck, self).__init__()
        self.conv1 = Conv2d(inplanes, planes, kernel_size=1, stride=stride, bias=False)
        self.bn1 = _freeze(BatchNorm2d(planes, affine=affine_par))
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=1, padding=dilation, bias=False,
                            dilation=dilation)
        self.bn2 = _freeze(BatchNorm2d(planes, affine=affine_par))
        self.conv3 = Conv2d(planes, planes * 4, kernel_size=1, bias=False)
        self.bn3 = _freeze(BatchNorm2d(planes * 4, affine=affine_par))
        self.relu = ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        # x's two readers accumulate their gradients into one buffer (nn.grad_join)
        join = grad_join(x, 2)
        skip = x if self.downsample is None else conv_bn(self.downsample[0], self.downsample[1], x, join=join)
        l1, l2 = BnBwdLink(), BnBwdLink()  # bn1 -> conv2, bn2 -> conv3 (single readers)
        t = conv_bn(self.conv1, self.bn1, x, "relu", join=join, out_link=l1)
        t = conv_bn(self.conv2, self.bn2, t, "relu", in_link=l1, out_link=l2)
        return conv_bn(self.conv3, self.bn3, t, "relu", skip,
                       res_join=join if self.downsample is None else None, in_link=l2)


class ClassifierModule(nn.Module):
    """ASPP (deeplabv2.py:50-66): out = sum_i conv_i(x), dilation = padding = 6/12/18/24."""

    def __init__(self, inplanes, dilation_series, padding_series, num_classes):
        super(ClassifierModule, self).__init__()
        self.conv2d_list = nn.ModuleList()
        for dilation, padding in zip(dilation_series, padding_series):
            self.conv2d_list.append(Conv2d(inplanes, num_classes, kernel_size=3, stride=1,
                                           padding=padding, dilation=dilation, bias=True))
        for m in self.conv2d_list:
            m.weight.data.normal_(0, 0.01)

    def forward(self, x):
        convs = list(self.conv2d_list)
        geoms = tuple((c.stride, c.padding, c.dilation) for c in convs)
        ws = [c.weight for c in convs]
        bs = [c.bias for c in convs]
        wqs = [_shadow(c.weight, x.dtype) for c in convs]
        return F.ConvSumFn.apply(x, geoms, *ws, *bs, *wqs)


class ResNetMulti(nn.Module):
    # forward() starts with nn.to_input: runtime.GraphedForward may capture from the packed input
    accepts_packed_input = True

    def __init__(self, block, layers, num_classes):
        self.inplanes = 64
        super(ResNetMulti, self).__init__()
        self.conv1 = Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = _freeze(BatchNorm2d(64, affine=affine_par))
        self.relu = ReLU(inplace=True)
        self.maxpool = MaxPool2d(kernel_size=3, stride=2, padding=1, ceil_mode=True)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=1, dilation=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=1, dilation=4)
        self.layer6 = ClassifierModule(2048, [6, 12, 18, 24], [6, 12, 18, 24], num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                m.weight.data.normal_(0, 0.01)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        self.multi_level = False

    def _make_layer(self, block, planes, blocks, stride=1, dilation=1):
        # deeplabv2.py:94-97 -- every stage of this network satisfies the condition
        down = nn.Sequential(
            Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
            _freeze(BatchNorm2d(planes * block.expansion, affine=affine_par)))
        layers = [block(self.inplanes, planes, stride, dilation=dilation, downsample=down)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, dilation=dilation))
        return nn.Sequential(*layers)

    def forward_lowres(self, x, main_only=False):
        """[(stride-8 logits, resize geometry)] -- forward() before its final bilinear resize
        (deeplabv2.py:126), so the training loop can fuse the resize into the loss."""
        _, _, H, W = x.size()
        t = to_input(x)
        t = conv_bn_relu_maxpool(self.conv1, self.bn1, self.maxpool, t)
        # runtime.grad_cut: under data parallelism the backward runs in phases split at layer2's
        # output, the middle of layer3 (23 blocks) and layer3's output, so G's 175 MB gradient
        # arena is all-reduced in ~4 buckets while the backward proceeds
        t = grad_cut(self.layer2(self.layer1(t)))
        for i, blk in enumerate(self.layer3):
            t = blk(t)
            if i == len(self.layer3) // 2:
                t = grad_cut(t)
        t = self.layer4(grad_cut(t))
        t = self.layer6(t)
        return [(t, F.upsample_geometry(t, size=(H, W)))]

    def forward(self, x):
        (t, geo), = self.forward_lowres(x)
        t = F.interpolate_geometry(t, geo)
        if self.training == True:  # noqa: E712  (reference contract, deeplabv2.py:128)
            return t, None, None
        return t

    def get_1x_lr_params_no_scale(self):
        for mod in (self.conv1, self.bn1, self.layer1, self.layer2, self.layer3, self.layer4):
            for m in mod.modules():
                for p in m.parameters(recurse=False):
                    if p.requires_grad:
                        yield p

    def get_10x_lr_params(self):
        for p in self.layer6.parameters():
            yield p

    def optim_parameters(self, lr):
        return [{"params": self.get_1x_lr_params_no_scale(), "lr": lr},
                {"params": self.get_10x_lr_params(), "lr": 10 * lr}]


def get_deeplab_v2(num_classes=19, pretrain=True,
                   pretrain_model_path="DeepLab_resnet_pretrained_imagenet.pth"):
    """deeplabv2.py:176-190.  The pretrained checkpoint is read with weights_only=True; keys
    lose their first dotted component (prefix stripping, deeplabv2.py:184-187)."""
    model = ResNetMulti(Bottleneck, [3, 4, 23, 3], num_classes)
    if pretrain:
        print("Deeplab pretraining loading...")
        saved = torch.load(pretrain_model_path, map_location="cpu", weights_only=True)
        new_params = model.state_dict().copy()
        for k in saved:
            new_params[".".join(k.split(".")[1:])] = saved[k]
        model.load_state_dict(new_params, strict=False)
    return model
