"""BiSeNet on the MI355X kernels -- drop-in for the reference's models/bisenet/build_bisenet.py.

Same classes, constructor arguments, attribute names (including the reference's
``saptial_path`` spelling), ``state_dict`` keys and train/eval output contract
(build_bisenet.py:141-172: training -> (result, cx1_sup, cx2_sup), eval -> result).
The forward runs NHWC in the runtime compute dtype with these fusions:
conv epilogues carry bias + ReLU/sigmoid, BatchNorm carries ReLU / sigmoid (ARM) and the
cat / channel-attention scaling are single kernels.  Input: NCHW fp32 images on a HIP
device; outputs: [N, num_classes, H, W] tensors in channels_last memory.
"""
import torch
from torch import nn

from rtsds_amd import functional as F
from rtsds_amd.nn import AdaptiveAvgPool2d, BatchNorm2d, Conv2d, ReLU, Sigmoid, _shadow, conv_bn, to_input
from rtsds_amd.runtime import BranchOut, branch_stream, branches_enabled

from .build_contextpath import build_contextpath


class ConvBlock(torch.nn.Module):
    """conv(no bias) -> BN -> ReLU (build_bisenet.py:8-18); BN+ReLU fused."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=2, padding=1):
        super().__init__()
        self.conv1 = Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                            padding=padding, bias=False)
        self.bn = BatchNorm2d(out_channels)
        self.relu = ReLU()

    def forward(self, input, out=None):
        """``out``: inference only, a destination channel slice (nn.conv_bn)."""
        return conv_bn(self.conv1, self.bn, input, "relu", out=out)


class Spatial_path(torch.nn.Module):
    """build_bisenet.py:21-32."""

    def __init__(self):
        super().__init__()
        self.convblock1 = ConvBlock(in_channels=3, out_channels=64)
        self.convblock2 = ConvBlock(in_channels=64, out_channels=128)
        self.convblock3 = ConvBlock(in_channels=128, out_channels=256)

    def forward(self, input, out=None):
        return self.convblock3(self.convblock2(self.convblock1(input)), out=out)


class AttentionRefinementModule(torch.nn.Module):
    """GAP -> 1x1 conv(bias) -> BN -> sigmoid -> x*a (build_bisenet.py:35-53).
    BN+sigmoid fused; BN statistics are over the N pooled vectors, as in the reference."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = Conv2d(in_channels, out_channels, kernel_size=1)
        self.bn = BatchNorm2d(out_channels)
        self.sigmoid = Sigmoid()
        self.in_channels = in_channels
        self.avgpool = AdaptiveAvgPool2d(output_size=(1, 1))

    def attention(self, input, pooled=None, join=None, pooled_join=None):
        """sigmoid(BN(conv(GAP(input)))) [N, C, 1, 1]; ``pooled``: GAP(input) when the caller
        already has it (BiSeNet's ARM2 reads the context path's tail, the same kernel on the
        same tensor); ``join``: GradJoin of input's two readers (the pool and the scale);
        ``pooled_join``: GradJoin of the caller's pooled tensor's readers."""
        if pooled is None:
            pooled = F.global_avg_pool(input, join)
        assert self.in_channels == pooled.size(1), \
            "in_channels and out_channels should all be {}".format(pooled.size(1))
        return conv_bn(self.conv, self.bn, pooled, "sigmoid", join=pooled_join)

    def forward(self, input, pooled=None, join=None, pooled_join=None):
        """``join``: the caller's GradJoin of input's readers (with ``pooled``: the pool that
        made it and this scale; without: this module's pool and scale plus the caller's other
        readers).  ``pooled_join``: see attention()."""
        # input's two readers (the pool and the scale) share one gradient buffer: the pool's
        # backward adds into the scale's (no autograd sum of two full-size gradients)
        if pooled is None and join is None:
            join = F.GradJoin(2) if torch.is_grad_enabled() and input.requires_grad else None
        att = self.attention(input, pooled, join if pooled is None else None, pooled_join)
        return F.channel_scale(input, att, join=join)


class FeatureFusionModule(torch.nn.Module):
    """build_bisenet.py:56-81: cat -> ConvBlock(s1) -> GAP -> 1x1+ReLU -> 1x1+sigmoid -> f*a + f."""

    # with autograd: the attention (two pooled 1x1 convs) as functional.PooledMlpFn, whose
    # backward is one launch instead of six (False: the per-conv chain, for A/B tests)
    fused_attention = True

    def __init__(self, num_classes, in_channels):
        super().__init__()
        self.in_channels = in_channels
        self.convblock = ConvBlock(in_channels=self.in_channels, out_channels=num_classes, stride=1)
        self.conv1 = Conv2d(num_classes, num_classes, kernel_size=1)
        self.relu = ReLU()
        self.conv2 = Conv2d(num_classes, num_classes, kernel_size=1)
        self.sigmoid = Sigmoid()
        self.avgpool = AdaptiveAvgPool2d(output_size=(1, 1))

    def forward(self, input_1, input_2=None, joins=None):
        # input_2 may be the (cx1, cx2) pair itself: one concat pass instead of the
        # reference's nested cat (build_bisenet.py:153 then :72), same channel order.
        # joins: GradJoin per concatenated input (functional.cat).  input_2 None: input_1 is
        # the concatenation already (BiSeNet's inference path writes it in place).
        if input_2 is None:
            x = input_1
        else:
            parts = [input_1, *input_2] if isinstance(input_2, (tuple, list)) else [input_1, input_2]
            x = F.cat(parts, joins)
        assert self.in_channels == x.size(1), \
            "in_channels of ConvBlock should be {}".format(x.size(1))
        feature = self.convblock(x)
        join = F.GradJoin(2) if torch.is_grad_enabled() and feature.requires_grad else None  # see ARM.forward
        pooled = F.global_avg_pool(feature, join)
        if self.fused_attention and torch.is_grad_enabled() and pooled.is_cuda and \
                F.pooled_mlp_ok(pooled, self.conv1.out_channels, self.conv2.out_channels):
            # the attention's backward in one launch (functional.PooledMlpFn)
            att = F.pooled_mlp(pooled, self.conv1.weight, self.conv1.bias, _shadow(self.conv1.weight, pooled.dtype),
                               self.conv2.weight, self.conv2.bias, _shadow(self.conv2.weight, pooled.dtype))
        else:
            att = self.conv2(self.conv1(pooled, act="relu"), act="sigmoid")
        return F.channel_scale(feature, att, residual=True, join=join)


_HEADS = {"resnet18": (256, 512), "resnet101": (1024, 2048)}


class BiSeNet(torch.nn.Module):
    """build_bisenet.py:84-172."""

    # training: spatial path on runtime.branch_stream beside the context path (bs 8 train step
    # +2.5 %; at inference the fork / join edges cost more than the overlap gains)
    branch_parallel = True
    # the spatial path starts at the fork point (an event after layer1) but is enqueued after the
    # whole context path: its autograd nodes then carry the highest sequence numbers, so the
    # engine enqueues its backward right after the fusion module's, ahead of the context path's
    # layer4..2 backward (the graph's dependencies are the same either way; the multi-queue
    # replay submits nodes in capture order): bs-8 step +0.25 % (profiles/r5ar_spatial_order_ab.txt)
    spatial_enqueued_last = True
    # inference (eval, no autograd): resizes written into the fusion module's concatenated input
    # and the attention tail + final 1x1 conv fused (False: the separate ops, for A/B tests)
    inference_fusions = True
    # forward() starts with nn.to_input: runtime.GraphedForward may capture from the packed input
    accepts_packed_input = True
    # the spatial path's last ConvBlock writes straight into the fusion module's concatenated
    # input and, in training, its BatchNorm backward reads its gradient slice in place (no copy
    # of the 256-channel map or its gradient)
    spatial_into_concat = True
    # training: the tensors read by two modules share one gradient buffer (functional.GradJoin
    # first_returns) instead of autograd's add: cx1 / cx2 (supervision conv, fusion-module
    # resize) and the tail (ARM2's attention conv, cx2's scale)
    feature_joins = True

    def __init__(self, num_classes, context_path, with_interpolation=True):
        super().__init__()
        self.with_interpolation = with_interpolation
        self.saptial_path = Spatial_path()
        self.context_path = build_contextpath(name=context_path)
        if context_path not in _HEADS:
            print("Error: unspport context_path network \n")
        c3, c4 = _HEADS.get(context_path, (256, 512))
        self.attention_refinement_module1 = AttentionRefinementModule(c3, c3)
        self.attention_refinement_module2 = AttentionRefinementModule(c4, c4)
        self.supervision1 = Conv2d(in_channels=c3, out_channels=num_classes, kernel_size=1)
        self.supervision2 = Conv2d(in_channels=c4, out_channels=num_classes, kernel_size=1)
        self.feature_fusion_module = FeatureFusionModule(num_classes, 256 + c3 + c4)
        self.conv = Conv2d(in_channels=num_classes, out_channels=num_classes, kernel_size=1)
        self.init_weight()
        self.mul_lr = [self.saptial_path, self.attention_refinement_module1,
                       self.attention_refinement_module2, self.supervision1, self.supervision2,
                       self.feature_fusion_module, self.conv]

    def init_weight(self):
        """kaiming fan_in on every conv outside the context path; BN 1/0 (build_bisenet.py:130-139)."""
        for name, m in self.named_modules():
            if "context_path" in name:
                continue
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_in", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                m.eps, m.momentum = 1e-5, 0.1
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _heads(self, input, main_only=False):
        """Everything up to the final resizes: [(low-res logits, resize geometry), ...] --
        the main head (conv before up8, see below) then, in training, the two supervision
        heads (build_bisenet.py:151-166).  main_only: skip the supervision heads (1x1 convs
        with no state; for callers that discard them, e.g. the DA target branch)."""
        x = to_input(input)
        # the fusion module's concatenated input, allocated up front: the spatial path's last
        # ConvBlock writes its channel slice in place (nn.conv_bn out=; inference: the folded conv
        # epilogue, training: the BatchNorm apply), the context resizes the rest
        into = None
        if self.spatial_into_concat and x.is_cuda:
            h8, w8 = x.shape[-2], x.shape[-1]
            for _ in range(3):  # three 3x3 stride-2 pad-1 convs
                h8, w8 = (h8 - 1) // 2 + 1, (w8 - 1) // 2 + 1
            into = F.empty_nhwc(x.shape[0], self.feature_fusion_module.in_channels, h8, w8, x.dtype, x.device)
        # the 1/32 features have two readers, the context path's GAP (the tail) and ARM2's scale:
        # one gradient buffer (functional.GradJoin).  Only when ARM2 runs with autograd below.
        j4 = F.GradJoin(2) if self.training and torch.is_grad_enabled() else None
        # the tail's readers (ARM2's attention conv, cx2's scale); not the 1/16 features' two
        # (layer4, ARM1): joining those would regroup the bf16 roundings of four contributions
        fj = self.training and torch.is_grad_enabled() and self.feature_joins
        jt = F.GradJoin(0, first_returns=True) if fj else None
        if self.branch_parallel and self.training and x.is_cuda and F.CONV_PROFILE is None and branches_enabled():
            # (not while bench.py event-times each conv: concurrent branches would inflate them)
            # spatial path on the branch stream, concurrently with the context path (forward and,
            # through autograd's per-op streams, backward); joined before the fusion module
            main = torch.cuda.current_stream(x.device)
            side = branch_stream(x.device)
            box = []

            def run_spatial():
                x.record_stream(side)  # read (and saved for backward) on the branch stream
                if into is not None:
                    into.record_stream(side)
                with torch.cuda.stream(side):
                    box.append(BranchOut.apply(self.saptial_path(x, out=None if into is None else (into, 0)), main, side))

            def fork():  # after the context path's layer1 (_ContextPath.fork_after): beside its later layers
                if self.spatial_enqueued_last:
                    ev = torch.cuda.Event()
                    ev.record(main)
                    box.append(ev)
                else:
                    side.wait_stream(main)
                    run_spatial()
            f3, f4, tail = self.context_path(x, mid=fork, tail_join=j4)
            if self.spatial_enqueued_last:
                side.wait_event(box.pop())
                run_spatial()
            sx = box[0]
            main.wait_stream(side)
            sx.record_stream(main)
        else:
            sx = self.saptial_path(x, out=None if into is None else (into, 0))
            f3, f4, tail = self.context_path(x, tail_join=j4)
        hw = sx.shape[-2:]
        heads = []
        cat = None
        infer = self.inference_fusions and not self.training and not torch.is_grad_enabled() and \
            sx.shape[1] + f3.shape[1] + f4.shape[1] == self.feature_fusion_module.in_channels
        if infer:
            # inference: the attention refinements' channel scales and the two resizes write
            # straight into the fusion module's concatenated input (the reference: scale, scale,
            # interpolate, interpolate, cat); ARM2's global average pool is the tail itself
            att1 = self.attention_refinement_module1.attention(f3)
            att2 = self.attention_refinement_module2.attention(f4, pooled=tail)
            cat = F.concat_resized_scaled_eval(sx, ((f3, (att1,)), (f4, (att2, tail))), hw, into=into)
        if cat is None:
            cx1 = self.attention_refinement_module1(f3)
            # ARM2's global average pool is the tail itself (same kernel, same f4)
            cx2 = F.channel_scale(self.attention_refinement_module2(f4, pooled=tail, join=j4, pooled_join=jt), tail,
                                  join_a=jt)
        if infer:
            if cat is None:  # a geometry outside the fused resize
                cat = F.concat_resized(sx, (cx1, cx2), hw)
            ffm = self.feature_fusion_module
            if self.with_interpolation and ffm.conv1.out_channels == 19 and \
                    (hw[0] * hw[1]) % (8 if sx.dtype == torch.bfloat16 else 4) == 0 and \
                    all(m.kernel_size == (1, 1) and m.in_channels == m.out_channels == ffm.conv1.in_channels
                        for m in (ffm.conv1, ffm.conv2, self.conv)):
                # attention tail + final 1x1 conv as one launch (functional.ffm_head_eval)
                feature = ffm.convblock(cat)
                ws = [_shadow(m.weight, feature.dtype) for m in (ffm.conv1, ffm.conv2, self.conv)]
                main = F.ffm_head_eval(feature, ws[0], ffm.conv1.bias, ws[1], ffm.conv2.bias, ws[2], self.conv.bias)
                return [(main, F.upsample_geometry(main, scale_factor=8))]
            result = ffm(cat)
            if self.with_interpolation:
                main = self.conv(result)
                return [(main, F.upsample_geometry(main, scale_factor=8))]
            return [(result, None)]
        aux_on = self.training and not main_only
        j1 = j2 = None
        if aux_on:
            # reference: supervision_i(interpolate(cx_i)) (build_bisenet.py:151-152, 156-157).  The
            # 1x1 conv commutes with the bilinear resize (as the main head's, below), so each
            # supervision conv runs on the un-resized map -- 1/4 (cx1) and 1/16 (cx2) of the
            # pixels, without reading the resized 256 / 512-channel maps -- and its 19-channel
            # output is resized instead; the loss then resizes it to full resolution as before.
            # cx1 / cx2 also feed the fusion module's resizes: one gradient buffer each, the
            # supervision conv's data gradient accumulating into the resize adjoint's (or the
            # reverse), instead of autograd's add of two full gradients; first_returns: correct
            # also when a caller leaves the supervision outputs out of its loss
            if torch.is_grad_enabled() and self.feature_joins:
                j1 = F.GradJoin(2, first_returns=True) if cx1.requires_grad else None
                j2 = F.GradJoin(2, first_returns=True) if cx2.requires_grad else None
            full = input.shape[-2:]
            s1 = F.interpolate_bilinear(self.supervision1(cx1, join=j1), size=hw)
            s2 = F.interpolate_bilinear(self.supervision2(cx2, join=j2), size=hw)
            aux = [(s1, F.upsample_geometry(s1, size=full)), (s2, F.upsample_geometry(s2, size=full))]
        # the two resizes write straight into the fusion module's concatenated input and read
        # their gradients straight from its gradient (functional.CatResizeFn; the reference:
        # interpolate, interpolate, cat)
        result = self.feature_fusion_module(F.concat_resized(sx, (cx1, cx2), hw, joins=(j1, j2), into=into))
        if self.with_interpolation:
            # reference: conv(up8(result)) (build_bisenet.py:165-167).  A 1x1 conv mixes channels
            # per pixel and bilinear resize mixes pixels per channel with weights summing to 1,
            # so up8(conv(result)) is the same function (bias included) at 1/64 of the conv work
            # and without the full-resolution intermediate.
            main = self.conv(result)
            heads.append((main, F.upsample_geometry(main, scale_factor=8)))
        else:
            heads.append((result, None))
        if aux_on:
            heads += aux
        return heads

    def forward_lowres(self, input, main_only=False):
        """Training-loop entry used by rtsds_amd.train: the heads before their final bilinear
        resize, so the resize can be fused into the loss (functional.upsample_cross_entropy).
        forward() is exactly these heads, resized."""
        return self._heads(input, main_only)

    def forward(self, input):
        outs = [t if geo is None else F.interpolate_geometry(t, geo) for t, geo in self._heads(input)]
        if self.training:
            return tuple(outs)
        return outs[0]
