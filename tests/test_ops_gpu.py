"""Per-op parity of the HIP kernels against the ATen CPU ops the reference calls
(torch.nn.functional on CPU, float64) -- forward and backward.  GPU only.

Tolerances: fp32 mode (exact-f32 MFMA) max|err| <= 1e-4 * max|ref| (+ tiny abs floor);
bf16 mode 3e-2 * max|ref| (bf16 operands, fp32 accumulation).
"""
import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

from rtsds_amd import functional as F  # noqa: E402
from rtsds_amd.nn import _shadow  # noqa: E402

DEV = "cuda"
CL = torch.channels_last
TOL = {torch.float32: 2e-4, torch.bfloat16: 3e-2}


def _close(got, ref, dt, what, tol=None):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = ref.abs().max().item() + 1e-12
    err = (got - ref).abs().max().item()
    t = tol if tol is not None else TOL[dt]
    assert err <= t * scale + 1e-6, f"{what}: max err {err:.3e} vs scale {scale:.3e} (tol {t})"


def _dev(t, dt):
    return t.to(DEV, dt).contiguous(memory_format=CL)


CONV_CASES = [
    # n, c, h, w, k, kh, stride, pad, dil, bias
    (2, 3, 32, 48, 64, 7, 2, 3, 1, False),     # ResNet stem (Cin=3, scalar gather)
    (2, 3, 32, 32, 64, 3, 2, 1, 1, False),     # spatial path conv1
    (2, 64, 16, 24, 64, 3, 1, 1, 1, False),    # BasicBlock 3x3
    (2, 64, 16, 16, 128, 3, 2, 1, 1, False),   # stride-2 3x3
    (2, 64, 16, 16, 128, 1, 2, 0, 1, False),   # downsample 1x1 s2
    (2, 19, 32, 64, 64, 4, 2, 1, 1, True),     # TinyD conv1 (Cin=19)
    (2, 64, 16, 32, 1, 4, 2, 1, 1, True),      # D classifier (Cout=1)
    (1, 64, 13, 17, 64, 3, 1, 2, 2, False),    # atrous d=2, odd sizes
    (1, 128, 9, 11, 19, 3, 1, 6, 6, True),     # ASPP-like, Cout=19
    (2, 19, 16, 16, 19, 1, 1, 0, 1, True),     # final 1x1 19->19
    (8, 256, 1, 1, 256, 1, 1, 0, 1, True),     # ARM 1x1 on pooled vectors
    (8, 512, 1, 1, 512, 1, 1, 0, 1, True),     # pooled, vector kernels (16-B chunks, butterfly dgrad)
    (5, 64, 1, 1, 40, 1, 1, 0, 1, True),       # pooled vector kernels: 5 rows, k < 64 lanes
    (12, 256, 1, 1, 128, 1, 1, 0, 1, True),    # pooled: 12 rows (32-row vector fwd, scalar dgrad)
    (2, 19, 1, 1, 19, 1, 1, 0, 1, True),       # pooled, C % 8 != 0: scalar kernels (FFM attention)
    (2, 1024, 8, 16, 19, 3, 1, 1, 1, False),   # FFM conv (K=9216, N=19)
    (2, 256, 8, 8, 512, 3, 2, 1, 1, False),    # layer4 conv1
    (1, 32, 13, 17, 64, 3, 2, 1, 1, False),    # stride-2 dgrad phases, odd sizes
    (2, 8, 9, 11, 16, 4, 2, 1, 1, True),       # k4 s2 phases, odd sizes
    (2, 16, 7, 9, 32, 1, 2, 0, 1, False),      # 1x1 s2: odd phases receive nothing
    (8, 128, 64, 64, 128, 3, 1, 1, 1, False),  # 128x128 LDS-DMA tiles (fwd and dgrad)
    (2, 128, 8, 128, 19, 3, 1, 1, 1, False),   # halo direct conv (hconv.hip): Cout 19, w % 64 == 0
    (1, 64, 12, 64, 32, 3, 1, 1, 1, True),     # hconv with bias, Cout 32, edge tiles on 3 row-blocks
    (1, 256, 8, 64, 64, 3, 1, 1, 1, True),     # hconv N-tiled (Cin >= 256, Cout 2 x 32), fwd and dgrad
    (2, 256, 6, 100, 19, 3, 1, 1, 1, False),   # halo weight gradient (nwgrad): 2 channel chunks, partial column tiles
    (1, 128, 5, 64, 32, 3, 1, 1, 1, True),     # nwgrad: Cout 32 (no dY pad), odd rows, dbias
    (2, 512, 16, 32, 512, 3, 1, 1, 1, False),  # layer4-like: DGRAD split-K (128x128 tiles, fp32 slabs)
    (2, 512, 16, 32, 512, 3, 1, 2, 2, False),  # dilated (DeepLab layer3-like, small M): DGRAD split-K
    (2, 256, 16, 32, 19, 3, 1, 2, 2, True),    # ASPP-like narrow output, few M tiles: FWD split-K slabs
    (2, 512, 32, 64, 19, 1, 1, 0, 1, True),    # supervision 1x1 (pw.hip backward): 1 row group
    (2, 40, 32, 64, 32, 1, 1, 0, 1, True),     # pw.hip: Cout 32, 12 row groups
    (4, 19, 32, 32, 19, 1, 1, 0, 1, True),     # pw.hip: final 19->19, odd Cin (scalar lanes)
    (1, 1024, 64, 64, 16, 1, 1, 0, 1, False),  # pw.hip: two lane passes over 1024 channels
    # persistent implicit-GEMM launches (more tiles than resident workgroups: a workgroup walks
    # several tiles, the next tile's first K-tile DMA in flight during the epilogue):
    (8, 128, 67, 131, 128, 3, 1, 1, 1, False),  # 549 ragged 128x128 FWD / DGRAD tiles
    (24, 64, 161, 97, 128, 3, 2, 1, 1, False),  # stride 2, odd sizes: FWD 745 tiles; DGRAD's
                                                # 4 parity phases of unequal rows (tile holes)
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(case, dt):
    n, c, h, w, k, kh, s, p, d, bias = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(k, c, kh, kh, generator=g, dtype=torch.float64) / (c * kh * kh) ** 0.5
    b = torch.randn(k, generator=g, dtype=torch.float64) if bias else None
    if dt == torch.bfloat16:  # compare against the bf16-rounded operands
        x, wt = x.bfloat16().double(), wt.bfloat16().double()
    xr, wr = x.clone().requires_grad_(), wt.clone().requires_grad_()
    br = b.clone().requires_grad_() if bias else None
    yr = TF.conv2d(xr, wr, br, s, p, d)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        gy = gy.bfloat16().double()
    yr.backward(gy)

    xd = _dev(x, dt).requires_grad_()
    wp = torch.nn.Parameter(wt.float().to(DEV).contiguous(memory_format=CL))
    bp = torch.nn.Parameter(b.float().to(DEV)) if bias else None
    y = F.conv2d(xd, wp, bp, _shadow(wp, dt), (s, s), (p, p), (d, d), 0)
    y.backward(_dev(gy, dt))
    torch.cuda.synchronize()
    _close(y, yr, dt, "y")
    _close(xd.grad, xr.grad, dt, "dx")
    _close(wp.grad, wr.grad, dt, "dw")
    if bias:
        _close(bp.grad, br.grad, dt, "db")


def test_dgrad_split_k_accumulate():
    """DGRAD split-K (small-M deep conv) with the accumulate flag: dx += dgrad."""
    import ctypes
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _conv_desc, _P
    from rtsds_amd.runtime import stream, workspace

    g = torch.Generator().manual_seed(5)
    n, c, h, w, k = 2, 512, 16, 32, 512
    dy = _dev(torch.randn(n, k, h, w, generator=g), torch.bfloat16)
    wq = _dev(torch.randn(k, c, 3, 3, generator=g) / (9 * c) ** 0.5, torch.bfloat16)
    x = _dev(torch.zeros(n, c, h, w), torch.bfloat16)
    d = _conv_desc(x, k, 3, 3, (1, 1), (1, 1), (1, 1))
    dx0 = _dev(torch.randn(n, c, h, w, generator=g), torch.bfloat16)
    dx, fresh = dx0.clone(), torch.empty_like(dx0)
    ws = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
    for out, acc in ((dx, 1), (fresh, 0)):
        assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wq), _P(out), acc, _P(ws), ws.numel(), stream()) == 0
    torch.cuda.synchronize()
    ref = TF.conv_transpose2d(dy.double().cpu(), wq.double().cpu(), padding=1)
    _close(fresh, ref, torch.bfloat16, "dx")
    _close(dx, dx0.double() + fresh.double(), torch.bfloat16, "dx accum", tol=1e-2)


@pytest.mark.parametrize("geo", [(1, 128, 8, 64, 19), (1, 96, 16, 32, 32)])
def test_hconv_dgrad_accumulate(geo):
    """Narrow-output data gradient (hconv_dgrad_nt_kernel: the dY halo staged once, the output
    channel tiles streamed; 64- and 32-wide maps) with and without the accumulate flag."""
    import ctypes
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _conv_desc, _P
    from rtsds_amd.runtime import stream, workspace

    n, c, h, w, k = geo
    g = torch.Generator().manual_seed(11)
    dy = _dev(torch.randn(n, k, h, w, generator=g), torch.bfloat16)
    wq = _dev(torch.randn(k, c, 3, 3, generator=g) / (9 * c) ** 0.5, torch.bfloat16)
    x = _dev(torch.zeros(n, c, h, w), torch.bfloat16)
    d = _conv_desc(x, k, 3, 3, (1, 1), (1, 1), (1, 1))
    dx0 = _dev(torch.randn(n, c, h, w, generator=g), torch.bfloat16)
    dx, fresh = dx0.clone(), torch.empty_like(dx0)
    ws = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
    for out, acc in ((dx, 1), (fresh, 0)):
        assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wq), _P(out), acc, _P(ws), ws.numel(), stream()) == 0
    torch.cuda.synchronize()
    ref = TF.conv_transpose2d(dy.double().cpu(), wq.double().cpu(), padding=1)
    _close(fresh, ref, torch.bfloat16, "dx")
    _close(dx, dx0.double() + fresh.double(), torch.bfloat16, "dx accum", tol=1e-2)


def test_fwd_split_k_accumulate():
    """FWD split-K (narrow output, few M tiles: DeepLab's ASPP branches) with bias and the
    accumulate flag (ConvSum: y += conv + bias), against the non-accumulating call."""
    import ctypes
    from rtsds_amd._lib import ACCUMULATE, lib
    from rtsds_amd.functional import _conv_desc, _P
    from rtsds_amd.runtime import stream, workspace

    g = torch.Generator().manual_seed(7)
    n, c, h, w, k = 2, 512, 13, 21, 19
    x = _dev(torch.randn(n, c, h, w, generator=g), torch.bfloat16)
    wq = _dev(torch.randn(k, c, 3, 3, generator=g) / (9 * c) ** 0.5, torch.bfloat16)
    b = torch.randn(k, generator=g).to(DEV)
    d = _conv_desc(x, k, 3, 3, (1, 1), (4, 4), (4, 4))
    y0 = _dev(torch.randn(n, k, h, w, generator=g), torch.bfloat16)
    y, fresh = y0.clone(), torch.empty_like(y0)
    ws = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), x.device)
    for out, acc in ((y, ACCUMULATE), (fresh, 0)):
        assert lib.rtsds_conv2d_fwd(ctypes.byref(d), _P(x), _P(wq), _P(b), _P(out), acc, None, _P(ws), ws.numel(),
                                    stream()) == 0
    torch.cuda.synchronize()
    ref = TF.conv2d(x.double().cpu(), wq.double().cpu(), b.double().cpu(), padding=4, dilation=4)
    _close(fresh, ref, torch.bfloat16, "y")
    _close(y, y0.double() + fresh.double(), torch.bfloat16, "y accum", tol=1e-2)


@pytest.mark.parametrize("hw", [(32, 64), (33, 63)])
@pytest.mark.parametrize("c", [512, 256, 19])
def test_pw_backward_accumulate(c, hw):
    """Narrow 1x1 backward with the accumulate flag (pw.hip dgrad, split-K GEMM wgrad): dx +=
    dgrad, dw/db += wgrad (the flat-arena gradient sink and ConvSum paths), checked against the
    non-accumulating call plus the prior contents (dx: bit-identical to adding the two bf16
    gradients, as autograd would; 33 x 63 leaves a partial pixel tile); the weight gradient
    against fp64, and for the 19-channel input also from the 32-channel padded image
    (RTSDS_INPUT_PADDED)."""
    import ctypes
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _conv_desc, _P
    from rtsds_amd.runtime import stream, workspace

    g = torch.Generator().manual_seed(c)
    n, (h, w), k = 2, hw, 19
    x = _dev(torch.randn(n, c, h, w, generator=g), torch.bfloat16)
    dy = _dev(torch.randn(n, k, h, w, generator=g), torch.bfloat16)
    wq = _dev(torch.randn(k, c, 1, 1, generator=g) / c ** 0.5, torch.bfloat16)
    d = _conv_desc(x, k, 1, 1, (1, 1), (0, 0), (1, 1))
    dx0 = _dev(torch.randn(n, c, h, w, generator=g), torch.bfloat16)
    dx = dx0.clone()
    dx_fresh = torch.empty_like(dx0)
    ws = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
    assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wq), _P(dx), 1, _P(ws), ws.numel(), stream()) == 0
    assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wq), _P(dx_fresh), 0, _P(ws), ws.numel(), stream()) == 0
    dw0 = torch.randn(k, c, generator=g).to(DEV)
    db0 = torch.randn(k, generator=g).to(DEV)
    dw, db = dw0.clone(), db0.clone()
    dw_f, db_f = torch.empty_like(dw0), torch.empty_like(db0)
    ws = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), x.device)
    for out_w, out_b, acc in ((dw, db, 1), (dw_f, db_f, 0)):
        assert lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(x), _P(dy), _P(out_w), _P(out_b), acc, _P(ws), ws.numel(),
                                      stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(dx, dx0 + dx_fresh)
    ref_dx = torch.einsum("nkhw,kc->nchw", dy.double(), wq.double().reshape(k, c))
    _close(dx_fresh, ref_dx, torch.bfloat16, "dx", tol=1e-2)
    _close(dw, dw0.double() + dw_f.double(), torch.float32, "dw accum", tol=1e-5)
    _close(db, db0.double() + db_f.double(), torch.float32, "db accum", tol=1e-5)
    ref_w = torch.einsum("nkhw,nchw->kc", dy.double(), x.double())
    _close(dw_f, ref_w, torch.float32, "dw", tol=1e-4)
    _close(db_f, dy.double().sum((0, 2, 3)), torch.float32, "db", tol=1e-4)
    if c % 8:
        xp = torch.nn.functional.pad(x.permute(0, 2, 3, 1), (0, 32 - c)).contiguous()  # NHWC, pitch 32
        dw_p, db_p = torch.empty_like(dw0), torch.empty_like(db0)
        assert lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(xp), _P(dy), _P(dw_p), _P(db_p), 0x400, _P(ws), ws.numel(),
                                      stream()) == 0
        torch.cuda.synchronize()
        assert torch.equal(dw_p, dw_f) and torch.equal(db_p, db_f)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_conv_fused_act(dt, act):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 12, 12, generator=g, dtype=torch.float64)
    wt = torch.randn(32, 64, 3, 3, generator=g, dtype=torch.float64) / 24
    b = torch.randn(32, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x, wt = x.bfloat16().double(), wt.bfloat16().double()
    xr, wr, br = x.clone().requires_grad_(), wt.clone().requires_grad_(), b.clone().requires_grad_()
    yr = TF.conv2d(xr, wr, br, 1, 1)
    yr = [yr, TF.relu(yr), TF.leaky_relu(yr, 0.2)][act]
    yr.sum().backward()
    xd = _dev(x, dt).requires_grad_()
    wp = torch.nn.Parameter(wt.float().to(DEV).contiguous(memory_format=CL))
    bp = torch.nn.Parameter(b.float().to(DEV))
    y = F.conv2d(xd, wp, bp, _shadow(wp, dt), (1, 1), (1, 1), (1, 1), act)
    y.backward(torch.ones_like(y))
    _close(y, yr, dt, "y")
    _close(xd.grad, xr.grad, dt, "dx")
    _close(wp.grad, wr.grad, dt, "dw")
    _close(bp.grad, br.grad, dt, "db")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,act,res", [((4, 64, 8, 12), 1, False), ((2, 128, 5, 7), 1, True),
                                           ((8, 512, 1, 1), 3, False), ((2, 19, 9, 9), 1, False),
                                           ((3, 2048, 3, 3), 0, True), ((2, 24, 7, 9), 2, False),
                                           ((8, 64, 48, 64), 1, False), ((4, 32, 40, 40), 2, True)])
def test_batchnorm_train(shape, act, res, dt):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(shape, generator=g, dtype=torch.float64) * 3 + 50  # large mean
    r = torch.randn(shape, generator=g, dtype=torch.float64)
    c = shape[1]
    gam = 1 + 0.1 * torch.randn(c, generator=g, dtype=torch.float64)
    bet = 0.1 * torch.randn(c, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x, r = x.bfloat16().double(), r.bfloat16().double()
    rm0 = 0.1 * torch.randn(c, generator=g, dtype=torch.float64)
    rv0 = 1 + torch.rand(c, generator=g, dtype=torch.float64)
    xr, gr, br = x.clone().requires_grad_(), gam.clone().requires_grad_(), bet.clone().requires_grad_()
    rr = r.clone().requires_grad_()
    rm, rv = rm0.clone(), rv0.clone()
    gy = torch.randn(shape, generator=g, dtype=torch.float64)
    xd = _dev(x, dt).requires_grad_()
    rd = _dev(r, dt).requires_grad_() if res else None
    gp = gam.float().to(DEV).requires_grad_()
    bp = bet.float().to(DEV).requires_grad_()
    rmd, rvd = rm0.float().to(DEV), rv0.float().to(DEV)
    y = F.batch_norm(xd, gp, bp, rmd, rvd, True, 0.1, 1e-5, act, rd)
    y.backward(_dev(gy, dt))

    yr = TF.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5)
    if res:
        yr = yr + rr
    if act in (1, 2):
        # ReLU / LeakyReLU: the backward is tested under the kernel's own activation mask.
        # Pre-activations within fp32 rounding of 0 (large-mean inputs: x*scale + shift cancels
        # ~50*scale) may take either side; the fp64 reference applies the same mask, the
        # forward values are compared below within tolerance either way.
        neg = (y.detach().double().cpu() <= 0) if act == 1 else (y.detach().double().cpu() < 0)
        yr = torch.where(neg, yr * (0.0 if act == 1 else 0.2), yr)
    elif act == 3:
        yr = torch.sigmoid(yr)
    yr.backward(gy)
    tol = 5e-4 if dt == torch.float32 else None
    _close(y, yr, dt, "y", tol)
    _close(xd.grad, xr.grad, dt, "dx", 2e-3 if dt == torch.float32 else 6e-2)
    _close(gp.grad, gr.grad, dt, "dgamma", 2e-3 if dt == torch.float32 else 6e-2)
    _close(bp.grad, br.grad, dt, "dbeta", tol)
    if res:
        _close(rd.grad, rr.grad, dt, "dres", tol)
    _close(rmd, rm, torch.float32, "running_mean", 1e-4)
    _close(rvd, rv, torch.float32, "running_var", 1e-3)


@pytest.mark.parametrize("shape,ld,off", [((2, 64, 9, 13), 96, 16), ((4, 256, 8, 16), 1024, 0), ((1, 8, 3, 5), 24, 8)])
def test_batchnorm_channel_slice_bit_identical(shape, ld, off):
    """Train-mode BatchNorm + ReLU writing y into a channel slice of a wider NHWC buffer
    (batch_norm out=, rtsds_bn_fwd_ld) and reading its gradient from such a slice in place
    (rtsds_bn_bwd_ld): y, dx, dgamma, dbeta and the running statistics bit-identical to the
    dense call; the rest of the buffer untouched."""
    g = torch.Generator().manual_seed(sum(shape) + ld)
    n, c, h, w = shape
    x = _dev(torch.randn(shape, generator=g) * 2 + 3, torch.bfloat16)
    gy = torch.randn(n, ld, h, w, generator=g).to(DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gam = (1 + 0.1 * torch.randn(c, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(c, generator=g)).to(DEV)
    outs = []
    for sliced in (False, True):
        xd = x.clone().requires_grad_()
        gp, bp = gam.clone().requires_grad_(), bet.clone().requires_grad_()
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        buf = None
        if sliced:
            buf = torch.full((n, ld, h, w), 7.0, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = F.batch_norm(xd, gp, bp, rm, rv, True, 0.1, 1e-5, 1, None, out=None if buf is None else (buf, off))
        if sliced:
            assert y.data_ptr() == buf.data_ptr() + 2 * off and y.stride(3) == ld
            assert torch.equal(buf[:, :off].float(), torch.full_like(buf[:, :off].float(), 7.0))
            assert torch.equal(buf[:, off + c:].float(), torch.full_like(buf[:, off + c:].float(), 7.0))
        y.backward(gy[:, off:off + c] if sliced else gy[:, off:off + c].contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
        outs.append([t.detach().float().cpu() for t in (y, xd.grad, gp.grad, bp.grad, rm, rv)])
    for a, b_, what in zip(outs[0], outs[1], ("y", "dx", "dgamma", "dbeta", "running_mean", "running_var")):
        assert torch.equal(a, b_), what


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_batchnorm_eval(dt):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 6, 6, generator=g, dtype=torch.float64)
    rm, rv = torch.randn(64, generator=g, dtype=torch.float64), 1 + torch.rand(64, generator=g, dtype=torch.float64)
    gam, bet = torch.randn(64, generator=g, dtype=torch.float64), torch.randn(64, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x = x.bfloat16().double()
    xr = x.clone().requires_grad_()
    yr = TF.relu(TF.batch_norm(xr, rm, rv, gam, bet, False, 0.1, 1e-5))
    gy = torch.randn(x.shape, generator=g, dtype=torch.float64)
    yr.backward(gy)
    xd = _dev(x, dt).requires_grad_()
    y = F.batch_norm(xd, gam.float().to(DEV), bet.float().to(DEV), rm.float().to(DEV),
                     rv.float().to(DEV), False, 0.1, 1e-5, 1, None)
    y.backward(_dev(gy, dt))
    _close(y, yr, dt, "y", 1e-4 if dt == torch.float32 else None)
    _close(xd.grad, xr.grad, dt, "dx", 1e-4 if dt == torch.float32 else None)


def test_batchnorm_module_counter():
    """num_batches_tracked is advanced by the finalize kernel in train mode only."""
    from rtsds_amd import nn as rnn
    bn = rnn.BatchNorm2d(16).to(DEV)
    x = torch.randn(2, 16, 4, 4, device=DEV).contiguous(memory_format=torch.channels_last)
    for _ in range(3):
        bn(x, act="relu")
    bn.eval()
    bn(x)
    assert int(bn.num_batches_tracked) == 3


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [(3, 2, 1, False, 17, 23), (3, 2, 1, True, 17, 23), (3, 2, 1, True, 16, 16),
                                 (3, 2, 1, False, 32, 64, "relu"), (3, 1, 1, False, 9, 12), (2, 2, 0, False, 8, 10),
                                 (3, 2, 0, False, 17, 23), (3, 2, 0, True, 16, 16), (3, 2, 1, False, 1, 5)])
def test_maxpool(geo, dt):
    """Incl. post-ReLU input (ties at 0: the first maximum in window order wins, as ATen)
    and the generic (non 3x3 / stride-2) kernels."""
    k, s, p, ceil, h, w = geo[:6]
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 8, h, w, generator=g, dtype=torch.float64)
    if len(geo) > 6:
        x = x.clamp_min(0)
    if dt == torch.bfloat16:
        x = x.bfloat16().double()
    xr = x.clone().requires_grad_()
    yr = TF.max_pool2d(xr, k, s, p, ceil_mode=ceil)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(gy)
    xd = _dev(x, dt).requires_grad_()
    y = F.max_pool2d(xd, k, s, p, ceil)
    y.backward(_dev(gy, dt))
    _close(y, yr, dt, "y", 0.0)
    _close(xd.grad, xr.grad, dt, "dx", 1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [((4, 8), (16, 32), None), ((16, 32), None, 8), ((65, 129), (512, 1024), None),
                                 ((5, 7), (9, 13), None), ((8, 8), (8, 8), None)])
def test_bilinear(geo, dt):
    (hi, wi), size, sf = geo
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 5, hi, wi, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x = x.bfloat16().double()
    xr = x.clone().requires_grad_()
    yr = TF.interpolate(xr, size=size, scale_factor=sf, mode="bilinear")
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(gy)
    xd = _dev(x, dt).requires_grad_()
    y = F.interpolate_bilinear(xd, size=size, scale_factor=sf)
    y.backward(_dev(gy, dt))
    _close(y, yr, dt, "y", 1e-5 if dt == torch.float32 else 1e-2)
    _close(xd.grad, xr.grad, dt, "dx", 1e-5 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [(16, 32, 64, 128, 64), (32, 64, 64, 128, 256), (13, 17, 97, 129, 16), (8, 8, 8, 8, 8),
                                 (32, 64, 64, 128, 19), (16, 32, 64, 128, 19), (13, 17, 97, 129, 19), (8, 8, 8, 8, 3)])
def test_bilinear_bwd_fused_bit_identical(geo, dt):
    """The one-pass backward -- bilinear_bwd_fused_vec_kernel (channel counts, dY pitch and
    offset multiples of 16 B) or, for channel counts off the vector width with a dense dY,
    bilinear_bwd_fused_kernel (the supervision heads' 19 classes) -- equals the two-pass W / H
    kernels bit for bit: the same dY read through a row pitch of c + 1 takes the two-pass
    route.  And both match torch fp64."""
    import ctypes
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _P, dcode
    from rtsds_amd.runtime import workspace
    hi, wi, ho, wo, c = geo
    n = 2
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, c, hi, wi, generator=g, dtype=torch.float64)
    gy = torch.randn(n, c, ho, wo, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        gy = gy.bfloat16().double()
    xr = x.clone().requires_grad_()
    TF.interpolate(xr, size=(ho, wo), mode="bilinear").backward(gy)
    geo_t = F.upsample_geometry(_dev(x, dt), size=(ho, wo))
    sh, sw = geo_t[2], geo_t[3]
    dy = gy.permute(0, 2, 3, 1).contiguous().to(DEV, dt)                      # pitch c
    dyp = torch.zeros(n, ho, wo, c + 1, dtype=dt, device=DEV)
    dyp[..., :c] = dy                                                         # pitch c + 1
    ws = workspace(lib.rtsds_bilinear_bwd_workspace(n, hi, wi, c, ho, wo), dy.device)
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for src, ld in ((dy, c), (dyp, c + 1)):
        dx = torch.empty(n, hi, wi, c, dtype=dt, device=DEV)
        assert lib.rtsds_bilinear_bwd(_P(src), _P(dx), n, hi, wi, c, ho, wo, sh, sw, ld, 0, dcode(dy), _P(ws), ws.numel(), st) == 0
        outs.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), int((outs[0] != outs[1]).sum())
    _close(outs[0].permute(0, 3, 1, 2), xr.grad, dt, "dx", 1e-5 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [((8, 16), None, 8), ((13, 17), (97, 129), None), ((64, 128), (512, 1024), None),
                                 ((9, 9), (9, 9), None), ((7, 5), (20, 31), None)])
def test_bilinear_narrow_channels(geo, dt):
    """19-class logits (channel count not a 16-B multiple): the row-group upsample kernel
    (bilinear_fwd_rowgroup_kernel) vs torch fp64, and bit-identical to the generic per-element
    path evaluating the same bil_mix expression (an output pitch forces that path)."""
    (hi, wi), size, sf = geo
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 19, hi, wi, generator=g, dtype=torch.float64) * 3
    if dt == torch.bfloat16:
        x = x.bfloat16().double()
    yr = TF.interpolate(x, size=size, scale_factor=sf, mode="bilinear")
    xd = _dev(x, dt)
    geo_ = F.upsample_geometry(xd, size=size, scale_factor=sf)
    y = F.interpolate_geometry(xd, geo_)
    _close(y, yr, dt, "y", 1e-5 if dt == torch.float32 else 1e-2)
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _P
    from rtsds_amd.runtime import stream
    ho, wo = yr.shape[2], yr.shape[3]
    wide = torch.zeros(2, ho, wo, 24, device=DEV, dtype=dt)
    lib.rtsds_bilinear_fwd(_P(xd), _P(wide), 2, hi, wi, 19, ho, wo, float(geo_[2]), float(geo_[3]), 24, 0,
                           0 if dt == torch.float32 else 1, stream())
    torch.cuda.synchronize()
    assert torch.equal(y.permute(0, 2, 3, 1), wide[..., :19])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [((16, 32), (32, 64)), ((8, 16), (32, 64)), ((13, 17), (50, 61)), ((9, 9), (9, 9))])
def test_bilinear_grouped_vectors(geo, dt):
    """Upsampling with 16-B channel vectors (bilinear_fwd_group_vec_kernel: taps gathered once per
    source row, all output rows of the group written from registers) vs torch fp64, into a
    pitched channel slice as the FFM concat uses it (output pitch 48, offset 16)."""
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _P
    from rtsds_amd.runtime import stream
    (hi, wi), (ho, wo) = geo
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 32, hi, wi, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x = x.bfloat16().double()
    yr = TF.interpolate(x, size=(ho, wo), mode="bilinear")
    xd = _dev(x, dt)
    y = F.interpolate_bilinear(xd, size=(ho, wo))
    _close(y, yr, dt, "y", 1e-5 if dt == torch.float32 else 1e-2)
    cat = torch.zeros(2, ho, wo, 48, device=DEV, dtype=dt)
    assert lib.rtsds_bilinear_fwd(_P(xd), _P(cat), 2, hi, wi, 32, ho, wo, hi / ho, wi / wo, 48, 16,
                                  0 if dt == torch.float32 else 1, stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(y.permute(0, 2, 3, 1), cat[..., 16:])
    assert not cat[..., :16].any()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_concat_resized_scaled_eval(dt):
    """BiSeNet eval: ARM channel scales folded into the resize taps (rtsds_bilinear_fwd_scaled)
    == channel_scale, channel_scale, concat_resized, bit for bit."""
    g = torch.Generator().manual_seed(8)
    sx = _dev(torch.randn(2, 16, 32, 64, generator=g), dt)
    f3 = _dev(torch.randn(2, 32, 16, 32, generator=g), dt)
    f4 = _dev(torch.randn(2, 64, 8, 16, generator=g), dt)
    a1, a2, t = (torch.rand(2, c, 1, 1, generator=g).to(DEV, dt) for c in (32, 64, 64))
    with torch.no_grad():
        ref = F.concat_resized(sx, (F.channel_scale(f3, a1), F.channel_scale(F.channel_scale(f4, a2), t)), (32, 64))
        got = F.concat_resized_scaled_eval(sx, ((f3, (a1,)), (f4, (a2, t))), (32, 64))
    assert got is not None
    assert torch.equal(got, ref)
    # a downsampling part is outside the fused kernel: None, the caller runs the separate ops
    big = _dev(torch.randn(2, 32, 64, 128, generator=g), dt)
    with torch.no_grad():
        assert F.concat_resized_scaled_eval(sx, ((big, (a1,)),), (32, 64)) is None


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gap_chscale_cat_act(dt):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(3, 24, 7, 9, generator=g, dtype=torch.float64)
    x2 = torch.randn(3, 16, 7, 9, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x, x2 = x.bfloat16().double(), x2.bfloat16().double()
    xr, x2r = x.clone().requires_grad_(), x2.clone().requires_grad_()
    a_r = torch.sigmoid(xr.mean((2, 3), keepdim=True))
    yr = torch.cat((xr * a_r + xr, x2r), 1)
    yr = TF.relu(yr)
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(gy)
    xd, x2d = _dev(x, dt).requires_grad_(), _dev(x2, dt).requires_grad_()
    a = F.sigmoid(F.global_avg_pool(xd))
    y = F.relu(F.cat([F.channel_scale(xd, a, residual=True), x2d]))
    y.backward(_dev(gy, dt))
    _close(y, yr, dt, "y", 1e-5 if dt == torch.float32 else 2e-2)
    _close(xd.grad, xr.grad, dt, "dx", 1e-4 if dt == torch.float32 else 5e-2)
    _close(x2d.grad, x2r.grad, dt, "dx2", 1e-6 if dt == torch.float32 else 1e-2)


@pytest.mark.parametrize("shape", [(8, 512, 16, 32), (8, 19, 64, 128), (3, 40, 33, 47)])
def test_gap_chscale_row_slices(shape):
    """Two-stage channel reductions (row-slice partials, ragged last slice, VEC 1 and 8):
    global average pool and the channel-scale weight gradient sum_hw dy * x."""
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g, dtype=torch.float64).bfloat16().double()
    a = torch.rand(shape[0], shape[1], 1, 1, generator=g, dtype=torch.float64).bfloat16().double()
    xr, ar = x.clone().requires_grad_(), a.clone().requires_grad_()
    yr = xr * ar
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64).bfloat16().double()
    yr.backward(gy)
    xd, ad = _dev(x, torch.bfloat16).requires_grad_(), a.to(DEV, torch.bfloat16).requires_grad_()
    y = F.channel_scale(xd, ad)
    y.backward(_dev(gy, torch.bfloat16))
    _close(ad.grad.reshape(ar.grad.shape), ar.grad, torch.bfloat16, "da", 1e-2)
    _close(F.global_avg_pool(xd), x.mean((2, 3), keepdim=True), torch.bfloat16, "gap", 1e-2)


@pytest.mark.parametrize("geo", [(2, 64, 32, 64, False), (2, 64, 33, 65, True), (1, 16, 20, 24, False)])
def test_bn_relu_maxpool_fused(geo):
    """The fused stem (BN train stats from the conv epilogue -> ReLU -> MaxPool 3/2/1) against
    the separate rtsds ops: pooled output and argmax bit-identical; gradients equal up to the
    bf16 rounding of the materialised pool gradient the unfused path sums in; BN buffers."""
    from rtsds_amd import nn as rnn
    n, c, h, w, ceil = geo
    g = torch.Generator().manual_seed(h * w)
    x = torch.randn(n, 3, 2 * h, 2 * w, generator=g).bfloat16()
    outs = []
    for fused in (True, False):
        torch.manual_seed(0)
        conv = rnn.Conv2d(3, c, 7, 2, 3, bias=False).to(DEV)
        bn = rnn.BatchNorm2d(c).to(DEV)
        pool = rnn.MaxPool2d(3, 2, 1, ceil_mode=ceil)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        xd = _dev(x.double(), torch.bfloat16).requires_grad_()
        if fused:
            y = rnn.conv_bn_relu_maxpool(conv, bn, pool, xd)
        else:
            y = pool(bn(conv(xd, bn_stats=True), act="relu"))
        gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(DEV, torch.bfloat16)
        y.backward(gy.contiguous(memory_format=CL))
        torch.cuda.synchronize()
        outs.append((y.detach().float().cpu(), xd.grad.float().cpu(), conv.weight.grad.cpu(), bn.weight.grad.cpu(),
                     bn.bias.grad.cpu(), bn.running_mean.cpu(), bn.running_var.cpu(), int(bn.num_batches_tracked)))
    (yf, dxf, dwf, dgf, dbf, rmf, rvf, nf), (yu, dxu, dwu, dgu, dbu, rmu, rvu, nu) = outs
    assert torch.equal(yf, yu)
    # the gather-in-BatchNorm backward entry (rtsds_bn_relu_maxpool_bwd) on the same tensors
    import ctypes
    from rtsds_amd._lib import lib
    from rtsds_amd.runtime import stream, workspace
    conv = rnn.Conv2d(3, c, 7, 2, 3, bias=False).to(DEV)
    bn = rnn.BatchNorm2d(c).to(DEV)
    with torch.no_grad():
        xc = conv(_dev(x.double(), torch.bfloat16))
        ho, wo = F.pool_out(h, 3, 2, 1, ceil), F.pool_out(w, 3, 2, 1, ceil)
        y = torch.empty((n, c, ho, wo), device=DEV, dtype=torch.bfloat16, memory_format=CL)
        idx = torch.empty((n, ho, wo, c), device=DEV, dtype=torch.uint8)
        sm, si = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
        ws = workspace(lib.rtsds_bn_workspace(n * h * w, c), xc.device)
        P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        lib.rtsds_bn_relu_maxpool_fwd(P(xc), P(y), P(idx), n, h, w, c, ho, wo, 1, P(bn.weight), P(bn.bias),
                                      P(bn.running_mean), P(bn.running_var), None, P(sm), P(si), 0.1, 1e-5, 1, None, 0,
                                      1, P(ws), ws.numel(), stream())
        dyp = torch.randn(y.shape, generator=torch.Generator().manual_seed(2)).to(DEV, torch.bfloat16)
        dyp = dyp.contiguous(memory_format=CL)
        outs2 = []
        for fusedb in (True, False):
            dx = torch.empty_like(xc)
            dg, db = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
            if fusedb:
                lib.rtsds_bn_relu_maxpool_bwd(P(dyp), P(idx), P(xc), P(dx), P(dg), P(db), n, h, w, c, ho, wo, 1,
                                              P(bn.weight), P(bn.bias), P(sm), P(si), 1, 0, 1, P(ws), ws.numel(), stream())
            else:
                gfull = torch.empty_like(xc)
                lib.rtsds_maxpool_bwd(P(dyp), P(idx), P(gfull), n, h, w, c, ho, wo, 3, 2, 1, 1, stream())
                lib.rtsds_bn_bwd(P(gfull), P(xc), None, P(dx), None, P(dg), P(db), n * h * w, c, P(bn.weight),
                                 P(bn.bias), P(sm), P(si), 1, 1, 0, 1, P(ws), ws.numel(), stream())
            outs2.append((dx.float().cpu(), dg.cpu(), db.cpu()))
        torch.cuda.synchronize()
    for a, b, nm in zip(outs2[0], outs2[1], ("dx", "dgamma", "dbeta")):
        _close(a, b.double(), torch.bfloat16, "gather-bwd " + nm, 2e-2)
    assert torch.equal(rmf, rmu) and torch.equal(rvf, rvu) and nf == nu == 1
    _close(dxf, dxu.double(), torch.bfloat16, "dx", 2e-2)
    _close(dwf, dwu.double(), torch.bfloat16, "dw", 2e-2)
    _close(dgf, dgu.double(), torch.bfloat16, "dgamma", 2e-2)
    _close(dbf, dbu.double(), torch.bfloat16, "dbeta", 2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_softmax_ce_argmax(dt):
    g = torch.Generator().manual_seed(9)
    x = torch.randn(2, 19, 12, 20, generator=g, dtype=torch.float64) * 3
    t = torch.randint(0, 20, (2, 12, 20), generator=g)
    if dt == torch.bfloat16:
        x = x.bfloat16().double()
    xr = x.clone().requires_grad_()
    lr = TF.cross_entropy(xr, t, ignore_index=19)
    sr = torch.softmax(xr, 1)
    gs = torch.randn(sr.shape, generator=g, dtype=torch.float64)
    (lr * 2.0 + (sr * gs).sum()).backward()

    xd = _dev(x, dt).requires_grad_()
    td = t.to(DEV)
    loss = F.cross_entropy(xd, td, ignore_index=19)
    s = F.softmax(xd, 1)
    loss.backward(torch.tensor(2.0, device=DEV), retain_graph=True)
    s.backward(_dev(gs, dt))
    _close(loss, lr, torch.float32, "ce", 1e-5 if dt == torch.float32 else 1e-2)
    _close(s, sr, dt, "softmax", 1e-5 if dt == torch.float32 else 1e-2)
    _close(xd.grad, xr.grad, dt, "dx", 1e-5 if dt == torch.float32 else 3e-2)

    # NCHW-strided logits work too
    xn = x.float().to(DEV).requires_grad_()
    ln = F.cross_entropy(xn, td, ignore_index=19)
    ln.backward()
    _close(ln, TF.cross_entropy(x, t, ignore_index=19), torch.float32, "ce_nchw", 1e-5)

    correct = torch.zeros(1, dtype=torch.int64, device=DEV)
    am = F.argmax_channels(_dev(x, torch.float32), td, correct)
    ref = x.argmax(1)
    assert torch.equal(am.cpu(), ref)
    assert int(correct.item()) == int((ref == t).sum())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("sizes", [((20, 40), (16, 32)), ((23, 37), (10, 13)), ((9, 9), (4, 7)),
                                   ((16, 32), (16, 32))])
def test_adaptive_avg_pool(sizes, dt):
    """F.adaptive_avg_pool2d (train.py:410,438,445) forward/backward vs ATen fp64."""
    (hi, wi), (ho, wo) = sizes
    g = torch.Generator().manual_seed(31)
    x = torch.randn(2, 19, hi, wi, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x = x.bfloat16().double()
    xr = x.clone().requires_grad_()
    yr = TF.adaptive_avg_pool2d(xr, (ho, wo))
    gy = torch.randn(yr.shape, generator=g, dtype=torch.float64)
    yr.backward(gy)
    xd = _dev(x, dt).requires_grad_()
    y = F.adaptive_avg_pool2d(xd, (ho, wo))
    y.backward(_dev(gy, dt))
    _close(y, yr, dt, "y", 1e-5 if dt == torch.float32 else None)
    _close(xd.grad, xr.grad, dt, "dx", 1e-5 if dt == torch.float32 else None)


def _upce_reference(heads, t, geo_args, ignore):
    """fp64 torch: sum_h CE(interpolate(head_h)), grads, and head-0 argmax matches."""
    hr = [h.clone().requires_grad_() for h in heads]
    ups = [TF.interpolate(h, mode="bilinear", align_corners=False, **geo_args) for h in hr]
    loss = None
    for u in ups:
        l = TF.cross_entropy(u, t, ignore_index=ignore)
        loss = l if loss is None else loss + l
    loss.backward()
    return loss.detach(), [h.grad for h in hr], int((ups[0].detach().argmax(1) == t).sum()), ups[0].detach()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [
    (2, 19, 8, 16, {"scale_factor": 8}, 3),          # BiSeNet heads, x8 (scale_factor form)
    (2, 19, 8, 16, {"size": (64, 128)}, 3),          # size form (aux heads)
    (1, 19, 13, 17, {"size": (97, 129)}, 2),         # non-integer scale, ragged tiles
    (2, 5, 7, 9, {"scale_factor": 4}, 1),            # other factor, few classes
    (1, 19, 9, 33, {"size": (72, 264)}, 1),          # several column tiles
    (2, 19, 8, 16, {"scale_factor": 8}, 2, 40.0),    # wide logit ranges (softmax shift, exp
    (2, 19, 8, 16, {"scale_factor": 8}, 1, 12.0),    # underflow of the far classes)
    (2, 19, 8, 16, {"scale_factor": 2}, 3),          # 3 heads at x2: no auxiliary wave (LDS cap)
    (2, 19, 8, 16, {"scale_factor": 2}, 2),          # 2 heads at x2: with it
    (2, 19, 8, 16, {"scale_factor": 4}, 3),          # 19 classes below x8: the tile width narrows
    (1, 19, 16, 40, {"scale_factor": 3}, 1),         # (several column tiles after narrowing)
])
def test_upsample_cross_entropy_fused(case, dt):
    """Fused resize+CE+accuracy (rtsds_upce_*) vs torch fp64 interpolate -> CrossEntropyLoss."""
    n, c, hl, wl, geo_args, k = case[:6]
    amp = case[6] if len(case) > 6 else 2.0
    g = torch.Generator().manual_seed(21)
    heads = [torch.randn(n, c, hl, wl, generator=g, dtype=torch.float64) * amp for _ in range(k)]
    if dt == torch.bfloat16:
        heads = [h.bfloat16().double() for h in heads]
    hd = [_dev(h, dt).requires_grad_() for h in heads]
    geo = F.upsample_geometry(hd[0], **geo_args)
    H, W = geo[0], geo[1]
    t = torch.randint(0, c + 1, (n, H, W), generator=g)
    t[t == c] = 255  # ignore label
    lr, gr, corr_r, up0 = _upce_reference(heads, t, geo_args, 255)
    assert F.upsample_cross_entropy_supported(hd, geo, 255)
    correct = torch.zeros(1, dtype=torch.int64, device=DEV)
    loss = F.upsample_cross_entropy(hd, t.to(DEV), geo, 255, correct)
    loss.backward(torch.tensor(1.5, device=DEV))
    _close(loss, lr, torch.float32, "loss", 1e-5 if dt == torch.float32 else 1e-4)
    for i in range(k):
        _close(hd[i].grad, gr[i] * 1.5, dt, f"dhead{i}", 1e-4 if dt == torch.float32 else 2e-2)
    # accuracy: exact against fp64 except pixels whose top-2 logits tie within fp32 noise
    top2 = up0.topk(2, dim=1).values
    near = int(((top2[:, 0] - top2[:, 1]) < 1e-4).sum())
    assert abs(int(correct.item()) - corr_r) <= near
    if dt == torch.float32:  # bit-identical to the unfused HIP chain (same taps/weights/expression)
        up = F.interpolate_geometry(_dev(heads[0], dt), geo)
        c2 = torch.zeros(1, dtype=torch.int64, device=DEV)
        F.argmax_channels(up, t.to(DEV), c2, want_map=False)
        assert int(c2.item()) == int(correct.item())


def test_upsample_cross_entropy_no_grad_and_fallback():
    x = _dev(torch.randn(2, 19, 8, 16), torch.float32)
    geo = F.upsample_geometry(x, scale_factor=8)
    t = torch.randint(0, 20, (2, 64, 128), device=DEV)
    with torch.no_grad():
        l = F.upsample_cross_entropy([x], t, geo, 19)
    ref = F.cross_entropy(F.interpolate_geometry(x, geo), t, 19)
    _close(l, ref, torch.float32, "loss", 1e-5)
    # downsampling and > 32 classes are outside the fused path
    assert not F.upsample_cross_entropy_supported([x], F.upsample_geometry(x, size=(4, 8)), 19)
    big = _dev(torch.randn(1, 40, 8, 8), torch.float32)
    assert not F.upsample_cross_entropy_supported([big], F.upsample_geometry(big, scale_factor=8), 19)


def test_bce():
    g = torch.Generator().manual_seed(6)
    x = torch.randn(8, 1, 1, 1, generator=g, dtype=torch.float64) * 4
    for tv in (0.0, 1.0):
        t = torch.full_like(x, tv)
        xr = x.clone().requires_grad_()
        lr = TF.binary_cross_entropy_with_logits(xr, t)
        lr.backward()
        xd = x.float().to(DEV).requires_grad_()
        l = F.bce_with_logits(xd, t.float().to(DEV))
        l.backward()
        _close(l, lr, torch.float32, "bce", 1e-6)
        _close(xd.grad, xr.grad, torch.float32, "dx", 1e-6)


def test_adam_matches_torch():
    from rtsds_amd._lib import lib
    from rtsds_amd.runtime import stream
    g = torch.Generator().manual_seed(8)
    p0 = torch.randn(10007, generator=g)
    grads = [torch.randn(10007, generator=g) for _ in range(3)]
    pr = p0.clone().requires_grad_()
    opt = torch.optim.Adam([pr], lr=1e-3, weight_decay=1e-4)
    pd = p0.to(DEV)
    m, v = torch.zeros_like(pd), torch.zeros_like(pd)
    sh = torch.empty(10007, dtype=torch.bfloat16, device=DEV)
    for i, gr in enumerate(grads, 1):
        pr.grad = gr.clone()
        opt.step()
        gd = gr.to(DEV)
        lib.rtsds_adam_step(pd.data_ptr(), gd.data_ptr(), m.data_ptr(), v.data_ptr(), sh.data_ptr(),
                            10007, 1e-3, 0.9, 0.999, 1e-8, 1e-4, i, 1.0, 0, stream())
    _close(pd, pr, torch.float32, "param", 1e-6)
    _close(sh.float(), pr.detach().bfloat16().float(), torch.float32, "shadow", 1e-2)


def test_confusion():
    g = torch.Generator().manual_seed(12)
    lab = torch.randint(0, 20, (3, 40, 50), generator=g)
    pred = torch.randint(0, 19, (3, 40, 50), generator=g)
    hist = torch.zeros(19 * 19, dtype=torch.int64, device=DEV)
    F.confusion(lab.to(DEV), pred.to(DEV), hist, 19)
    k = (lab >= 0) & (lab < 19)
    ref = torch.bincount(19 * lab[k] + pred[k], minlength=361)
    assert torch.equal(hist.cpu(), ref)


FOLD_CASES = [
    # n, c, h, w, k, kh, stride, pad, bias, act, residual
    (2, 3, 32, 48, 64, 7, 2, 3, False, 1, False),    # stem conv + bn1 + relu
    (2, 64, 16, 24, 64, 3, 1, 1, False, 1, True),    # BasicBlock conv2 + bn2 + identity + relu
    (2, 64, 16, 16, 128, 1, 2, 0, False, 0, False),  # downsample 1x1 s2 + bn
    (8, 256, 1, 1, 256, 1, 1, 0, True, 3, False),    # ARM 1x1(bias) + bn + sigmoid (pooled-vector kernel)
    (5, 19, 1, 1, 19, 1, 1, 0, True, 1, False),      # pooled, C % 8 != 0: scalar kernel with the fold
    (2, 1024, 8, 16, 19, 3, 1, 1, False, 1, False),  # FFM ConvBlock (N=19: scalar epilogue)
    (8, 128, 64, 64, 128, 3, 1, 1, False, 1, True),  # 128x128 LDS-DMA tile + residual
    (2, 256, 8, 64, 256, 3, 1, 1, False, 1, True),   # halo conv (bf16), 4 x 64 tiles + residual
    (2, 512, 8, 32, 512, 3, 1, 1, False, 1, True),   # halo conv (bf16), 8 x 32 tiles (layer4) + residual
]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", FOLD_CASES)
def test_conv_bn_eval_fold(case, dt):
    """Inference conv -> BN(running stats) [+res] [-> act] as one launch vs ATen fp64."""
    n, c, h, w, k, kh, s, p, has_bias, act, has_res = case
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(k, c, kh, kh, generator=g, dtype=torch.float64) / (c * kh * kh) ** 0.5
    b = torch.randn(k, generator=g, dtype=torch.float64) if has_bias else None
    rm, rv = torch.randn(k, generator=g, dtype=torch.float64), 0.5 + torch.rand(k, generator=g, dtype=torch.float64)
    gam, bet = torch.randn(k, generator=g, dtype=torch.float64), torch.randn(k, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x, wt = x.bfloat16().double(), wt.bfloat16().double()
    y0 = TF.batch_norm(TF.conv2d(x, wt, b, s, p), rm, rv, gam, bet, False, 0.1, 1e-5)
    res = torch.randn(y0.shape, generator=g, dtype=torch.float64) if has_res else None
    if res is not None:
        if dt == torch.bfloat16:
            res = res.bfloat16().double()
        y0 = y0 + res
    yr = {0: y0, 1: TF.relu(y0), 3: torch.sigmoid(y0)}[act]
    wd = wt.float().to(DEV).contiguous(memory_format=CL)
    dv = lambda t: None if t is None else t.float().to(DEV)  # noqa: E731
    with torch.no_grad():
        y = F.conv_bn_eval(_dev(x, dt), wd, dv(b), _shadow(wd, dt), (s, s), (p, p), (1, 1), dv(gam), dv(bet),
                           dv(rm), dv(rv), 1e-5, act, None if res is None else _dev(res, dt))
    _close(y, yr, dt, "y", 2e-4 if dt == torch.float32 else 3e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [(2, 128, 32, 64, 256, 3, 2, 1, 1024, 0),   # the spatial path's conv3 into the FFM input
                                 (2, 64, 16, 24, 64, 3, 2, 1, 96, 32),      # 64 x 64 tiles, offset slice
                                 (1, 32, 9, 13, 32, 3, 2, 1, 40, 8)])       # ragged M tiles
def test_conv_bn_eval_into_slice(geo, dt):
    """conv_bn_eval(out=(buf, off)) -- rtsds_conv2d_fwd_bn_ld, the row-pitched epilogue --
    writes exactly the plain conv_bn_eval result into channels [off, off + k) of the wider
    tensor and leaves the other channels untouched."""
    n, c, h, w, k, kh, s, p, ct, off = geo
    g = torch.Generator().manual_seed(12)
    x = _dev(torch.randn(n, c, h, w, generator=g), dt)
    wt = (torch.randn(k, c, kh, kh, generator=g) / (c * kh * kh) ** 0.5).to(DEV).contiguous(memory_format=CL)
    rm, rv = torch.randn(k, generator=g).to(DEV), (0.5 + torch.rand(k, generator=g)).to(DEV)
    gam, bet = torch.randn(k, generator=g).to(DEV), torch.randn(k, generator=g).to(DEV)
    args = (wt, None, _shadow(wt, dt), (s, s), (p, p), (1, 1), gam, bet, rm, rv, 1e-5, 1)
    with torch.no_grad():
        ref = F.conv_bn_eval(x, *args)
        buf = _dev(torch.randn(n, ct, ref.shape[2], ref.shape[3], generator=g), dt)
        before = buf.clone()
        got = F.conv_bn_eval(x, *args, out=(buf, off))
    torch.cuda.synchronize()
    assert got.data_ptr() == buf.data_ptr() + off * buf.element_size()
    assert torch.equal(buf[:, off:off + k], ref)
    assert torch.equal(buf[:, :off], before[:, :off]) and torch.equal(buf[:, off + k:], before[:, off + k:])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [(2, 64, 128), (3, 8, 40), (1, 16, 17)])
def test_ffm_head_eval(geo, dt):
    """FeatureFusionModule attention tail + final 1x1 conv (rtsds_ffm_head_eval: GAP partials per
    256-pixel slice, then one workgroup per slice) vs fp64: conv3(f * a + f) + b3 with
    a = sigmoid(conv2(relu(conv1(GAP(f)) + b1)) + b2); last slices partial (8 x 40, 16 x 17)."""
    n, h, w = geo
    if (h * w) % (8 if dt == torch.bfloat16 else 4):
        pytest.skip("hw must be a multiple of the vector length")
    g = torch.Generator().manual_seed(21)
    c = 19
    f = torch.randn(n, c, h, w, generator=g, dtype=torch.float64)
    ws = [torch.randn(c, c, 1, 1, generator=g, dtype=torch.float64) / c ** 0.5 for _ in range(3)]
    bs = [torch.randn(c, generator=g, dtype=torch.float64) for _ in range(3)]
    if dt == torch.bfloat16:
        f = f.bfloat16().double()
        ws = [t.bfloat16().double() for t in ws]
    a = torch.sigmoid(TF.conv2d(torch.relu(TF.conv2d(f.mean((2, 3), keepdim=True), ws[0], bs[0])), ws[1], bs[1]))
    ref = TF.conv2d(f * a + f, ws[2], bs[2])
    with torch.no_grad():
        got = F.ffm_head_eval(_dev(f, dt), *[t.to(DEV, dt) for t in ws[:1]], bs[0].float().to(DEV),
                              ws[1].to(DEV, dt), bs[1].float().to(DEV), ws[2].to(DEV, dt), bs[2].float().to(DEV))
    _close(got, ref, dt, "out", 1e-4 if dt == torch.float32 else 3e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_bisenet_eval_fold_and_graph(dt):
    """BiSeNet eval forward: folded conv+BN path == unfused path (autograd-enabled eval), and a
    hipGraph replay (runtime.GraphedForward) == eager."""
    import rtsds_amd
    from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
    from rtsds_amd.runtime import GraphedForward
    torch.manual_seed(0)
    with rtsds_amd.precision(dt):
        net = BiSeNet(19, "resnet18").to(DEV)
        # non-trivial running statistics: a few train-mode forwards
        xs = torch.randn(2, 3, 64, 128, device=DEV)
        with torch.no_grad():
            for _ in range(2):
                net(xs)
        net.eval()
        x = torch.randn(2, 3, 64, 128, device=DEV)
        ref = net(x.requires_grad_()).detach()  # autograd on: unfused conv -> BN chain
        x = x.detach()
        with torch.no_grad():
            fused = net(x)
        gf = GraphedForward(net, x)
        x2 = torch.randn_like(x)
        with torch.no_grad():
            eager2 = net(x2)
        rep2 = gf(x2).clone()
        rep1 = gf(x).clone()
    tol = 1e-3 if dt == torch.float32 else 5e-2
    scale = ref.abs().max().item()
    assert (fused.float() - ref.float()).abs().max().item() <= tol * scale
    assert torch.equal(rep1, fused) and torch.equal(rep2, eager2)


@pytest.mark.parametrize("shape", [(2, 128, 8, 128, 19), (2, 64, 8, 64, 32), (2, 64, 6, 20, 19), (2, 256, 8, 64, 64)])
def test_conv_bn_stats_epilogue(shape):
    """Train-mode ConvBlock (conv -> BN with batch statistics from the conv epilogue -> ReLU):
    the GEMM epilogue and the halo direct conv (hconv.hip, w % 64 == 0) both against ATen."""
    from rtsds_amd import nn as rnn
    n, c, h, w, k = shape
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, c, h, w, generator=g, dtype=torch.float64).bfloat16().double()
    conv = rnn.Conv2d(c, k, 3, padding=1, bias=False).to(DEV)
    bn = rnn.BatchNorm2d(k).to(DEV)
    with torch.no_grad():
        conv.weight.copy_((torch.randn(k, c, 3, 3, generator=g) / (9 * c) ** 0.5).bfloat16().float())
    wr = conv.weight.detach().double().cpu()
    yr = TF.relu(TF.batch_norm(TF.conv2d(x, wr, None, 1, 1), None, None, None, None, True, 0.1, 1e-5))
    y = rnn.conv_bn(conv, bn, _dev(x, torch.bfloat16), "relu")
    _close(y, yr, torch.bfloat16, "y")
    rm_ref = 0.1 * TF.conv2d(x, wr, None, 1, 1).mean(dim=(0, 2, 3))
    _close(bn.running_mean, rm_ref, torch.bfloat16, "running_mean")


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [((2, 19, 16, 32), (128, 256)), ((1, 19, 13, 17), (97, 129)), ((2, 7, 9, 40), (64, 96))])
def test_upsample_softmax_fused(dt, geo):
    """functional.upsample_softmax (rtsds_upsoftmax_fwd / _bwd): forward and input gradient vs
    torch fp64 (interpolate bilinear + softmax), bit-identical to the unfused HIP chain
    (interpolate_geometry -> softmax), and zero in the padding channels."""
    (n, c, h, w), (ho, wo) = geo
    g = torch.Generator().manual_seed(n * 7 + h)
    x = torch.randn(n, c, h, w, generator=g, dtype=torch.float64) * 3
    gy = torch.randn(n, c, ho, wo, generator=g, dtype=torch.float64)
    if dt == torch.bfloat16:
        x, gy = x.bfloat16().double(), gy.bfloat16().double()
    xr = x.clone().requires_grad_()
    yr = torch.softmax(TF.interpolate(xr, size=(ho, wo), mode="bilinear", align_corners=False), dim=1)
    yr.backward(gy)
    xd = _dev(x, dt).requires_grad_()
    geo_ = F.upsample_geometry(xd, size=(ho, wo))
    y = F.upsample_softmax(xd, geo_)
    assert F.is_padded_input(y)
    y.backward(_dev(gy, dt))
    pad = y.as_strided((n, ho, wo, 32), (ho * wo * 32, wo * 32, 32, 1))[..., c:]
    assert float(pad.abs().max()) == 0.0
    _close(y, yr, dt, "y")
    _close(xd.grad, xr.grad, dt, "dx", tol=2e-4 if dt == torch.float32 else 5e-2)
    # the unfused chain on the same input
    x2 = _dev(x, dt).requires_grad_()
    y2 = F.softmax(F.interpolate_geometry(x2, geo_), dim=1)
    y2.backward(_dev(gy, dt))
    assert torch.equal(y.detach().float(), y2.detach().float())
    assert torch.equal(xd.grad, x2.grad)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 3, 64, 96), (3, 3, 7, 9), (1, 2, 4, 5)])
def test_nchw_to_nhwc_pad(shape, dt):
    """rtsds_nchw_to_nhwc_pad: NCHW fp32 -> NHWC with a 4-channel pitch, pad channels zero (the
    4-pixel vector kernel for planes of a multiple of 4 pixels, the per-pixel one otherwise)."""
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _P
    from rtsds_amd.runtime import stream
    n, c, h, w = shape
    x = (torch.randn(shape, generator=torch.Generator().manual_seed(3)) * 30).to(DEV)
    y = torch.full((n, h, w, 4), 7.0, device=DEV, dtype=dt)
    assert lib.rtsds_nchw_to_nhwc_pad(_P(x), _P(y), n, c, h, w, 4, 0 if dt == torch.float32 else 1, stream()) == 0
    torch.cuda.synchronize()
    assert torch.equal(y[..., :c], x.permute(0, 2, 3, 1).to(dt))
    assert not y[..., c:].any()


@pytest.mark.parametrize("kh,pad", [(7, 3), (3, 1)])
def test_padded_image_input_bit_identical(kh, pad):
    """pack_input writes a 3-channel bf16 image with the 4-channel pitch of the superpixel
    stem / spatial-path convs (RTSDS_INPUT_PADDED, no pad pass): forward, weight gradient and
    the eval-mode folded conv equal the same convs on an ordinary NHWC copy bit for bit."""
    g = torch.Generator().manual_seed(17)
    x = torch.randn(2, 3, 64, 96, generator=g) * 50
    xp = F.pack_input(x.to(DEV), torch.bfloat16)
    assert F.is_padded_input(xp) and xp.shape == (2, 3, 64, 96) and xp._rt_cpad == 4
    xu = xp.contiguous(memory_format=CL)
    assert not F.is_padded_input(xu)
    assert torch.equal(xu.float().cpu(), x.bfloat16().float())
    wt = torch.randn(64, 3, kh, kh, generator=g) / (3 * kh * kh) ** 0.5
    gy = None
    outs = []
    for xi in (xp, xu):
        wp = torch.nn.Parameter(wt.to(DEV).contiguous(memory_format=CL))
        y = F.conv2d(xi, wp, None, _shadow(wp, torch.bfloat16), (2, 2), (pad, pad), (1, 1), 0)
        if gy is None:
            gy = torch.randn(y.shape, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
        y.backward(gy)
        with torch.no_grad():
            k = 64
            ye = F.conv_bn_eval(xi, wp.detach(), None, _shadow(wp.detach(), torch.bfloat16), (2, 2), (pad, pad),
                                (1, 1), torch.ones(k, device=DEV), torch.zeros(k, device=DEV),
                                torch.zeros(k, device=DEV), torch.ones(k, device=DEV), 1e-5, 1)
        torch.cuda.synchronize()
        outs.append((y.detach().float().cpu(), wp.grad.float().cpu(), ye.float().cpu()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("case", [
    (2, 64, 16, 24, 64, 3, 1, 1, 1),      # stride-1 GEMM route
    (2, 64, 16, 16, 128, 3, 2, 1, 1),     # stride-2 parity phases
    (1, 32, 13, 17, 64, 3, 2, 1, 1),      # stride-2 phases, odd sizes
    (2, 64, 16, 16, 128, 1, 2, 0, 1),     # 1x1 s2: phases without taps
    (2, 128, 8, 128, 19, 3, 1, 1, 1),     # halo route (flipped weights), Cout padded to 32
    (2, 512, 16, 32, 512, 3, 1, 1, 1),    # DGRAD split-K
    (1, 64, 13, 17, 64, 3, 1, 2, 2),      # dilated
    (2, 512, 32, 64, 19, 1, 1, 0, 1),     # narrow 1x1 (pw.hip): no packed copy
])
def test_dgrad_packed_weights_bit_identical(case):
    """rtsds_conv2d_dgrad_pack_many (all cases in one call) + RTSDS_WEIGHT_PACKED equals the
    per-call repack bit for bit: plain, accumulate and the LeakyReLU-masked variant."""
    import ctypes
    from rtsds_amd._lib import ConvDesc, WEIGHT_PACKED, lib
    from rtsds_amd.functional import _conv_desc, _P
    from rtsds_amd.runtime import stream, workspace

    n, c, h, w, k, kh, s, p, dil = case
    g = torch.Generator().manual_seed(23)
    x = _dev(torch.randn(n, c, h, w, generator=g), torch.bfloat16)
    wq = _dev(torch.randn(k, c, kh, kh, generator=g) / (kh * kh * c) ** 0.5, torch.bfloat16)
    d = _conv_desc(x, k, kh, kh, (s, s), (p, p), (dil, dil))
    nb = lib.rtsds_conv2d_dgrad_pack_bytes(ctypes.byref(d))
    if case[4] == 19 and kh == 1:
        assert nb == 0
        return
    assert nb > 0
    dy = _dev(torch.randn(n, k, d.ho, d.wo, generator=g), torch.bfloat16)
    pk = torch.full((nb // 2,), float("nan"), dtype=torch.bfloat16, device=DEV)
    descs = (ConvDesc * 1)(d)
    assert lib.rtsds_conv2d_dgrad_pack_many(1, descs, (ctypes.c_void_p * 1)(wq.data_ptr()),
                                            (ctypes.c_void_p * 1)(pk.data_ptr()), stream()) == 0
    ws = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), x.device)
    base = _dev(torch.randn(n, c, h, w, generator=g), torch.bfloat16)
    outs = []
    for wt, flag in ((wq, 0), (pk, WEIGHT_PACKED)):
        a, b, m = torch.empty_like(x), base.clone(), torch.empty_like(x)
        assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wt), _P(a), flag, _P(ws), ws.numel(), stream()) == 0
        assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dy), _P(wt), _P(b), 1 | flag, _P(ws), ws.numel(), stream()) == 0
        assert lib.rtsds_conv2d_dgrad_act(ctypes.byref(d), _P(dy), _P(wt), _P(m), _P(x), 2 | flag, _P(ws), ws.numel(),
                                          stream()) == 0
        torch.cuda.synchronize()
        outs.append((a.float().cpu(), b.float().cpu(), m.float().cpu()))
    for u, v in zip(*outs):
        assert torch.equal(u, v)
    ref = TF.conv_transpose2d(dy.double().cpu(), wq.double().cpu(), stride=s, padding=p, dilation=dil,
                              output_padding=(h - ((d.ho - 1) * s - 2 * p + dil * (kh - 1) + 1),
                                              w - ((d.wo - 1) * s - 2 * p + dil * (kh - 1) + 1)))
    _close(outs[1][0], ref, torch.bfloat16, "dx")


def test_dgrad_packs_in_training_bit_identical():
    """Three BiSeNet bf16 seg iterations and two DA iterations with the optimizer-maintained
    packed dgrad weights (default) leave parameters, optimizer state and BN buffers identical to
    the per-call repack (functional.set_dgrad_packs(False))."""
    import rtsds_amd
    from rtsds_amd import losses, optim
    from rtsds_amd import train as rtrain
    from rtsds_amd.models.bisenet.build_bisenet import BiSeNet
    from rtsds_amd.models.domain_shift.adversarial.model import TinyDomainDiscriminator

    g = torch.Generator().manual_seed(29)
    x = torch.randn(2, 3, 64, 128, generator=g).to(DEV)
    xt = torch.randn(2, 3, 64, 128, generator=g).to(DEV)
    y = torch.randint(0, 20, (2, 64, 128), generator=g).to(DEV)
    ce, bce = losses.CrossEntropyLoss(ignore_index=19), losses.BCEWithLogitsLoss()
    states = []
    try:
        for on in (False, True):
            F.set_dgrad_packs(on)
            with rtsds_amd.precision(torch.bfloat16):
                torch.manual_seed(3)
                net = BiSeNet(19, "resnet18").to(DEV).train()
                disc = TinyDomainDiscriminator(19).to(DEV).train()
                opt = optim.Adam(net.parameters(), lr=1e-3)
                dopt = optim.Adam(disc.parameters(), lr=1e-3, weight_decay=1e-4)
                for _ in range(3):
                    rtrain.seg_step(net, ce, opt, x, y)
                for _ in range(2):
                    rtrain.da_step(net, disc, opt, dopt, ce, bce, x, y, xt, 0.1, 100)
                torch.cuda.synchronize()
                if on:
                    assert any(getattr(p, "_rt_dpack", None) is not None and p._rt_dpack.valid is not None
                               for p in net.parameters())
                states.append({k: v.detach().float().cpu().clone() for k, v in
                               list(net.state_dict().items()) + list(disc.state_dict().items())})
    finally:
        F.set_dgrad_packs(True)
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), k


@pytest.mark.parametrize("kh,pad,bias", [(7, 3, False), (3, 1, True)])
@pytest.mark.parametrize("hw", [(38, 150), (64, 256)])
def test_image_conv_direct(kh, pad, bias, hw):
    """The 3-channel stride-2 image convs (imgconv.hip: stem 7x7 s2 p3, spatial-path 3x3 s2 p1)
    at output sizes that do / do not divide the 4 x 64 tile: forward vs ATen fp64, the
    train-mode ConvBlock with the BatchNorm statistics from the conv epilogue (output and
    running statistics), and the eval-mode folded conv + BN + ReLU."""
    from rtsds_amd import nn as rnn
    h, w = hw
    g = torch.Generator().manual_seed(kh * 100 + h)
    x = (torch.randn(2, 3, h, w, generator=g, dtype=torch.float64) * 40).bfloat16().double()
    conv = rnn.Conv2d(3, 64, kh, stride=2, padding=pad, bias=bias).to(DEV)
    bn = rnn.BatchNorm2d(64).to(DEV)
    with torch.no_grad():
        conv.weight.copy_((torch.randn(64, 3, kh, kh, generator=g) / (3 * kh * kh) ** 0.5).bfloat16().float())
        if bias:
            conv.bias.copy_(torch.randn(64, generator=g))
    wr = conv.weight.detach().double().cpu()
    br = conv.bias.detach().double().cpu() if bias else None
    y0 = TF.conv2d(x, wr, br, 2, pad)
    y = F.conv2d(_dev(x, torch.bfloat16), conv.weight, conv.bias, _shadow(conv.weight, torch.bfloat16), (2, 2),
                 (pad, pad), (1, 1), 0)
    _close(y, y0, torch.bfloat16, "conv")
    yb = rnn.conv_bn(conv, bn, _dev(x, torch.bfloat16), "relu")
    _close(yb, TF.relu(TF.batch_norm(y0, None, None, None, None, True, 0.1, 1e-5)), torch.bfloat16, "conv+bn+relu")
    _close(bn.running_mean, 0.1 * y0.mean(dim=(0, 2, 3)), torch.bfloat16, "running_mean")
    _close(bn.running_var, 0.9 + 0.1 * y0.var(dim=(0, 2, 3)), torch.bfloat16, "running_var")
    conv.eval()
    bn.eval()
    with torch.no_grad():
        ye = rnn.conv_bn(conv, bn, _dev(x, torch.bfloat16), "relu")
    rm, rv = bn.running_mean.double().cpu(), bn.running_var.double().cpu()
    _close(ye, TF.relu(TF.batch_norm(y0, rm, rv, None, None, False, 0.1, 1e-5)), torch.bfloat16, "eval fold")


@pytest.mark.parametrize("hw,ceil", [((64, 96), False), ((38, 150), False), ((38, 150), True), ((70, 134), True)])
def test_stem_conv_bn_maxpool_eval_fused(hw, ceil):
    """Inference stem (imgconv_pool_kernel: conv 7x7 s2 + folded BN + ReLU + MaxPool 3/2/1 in one
    launch) equals the folded conv followed by the pool bit for bit, incl. ceil mode and tiles
    past the output edge; and the module path (nn.conv_bn_relu_maxpool) takes it."""
    from rtsds_amd import nn as rnn
    h, w = hw
    g = torch.Generator().manual_seed(h + w)
    x = F.pack_input((torch.randn(2, 3, h, w, generator=g) * 40).to(DEV), torch.bfloat16)
    conv = rnn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(DEV)
    bn = rnn.BatchNorm2d(64).to(DEV)
    pool = rnn.MaxPool2d(3, 2, 1, ceil_mode=ceil)
    with torch.no_grad():
        conv.weight.copy_(torch.randn(64, 3, 7, 7, generator=g) / 12)
        bn.running_mean.copy_(torch.randn(64, generator=g))
        bn.running_var.copy_(0.5 + torch.rand(64, generator=g))
        bn.weight.copy_(torch.randn(64, generator=g))
        bn.bias.copy_(torch.randn(64, generator=g))
    conv.eval()
    bn.eval()
    with torch.no_grad():
        wq = _shadow(conv.weight, torch.bfloat16)
        fused = F.conv_bn_maxpool_eval(x, conv.weight, None, wq, (2, 2), (3, 3), (1, 1), bn.weight, bn.bias,
                                       bn.running_mean, bn.running_var, bn.eps, 1, 3, 2, 1, ceil)
        y = F.conv_bn_eval(x, conv.weight, None, wq, (2, 2), (3, 3), (1, 1), bn.weight, bn.bias, bn.running_mean,
                           bn.running_var, bn.eps, 1)
        ref = F.max_pool2d(y, 3, 2, 1, ceil)
        mod = rnn.conv_bn_relu_maxpool(conv, bn, pool, x)
    assert fused is not None and fused.shape == ref.shape, (None if fused is None else fused.shape, ref.shape)
    assert torch.equal(fused.float(), ref.float())
    assert torch.equal(mod.float(), ref.float())


@pytest.mark.parametrize("geo", [(2, 18, 120), (1, 7, 56)])
def test_tapconv_partial_tiles(geo):
    """The register-weight direct 3x3 64 -> 64 conv (tapconv.hip, ResNet layer1) through the C ABI
    on geometries with partial tiles: widths with w % 64 in 49..63 (a last column tile with
    valid columns < 64) and heights that end inside a 4-row tile, so the edge columns / rows, the
    out-of-range buffer stores and the Chan merge of the statistics over tiles with unequal
    counts all run.  Every epilogue the networks launch, against float64 on the bf16 operands:
    forward (plain, ReLU, BatchNorm statistics, eval BN scale / shift + residual + ReLU), data
    gradient (plain, accumulate, ReLU mask, BatchNorm-backward statistics), and the same convs'
    weight gradient (split-K implicit GEMM + split reduce; plain and accumulating)."""
    import ctypes
    from rtsds_amd._lib import lib
    from rtsds_amd.functional import _conv_desc, _P
    from rtsds_amd.runtime import stream, workspace

    n, h, w = geo
    c = 64
    g = torch.Generator().manual_seed(n * 1000 + h * 10 + w)
    bf = torch.bfloat16

    def rnd(*shape, scale=1.0):
        return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale).bfloat16().double()
    x, wt, dy, res, aux = rnd(n, c, h, w), rnd(c, c, 3, 3, scale=(9 * c) ** -0.5), rnd(n, c, h, w), rnd(n, c, h, w), \
        rnd(n, c, h, w)
    bias, scale, shift = torch.randn(c, generator=g).double(), torch.rand(c, generator=g).double() + 0.5, \
        torch.randn(c, generator=g).double()
    xd, wd, dyd, resd, auxd = (_dev(t, bf) for t in (x, wt, dy, res, aux))
    d = _conv_desc(xd, c, 3, 3, (1, 1), (1, 1), (1, 1))
    st = stream()
    wsf = workspace(lib.rtsds_conv2d_fwd_workspace(ctypes.byref(d)), xd.device)
    wsd = workspace(lib.rtsds_conv2d_dgrad_workspace(ctypes.byref(d)), xd.device)
    conv = TF.conv2d(x, wt, None, 1, 1)
    dgr = TF.conv_transpose2d(dy, wt, padding=1)
    f32 = lambda t: t.float().to(DEV).contiguous()  # noqa: E731

    def fwd(b, act, stats=None):
        y = torch.empty_like(xd)
        assert lib.rtsds_conv2d_fwd(ctypes.byref(d), _P(xd), _P(wd), None if b is None else _P(b), _P(y), act,
                                    None if stats is None else _P(stats), _P(wsf), wsf.numel(), st) == 0
        return y
    _close(fwd(None, 0), conv, bf, "fwd plain", tol=1e-2)
    _close(fwd(f32(bias), 1), TF.relu(conv + bias.view(1, -1, 1, 1)), bf, "fwd bias relu", tol=1e-2)
    tiles = lib.rtsds_conv2d_fwd_stats_tiles(ctypes.byref(d))
    stats = torch.zeros(c, tiles, 4, device=DEV)
    _close(fwd(None, 0, stats), conv, bf, "fwd stats y", tol=1e-2)
    s = stats.double().cpu()
    cnt = s[:, :, 0]
    tot = cnt.sum(1)
    mean = (cnt * s[:, :, 1]).sum(1) / tot
    m2 = (s[:, :, 2] + cnt * (s[:, :, 1] - mean[:, None]) ** 2).sum(1)
    assert torch.all(tot == n * h * w), tot
    _close(mean, conv.mean(dim=(0, 2, 3)), bf, "stats mean", tol=1e-4)
    _close(m2 / tot, conv.var(dim=(0, 2, 3), unbiased=False), bf, "stats var", tol=1e-4)
    y = torch.empty_like(xd)
    assert lib.rtsds_conv2d_fwd_bn(ctypes.byref(d), _P(xd), _P(wd), _P(f32(scale)), _P(f32(shift)), _P(resd), _P(y), 1,
                                   _P(wsf), wsf.numel(), st) == 0
    _close(y, TF.relu(conv * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1) + res), bf, "fwd bn res relu",
           tol=1e-2)

    dx = torch.empty_like(xd)
    assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dyd), _P(wd), _P(dx), 0, _P(wsd), wsd.numel(), st) == 0
    _close(dx, dgr, bf, "dgrad", tol=1e-2)
    dxa = auxd.clone()
    assert lib.rtsds_conv2d_dgrad(ctypes.byref(d), _P(dyd), _P(wd), _P(dxa), 1, _P(wsd), wsd.numel(), st) == 0
    _close(dxa, dgr + aux, bf, "dgrad accumulate", tol=1e-2)
    dxm = torch.empty_like(xd)
    assert lib.rtsds_conv2d_dgrad_act(ctypes.byref(d), _P(dyd), _P(wd), _P(dxm), _P(auxd), 1, _P(wsd), wsd.numel(),
                                      st) == 0
    _close(dxm, dgr * (aux > 0), bf, "dgrad relu mask", tol=1e-2)
    btiles = lib.rtsds_conv2d_dgrad_bnstats_tiles(ctypes.byref(d))
    assert btiles > 0
    gamma, beta = torch.rand(c, generator=g).double() + 0.5, torch.randn(c, generator=g).double() * 0.2
    bmean, binv = torch.randn(c, generator=g).double() * 0.1, torch.rand(c, generator=g).double() + 0.5
    part = torch.zeros(c, btiles, 2, device=DEV)
    dxb = torch.empty_like(xd)
    assert lib.rtsds_conv2d_dgrad_bnstats(ctypes.byref(d), _P(dyd), _P(wd), _P(dxb), _P(auxd), _P(f32(gamma)),
                                          _P(f32(beta)), _P(f32(bmean)), _P(f32(binv)), 1, _P(part), _P(wsd),
                                          wsd.numel(), st) == 0
    torch.cuda.synchronize()
    _close(dxb, dgr, bf, "dgrad bnstats dx", tol=1e-2)
    # the statistics are taken from the stored (bf16-rounded) dx values
    dxs = dxb.double().cpu()
    sc = (gamma * binv).view(1, -1, 1, 1)
    pre = aux * sc + (beta.view(1, -1, 1, 1) - bmean.view(1, -1, 1, 1) * sc)
    gg = dxs * (pre > 0)
    p = part.double().cpu().sum(1)
    _close(p[:, 0], gg.sum(dim=(0, 2, 3)), bf, "bnstats sum g", tol=1e-4)
    _close(p[:, 1], (gg * (aux - bmean.view(1, -1, 1, 1))).sum(dim=(0, 2, 3)), bf, "bnstats sum g(x-mean)", tol=1e-4)
    # weight gradient (split-K slabs + the split reduce), plain and accumulating into an
    # existing gradient
    wsw = workspace(lib.rtsds_conv2d_wgrad_workspace(ctypes.byref(d)), xd.device)
    dwr = torch.nn.grad.conv2d_weight(x, wt.shape, dy, padding=1).permute(0, 2, 3, 1)  # [k][kh][kw][c]
    dw = torch.empty(c, 3, 3, c, device=DEV)
    assert lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(xd), _P(dyd), _P(dw), None, 0, _P(wsw), wsw.numel(), st) == 0
    dw0 = torch.randn(c, 3, 3, c, generator=g).to(DEV)
    dwa = dw0.clone()
    assert lib.rtsds_conv2d_wgrad(ctypes.byref(d), _P(xd), _P(dyd), _P(dwa), None, 1, _P(wsw), wsw.numel(), st) == 0
    torch.cuda.synchronize()
    _close(dw, dwr, torch.float32, "wgrad", tol=1e-4)
    _close(dwa, dwr + dw0.double().cpu(), torch.float32, "wgrad accumulate", tol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,c0,c1,c2,bias", [(2, 19, 19, 19, True), (8, 61, 13, 61, False), (1, 3, 5, 7, True)])
def test_pooled_mlp_matches_conv_chain(dt, n, c0, c1, c2, bias):
    """rtsds_pooled_mlp_fwd / _bwd (the FFM attention, build_bisenet.py:67-70, one launch each)
    equal the pooled 1x1 conv chain (conv + ReLU, conv + sigmoid) bit for bit: outputs, dL/dp
    and the weight / bias gradients."""
    g = torch.Generator().manual_seed(n * 100 + c0)
    p = torch.randn(n, c0, 1, 1, generator=g).to(DEV, dt)
    w1 = (torch.randn(c1, c0, 1, 1, generator=g) * 0.3).to(DEV)
    w2 = (torch.randn(c2, c1, 1, 1, generator=g) * 0.3).to(DEV)
    b1 = torch.randn(c1, generator=g).to(DEV) if bias else None
    b2 = torch.randn(c2, generator=g).to(DEV) if bias else None
    da = torch.randn(n, c2, 1, 1, generator=g).to(DEV, dt)
    assert F.pooled_mlp_ok(p, c1, c2)
    outs = []
    for fused in (False, True):
        ps = p.clone().requires_grad_(True)
        ws = [t.clone().requires_grad_(True) if t is not None else None for t in (w1, b1, w2, b2)]
        q1, q2 = _shadow(ws[0], dt), _shadow(ws[2], dt)
        if fused:
            a = F.pooled_mlp(ps, ws[0], ws[1], q1, ws[2], ws[3], q2)
        else:
            h = F.conv2d(ps, ws[0], ws[1], q1, act=1)
            a = F.conv2d(h, ws[2], ws[3], q2, act=3)
        a.backward(da)
        torch.cuda.synchronize()
        outs.append([a.detach().float().cpu(), ps.grad.float().cpu()] +
                    [t.grad.cpu() for t in ws if t is not None])
    for u, v in zip(*outs):
        assert torch.equal(u, v)
    ref = torch.sigmoid(TF.conv2d(torch.relu(TF.conv2d(p.double(), w1.double(), b1.double() if bias else None)),
                                  w2.double(), b2.double() if bias else None))
    tol = 2e-2 if dt == torch.bfloat16 else 1e-5
    assert (outs[1][0].double() - ref.cpu()).abs().max() < tol
