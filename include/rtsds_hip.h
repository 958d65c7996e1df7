/*
 * rtsds_hip.h -- C ABI of librtsds_hip.so, the MI355X (gfx950 / CDNA4) kernels behind the
 * RTSDS hot path (BiSeNet / DeepLabV2 forward+backward + adversarial DA discriminator step).
 *
 * The reference (sina-behnam/RTSDS @ 2024-08-07) is pure PyTorch: every kernel on its hot
 * path is an implicit ATen op reached through torch.nn.  Each entry point below names the
 * reference call site(s) whose ATen kernel it replaces.
 *
 * Conventions:
 *  - Activations are NHWC ("channels_last"), dtype RTSDS_F32 or RTSDS_BF16; weights are
 *    [Cout][KH][KW][Cin] in the same dtype; statistics, biases, losses and optimizer state
 *    are fp32.
 *  - Pointers are device pointers owned by the caller (PyTorch caching allocator).  The
 *    library never allocates or frees; scratch comes in as (ws, ws_bytes).
 *  - `stream` is a hipStream_t passed as void*.  Every call is stream-ordered, stateless,
 *    re-entrant and performs no host synchronisation (graph-capture safe).
 *  - Return value: RTSDS_OK or one of the RTSDS_ERR_* codes; the Python layer raises.
 */
#ifndef RTSDS_HIP_H
#define RTSDS_HIP_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { RTSDS_F32 = 0, RTSDS_BF16 = 1, RTSDS_F16 = 2 /* the gradient wire only: rtsds_cast, optimizer grad_dtype */ };
enum {
  RTSDS_OK = 0,
  RTSDS_ERR_SHAPE = 1,        /* inconsistent / out-of-range shape */
  RTSDS_ERR_UNSUPPORTED = 2,  /* configuration the kernels do not implement */
  RTSDS_ERR_LAUNCH = 3,       /* HIP launch failure */
  RTSDS_ERR_WORKSPACE = 4     /* ws_bytes smaller than the *_workspace() query */
};
enum { RTSDS_ACT_NONE = 0, RTSDS_ACT_RELU = 1, RTSDS_ACT_LEAKY = 2, RTSDS_ACT_SIGMOID = 3 };
#define RTSDS_ACCUMULATE 0x100 /* conv fwd flag: y += conv(...) (ASPP sum, deeplabv2.py:62-66) */
/* conv fwd (act) / wgrad (accumulate) flag: x is already stored with the padded channel pitch
 * the GEMM gathers (rtsds_conv2d_input_pitch: 19 -> 32 for the discriminator's class-probability
 * input, written by rtsds_upsoftmax_fwd; 3 -> 4 for the image of the stem / spatial-path convs,
 * written by rtsds_nchw_to_nhwc_pad) and zero in channels c..pitch-1: the internal pad pass is
 * skipped.  Rejected (RTSDS_ERR_UNSUPPORTED) where the pitch is c itself.                   */
#define RTSDS_INPUT_PADDED 0x400
/* conv dgrad flag (rtsds_conv2d_dgrad: accumulate; _act / _bnstats: act): w is the packed
 * copy rtsds_conv2d_dgrad_pack_many wrote for this descriptor, not the [Cout][KH][KW][Cin]
 * weight -- the per-call repack is skipped.                                                 */
#define RTSDS_WEIGHT_PACKED 0x800

typedef struct {
  int n, h, w, c;   /* input  [n][h][w][c]                                     */
  int ho, wo, k;    /* output [n][ho][wo][k]                                   */
  int kh, kw;       /* filter size                                             */
  int sh, sw;       /* stride                                                  */
  int ph, pw;       /* zero padding                                            */
  int dh, dw;       /* dilation                                                */
  int dtype;        /* RTSDS_F32 / RTSDS_BF16 for x, w, y                      */
} rtsds_conv_desc;

/* ---------------------------------------------------------------- convolution
 * Replaces nn.Conv2d (ATen convolution fwd / grad_input / grad_weight) at
 * build_bisenet.py:11-12,38,65,67,99-100,109-110,117; torchvision ResNet convs reached via
 * build_contextpath.py:19-24; deeplabv2.py:13,19,24,56,73,99; model.py:54-58,69-70.
 * Implicit GEMM on MFMA (bf16: v_mfma_f32_16x16x32_bf16, f32: v_mfma_f32_16x16x4_f32).  */

/* y = act(conv(x, w) + bias [+ y if act & RTSDS_ACCUMULATE]).  bias may be NULL (fp32 [k]).
 * bn_stats (may be NULL; act must be NONE): receives the following BatchNorm's per-tile
 * partial statistics, fp32 [k][rtsds_conv2d_fwd_stats_tiles(d)][count, mean, M2, 0] (channel-major), consumed
 * by rtsds_bn_fwd(stats_part=...) -- the statistics pass over y is then skipped.
 * ws >= rtsds_conv2d_fwd_workspace(d) (non-zero only when Cin needs channel padding).   */
size_t rtsds_conv2d_fwd_workspace(const rtsds_conv_desc* d);
/* Channel pitch of x that the forward / weight-gradient gathers of d read (0: bad descriptor). */
int rtsds_conv2d_input_pitch(const rtsds_conv_desc* d);
int rtsds_conv2d_fwd_stats_tiles(const rtsds_conv_desc* d);
int rtsds_conv2d_fwd(const rtsds_conv_desc* d, const void* x, const void* w, const float* bias,
                     void* y, int act, float* bn_stats, void* ws, size_t ws_bytes, void* stream);
/* Eval-mode conv + BatchNorm(running stats) (+ residual) (+ act) in one launch (inference
 * path of build_bisenet.py:16-18 ConvBlock, torchvision BasicBlock / Bottleneck,
 * deeplabv2.py:32-47): y = act(conv(x, w) * scale[k] + shift[k] + res), res NHWC like y (may
 * be NULL); scale / shift from rtsds_bn_fold.  Same workspace as rtsds_conv2d_fwd.         */
int rtsds_conv2d_fwd_bn(const rtsds_conv_desc* d, const void* x, const void* w, const float* scale,
                        const float* shift, const void* res, void* y, int act, void* ws, size_t ws_bytes,
                        void* stream);
/* rtsds_conv2d_fwd_bn (no residual) writing y as a channel slice of a wider NHWC tensor: row
 * pitch ldy elements (>= d->k; y 16-B aligned, ldy and d->k multiples of 8 for bf16 / 4 for f32)
 * -- the inference spatial path writes its output straight into the fusion module's
 * concatenated input (build_bisenet.py:153, :72).  RTSDS_ERR_UNSUPPORTED outside the
 * implicit-GEMM route (the caller then writes a plain tensor and copies).                   */
int rtsds_conv2d_fwd_bn_ld(const rtsds_conv_desc* d, const void* x, const void* w, const float* scale,
                           const float* shift, void* y, long ldy, int act, void* ws, size_t ws_bytes, void* stream);
/* Inference stem: eval conv + BatchNorm(running stats) + act + MaxPool2d(3, 2, pool_pad) in one
 * launch (torchvision ResNet conv1 -> bn1 -> relu -> maxpool, deeplabv2.py:106-110): y is the
 * pooled [n][hp][wp][k] NHWC output (hp / wp from the caller: floor or ceil mode); windows
 * skip positions outside the conv output.  Equal to rtsds_conv2d_fwd_bn + rtsds_maxpool_fwd.
 * RTSDS_ERR_UNSUPPORTED outside the 3-channel 7x7 stride-2 image conv with 64 outputs (bf16).
 * Same workspace as rtsds_conv2d_fwd.                                                       */
int rtsds_conv2d_fwd_bn_maxpool(const rtsds_conv_desc* d, const void* x, const void* w, const float* scale,
                                const float* shift, void* y, int act, int hp, int wp, int pool_pad, void* ws,
                                size_t ws_bytes, void* stream);
/* dx (+)= conv_transpose(dy, w) (accumulate != 0: dx += ...).  Needs ws >=
 * rtsds_conv2d_dgrad_workspace(d).  Strides 1 and 2 only.                               */
size_t rtsds_conv2d_dgrad_workspace(const rtsds_conv_desc* d);
/* Pre-packed data-gradient weights: bytes of d's packed copy (0: its route reads w as is --
 * pooled / narrow 1x1 -- and takes no RTSDS_WEIGHT_PACKED); pack_many writes the packed copies
 * wt[i] of count convs (descs[i], weights w[i] in [Cout][KH][KW][Cin]) in one launch per 16
 * segments -- the optimizer's per-step refresh after its update (optim.py).                 */
size_t rtsds_conv2d_dgrad_pack_bytes(const rtsds_conv_desc* d);
int rtsds_conv2d_dgrad_pack_many(int count, const rtsds_conv_desc* descs, const void* const* w, void* const* wt,
                                 void* stream);
int rtsds_conv2d_dgrad(const rtsds_conv_desc* d, const void* dy, const void* w, void* dx,
                       int accumulate, void* ws, size_t ws_bytes, void* stream);
/* dx = conv_transpose(dy, w) * act'(x_act): the data gradient of this conv followed by the
 * backward of the ReLU (act 1) / LeakyReLU(0.2) (act 2) that produced its input x_act (NHWC
 * [n][h][w][c], the activation's output) -- the discriminator's conv -> LeakyReLU -> conv
 * chains (model.py:54-58,69-70), applied in the GEMM epilogue (else as a second pass).
 * Values equal rtsds_conv2d_dgrad followed by rtsds_act_bwd.  Same workspace as dgrad.   */
int rtsds_conv2d_dgrad_act(const rtsds_conv_desc* d, const void* dy, const void* w, void* dx, const void* x_act,
                           int act, void* ws, size_t ws_bytes, void* stream);
/* dx = conv_transpose(dy, w), plus -- from the stored dx values -- the backward statistics of
 * the train-mode BatchNorm (+ ReLU / LeakyReLU, act) whose output is this conv's input
 * (ResNet BasicBlock bn1 -> conv2, Bottleneck bn1 -> conv2, bn2 -> conv3): per M tile t and
 * channel ch, part[(ch * tiles + t) * 2 + {0, 1}] = (sum g, sum g (bn_x - mean)),
 * g = dx * act'(bn_x * gamma * invstd + beta - mean * gamma * invstd) -- what rtsds_bn_bwd's
 * first pass computes, handed to rtsds_bn_bwd_part (the BatchNorm backward then skips it).
 * tiles = rtsds_conv2d_dgrad_bnstats_tiles(d); 0 = route not available (bf16, stride 1 and
 * the plain GEMM route only): call rtsds_conv2d_dgrad instead.                             */
int rtsds_conv2d_dgrad_bnstats_tiles(const rtsds_conv_desc* d);
int rtsds_conv2d_dgrad_bnstats(const rtsds_conv_desc* d, const void* dy, const void* w, void* dx, const void* bn_x,
                               const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                               int act, float* part, void* ws, size_t ws_bytes, void* stream);
/* dw (fp32 [k][kh][kw][c]) = sum_pixels dy (x) patch(x); dbias (fp32 [k], may be NULL) =
 * sum_pixels dy.  accumulate != 0 adds into dw / dbias instead of overwriting (gradients go
 * straight into the optimizer's flat gradient arena, replacing autograd's AccumulateGrad).  */
size_t rtsds_conv2d_wgrad_workspace(const rtsds_conv_desc* d);
int rtsds_conv2d_wgrad(const rtsds_conv_desc* d, const void* x, const void* dy, float* dw,
                       float* dbias, int accumulate, void* ws, size_t ws_bytes, void* stream);
/* Deferred split-K reduction of a weight gradient.  rtsds_conv2d_wgrad_deferred launches every
 * kernel of rtsds_conv2d_wgrad except the final reduction of the fp32 split slabs (which stay in
 * ws) into dw, and describes that reduction in *pending (pending->nv == 0: nothing deferred --
 * the call completed dw itself).  rtsds_split_reduce_many then performs up to n pending
 * reductions in ONE launch (the backward pass's wgrads reduced together instead of one small
 * launch each); descs must target distinct dw, and ws must stay allocated until it has run.  */
typedef struct {
  const float* slab;  /* [splits][k * kh * kw * cp] fp32 partials (in the wgrad's workspace) */
  float* dw;          /* [k][kh][kw][c] fp32                                                   */
  long slab_stride;   /* elements between splits                                              */
  int nv;             /* float4 outputs: k * kh * kw * c / 4                                    */
  int cv, cp;         /* c / 4; the slab's (padded) channel pitch                              */
  int splits, accumulate;
} rtsds_split_reduce_desc;
int rtsds_conv2d_wgrad_deferred(const rtsds_conv_desc* d, const void* x, const void* dy, float* dw,
                                float* dbias, int accumulate, void* ws, size_t ws_bytes,
                                rtsds_split_reduce_desc* pending, void* stream);
int rtsds_split_reduce_many(int n, const rtsds_split_reduce_desc* descs, void* stream);

/* ---------------------------------------------------------------- batch norm (train/eval)
 * Replaces nn.BatchNorm2d at build_bisenet.py:13,39; torchvision ResNet bn*; deeplabv2.py:14-27,
 * 75,101 (frozen affine, train-mode batch statistics).  x, y, res, dy, dx: NHWC [rows][c]
 * with rows = n*h*w.
 * Forward (training): mean/invstd of the batch are written to save_mean / save_invstd, the
 * running buffers are updated in place with the unbiased variance, momentum m, and
 * *num_batches_tracked (int64, may be NULL) is incremented on the device (PyTorch
 * semantics).  Forward (eval): running stats are used and copied to save_* when non-NULL.
 * y = act(gamma * (x - mean) * invstd + beta [+ res]).  gamma/beta may be NULL (1 / 0).   */
size_t rtsds_bn_workspace(long rows, int c);
/* stats_part (may be NULL): [c][stats_nrb][count, mean, M2, 0] partials from the producing
 * conv (rtsds_conv2d_fwd bn_stats) -- training mode then skips its own statistics pass.   */
int rtsds_bn_fwd(const void* x, const void* res, void* y, long rows, int c, const float* gamma,
                 const float* beta, float* running_mean, float* running_var,
                 long long* num_batches_tracked, float* save_mean,
                 float* save_invstd, float momentum, float eps, int training, int act,
                 const float* stats_part, int stats_nrb, int dtype, void* ws, size_t ws_bytes,
                 void* stream);
/* rtsds_bn_fwd with y's row pitch ldy >= c (ldy == c: rtsds_bn_fwd): y is a channel slice of a
 * wider NHWC tensor -- the spatial path's output written into the fusion module's concatenated
 * input (build_bisenet.py:153,72).  ldy != c: bf16, c % 8 == 0, ldy % 8 == 0.              */
int rtsds_bn_fwd_ld(const void* x, const void* res, void* y, long ldy, long rows, int c,
                    const float* gamma, const float* beta, float* running_mean, float* running_var,
                    long long* num_batches_tracked, float* save_mean, float* save_invstd,
                    float momentum, float eps, int training, int act, const float* stats_part,
                    int stats_nrb, int dtype, void* ws, size_t ws_bytes, void* stream);
/* Eval-mode fold of BatchNorm2d(running stats) into the preceding conv (+ its bias, may be
 * NULL): scale = gamma / sqrt(running_var + eps), shift = beta + (bias - running_mean) * scale
 * (fp32 [c]; gamma / beta may be NULL = 1 / 0).                                            */
int rtsds_bn_fold(const float* gamma, const float* beta, const float* running_mean,
                  const float* running_var, const float* conv_bias, float eps, int c, float* scale,
                  float* shift, void* stream);
/* Backward of the fused BN(+res)(+act) above.  y (post-activation output) gives the
 * activation mask; it may be NULL without a residual for act NONE/RELU/LEAKY, when the mask
 * is recomputed bit-exactly from x, gamma, beta and save_*.  dx, dres (may be NULL),
 * dgamma/dbeta (fp32, may be NULL; overwritten, or added to when accumulate_params != 0).
 * training=0: eval-mode backward (constant stats).                                        */
int rtsds_bn_bwd(const void* dy, const void* x, const void* y, void* dx, void* dres,
                 float* dgamma, float* dbeta, long rows, int c, const float* gamma,
                 const float* beta, const float* save_mean, const float* save_invstd, int training, int act,
                 int accumulate_params, int dtype, void* ws, size_t ws_bytes, void* stream);
/* rtsds_bn_bwd reading dy with row pitch ldy >= c (a channel slice of the concatenated
 * input's gradient; ldy != c: bf16, c % 8 == 0, ldy % 8 == 0).                              */
int rtsds_bn_bwd_ld(const void* dy, long ldy, const void* x, const void* y, void* dx, void* dres,
                    float* dgamma, float* dbeta, long rows, int c, const float* gamma,
                    const float* beta, const float* save_mean, const float* save_invstd, int training,
                    int act, int accumulate_params, int dtype, void* ws, size_t ws_bytes, void* stream);
/* rtsds_bn_bwd without its statistics pass: part / nrb = the channel-major (sum g,
 * sum g (x - mean)) partials of rtsds_conv2d_dgrad_bnstats (bf16, c % 8 == 0, no residual).  */
int rtsds_bn_bwd_part(const void* dy, const void* x, void* dx, float* dgamma, float* dbeta, long rows, int c,
                      const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                      int training, int act, int accumulate_params, const float* part, int nrb, int dtype, void* ws,
                      size_t ws_bytes, void* stream);

/* BatchNorm2d + ReLU + MaxPool2d(3, 2, p in {0,1}) fused -- the ResNet stem bn1 -> relu ->
 * maxpool (build_contextpath.py:15-18 via torchvision resnet.py; deeplabv2.py:106-110, ceil
 * mode via ho / wo).  bf16, c % 8 == 0.  x: the conv output [n][h][w][c]; y: pooled
 * [n][ho][wo][c]; idx: window argmax 0..8 per output element (first maximum in window order,
 * as ATen).  Statistics, running buffers and workspace as rtsds_bn_fwd (rows = n*h*w).  The
 * backward gathers dy_pool through idx inside the BatchNorm backward passes: dx = d(bn+relu)
 * of the pooled gradient; dgamma / dbeta as rtsds_bn_bwd.                                  */
int rtsds_bn_relu_maxpool_fwd(const void* x, void* y, uint8_t* idx, int n, int h, int w, int c, int ho, int wo,
                              int p, const float* gamma, const float* beta, float* running_mean,
                              float* running_var, long long* num_batches_tracked, float* save_mean,
                              float* save_invstd, float momentum, float eps, int training,
                              const float* stats_part, int stats_nrb, int dtype, void* ws, size_t ws_bytes,
                              void* stream);
int rtsds_bn_relu_maxpool_bwd(const void* dy_pool, const uint8_t* idx, const void* x, void* dx, float* dgamma,
                              float* dbeta, int n, int h, int w, int c, int ho, int wo, int p,
                              const float* gamma, const float* beta, const float* save_mean,
                              const float* save_invstd, int training, int accumulate_params, int dtype,
                              void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- layout / dtype
 * Input images arrive NCHW fp32 from the reference's loaders (datasets/cityscapes.py:62,
 * main.py:69-72).  cast: weight shadows (fp32 master -> bf16) and dtype round trips.
 * copy_channels: torch.cat along channels and its backward split (build_bisenet.py:72,153);
 * accumulate != 0: dst += src (a split slice whose tensor also has another reader).      */
int rtsds_nchw_to_nhwc(const float* x, void* y, int n, int c, int h, int w, int dtype, void* stream);
/* Same, written with channel pitch `pitch` (channels c..pitch-1 zero; pitch 4): the 3-channel
 * image batch in the layout rtsds_conv2d_input_pitch reports for the stem / spatial-path convs,
 * passed to them with RTSDS_INPUT_PADDED (main.py:46-108 loaders -> model input).           */
int rtsds_nchw_to_nhwc_pad(const float* x, void* y, int n, int c, int h, int w, int pitch, int dtype, void* stream);
int rtsds_cast(const void* src, int src_dtype, void* dst, int dst_dtype, long n, void* stream);
int rtsds_copy_channels(const void* src, int src_ld, int src_off, void* dst, int dst_ld, int dst_off,
                        long rows, int cnt, int accumulate, int dtype, void* stream);

/* ---------------------------------------------------------------- pointwise activations
 * act 1 ReLU (build_bisenet.py:77), 2 LeakyReLU(0.2) (model.py:62,73), 3 sigmoid
 * (build_bisenet.py:49,78).  Backward from the forward output y; act 0 = dx = alpha*dy
 * (GradientReversalFunction, model.py:9-17).                                              */
int rtsds_act_fwd(const void* x, void* y, long n, int act, int dtype, void* stream);
int rtsds_act_bwd(const void* dy, const void* y, void* dx, long n, int act, float alpha, int dtype,
                  void* stream);

/* ---------------------------------------------------------------- pooling
 * MaxPool2d (build_contextpath.py:21 via torchvision; deeplabv2.py:79 ceil_mode -- the
 * caller sizes ho/wo).  idx: uint8 tap index per output, consumed by the backward; NULL for
 * inference (3x3 windows with 16-B channel vectors only, else RTSDS_ERR_UNSUPPORTED).     */
int rtsds_maxpool_fwd(const void* x, void* y, uint8_t* idx, int n, int h, int w, int c, int ho,
                      int wo, int k, int s, int p, int dtype, void* stream);
int rtsds_maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int n, int h, int w, int c,
                      int ho, int wo, int k, int s, int p, int dtype, void* stream);
/* Global average pool over H*W (build_bisenet.py:46,75; build_contextpath.py:27-28;
 * model.py:63,82).  y: [n][c].  ws: rtsds_gap_workspace(n, hw, c) bytes (row-slice
 * partials of the two-stage reduction; also used by rtsds_chscale_bwd's da).              */
size_t rtsds_gap_workspace(int n, long hw, int c);
int rtsds_gap_fwd(const void* x, void* y, int n, long hw, int c, int dtype, void* ws, size_t ws_bytes,
                  void* stream);
/* dx (+)= broadcast(dy) / hw; accumulate: add into dx (the gradient another reader of x already
 * wrote there -- functional.GradJoin; same roundings as a separate elementwise add).          */
int rtsds_gap_bwd(const void* dy, void* dx, int n, long hw, int c, int accumulate, int dtype, void* stream);

/* ---------------------------------------------------------------- channel attention
 * mode 0: y = x*a[n][c] (build_bisenet.py:52,149); mode 1: y = x*a + x (build_bisenet.py:79-80).
 * Backward: dx (may be NULL), da[n][c] = sum_hw dy*x (may be NULL; needs
 * ws = rtsds_gap_workspace(n, hw, c) bytes).                                              */
/* Inference tail of FeatureFusionModule + the final 1x1 conv (build_bisenet.py:75-80, 167), two
 * launches: out = conv3(f * a + f) + b3 with a = sigmoid(conv2(relu(conv1(GAP(f)) + b1)) + b2);
 * f / out NHWC [n][hw][c] (c = 19 -- the class maps -- and hw a multiple of the 16-B vector length,
 * else RTSDS_ERR_UNSUPPORTED); w1..w3 [c][c] in the compute dtype, biases fp32 (NULL = 0).  Needs
 * ws >= rtsds_ffm_head_eval_workspace(n, hw, c) bytes (the GAP partials).                     */
size_t rtsds_ffm_head_eval_workspace(int n, long hw, int c);
int rtsds_ffm_head_eval(const void* f, const void* w1, const float* b1, const void* w2, const float* b2,
                        const void* w3, const float* b3, void* out, int n, long hw, int c, int dtype, void* ws,
                        size_t ws_bytes, void* stream);
int rtsds_chscale_fwd(const void* x, const void* a, void* y, int n, long hw, int c, int mode,
                      int dtype, void* stream);
int rtsds_chscale_bwd(const void* dy, const void* x, const void* a, void* dx, void* da, int n,
                      long hw, int c, int mode, int dtype, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- bilinear resize
 * F.interpolate(mode='bilinear', align_corners=False) (build_bisenet.py:151-152,158-159,166;
 * deeplabv2.py:126; model.py:23).  scale = in/out (size=) or 1/scale_factor, in fp32 as
 * ATen computes it.  The output (forward) / incoming grad (backward) may be a channel slice
 * of a wider NHWC tensor: pixel pitch *_ld (0 = c), channel offset *_off.               */
int rtsds_bilinear_fwd(const void* x, void* y, int n, int hi, int wi, int c, int ho, int wo,
                       float scale_h, float scale_w, int y_ld, int y_off, int dtype, void* stream);
/* Inference: rtsds_bilinear_fwd of (x * s1) * s2 (s1 / s2: optional [n][c] channel scales in the
 * activation dtype, each product rounded to it as rtsds_chscale_fwd mode 0 stores it) -- the
 * attention refinement's channel scales (build_bisenet.py:52-53, 157-159) folded into the
 * eval forward's resize.  Upsampling (ho >= hi) with c, y_ld, y_off multiples of a 16-B vector
 * only; RTSDS_ERR_UNSUPPORTED otherwise (the caller scales and resizes separately).      */
int rtsds_bilinear_fwd_scaled(const void* x, const void* s1, const void* s2, void* y, int n, int hi, int wi,
                              int c, int ho, int wo, float scale_h, float scale_w, int y_ld, int y_off,
                              int dtype, void* stream);
/* Backward = separable two-pass gather (W then H) through an fp32 workspace of
 * rtsds_bilinear_bwd_workspace() bytes; deterministic (no atomics).                      */
size_t rtsds_bilinear_bwd_workspace(int n, int hi, int wi, int c, int ho, int wo);
int rtsds_bilinear_bwd(const void* dy, void* dx, int n, int hi, int wi, int c, int ho, int wo,
                       float scale_h, float scale_w, int dy_ld, int dy_off, int dtype, void* ws,
                       size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- adaptive average pool
 * F.adaptive_avg_pool2d(x, (ho, wo)) of adversarial_train_2 (train.py:410,438,445): window
 * rows [floor(o*hi/ho), ceil((o+1)*hi/ho)), same for columns (ATen semantics), NHWC.
 * Backward gathers each input pixel's share of every window containing it (no atomics).   */
int rtsds_adaptive_avgpool_fwd(const void* x, void* y, int n, int hi, int wi, int c, int ho, int wo,
                               int dtype, void* stream);
int rtsds_adaptive_avgpool_bwd(const void* dy, void* dx, int n, int hi, int wi, int c, int ho, int wo,
                               int dtype, void* stream);

/* ---------------------------------------------------------------- softmax / losses
 * Logits addressed by element strides (sn, sc, shw) per (image, channel, pixel): NHWC and
 * NCHW both work.  Softmax over channels (train.py:225,245,256) writes NHWC with pitch
 * y_ld >= c (extra channels zeroed).                                                      */
int rtsds_softmax_fwd(const void* x, long sn, long sc, long shw, void* y, int y_ld, int n, long hw,
                      int c, int dtype, void* stream);
int rtsds_softmax_bwd(const void* dy, const void* y, int ld, void* dx, long sn, long sc, long shw,
                      int n, long hw, int c, int dtype, void* stream);
/* nn.CrossEntropyLoss(ignore_index) mean over valid pixels (main.py:124-130).  The forward
 * leaves the valid count at ((float*)ws)[2048]; pass that pointer as `count` to the bwd.  */
size_t rtsds_ce_workspace(void);
/* ws + 2048 floats holds (valid count C, loss sum S); rtsds_ce_finish sets loss = S / C after
 * the caller summed C over data-parallel ranks (the backward reads the same C).           */
int rtsds_ce_finish(const void* ws, float* loss, void* stream);
int rtsds_ce_fwd(const void* x, long sn, long sc, long shw, const int64_t* target, float* loss, int n,
                 long hw, int c, int ignore_index, int dtype, void* ws, size_t ws_bytes, void* stream);
int rtsds_ce_bwd(const void* x, long sn, long sc, long shw, const int64_t* target,
                 const float* grad_loss, const float* count, void* dx, int n, long hw, int c,
                 int ignore_index, int dtype, void* stream);
/* nn.BCEWithLogitsLoss() mean (main.py:131-132), fp32.                                  */
int rtsds_bce_fwd(const float* x, const float* target, float* loss, int n, void* stream);
int rtsds_bce_bwd(const float* x, const float* target, const float* grad_loss, float* dx, int n,
                  void* stream);

/* ---------------------------------------------------------------- optimizer
 * torch.optim.Adam step (main.py:116-117) over flat fp32 arenas; grad is multiplied by
 * grad_scale first (data-parallel 1/world).  bf16_shadow (may be NULL) receives bf16(param).
 * grad_dtype: RTSDS_F32, or RTSDS_F16 / RTSDS_BF16 for the all-reduced reduced-precision wire
 * copy of the gradients, read directly (no cast back into the fp32 gradient arena).         */
int rtsds_adam_step(float* param, const void* grad, float* exp_avg, float* exp_avg_sq,
                    void* bf16_shadow, long n, float lr, float beta1, float beta2, float eps,
                    float weight_decay, int step, float grad_scale, int grad_dtype, void* stream);

/* The same update with hyper = {lr, 1 - beta1^step, sqrt(1 - beta2^step)} (fp32, device
 * memory) read by the kernel: a captured hipGraph of the training step replays correct
 * updates while the host advances lr and step between replays.                            */
int rtsds_adam_step_dev(float* param, const void* grad, float* exp_avg, float* exp_avg_sq,
                        void* bf16_shadow, long n, const float* hyper, float beta1, float beta2,
                        float eps, float weight_decay, float grad_scale, int grad_dtype, void* stream);

/* torch.optim.SGD step (main.py:118-120) over a flat fp32 arena: d = grad*grad_scale
 * (+ weight_decay*param); with momentum, buf = d on the first step (first != 0), else
 * buf = momentum*buf + (1-dampening)*d; d = nesterov ? d + momentum*buf : buf;
 * param -= lr*d.  hyper (device fp32 {lr, first}, may be NULL) overrides lr / first for
 * hipGraph replays.  bf16_shadow (may be NULL) receives bf16(param).                       */
int rtsds_sgd_step(float* param, const void* grad, float* momentum_buf, void* bf16_shadow,
                   long n, const float* hyper, float lr, float momentum, float dampening,
                   float weight_decay, int nesterov, int first, float grad_scale, int grad_dtype, void* stream);

/* ---------------------------------------------------------------- metrics
 * argmax over channels, first maximum wins (train.py:102-106,272-275; validation.py:51).
 * out (int64 [n*hw]) may be NULL; if target and correct are given, *correct += #matches.
 * confusion: hist[nc*nc] += bincount(nc*label + pred) for 0 <= label < nc (utils.py:52-58). */
int rtsds_argmax(const void* x, long sn, long sc, long shw, int64_t* out, const int64_t* target,
                 unsigned long long* correct, int n, long hw, int c, int dtype, void* stream);
int rtsds_confusion(const int64_t* label, const int64_t* pred, unsigned long long* hist, long total,
                    int nc, void* stream);

/* ---------------------------------------------------------------- fused upsample + CE
 * Replaces, for nheads (<= 4) low-resolution NHWC logit maps of the same geometry
 * [n][hl][wl][c] (c <= 32), the chain F.interpolate(bilinear, align_corners=False) to
 * [n][c][H][W] -> nn.CrossEntropyLoss(ignore_index) per head -> (head 0) argmax == target
 * pixel count: build_bisenet.py:151-152,158-159,166, deeplabv2.py:126, train.py:86-106.
 * logits / dlogits: host arrays of nheads device pointers.  scale_h/w: ATen source scales
 * (in/out for size=, 1/scale_factor for scale_factor=; upsampling only, <= 1).
 * Forward writes loss[nheads] (mean over non-ignored pixels; may be NULL) and *loss_sum (their
 * sum in head order; may be NULL), adds the head-0 argmax matches to *correct (may be NULL;
 * overwrites it instead when want_grad carries RTSDS_UPCE_SET_CORRECT, so the caller need not
 * zero it) and, when want_grad & 1, keeps unscaled low-res gradient partials in ws.  Backward:
 * dlogits[h] = grad_loss[h * grad_stride] * d loss[h] / d logits[h] from those partials (ws
 * must be the forward's; grad_stride 0 = one upstream gradient for loss_sum).  Full-resolution logits are never materialised.  workspace()
 * returns 0 for geometries the fused path does not cover.                                 */
#define RTSDS_UPCE_SET_CORRECT 2
size_t rtsds_upce_workspace(int nheads, int n, int hl, int wl, int c, int H, int W, float scale_h,
                            float scale_w);
int rtsds_upce_fwd(int nheads, const void* const* logits, const int64_t* target, int n, int hl,
                   int wl, int c, int H, int W, float scale_h, float scale_w, int ignore_index,
                   float* loss, float* loss_sum, unsigned long long* correct, int want_grad,
                   int dtype, void* ws, size_t ws_bytes, void* stream);
/* Data-parallel global mean: ws starts with float stat[1 + nheads] = (valid-pixel count,
 * per-head loss sums).  After the caller sums stat[0] over ranks (a 1-element all-reduce),
 * rtsds_upce_finish recomputes loss / loss_sum = this rank's sums / global count, and
 * rtsds_upce_bwd scales by the global count: the ranks' losses and gradients sum to the
 * single-device mean over the gathered batch exactly.                                     */
int rtsds_upce_finish(int nheads, const void* ws, float* loss, float* loss_sum, void* stream);
int rtsds_upce_bwd(int nheads, const float* grad_loss, int grad_stride, void* const* dlogits,
                   int n, int hl, int wl, int c, int H, int W, float scale_h, float scale_w,
                   int dtype, const void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- discriminator input
 * softmax(interpolate_bilinear(x)) over classes (train.py:225,245,256) in one pass: x NHWC
 * [n][hi][wi][c], y NHWC [n][ho][wo][y_ld] with channels c..y_ld-1 zero (the padded input of
 * the discriminator's first conv, RTSDS_INPUT_PADDED).  Bit-identical to rtsds_bilinear_fwd
 * followed by the channel softmax.  rtsds_upsoftmax_bwd: dx = resize_adjoint(softmax_bwd(dy,
 * y)) (dy with row pitch dy_ld), bit-identical to the unfused backward chain.  c <= 32.      */
int rtsds_upsoftmax_fwd(const void* x, void* y, int n, int hi, int wi, int c, int ho, int wo,
                        float scale_h, float scale_w, int y_ld, int dtype, void* stream);
size_t rtsds_upsoftmax_bwd_workspace(int n, int hi, int wi, int c, int ho, int wo);
int rtsds_upsoftmax_bwd(const void* dy, int dy_ld, const void* y, int y_ld, void* dx, int n, int hi,
                        int wi, int c, int ho, int wo, float scale_h, float scale_w, int dtype,
                        void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- input pipeline
 * The reference's per-sample torchvision transforms (main.py:60-108; datasets/cityscapes.py:
 * 56-68, datasets/gta5.py:69-118) on a decoded HWC image in device memory.
 * rtsds_resize_aa: Resize((ho, wo), antialias=True) == F.interpolate(bilinear,
 *   align_corners=False, antialias=True) of the float image, optionally of its horizontal
 *   mirror (flip != 0: RandomHorizontalFlip applied before the resize), with the epilogue of
 *   kind 0: f32 HWC, 1: bf16 HWC (both (v - mean[c]) / std[c] when mean/std are given:
 *   Normalize on the 0-255 scale), 2: int64 label (round half-to-even, clamp to
 *   [clamp_lo, clamp_hi] when clamp_lo <= clamp_hi: IntRangeTransformer).  src_u8 selects a
 *   uint8 (else fp32) source.  dst is the image's slot in an NHWC batch.
 * rtsds_gaussian_blur: GaussianBlur((kx, ky), sigma) of a HWC image (uint8 or fp32 source),
 *   fp32 HWC out, reflect padding.
 * rtsds_gta5_decode: RGB label (HWC uint8) -> train id 0..18 (unmatched colours -> 0).      */
size_t rtsds_resize_aa_workspace(int c, int h, int w, int ho, int wo);
int rtsds_resize_aa(const void* src, int src_u8, int c, int h, int w, void* dst, int kind, int ho, int wo,
                    int flip, const float* mean, const float* std, int clamp_lo, int clamp_hi, void* ws,
                    size_t ws_bytes, void* stream);
int rtsds_gaussian_blur(const void* src, int src_u8, float* dst, int c, int h, int w, int kx, int ky,
                        float sigma_x, float sigma_y, void* stream);
int rtsds_gta5_decode(const uint8_t* rgb, int64_t* out, int h, int w, void* stream);

/* ---------------------------------------------------------------- graph replay
 * Replaces hipGraphLaunch of a captured multi-stream iteration (runtime.GraphedStep /
 * GraphedForward; the reference has no graphs: its train.py:65-113 / 172-284 loop bodies
 * launch every ATen kernel from the host).  rtsds_graph_split decomposes a captured hipGraph
 * (kernel / memcpy / memset / empty nodes) into at most max_lanes chains, cuts each chain at its
 * cross-chain edges into linear segments and instantiates one executable graph per segment;
 * rtsds_graph_split_launch replays them on one stream per chain (chain 0 = `stream`, which
 * also waits for the other chains at the end), with events for the cross-chain edges.  The
 * captured graph is only read (the caller keeps it and the memory it references alive).
 * Returns RTSDS_ERR_UNSUPPORTED for other node types (the caller replays the graph itself). */
int rtsds_graph_split(void* graph, int max_lanes, void** handle, int* n_segments, int* n_lanes);
/* Number of chains (<= max_lanes) rtsds_graph_split would use for `graph` -- 1 for a linear
 * (single-stream) capture; a negative RTSDS_ERR_* code on failure.  Nothing is instantiated. */
int rtsds_graph_lanes(void* graph, int max_lanes);
/* Number of nodes of a captured hipGraph (negative status on error); GraphedStep drops empty
 * segments (a capture between two back-to-back collectives). */
int rtsds_graph_nodes(void* graph);
/* Nodes captured so far by the capture `stream` records into (negative status when it is not
 * capturing); GraphedStep ends a graph segment at a collective only when it has nodes.        */
int rtsds_capture_nodes(void* stream);
int rtsds_graph_split_launch(void* handle, void* stream);
int rtsds_graph_split_destroy(void* handle);

/* Backward of the FFM attention on pooled vectors (build_bisenet.py:67-70): h = relu(conv1(p)),
 * a = sigmoid(conv2(h)), 1x1 convs on [n][c] rows (n <= 8, channels <= 64).  From da = dL/da:
 * dw2 / db2, dw1 / db1 (fp32 [cout][cin] / [cout]; overwritten, or added to when accumulate),
 * dp = dL/dp (stored).  w1 [c1][c0], w2 [c2][c1] in the compute dtype.  One launch; the
 * results equal the unfused chain's (act backward, pooled data / weight gradients) bit for bit
 * for channel counts that are not vector multiples (c % 8 bf16, c % 4 fp32).               */
int rtsds_pooled_mlp_bwd(const void* da, const void* a, const void* h, const void* p, const void* w1,
                         const void* w2, float* dw1, float* db1, float* dw2, float* db2, void* dp,
                         int n, int c0, int c1, int c2, int accumulate, int dtype, void* stream);

/* Its forward in one launch: h = relu(conv1(p) + b1), a = sigmoid(conv2(h) + b2) (b1 / b2 may
 * be NULL), h and a stored [n][c1] / [n][c2]; equal bit for bit to the two pooled 1x1 conv
 * launches of rtsds_conv2d_fwd for the same shapes (same limits as rtsds_pooled_mlp_bwd).     */
int rtsds_pooled_mlp_fwd(const void* p, const void* w1, const float* b1, const void* w2, const float* b2, void* h,
                         void* a, int n, int c0, int c1, int c2, int dtype, void* stream);

/* ABI revision of this header (RTSDS_ABI_VERSION): bumped whenever an entry point's signature
 * changes.  The Python loader refuses a library whose revision differs (A/B variant libraries
 * built from older sources would otherwise be called with the wrong argument lists). */
#define RTSDS_ABI_VERSION 10
int rtsds_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RTSDS_HIP_H */
