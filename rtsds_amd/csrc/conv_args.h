// Implicit-GEMM convolution: the kernel arguments and the tile choice shared by the host code
// (conv.hip) and the kernel translation units (conv_gemm_{fwd,dgrad,wgrad}.hip).
#pragma once
#include "common.h"

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

struct ConvArgs {
  const void* a;      // FWD: x   DGRAD: dy  WGRAD: dy
  const void* b;      // FWD: w   DGRAD: w^T (repacked [ci][r][s][co])  WGRAD: x
  const float* bias;  // FWD only
  void* out;          // FWD: y (T)  DGRAD: dx (T)  WGRAD: fp32 partials [split][M][N]
  int M, N, K;        // GEMM extents; K = reduction length
  int n, h, w, c, ho, wo, k, kh, kw, sh, sw, ph, pw, dh, dw;
  FastDiv f_howo, f_wo, f_hw, f_w, f_c, f_k, f_kw;
  int tiles_per_split;
  int wg_rows;        // WGRAD: 64-pixel K-tiles never straddle an image and map to whole / part
                      // output rows (ho*wo % 64 == 0 and wo | 64 or 64 | wo) -> affine gathers
  // DGRAD stride-phase decomposition (normal mode: tkw=kw, r0=0, rstep=1, psh=1, off=0,
  // hp=h, wp=w): output rows enumerate the pixels ih = th*psh + offh of one parity phase,
  // and the reduction runs over that phase's taps r = r0 + rr*rstep only.
  int tkw, r0h, r0w, rstep, psh, offh, offw, hp, wp;
  FastDiv f_tkw;
  int act;
  int accum;          // FWD/DGRAD: y += result
  // DGRAD: dx = result * act'(mask) -- the backward of the activation (ReLU / LeakyReLU) that
  // produced this conv's input (mask = that input, NHWC like dx), fused into the epilogue
  const void* mask;
  int mask_act;
  // DGRAD: the backward statistics of the BatchNorm (+ ReLU / LeakyReLU) that produced this
  // conv's input, from the stored dx values: per M tile and channel (sum g, sum g (x - mean)),
  // g = dx * act'(x * scale + shift) -- bn_bwd_stats_kernel's quantities, [N][mtile][2]
  float* bnb_part;
  const void* bnb_x;               // the BatchNorm's input, NHWC like dx
  const float *bnb_gamma, *bnb_beta, *bnb_mean, *bnb_invstd;
  int bnb_act;
  float* stats;       // FWD: per-M-tile BatchNorm partials [N][mtile][count, mean, M2, 0] (or null)
  long split_stride;  // elements between WGRAD split slabs (and DGRAD split-K slabs)
  float* slab;        // DGRAD split-K: fp32 partials [split][M][N] instead of the bf16 epilogue
  // FWD eval-mode BatchNorm fold: y = act(acc * scale[co] + bias[co] (+ res)), scale/bias the
  // running-statistics BN folded with the conv bias (rtsds_bn_fold); res = residual, same
  // layout as y (or null).
  const float* scale;
  const void* res;
  // FWD: row pitch of y in elements when y is a channel slice of a wider NHWC tensor (0 = N);
  // plain forward only (no residual / accumulate), checked by the host
  int ldo;
  int gbuf;           // operand tensors < 2 GiB: buffer-resource DMA with 32-bit offsets allowed
  // DGRAD stride-2: the parity phases of one conv in ONE launch (blockIdx.z = phase); each
  // phase patches the phase-dependent fields below over the shared ones.
  int nph;
  struct Phase {
    int hp, wp, offh, offw, r0h, r0w, tkw, M, K;
    FastDiv f_tkw, f_hw, f_w;
    long boff;  // element offset of the phase's repacked weights
  } phs[4];
};

// Tile selection for FWD / DGRAD (occupancy-aware): the widest tile that still puts >= 256
// workgroups on the 256 CUs.  bf16: 128x128 (or 160x128, see below) / 128x64 / 256x32 (19- and
// 1-channel outputs), falling back to 64x64 / 128x32 for small-M layers (ResNet layer4, pooled
// vectors).
static inline void pick_tile(long M, int N, bool b16, int& bm, int& bn, bool fwd = false, long K = 0, bool m160 = false) {
  auto blocks = [&](int a, int b) { return ((M + a - 1) / a) * (long)((N + b - 1) / b); };
  if (b16) {
    // short reductions (K <= 512: 1-8 K-steps, DeepLab's layer1-3 1x1 convs) cannot hide the
    // gather latency or the epilogue inside one workgroup; 128 x 64 tiles (48 KB of LDS: 3
    // groups per CU instead of 2) overlap more of them across workgroups (64 -> 256 1x1
    // forward 44 -> 33 us, 1024 -> 256 data gradient 72 -> 66 us; profiles/r2_conv_shortk_ab.txt)
    if (N > 64 && K > 0 && K <= 512 && blocks(128, 64) >= 1024) { bm = 128; bn = 64; return; }
    // (data gradients keep 128 rows: 4 groups per CU instead of 2 hide more of the gather
    // latency -- TinyD conv1's dgrad on the padded probabilities 313 -> 296 us at bs 8, 140 ->
    // 119 us at 1280x720 bs 2)
    if (N <= 32) { bn = 32; bm = fwd && blocks(256, 32) >= 256 ? 256 : 128; }
    else if (N <= 64) { bn = 64; bm = blocks(128, 64) >= 256 ? 128 : 64; }
    else if (blocks(128, 128) >= 512) {
      // tail quantisation: 2 workgroups per CU = 512 slots per round.  A 160-row tile (still 2
      // per CU in FWD: 113 VGPRs; the DGRAD instantiation needs 181 and would run 1 per CU)
      // when it needs fewer row-weighted rounds -- DeepLab's M = 33,540 rows: 526 tiles of
      // 128 (2 rounds, the second 3 % full) vs 420 of 160 (1 round)
      bn = 128;
      const long r128 = (blocks(128, 128) + 511) / 512, r160 = (blocks(160, 128) + 511) / 512;
      bm = (fwd || m160) && r160 * 160 < r128 * 128 ? 160 : 128;
    }
    else if (blocks(128, 64) >= 384) { bm = 128; bn = 64; }
    else { bm = 64; bn = 64; }
  } else {
    if (N <= 32) { bm = 128; bn = 32; } else { bm = 64; bn = 64; }
  }
}

// Entry points of the kernel translation units (explicit instantiations): dispatch_align picks
// the tile for FWD / DGRAD, launch_al runs one fixed tile (DGRAD split-K), wgrad_launch the
// WGRAD tiles.
template <typename T, int MODE> void dispatch_align(const ConvArgs& p, int cr, hipStream_t st, int splits = 1);
template <typename T, int MODE, int BM, int BN, int BK, int WM, int WN>
void launch_al(const ConvArgs& p, int cr, hipStream_t st, int splits = 1);
template <typename T> void wgrad_launch(const ConvArgs& p, int bm, int bn, int splits, hipStream_t st);
