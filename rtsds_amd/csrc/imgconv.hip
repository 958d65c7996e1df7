// Direct MFMA convolution for the 3-channel stride-2 image convs: the ResNet stem 7x7 s2 p3
// (build_contextpath.py via torchvision conv1; deeplabv2.py:106) and the spatial path's first
// ConvBlock 3x3 s2 p1 (build_bisenet.py:9-14, 21), 64 output channels, forward only (the image
// needs no data gradient; the weight gradient stays on the implicit GEMM's superpixel path).
//
// These convs are epilogue-bound, not MFMA-bound: 2 x 3.6-13 GFLOP against a 134 MB output at bs 8
// 1024x512.  As an implicit GEMM each 128-row tile ran 2-7 K-steps behind a register-staged
// gather, then a full epilogue -- 73 / 112 us per launch (30 % of the HBM bound).  Here a
// workgroup owns a 4 x 64 output tile with all 64 channels:
//  * the tile's input rows are staged ONCE into LDS as 16-B "superpixels" (two horizontally
//    adjacent pixels of the 4-channel-padded image, conv.hip sp_path): (2*4 + kh - 2) rows x
//    (64 + (kw+1)/2 - 1) superpixels, one buffer-resource LDS-DMA per 16 B, padding zero-filled
//    by the DMA (offsets past num_records);
//  * with odd padding, taps s = 2p - 1 + q of output column ow read superpixel ow - (pw+1)/2 + p,
//    so in superpixel units the conv is stride 1 horizontally: an A fragment (16 pixels x one
//    superpixel of K) is one ds_read_b128 of 16 consecutive LDS superpixels;
//  * wave w computes output channels 16w..16w+15 for all 256 pixels: its B fragments (kh *
//    (kw+1)/2 superpixel slots of 8 weights, zero for the padding channel / taps outside the
//    kernel) are built once in registers from the [64][kh][kw][3] weights (DMA-staged raw
//    into LDS beside the input rows) -- no repack launch;
//  * K order (row tap, superpixel, 8 elements) in 32-deep MFMA steps, identical to the
//    superpixel GEMM's BK = 32 K-steps, so the accumulators match it bit for bit;
//  * epilogue: bias or eval-BN scale / shift, activation, the following BatchNorm's per-tile
//    (count, mean, M2) from the fp32 values, and 8-B stores of 4 channels per pixel straight
//    from the (transposed) accumulators.
// Inference also has a variant with the stem's 3x3 stride-2 max pool in the epilogue
// (imgconv_pool_kernel): the full-resolution activation is never written.
#include "common.h"

template <int N> RT_DEV void wait_vmcnt_img() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// Sum over the 16 lanes of a DPP row (every lane of the row ends with the total): quad_perm
// [1,0,3,2], [2,3,0,1], then row_half_mirror, row_mirror -- VALU ops, no LDS round trip.
RT_DEV float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
// 8-B buffer store; an offset past num_records is dropped by the hardware
RT_DEV void store8(rsrc_t r, bf16x4 v, int off) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
#endif
}

// Activation of the epilogues.  ACT >= 0: the activation fixed at compile time (RTSDS_ACT_NONE /
// RTSDS_ACT_RELU, the ones the image convs run with), ACT < 0: chosen per launch.  With the
// runtime choice every value paid the uniform compare-and-branch chain of the switch (~200
// scalar branches per tile in the pooled stem); the fixed forms are one VALU op or none.
template <int ACT>
RT_DEV float img_act(float t, int act) {
  const int a = ACT >= 0 ? ACT : act;
  if (a == RTSDS_ACT_RELU) return fmaxf(t, 0.f);
  if (a == RTSDS_ACT_LEAKY) return t > 0.f ? t : 0.2f * t;
  if (a == RTSDS_ACT_SIGMOID) return 1.f / (1.f + expf(-t));
  return t;
}
static int img_act_variant(int act) { return act == RTSDS_ACT_NONE ? 0 : act == RTSDS_ACT_RELU ? 1 : -1; }

namespace {
constexpr int kTH = 4, kTW = 64;   // output tile rows x columns (all 64 channels)
constexpr int kCo = 64;            // output channels (4 waves x 16)
}  // namespace

struct ImgArgs {
  const bf16* x4;      // [n][h][w][4], channel 3 zero
  const bf16* wt;      // [64][kh][kw][3]
  const float* bias;   // [64] or null (eval fold: shift)
  const float* scale;  // [64] or null (eval fold)
  bf16* y;             // [n][ho][wo][64]
  float* stats;        // [64][tiles][4] (count, mean, M2, 0) or null
  int n, h, w, ho, wo, ph, pw, act;
  int tiles, per;      // tiles, tiles per workgroup (a contiguous run)
};

// WP x WC waves: WP pixel halves (8 groups each) x WC channel slices of 64 / WC
template <int KH, int KW, int WP, int ACT>
__global__ void __launch_bounds__(256, (KH == 7 || WP != 1) ? 2 : 3) imgconv_fwd_kernel(const ImgArgs P) {
  constexpr int WC = 4 / WP, GP = 16 / WP, NCB = kCo / WC / 16;  // pixel groups, 16-channel blocks per wave
  constexpr int KWP = (KW + 1) / 2;          // superpixels per row tap
  constexpr int NQ = KH * KWP;               // superpixel slots of K
  constexpr int KS = (NQ + 3) / 4;           // 32-deep MFMA steps
  constexpr int NR = 2 * kTH + KH - 2;       // staged input rows
  constexpr int NC = kTW + KWP - 1;          // staged superpixels per row
  constexpr int NP = NR * NC;                // 16-B pieces
  constexpr int NI = (NP + 63) / 64;         // DMA wave-instructions per tile
  constexpr int NIW = (NI + 3) / 4;          // per wave
  constexpr int W_EL = kCo * KH * KW * 3;    // raw weights
  constexpr int NWI = (W_EL * 2 + 1023) / 1024, NWIW = (NWI + 3) / 4;
  constexpr int A_BYTES = NI * 1024;
  __shared__ __attribute__((aligned(16))) unsigned char lds[NWI * 1024 + 2 * A_BYTES];
  unsigned char* const abuf = lds + NWI * 1024;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid;
  {  // XCD-aware bijective remap: the workgroups of one XCD take adjacent runs of tiles
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int t0 = bid * P.per, t1 = min(P.tiles, t0 + P.per);
  const int tw_n = (P.wo + kTW - 1) / kTW, th_n = (P.ho + kTH - 1) / kTH;
  const int spw = P.w >> 1;                  // superpixels per image row
  const int pwp = (P.pw + 1) >> 1;
  const rsrc_t rx = make_rsrc(P.x4, P.n * P.h * P.w * 8);
  const rsrc_t ry = make_rsrc(P.y, P.n * P.ho * P.wo * kCo * 2);
  auto tile_xy = [&](int t, int& img, int& oh0, int& ow0) {
    img = t / (th_n * tw_n);
    const int rem = t - img * th_n * tw_n, trow = rem / tw_n;
    oh0 = trow * kTH;
    ow0 = (rem - trow * tw_n) * kTW;
  };
  // input rows of tile t (zero outside the image) -> A buffer b
  auto issue = [&](int t, int b) {
    int img, oh0, ow0;
    tile_xy(t, img, oh0, ow0);
    const int ih0 = 2 * oh0 - P.ph, j0 = ow0 - pwp;
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const int ins = wave + 4 * i;
      if (ins < NI) {
        const int piece = ins * 64 + lane;
        const int row = piece / NC, col = piece - row * NC;
        const int ih = ih0 + row, j = j0 + col;
        const bool ok = piece < NP && (unsigned)ih < (unsigned)P.h && (unsigned)j < (unsigned)spw;
        buf_lds16(rx, abuf + b * A_BYTES + ins * 1024, ok ? ((img * P.h + ih) * spw + j) * 16 : (int)0x80000000, 0);
      }
    }
  };

  // ---- raw weights (once per workgroup), then the first tile's input
  const rsrc_t rw = make_rsrc(P.wt, W_EL * 2);
#pragma unroll
  for (int i = 0; i < NWIW; ++i) {
    const int ins = wave + 4 * i;
    if (ins < NWI) buf_lds16(rw, lds + ins * 1024, (ins * 64 + lane) * 16, 0);
  }
  issue(t0, 0);
  const int fr = lane & 15, fc = lane >> 4;
  const int wp = wave / WC, c0 = (wave % WC) * (kCo / WC);  // pixel half, first channel
  // this lane's output channels: c0 + 16 cb + 4 (lane >> 4) + e
  float bv[NCB][4], sv[NCB][4];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ch = c0 + 16 * cb + 4 * fc + e;
      bv[cb][e] = P.bias ? P.bias[ch] : 0.f;
      sv[cb][e] = P.scale ? P.scale[ch] : 1.f;
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- weight fragments (the MFMA's A operand: rows = channels c0 + 16 cb + (lane & 15), K
  // slot q = 4 ks + (lane >> 4)) and the per-slot LDS offsets of the pixel fragments
  const bf16* ws = (const bf16*)lds;
  bf16x8 fw[NCB][KS];
  int koff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int q = 4 * ks + fc;
    const int r = q / KWP, p = q - r * KWP;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      const int n = c0 + 16 * cb + fr;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int s = 2 * p - 1 + (e >> 2), ch = e & 3;
        bf16 v = (bf16)0.f;
        if (q < NQ && ch < 3 && s >= 0 && s < KW) v = ws[((n * KH + r) * KW + s) * 3 + ch];
        fw[cb][ks][e] = v;
      }
    }
    // slots past NQ carry zero weights: read any staged (finite) superpixel for them
    const int qq = q < NQ ? q : 0;
    koff[ks] = ((qq / KWP) * NC + (qq % KWP) + fr) * 16;
  }
  auto act_f = [&](float t) { return img_act<ACT>(t, P.act); };

  float rn = 0.f, rmean[NCB][4], rm2[NCB][4];  // running BatchNorm statistics of this wave's channels
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
    for (int e = 0; e < 4; ++e) rmean[cb][e] = rm2[cb][e] = 0.f;
  for (int t = t0; t < t1; ++t) {
    const int b = (t - t0) & 1;
    // tile t's input landed (the GP * NCB newest VMEM ops are the previous tile's output stores,
    // issued after this DMA), every wave is done with the other buffer: refill it
    if (t > t0) wait_vmcnt_img<GP * NCB>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < t1) issue(t + 1, b ^ 1);
    int img, oh0, ow0;
    tile_xy(t, img, oh0, ow0);

    // ---- this wave's GP pixel groups (group g = GP wp + i: tile row g / 4, columns 16 (g % 4)
    // + (lane & 15)) x NCB channel blocks: C^T = W x X^T, so each lane ends with 4 consecutive
    // channels of one pixel per block
    f32x4 acc[GP][NCB];
#pragma unroll
    for (int i = 0; i < GP; ++i)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[i][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned char* ab = abuf + b * A_BYTES;
    // group-major with one group of look-ahead: group i + 1's KS fragments are read before
    // group i's MFMAs (two register sets; the scheduling barriers keep the reads where they
    // are placed -- left alone the scheduler hoisted all GP x KS reads and spilled, and reading
    // each group right before its MFMAs exposed the LDS latency once per group)
    auto rdg = [&](int i, bf16x8* fa) {
      const int g = GP * wp + i;
      const int goff = ((2 * (g >> 2)) * NC + (g & 3) * 16) * 16;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) fa[ks] = *(const bf16x8*)(ab + koff[ks] + goff);
    };
    bf16x8 fa0[KS], fa1[KS];
    rdg(0, fa0);
#pragma unroll
    for (int i = 0; i < GP; ++i) {
      bf16x8* fa = (i & 1) ? fa1 : fa0;
      if (i + 1 < GP) rdg(i + 1, (i & 1) ? fa0 : fa1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
          acc[i][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[cb][ks], fa[ks], acc[i][cb], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: acc[i][cb][e] = C[channel c0 + 16 cb + 4 (lane >> 4) + e][pixel]
    const int vrows = min(kTH, P.ho - oh0), vcols = min(kTW, P.wo - ow0);
#pragma unroll
    for (int i = 0; i < GP; ++i)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][cb][e] = fmaf(acc[i][cb][e], sv[cb][e], bv[cb][e]);
    auto pix_ok = [&](int g) { return (g >> 2) < vrows && (g & 3) * 16 + fr < vcols; };
    if (P.stats) {
      // per-channel (count, mean, M2) over the valid pixels of this wave's part of the tile,
      // exact two-pass: lane sums over its GP pixels, then over the 16 lanes holding the same
      // channels; merged (Chan) into the workgroup's running statistics
      int nv = 0;
#pragma unroll
      for (int i = 0; i < GP; ++i) {
        const int g = GP * wp + i;
        nv += (g >> 2) < vrows ? max(0, min(16, vcols - (g & 3) * 16)) : 0;
      }
      const float cnt = (float)nv;
      const float rn1 = rn + cnt;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        float mean[4];
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          float sacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < GP; ++i) {
            const bool ok = pix_ok(GP * wp + i);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float d = pass == 0 ? acc[i][cb][e] : acc[i][cb][e] - mean[e];
              if (ok) sacc[e] += pass == 0 ? d : d * d;
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sacc[e] = row16_sum(sacc[e]);
            if (pass == 0) mean[e] = nv ? sacc[e] / cnt : 0.f;
          }
          if (pass == 1 && nv) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if (rn == 0.f) {
                rmean[cb][e] = mean[e];
                rm2[cb][e] = sacc[e];
              } else {
                const float dd = mean[e] - rmean[cb][e];
                rmean[cb][e] += dd * (cnt / rn1);
                rm2[cb][e] += sacc[e] + dd * dd * (rn * cnt / rn1);
              }
            }
          }
        }
      }
      rn = rn1;
    }
    // ---- 8-B stores of 4 channels per pixel; rows / columns past the output fall past
    // num_records and are dropped (every wave issues exactly GP * NCB stores per tile)
#pragma unroll
    for (int i = 0; i < GP; ++i) {
      const int g = GP * wp + i;
      const int oh = oh0 + (g >> 2), ow = ow0 + (g & 3) * 16 + fr;
      const bool ok = pix_ok(g);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)act_f(acc[i][cb][e]);
        const int off = ok ? (((img * P.ho + oh) * P.wo + ow) * kCo + c0 + 16 * cb + 4 * fc) * 2 : (int)0x80000000;
        store8(ry, o, off);
      }
    }
  }
  if (P.stats && fr == 0) {  // partial-statistics row WP bid + wp: [channel][row][4]
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        *(f32x4*)(P.stats + ((long)(c0 + 16 * cb + 4 * fc + e) * gridDim.x * WP + WP * bid + wp) * 4) =
            f32x4{rn, rmean[cb][e], rm2[cb][e], 0.f};
  }
}

// ---- conv + eval BatchNorm (folded scale / shift) + activation + MaxPool2d(3, 2, pp) (the
// ResNet stem at inference: build_contextpath.py via torchvision resnet; deeplabv2.py:106-110,
// ceil mode).  A tile is PH pooled rows x 31 pooled columns: conv rows 2 po0 - pp .. + 2 PH and
// 64 conv columns from 2 pc0 - pp (the 31 windows need 63 of them), (2 PH + 1) x 4 MFMA pixel
// groups per wave (4 waves x 16 channels).  Each conv value is rounded to bf16 exactly as the conv kernel stores
// it; the window maximum is taken vertically in registers and horizontally across lanes
// (ds_bpermute), conv positions outside the conv output are skipped (padding / ceil-mode
// windows), so the result equals imgconv_fwd_kernel followed by maxpool_fwd_k3 bit for bit.
namespace {
constexpr int kPW = 31;  // pooled columns per tile
}
struct ImgPoolArgs {
  const bf16* x4;
  const bf16* wt;
  const float* shift;
  const float* scale;
  bf16* y;             // [n][hp][wp][64]
  int n, h, w, ho, wo, ph, pw, act;
  int hp, wp, pp;      // pooled output size, pool padding
  int tiles, per;
};
template <int KH, int KW, int PH, int ACT>
__global__ void __launch_bounds__(256, 2) imgconv_pool_kernel(const ImgPoolArgs P) {
  constexpr int KWP = (KW + 1) / 2, NQ = KH * KWP, KS = (NQ + 3) / 4;
  constexpr int CR = 2 * PH + 1, NG = 4 * CR;  // conv rows, pixel groups per tile
  constexpr int NR = 2 * (CR - 1) + KH;      // input rows of the CR conv rows (stride 2)
  constexpr int NC = 64 + KWP - 1;
  constexpr int NP = NR * NC, NI = (NP + 63) / 64, NIW = (NI + 3) / 4;
  constexpr int W_EL = kCo * KH * KW * 3;
  constexpr int NWI = (W_EL * 2 + 1023) / 1024, NWIW = (NWI + 3) / 4;
  constexpr int A_BYTES = NI * 1024;
  constexpr int NST = 4 * PH;                // output store instructions per wave and tile
  __shared__ __attribute__((aligned(16))) unsigned char lds[NWI * 1024 + 2 * A_BYTES];
  unsigned char* const abuf = lds + NWI * 1024;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid;
  {
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int t0 = bid * P.per, t1 = min(P.tiles, t0 + P.per);
  const int tw_n = (P.wp + kPW - 1) / kPW, th_n = (P.hp + PH - 1) / PH;
  const int spw = P.w >> 1, pwp = (P.pw + 1) >> 1;
  const rsrc_t rx = make_rsrc(P.x4, P.n * P.h * P.w * 8);
  const rsrc_t ry = make_rsrc(P.y, P.n * P.hp * P.wp * kCo * 2);
  auto tile_xy = [&](int t, int& img, int& po, int& pc0) {  // po: the tile's first pooled row
    img = t / (th_n * tw_n);
    const int rem = t - img * th_n * tw_n, tr = rem / tw_n;
    po = tr * PH;
    pc0 = (rem - tr * tw_n) * kPW;
  };
  auto issue = [&](int t, int b) {
    int img, po, pc0;
    tile_xy(t, img, po, pc0);
    const int cr0 = 2 * po - P.pp, cc0 = 2 * pc0 - P.pp;
    const int ih0 = 2 * cr0 - P.ph, j0 = cc0 - pwp;
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const int ins = wave + 4 * i;
      if (ins < NI) {
        const int piece = ins * 64 + lane;
        const int row = piece / NC, col = piece - row * NC;
        const int ih = ih0 + row, j = j0 + col;
        const bool ok = piece < NP && (unsigned)ih < (unsigned)P.h && (unsigned)j < (unsigned)spw;
        buf_lds16(rx, abuf + b * A_BYTES + ins * 1024, ok ? ((img * P.h + ih) * spw + j) * 16 : (int)0x80000000, 0);
      }
    }
  };
  const rsrc_t rw = make_rsrc(P.wt, W_EL * 2);
#pragma unroll
  for (int i = 0; i < NWIW; ++i) {
    const int ins = wave + 4 * i;
    if (ins < NWI) buf_lds16(rw, lds + ins * 1024, (ins * 64 + lane) * 16, 0);
  }
  if (t0 < t1) issue(t0, 0);
  const int fr = lane & 15, fc = lane >> 4;
  const int nb = wave * 16 + 4 * fc;         // this lane's output channels nb .. nb + 3
  float bv[4], sv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    bv[e] = P.shift ? P.shift[nb + e] : 0.f;
    sv[e] = P.scale ? P.scale[nb + e] : 1.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const bf16* ws = (const bf16*)lds;
  bf16x8 fw[KS];
  int koff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int q = 4 * ks + fc;
    const int r = q / KWP, p = q - r * KWP;
    const int n = wave * 16 + fr;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int s = 2 * p - 1 + (e >> 2), ch = e & 3;
      bf16 v = (bf16)0.f;
      if (q < NQ && ch < 3 && s >= 0 && s < KW) v = ws[((n * KH + r) * KW + s) * 3 + ch];
      fw[ks][e] = v;
    }
    const int qq = q < NQ ? q : 0;
    koff[ks] = ((qq / KWP) * NC + (qq % KWP) + fr) * 16;
  }
  auto act_f = [&](float t) { return img_act<ACT>(t, P.act); };
  // window maximum with maxpool_fwd_k3's rule (a NaN wins)
  auto mx = [](float best, float f) { return (f > best || (f != f && best == best)) ? f : best; };

  for (int t = t0; t < t1; ++t) {
    const int b = (t - t0) & 1;
    if (t > t0) wait_vmcnt_img<NST>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < t1) issue(t + 1, b ^ 1);
    int img, po, pc0;
    tile_xy(t, img, po, pc0);
    const int cr0 = 2 * po - P.pp, cc0 = 2 * pc0 - P.pp;

    // NG pixel groups: conv row g / 4, columns 16 (g % 4) + (lane & 15)
    f32x4 acc[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned char* ab = abuf + b * A_BYTES;
    // (no look-ahead here, unlike imgconv_fwd_kernel: its second fragment set costs this kernel
    // a workgroup per CU -- 155 -> 194 VGPRs, eval stem 70 -> 78 us)
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int goff = ((2 * (g >> 2)) * NC + (g & 3) * 16) * 16;
      bf16x8 fa[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) fa[ks] = *(const bf16x8*)(ab + koff[ks] + goff);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ks], fa[ks], acc[g], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // the conv outputs as stored by the conv kernel (folded BN, activation, bf16 rounding), in
    // place; a NaN anywhere in the wave's tile sends the wave down the exact NaN-ordered path
    float probe = 0.f;
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[g][e] = (float)(bf16)act_f(fmaf(acc[g][e], sv[e], bv[e]));
        probe = fmaf(acc[g][e], 0.f, probe);  // NaN iff some value is NaN or infinite
      }
    const bool exact = __builtin_amdgcn_ballot_w64(probe != probe) != 0;  // wave-uniform
#pragma unroll
    for (int pr = 0; pr < PH; ++pr) {
      // vertical maxima (invalid conv positions skipped: -inf)
      float vm[4][4];
#pragma unroll
      for (int cg = 0; cg < 4; ++cg) {
        const int cc = cc0 + cg * 16 + fr;
        const bool cok = (unsigned)cc < (unsigned)P.wo;
#pragma unroll
        for (int e = 0; e < 4; ++e) vm[cg][e] = -INFINITY;
        if (exact) {
          bool any = false;
#pragma unroll
          for (int tr = 0; tr < 3; ++tr) {
            const int cr = cr0 + 2 * pr + tr;
            if ((unsigned)cr < (unsigned)P.ho && cok) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float v = acc[(2 * pr + tr) * 4 + cg][e];
                vm[cg][e] = any ? mx(vm[cg][e], v) : v;
              }
              any = true;
            }
          }
        } else {  // no NaN: compare-and-select from -inf gives the same maximum (and the same zero sign)
#pragma unroll
          for (int tr = 0; tr < 3; ++tr) {
            const int cr = cr0 + 2 * pr + tr;
            if ((unsigned)cr < (unsigned)P.ho) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float v = cok ? acc[(2 * pr + tr) * 4 + cg][e] : -INFINITY;
                vm[cg][e] = v > vm[cg][e] ? v : vm[cg][e];
              }
            }
          }
        }
      }
      // horizontal: pooled column j = 8 cg + fr / 2 (even lanes) covers local conv columns
      // fr, fr + 1, fr + 2 of group cg (fr + 2 = 16: lane 0 of group cg + 1)
#pragma unroll
      for (int cg = 0; cg < 4; ++cg) {
        const int l1 = (lane & ~15) | ((fr + 1) & 15), l2 = (lane & ~15) | ((fr + 2) & 15);
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a1 = __shfl(vm[cg][e], l1, 64);
          const float a2s = __shfl(vm[cg][e], l2, 64), a2n = __shfl(vm[cg < 3 ? cg + 1 : cg][e], l2, 64);
          const float a2 = fr + 2 < 16 ? a2s : a2n;  // (the selection is the reader's)
          // window order: left column, then middle, then right (skip -inf = no valid position)
          float best = vm[cg][e];
          if (exact) {
            best = a1 == -INFINITY ? best : (best == -INFINITY ? a1 : mx(best, a1));
            best = a2 == -INFINITY ? best : (best == -INFINITY ? a2 : mx(best, a2));
          } else {
            best = a1 > best ? a1 : best;
            best = a2 > best ? a2 : best;
          }
          o[e] = best;
        }
        const int pc = pc0 + cg * 8 + (fr >> 1), pry = po + pr;
        const bool ok = (fr & 1) == 0 && cg * 8 + (fr >> 1) < kPW && pry < P.hp && pc < P.wp;
        bf16x4 ov;
#pragma unroll
        for (int e = 0; e < 4; ++e) ov[e] = (bf16)o[e];
        store8(ry, ov, ok ? (((img * P.hp + pry) * P.wp + pc) * kCo + nb) * 2 : (int)0x80000000);
      }
    }
  }
}

// ---- host -------------------------------------------------------------------------------
// The superpixel geometry of conv.hip's sp_path with 64 output channels and a 7x7 or 3x3 kernel.
bool imgconv_ok(const rtsds_conv_desc* d) {
  if (!(d->dtype == RTSDS_BF16 && d->c == 3 && d->k == kCo && d->sh == 2 && d->sw == 2 && d->dh == 1 && d->dw == 1 &&
        (d->pw & 1) == 1 && (d->w & 1) == 0))
    return false;
  if (!((d->kh == 7 && d->kw == 7) || (d->kh == 3 && d->kw == 3))) return false;
  return (long)d->n * d->h * d->w * 8 < (1L << 31) && (long)d->n * d->ho * d->wo * kCo * 2 < (1L << 31);
}
// Wave layouts (measured, tools/ab_imgconv.sh, bs 8 1024x512): the 7x7 stem in 2 pixel halves x
// 2 channel halves (71.5 / 57 us train / eval vs 74 / 60.5 in 4 channel quarters); the 3x3
// spatial-path conv in channel quarters with the statistics epilogue (54 vs 58 us) and pixel
// halves without it (41.5 vs 45.8 us).
template <int ACT>
static const void* img_kernel_act(int kh, bool stats) {
  if (kh == 7) return (const void*)imgconv_fwd_kernel<7, 7, 2, ACT>;
  return stats ? (const void*)imgconv_fwd_kernel<3, 3, 1, ACT> : (const void*)imgconv_fwd_kernel<3, 3, 2, ACT>;
}
static const void* img_kernel(int kh, bool stats, int act) {
  const int v = img_act_variant(act);
  return v == 0 ? img_kernel_act<0>(kh, stats) : v == 1 ? img_kernel_act<1>(kh, stats) : img_kernel_act<-1>(kh, stats);
}
static int img_wp(int kh, bool stats) { return kh == 7 ? 2 : (stats ? 1 : 2); }
static int img_tiles(const rtsds_conv_desc* d) { return d->n * rt_cdiv(d->ho, kTH) * rt_cdiv(d->wo, kTW); }
// Persistent grid: every workgroup walks a contiguous run of `per` tiles (weights staged once,
// the next tile's input DMA in flight behind the current tile's MFMAs and stores); enough
// workgroups for the resident slots of all CUs.  Every workgroup gets >= 1 tile.
static void img_grid(const rtsds_conv_desc* d, bool stats, int& grid, int& per) {
  static int occ[3] = {0, 0, 0}, cus = 0;
  const int v = d->kh == 7 ? 2 : (stats ? 1 : 0);
  // (the activation variants share the launch bounds and register budget: ReLU's stands for all)
  if (!occ[v] && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[v], img_kernel(d->kh, stats, RTSDS_ACT_RELU), 256, 0) != hipSuccess ||
                  occ[v] < 1))
    occ[v] = 1;
  if (!cus && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus < 1)) cus = 256;
  const int tiles = img_tiles(d), slots = cus * occ[v];
  per = (tiles + slots - 1) / slots;
  grid = (tiles + per - 1) / per;
}
// BatchNorm partial-statistics rows of the training launch: one per workgroup and pixel part
int imgconv_tiles(const rtsds_conv_desc* d) {
  int grid, per;
  img_grid(d, true, grid, per);
  return grid * img_wp(d->kh, true);
}
void imgconv_fwd(const rtsds_conv_desc* d, const void* x4, const void* w, const float* bias, const float* scale, void* y,
                 int act, float* stats, hipStream_t st) {
  ImgArgs a;
  a.x4 = (const bf16*)x4; a.wt = (const bf16*)w; a.bias = bias; a.scale = scale; a.y = (bf16*)y; a.stats = stats;
  a.n = d->n; a.h = d->h; a.w = d->w; a.ho = d->ho; a.wo = d->wo; a.ph = d->ph; a.pw = d->pw; a.act = act;
  a.tiles = img_tiles(d);
  int grid;
  img_grid(d, stats != nullptr, grid, a.per);
  void* args[] = {&a};
  (void)hipLaunchKernel(img_kernel(d->kh, stats != nullptr, act), dim3(grid), dim3(256), args, 0, st);
}

// Pooled stem at inference (imgconv_pool_kernel): conv + folded BN + act + MaxPool2d(3, 2, pp).
bool imgconv_pool_ok(const rtsds_conv_desc* d, int hp, int wp) {
  return imgconv_ok(d) && d->kh == 7 && hp > 0 && wp > 0 && (long)d->n * hp * wp * kCo * 2 < (1L << 31);
}
void imgconv_pool_fwd(const rtsds_conv_desc* d, const void* x4, const void* w, const float* shift, const float* scale, void* y,
                      int act, int hp, int wp, int pp, hipStream_t st) {
  ImgPoolArgs a;
  a.x4 = (const bf16*)x4; a.wt = (const bf16*)w; a.shift = shift; a.scale = scale; a.y = (bf16*)y;
  a.n = d->n; a.h = d->h; a.w = d->w; a.ho = d->ho; a.wo = d->wo; a.ph = d->ph; a.pw = d->pw; a.act = act;
  a.hp = hp; a.wp = wp; a.pp = pp;
// 2 pooled rows per tile (tools/ab_pool.sh, bs 8 1024x512: 106 us vs 111 at 1 row, 155 at 3 with
// one group per CU; the separate folded conv + pool take 59 + 63 us)
static constexpr auto kImgPoolPH = 2;
  a.tiles = d->n * rt_cdiv(hp, kImgPoolPH) * rt_cdiv(wp, kPW);
  const int v = img_act_variant(act);
  const void* k = v == 0 ? (const void*)imgconv_pool_kernel<7, 7, kImgPoolPH, 0>
                : v == 1 ? (const void*)imgconv_pool_kernel<7, 7, kImgPoolPH, 1>
                         : (const void*)imgconv_pool_kernel<7, 7, kImgPoolPH, -1>;
  static int occ = 0, cus = 0;
  if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)imgconv_pool_kernel<7, 7, kImgPoolPH, 1>, 256, 0) != hipSuccess ||
               occ < 1))
    occ = 1;
  if (!cus && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus < 1)) cus = 256;
  const int slots = cus * occ;
  a.per = (a.tiles + slots - 1) / slots;
  const int grid = (a.tiles + a.per - 1) / a.per;
  void* args[] = {&a};
  (void)hipLaunchKernel(k, dim3(grid), dim3(256), args, 0, st);
}
