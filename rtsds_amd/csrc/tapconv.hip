// Register-resident-weight direct 3x3 convolution for 64 -> 64 channels, stride 1, same padding:
// ResNet layer1's BasicBlock convs (torchvision BasicBlock via build_contextpath.py:22; the
// 3x3 64-channel Bottleneck convs of deeplabv2.py:32-47 layer1), forward and data gradient (the
// data gradient of a 3x3 same-padding stride-1 conv is the same conv over dY with the weights
// flipped and transposed, rtsds_conv2d_dgrad_pack_many's halo layout).
//
// As an implicit GEMM these convs stage 24-32 KB of operands per 64-deep K-step (the input
// re-gathered once per tap, the weights once per M tile) for 1-2 MFLOP: ~43 flop per staged
// byte, and the L2 -> LDS gather rate the LDS can keep in flight sets the speed (~380 TF/s).
// Here:
//  * the weights never touch LDS: each wave holds the MFMA fragments of all 64 output channels
//    x 576 K in 288 VGPRs for the whole (persistent) launch (one wave per SIMD);
//  * a workgroup walks a contiguous run of 4 x 64-pixel output tiles; each tile's 6 x 66-pixel
//    input halo with all 64 channels (50 KB) is staged ONCE by buffer-resource LDS-DMA while the
//    previous tile computes (double-buffered), and the 9 taps read shifted windows of it:
//    ~370 flop per staged byte;
//  * 16-B chunk c of halo pixel f sits at slot c ^ (f & 7): the pixel fragments (16 consecutive
//    pixels x one 16-B chunk each) are conflict-free ds_read_b128 for every tap shift;
//  * the MFMA computes C^T = W X^T, so each lane ends with 4 consecutive channels of one pixel:
//    8-B stores (and 8-B residual / accumulate / BatchNorm-input loads) straight from the
//    accumulators, no LDS staging.
// Epilogues: FWD -- bias or eval-BN scale / shift, residual, activation; or the following
// BatchNorm's (count, mean, M2) merged per wave over its tiles (Chan).  DGRAD -- accumulate
// (GradJoin), the LeakyReLU / ReLU backward of the input's activation (mask), or the backward
// statistics (sum g, sum g (x - mean)) of the BatchNorm + activation that produced the input.
#include "common.h"

namespace {
constexpr int kC = 64;                    // input = output channels
constexpr int kWaves = 8;                 // 512-thread workgroups, one per CU (two waves per SIMD)
constexpr int kTH = 4, kTW = 64;          // output tile rows x columns
constexpr int kNCB = 2;                   // 16-channel blocks per wave (32 of the 64 outputs)
constexpr int kHR = kTH + 2, kHC = kTW + 2;
constexpr int kHalo = kHR * kHC;          // 396 halo pixels x 128 B
constexpr int kHInstr = (kHalo + 7) / 8;  // 50 LDS-DMA wave-instructions (8 pixels each)
constexpr int kHInstrW = (kHInstr + kWaves - 1) / kWaves;
constexpr int kHBytes = kHInstrW * kWaves * 1024;  // 56 KB per stage (the 6 pad instructions unused)
constexpr int kWHalf = 32 * 9 * kC * 2;   // weights of 32 output channels: 36 KB
constexpr int kStores = kTH * kTW * kC * 2 / 16 / (64 * kWaves);  // 16-B output stores per thread and tile (4)
}  // namespace

struct TapArgs {
  const bf16* x;       // NHWC [n][h][w][64] (DGRAD: dy)
  const bf16* wt;      // [64 out][3][3][64 in] (DGRAD: the flipped, transposed pack)
  const float* bias;   // [64] or null (eval fold: shift)
  const float* scale;  // [64] or null (eval fold)
  const bf16* res;     // FWD: residual, NHWC like y, or null
  const bf16* aux;     // DGRAD: mask input (act') or BatchNorm input (bnb), NHWC like y
  bf16* y;             // NHWC [n][h][w][64] (DGRAD: dx)
  float* stats;        // FWD: [64][rows][4] (count, mean, M2, 0); DGRAD bnb: [64][rows][2]
  const float *bn_gamma, *bn_beta, *bn_mean, *bn_invstd;  // DGRAD bnb
  int n, h, w, act, accum, mask_act, bnb_act;
  int tiles, per;
  FastDiv f_tpi, f_tw;  // tiles per image, tile columns per row
};

RT_DEV float tap_row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}
RT_DEV void tap_store16(rsrc_t r, bf16x8 v, int off) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, v), r, off, 0, 0);
#endif
}
RT_DEV bf16x4 tap_load8(rsrc_t r, int off) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
#else
  return bf16x4{};
#endif
}

// Wave w: output row (w >> 1) of the 4 x 64 tile (4 groups of 16 pixels) x channels 32 (w & 1)
// .. + 32; one 8-wave workgroup per CU (two waves per SIMD), so the weights are read from L2
// once per CU (staged through LDS) and the 6 x 66 halo feeds 256 output pixels.
template <int DGRAD, int EPI>
__global__ void __launch_bounds__(512, 1) tapconv_kernel(const TapArgs P) {
  // epilogue flags: compile-time for the modes the networks launch (tap_epi), read from P for
  // EPI < 0 -- per-element uniform branches on P's fields cost ~10 us per launch otherwise
  constexpr bool kGen = EPI < 0;
  const bool f_stats = kGen ? P.stats != nullptr : EPI == 1;
  const bool f_res = !DGRAD && (kGen ? P.res != nullptr : EPI == 3);
  const int f_act = DGRAD ? RTSDS_ACT_NONE : (kGen ? P.act : (EPI >= 2 ? RTSDS_ACT_RELU : RTSDS_ACT_NONE));
  const bool f_accum = DGRAD && (kGen ? P.accum != 0 : EPI == 3);
  const bool f_aux = DGRAD && (kGen ? P.aux != nullptr : (EPI == 1 || EPI == 2));
  const int f_mask_act = kGen ? P.mask_act : RTSDS_ACT_RELU;
  const int f_bnb_act = kGen ? P.bnb_act : RTSDS_ACT_RELU;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * kHBytes + kWHalf];
  // running statistics of the wave's channels across its tiles (kept here, not in registers):
  // FWD (mean, M2) per channel, DGRAD bnb (sum g, sum g (x - mean))
  __shared__ float srun[kWaves][32][2];
  // (wave index in an SGPR: the DMA destinations are then scalar, set straight into M0)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fc = lane >> 4;
  const int prow = wave >> 1, c0 = (wave & 1) * 32;
  int bid;
  {  // XCD-aware bijective remap: the workgroups of one XCD take adjacent runs of tiles
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int t0 = bid * P.per, t1 = min(P.tiles, t0 + P.per);
  const int npix = P.n * P.h * P.w;
  const rsrc_t rx = make_rsrc(P.x, npix * kC * 2);
  const rsrc_t ry = make_rsrc(P.y, npix * kC * 2);
  const rsrc_t rr = make_rsrc(DGRAD ? (const void*)P.aux : (const void*)P.res, npix * kC * 2);
  auto tile_xy = [&](int t, int& img, int& oh0, int& ow0) {
    img = (int)fdiv((uint32_t)t, P.f_tpi);
    const int rem = t - img * (int)P.f_tpi.d, trow = (int)fdiv((uint32_t)rem, P.f_tw);
    oh0 = trow * kTH;
    ow0 = (rem - trow * (int)P.f_tw.d) * kTW;
  };
  // this lane's DMA pieces: halo pixel f = 8 * instr + (lane >> 3), LDS slot lane & 7 holds
  // source chunk (lane & 7) ^ (f & 7), recomputed per tile from an opaque lane id (hoisted out
  // of the tile loop, the per-piece geometry would be held in -- and spill -- registers)
  auto issue = [&](int t, int b) {
    int img, oh0, ow0;
    tile_xy(t, img, oh0, ow0);
    int lz = lane;
    asm volatile("" : "+v"(lz));
#pragma unroll
    for (int u = 0; u < kHInstrW; ++u) {
      const int f = 8 * (wave + kWaves * u) + (lz >> 3);
      const int hr = f / kHC, hc = f - hr * kHC;
      const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
      const bool ok = f < kHalo && (unsigned)ih < (unsigned)P.h && (unsigned)iw < (unsigned)P.w;
      buf_lds16(rx, lds + b * kHBytes + (wave + kWaves * u) * 1024,
                ok ? ((img * P.h + ih) * P.w + iw) * (kC * 2) + (((lz & 7) ^ (f & 7)) << 4) : (int)0x80000000, 0);
    }
  };
  issue(t0, 0);
  if (f_stats) srun[wave][lane & 31][lane >> 5] = 0.f;

  // weight fragments (the MFMA's A operand): row = output channel c0 + 16 cb + fr, K slot =
  // channels 32 kk + 8 fc .. + 8 of tap (r, s).  Each 32-channel half of the weights is copied
  // once per workgroup into LDS (LDS-DMA, beside the first halo) and the four waves of that
  // channel half read their fragments from there: one L2 read of the 72 KB per CU instead of one
  // per wave (all workgroups read the same lines at launch).
  bf16x8 fw[kNCB][9][2];
  {
    const rsrc_t rw = make_rsrc(P.wt, 2 * kWHalf);
    unsigned char* wl = lds + 2 * kHBytes;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      // 16-B chunk j of weight row r (72 per row) sits at LDS chunk 72 r + (j ^ (r & 7)): the
      // fragment reads (16 rows at one chunk) then hit distinct bank groups (2-way at worst)
#pragma unroll
      for (int u = 0; u < (kWHalf / 1024 + kWaves - 1) / kWaves; ++u) {
        const int ins = wave + kWaves * u;
        const int c = ins * 64 + lane, r = c / 72, j = c - 72 * r;
        if (ins < kWHalf / 1024) buf_lds16(rw, wl + ins * 1024, h * kWHalf + (72 * r + (j ^ (r & 7))) * 16, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if ((c0 >> 5) == h) {
#pragma unroll
        for (int cb = 0; cb < kNCB; ++cb)
#pragma unroll
          for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
              fw[cb][tap][kk] = *(const bf16x8*)(wl + (72 * (16 * cb + fr) + ((8 * tap + 4 * kk + fc) ^ (fr & 7))) * 16);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // per-lane epilogue constants of channel c0 + 16 cb + 4 fc + e, read (L1 / L2 hits) in the
  // epilogue rather than held across the tile loop: the registers go to the weights
  auto ld4 = [&](const float* p, int cb, float dflt, float* v) {
    if (p) {
      const f32x4 q = *(const f32x4*)(p + c0 + 16 * cb + 4 * fc);
      v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
    } else {
      v[0] = v[1] = v[2] = v[3] = dflt;
    }
  };
  auto act_f = [&](float t) {
    if (f_act == RTSDS_ACT_RELU) return fmaxf(t, 0.f);
    if (f_act == RTSDS_ACT_LEAKY) return t > 0.f ? t : 0.2f * t;
    if (f_act == RTSDS_ACT_SIGMOID) return 1.f / (1.f + expf(-t));
    return t;
  };
  float rn = 0.f;  // FWD statistics: pixels merged so far (uniform over the wave)

  for (int t = t0; t < t1; ++t) {
    const int b = (t - t0) & 1;
    // tile t's halo landed (the kStores newest VMEM ops are the previous tile's output stores,
    // issued after this DMA; the first tile waits for everything, weights included), and every
    // wave is done reading the other buffer: refill it with tile t + 1
    if (t > t0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kStores) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < t1) issue(t + 1, b ^ 1);

    f32x4 acc[4][kNCB];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int cb = 0; cb < kNCB; ++cb) acc[g][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 18 K-steps (tap, 32-channel half); the pixel fragments of step i + 1 are read before the
    // MFMAs of step i (two fragment sets; the scheduling barriers keep the reads where they are
    // placed).  Fragment g of a step sits 16 pixels (2 KB) after fragment 0 with the same swizzle
    // (16 g = 0 mod 8): one address per step, from an opaque lane id (not hoisted and held).
    int lz = lane;
    asm volatile("" : "+v"(lz));
    const int frz = lz & 15, fcz = lz >> 4;
    const unsigned char* hrow = lds + b * kHBytes + (prow * kHC + frz) * (kC * 2);
    bf16x8 fx0[4], fx1[4];
    auto rd = [&](int step, bf16x8* fx) {
      const int tap = step >> 1, kk = step & 1, r = tap / 3, s = tap - 3 * r;
      const int fl = (frz + s + 2 * (prow + r)) & 7;  // (f & 7), f = (prow + r) * 66 + 16 g + fr + s
      const unsigned char* p = hrow + (r * kHC + s) * (kC * 2) + (((4 * kk + fcz) ^ fl) << 4);
#pragma unroll
      for (int g = 0; g < 4; ++g) fx[g] = *(const bf16x8*)(p + g * 16 * (kC * 2));
    };
    rd(0, fx0);
#pragma unroll
    for (int step = 0; step < 18; ++step) {
      bf16x8* cur = (step & 1) ? fx1 : fx0;
      bf16x8* nxt = (step & 1) ? fx0 : fx1;
      if (step + 1 < 18) rd(step + 1, nxt);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int cb = 0; cb < kNCB; ++cb)
          acc[g][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[cb][step >> 1][step & 1], cur[g], acc[g][cb], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue, one 16-channel block at a time: acc[g][cb][e] = C[channel c0 + 16 cb + 4 fc
    // + e][pixel 16 g + fr of row prow]
    int img, oh0, ow0;
    tile_xy(t, img, oh0, ow0);
    const int oh = oh0 + prow;
    const int vcols = oh < P.h ? min(kTW, P.w - ow0) : 0;
    const int pix0 = ((img * P.h + oh) * P.w + ow0) * kC + c0 + 4 * fc;
    const float cnt = (float)vcols, rn1 = rn + cnt;
    // the output tile is staged in this tile's halo buffer (every wave is done reading it after
    // this barrier) and leaves as coalesced 16-B row chunks: 8-B stores straight from the
    // accumulators wrote 32-B pieces of 16 different 128-B rows per instruction (14 of 39 us)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    unsigned char* stage = lds + b * kHBytes;
#pragma unroll
    for (int cb = 0; cb < kNCB; ++cb) {
      int off[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) off[g] = 16 * g + fr < vcols ? (pix0 + (16 * g + fr) * kC + 16 * cb) * 2 : (int)0x80000000;
      // operand of the epilogue (residual / accumulate target / mask / BatchNorm input)
      const bool need_r = DGRAD ? (f_accum || f_aux) : f_res;
      bf16x4 ro[4];
      if (need_r) {
        const rsrc_t rsrc = f_accum ? ry : rr;
#pragma unroll
        for (int g = 0; g < 4; ++g) ro[g] = tap_load8(rsrc, off[g]);
      }
      float bv[4], sv[4];
      ld4(DGRAD ? nullptr : P.bias, cb, 0.f, bv);
      ld4(DGRAD ? nullptr : P.scale, cb, 1.f, sv);
      bf16x4 ov[4];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (!DGRAD) {
            float v = fmaf(acc[g][cb][e], sv[e], bv[e]);
            if (f_res) v = (float)(bf16)v + (float)ro[g][e];
            ov[g][e] = (bf16)act_f(v);
            acc[g][cb][e] = v;  // (statistics: the pre-rounding value, as the GEMM epilogue)
          } else {
            const bf16 q = (bf16)acc[g][cb][e];
            float v = (float)q;
            if (f_accum) v += (float)ro[g][e];
            else if (f_aux && !f_stats) {  // mask: the backward of the input's activation
              const float xv = (float)ro[g][e];
              v = xv > 0.f ? v : (f_mask_act == RTSDS_ACT_LEAKY ? 0.2f * v : 0.f);
            }
            ov[g][e] = (f_accum || (f_aux && !f_stats)) ? (bf16)v : q;
          }
        }
      if (!DGRAD && f_stats) {
        // per-channel (count, mean, M2) over this wave's valid pixels of the tile (two-pass),
        // merged (Chan) into the wave's running statistics in LDS
        float mean[4];
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
          float sacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float d = pass == 0 ? acc[g][cb][e] : acc[g][cb][e] - mean[e];
              if (16 * g + fr < vcols) sacc[e] += pass == 0 ? d : d * d;
            }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sacc[e] = tap_row16_sum(sacc[e]);
            if (pass == 0) mean[e] = vcols ? sacc[e] / cnt : 0.f;
          }
          if (pass == 1 && vcols && fr == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float* st = srun[wave][16 * cb + 4 * fc + e];
              if (rn == 0.f) {
                st[0] = mean[e];
                st[1] = sacc[e];
              } else {
                const float dd = mean[e] - st[0];
                st[0] += dd * (cnt / rn1);
                st[1] += sacc[e] + dd * dd * (rn * cnt / rn1);
              }
            }
          }
        }
      }
      if (DGRAD && f_stats) {
        // BatchNorm backward statistics from the stored dx: g = dx * act'(x * scale + shift)
        float ga[4], be[4], mu[4], is[4], sg[4] = {0.f, 0.f, 0.f, 0.f}, sgx[4] = {0.f, 0.f, 0.f, 0.f};
        ld4(P.bn_gamma, cb, 1.f, ga);
        ld4(P.bn_beta, cb, 0.f, be);
        ld4(P.bn_mean, cb, 0.f, mu);
        ld4(P.bn_invstd, cb, 1.f, is);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (16 * g + fr >= vcols) continue;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sc = ga[e] * is[e], sh = fmaf(-mu[e], sc, be[e]);
            const float xv = (float)ro[g][e];
            float gv = (float)ov[g][e];
            gv *= fmaf(xv, sc, sh) > 0.f ? 1.f : (f_bnb_act == RTSDS_ACT_LEAKY ? 0.2f : 0.f);
            sg[e] += gv;
            sgx[e] = fmaf(gv, xv - mu[e], sgx[e]);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sg[e] = tap_row16_sum(sg[e]);
          sgx[e] = tap_row16_sum(sgx[e]);
          if (fr == 0) {
            float* st = srun[wave][16 * cb + 4 * fc + e];
            st[0] += sg[e];
            st[1] += sgx[e];
          }
        }
      }
      // staged as [pixel][64 ch] bf16 rows, 16-B chunk j of pixel px at slot j ^ (px & 7)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int px = prow * kTW + 16 * g + fr, j = (c0 >> 3) + 2 * cb + (fc >> 1);
        *(bf16x4*)(stage + px * (kC * 2) + ((j ^ (px & 7)) << 4) + (fc & 1) * 8) = ov[g];
      }
    }
    rn = rn1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // 16-B stores; pixels outside the output fall past num_records (every thread issues exactly
    // kStores stores per tile: the vmcnt accounting above relies on it)
#pragma unroll
    for (int i = 0; i < kStores; ++i) {
      const int q = tid + 64 * kWaves * i, px = q >> 3, j = q & 7;
      const int row = px / kTW, col = px - row * kTW;
      const bool ok = oh0 + row < P.h && ow0 + col < P.w;
      const bf16x8 v = *(const bf16x8*)(stage + px * (kC * 2) + ((j ^ (px & 7)) << 4));
      tap_store16(ry, v, ok ? (((img * P.h + oh0 + row) * P.w + ow0 + col) * kC + 8 * j) * 2 : (int)0x80000000);
    }
  }
  if (f_stats && lane < 32) {  // partial-statistics row 2 bid + prow of the wave's 32 channels
    const int rows = kTH * gridDim.x, row = kTH * bid + prow, ch = c0 + lane;
    const float* st = srun[wave][lane];
    if (!DGRAD) *(f32x4*)(P.stats + ((long)ch * rows + row) * 4) = f32x4{rn, st[0], st[1], 0.f};
    else *(f32x2*)(P.stats + ((long)ch * rows + row) * 2) = f32x2{st[0], st[1]};
  }
}

// ---- host -------------------------------------------------------------------------------
static bool tap_geom(const rtsds_conv_desc* d) {
  // widths that leave a nearly empty last column tile (DeepLab's 257 / 321: 64-pixel tiles with
  // one valid column) stay on the implicit GEMM, which measured faster there
  return d->dtype == RTSDS_BF16 && d->c == kC && d->k == kC && d->kh == 3 && d->kw == 3 && d->sh == 1 && d->sw == 1 &&
         d->ph == 1 && d->pw == 1 && d->dh == 1 && d->dw == 1 && (d->w % kTW == 0 || d->w % kTW > 3 * kTW / 4) &&
         (long)d->n * d->h * d->w * kC * 2 < (1L << 31);
}
bool tapconv_ok(const rtsds_conv_desc* d) {
  return tap_geom(d);
}
static int tap_tiles(const rtsds_conv_desc* d) { return d->n * ((d->h + kTH - 1) / kTH) * ((d->w + kTW - 1) / kTW); }
static void tap_geom_args(const rtsds_conv_desc* d, TapArgs& a) {
  const int tw = (d->w + kTW - 1) / kTW, th = (d->h + kTH - 1) / kTH;
  a.tiles = tap_tiles(d);
  a.f_tpi = fastdiv_make(th * tw);
  a.f_tw = fastdiv_make(tw);
}
template <int DGRAD>
static void tap_grid(const rtsds_conv_desc* d, int& grid, int& per) {
  static int occ = 0, cus = 0;
  if (!occ && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)tapconv_kernel<DGRAD, -1>, 64 * kWaves, 0) != hipSuccess ||
               occ < 1))
    occ = 1;
  if (!cus && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus < 1)) cus = 256;
  const int tiles = tap_tiles(d), slots = cus * occ;
  per = (tiles + slots - 1) / slots;
  grid = (tiles + per - 1) / per;
}
template <int DGRAD>
static void tap_launch(int epi, int grid, const TapArgs& a, hipStream_t st) {
  const dim3 g(grid), b(64 * kWaves);
  switch (epi) {
    case 0: hipLaunchKernelGGL((tapconv_kernel<DGRAD, 0>), g, b, 0, st, a); break;
    case 1: hipLaunchKernelGGL((tapconv_kernel<DGRAD, 1>), g, b, 0, st, a); break;
    case 2: hipLaunchKernelGGL((tapconv_kernel<DGRAD, 2>), g, b, 0, st, a); break;
    case 3: hipLaunchKernelGGL((tapconv_kernel<DGRAD, 3>), g, b, 0, st, a); break;
    default: hipLaunchKernelGGL((tapconv_kernel<DGRAD, -1>), g, b, 0, st, a); break;
  }
}
// partial-statistics rows of a launch: one per workgroup and output row of the tile
int tapconv_rows(const rtsds_conv_desc* d, int dgrad) {
  int grid, per;
  if (dgrad) tap_grid<1>(d, grid, per);
  else tap_grid<0>(d, grid, per);
  return kTH * grid;
}
void tapconv_fwd(const rtsds_conv_desc* d, const void* x, const void* w, const float* bias, const float* scale, const void* res,
                 void* y, int act, float* stats, hipStream_t st) {
  TapArgs a = {};
  a.x = (const bf16*)x; a.wt = (const bf16*)w; a.bias = bias; a.scale = scale; a.res = (const bf16*)res; a.y = (bf16*)y;
  a.stats = stats; a.n = d->n; a.h = d->h; a.w = d->w; a.act = act;
  tap_geom_args(d, a);
  int grid;
  tap_grid<0>(d, grid, a.per);
  // epilogue modes: 1 BatchNorm statistics, 2 ReLU, 3 residual + ReLU, 0 plain, -1 anything else
  const int epi = stats ? (!res && act == RTSDS_ACT_NONE ? 1 : -1)
                : act == RTSDS_ACT_RELU ? (res ? 3 : 2)
                : (act == RTSDS_ACT_NONE && !res ? 0 : -1);
  tap_launch<0>(epi, grid, a, st);
}
// dx (+)= conv(dy, wt_flipped) (wt: [c][3][3][k], rtsds_conv2d_dgrad_pack_many's halo layout);
// mask: act' of the input's activation; bnb: BatchNorm backward statistics [c][rows][2]
void tapconv_dgrad(const rtsds_conv_desc* d, const void* dy, const void* wt, void* dx, int accumulate, const void* mask,
                   int mask_act, float* bnb_part, const void* bnb_x, const float* gamma, const float* beta, const float* mean,
                   const float* invstd, int bnb_act, hipStream_t st) {
  TapArgs a = {};
  a.x = (const bf16*)dy; a.wt = (const bf16*)wt; a.y = (bf16*)dx; a.n = d->n; a.h = d->h; a.w = d->w;
  a.accum = accumulate ? 1 : 0;
  a.aux = (const bf16*)(bnb_part ? bnb_x : mask);
  a.mask_act = mask_act;
  a.stats = bnb_part;
  a.bn_gamma = gamma; a.bn_beta = beta; a.bn_mean = mean; a.bn_invstd = invstd; a.bnb_act = bnb_act;
  tap_geom_args(d, a);
  int grid;
  tap_grid<1>(d, grid, a.per);
  // epilogue modes: 1 ReLU BatchNorm-backward statistics, 2 ReLU mask, 3 accumulate, 0 plain
  int epi = -1;
  if (bnb_part) epi = (!accumulate && bnb_act == RTSDS_ACT_RELU) ? 1 : -1;
  else if (mask) epi = (!accumulate && mask_act == RTSDS_ACT_RELU) ? 2 : -1;
  else epi = accumulate ? 3 : 0;
  tap_launch<1>(epi, grid, a, st);
}
