// Halo-resident direct 3x3 convolution for narrow outputs (Cout <= 32) -- the BiSeNet feature
// fusion ConvBlock, 1024 -> 19 channels at 1/8 resolution (build_bisenet.py:64-65 via
// ConvBlock build_bisenet.py:9-18): forward (hconv_fwd_kernel, also the N-tiled deep 3x3 convs
// and the data gradients over multi-chunk dY), the single-chunk data gradient
// (hconv_dgrad_nt_kernel) and the weight gradient (nwgrad_kernel), each further below.
//
// As an implicit GEMM this conv is N = 19 wide: every input byte the im2col gathers feeds only
// 19 outputs, and the 3x3 taps gather each input pixel 9 times, so the generic kernel is bound
// by LDS-DMA throughput (36 KB staged per 64-deep K-step for 256 x 32 outputs).  Here a
// workgroup owns a 4 x 64 output tile and walks the input channels in chunks of 32: per chunk
// it stages the (4+2) x (64+2) input halo ONCE (25 KB) plus the chunk's weights for all 9 taps
// (32 x 9 x 32, 18 KB) and runs the 9 taps out of LDS -- 1.7x fewer staged bytes per MFMA
// than one tap per K-step, and no per-tap re-gather.  Both LDS images are double-buffered
// (the next chunk's DMA is in flight while this one computes) and XOR-swizzled for
// conflict-free ds_read_b128 fragments: 16-B chunk c of halo pixel p (weight row n) sits at
// slot c ^ ((p >> 2) & 3) (c ^ ((n >> 2) & 3)).
//
// Wave w computes output row w of the tile: 4 x 2 MFMA 16x16x32 tiles (64 pixels x 32
// channels).  Epilogue: bias (or eval-BN scale/shift), activation, the following BatchNorm's
// per-tile partial statistics (count, mean, M2 -- the exact two-pass form, as the GEMM
// epilogue), scalar bf16 stores of the Cout valid channels.
#include "common.h"
#include <algorithm>
#include <utility>

namespace {
// A tile is 256 output pixels: 4 rows x 64 columns, or 8 x 32 for 32-wide maps (ResNet layer4
// at 1024 x 512: 16 x 32); wave w computes pixels 64 w .. 64 w + 63 of the row-major tile.
constexpr int kCK = 32;
template <int TC> struct HTile {
  static constexpr int TR = 256 / TC, HR = TR + 2, HC = TC + 2, HaloPix = HR * HC;  // 396 / 340
  // 16-B DMA pieces (4 per halo pixel) in wave-instructions, padded to a multiple of 4 waves
  static constexpr int HaloInstr = ((HaloPix * 4 + 63) / 64 + 3) / 4 * 4;           // 28 / 24
  static constexpr int HaloBytes = HaloInstr * 1024;
};
constexpr int kWInstr = 20;     // 9 taps x 32 rows x 4 chunks / 64 = 18, padded to 5 per wave
constexpr int kWBytes = kWInstr * 1024;
}  // namespace

struct HconvArgs {
  const bf16* x;       // NHWC [n][h][w][c]
  const bf16* wt;      // [k][3][3][c]
  const float* bias;   // [k] or null (eval fold: shift)
  const float* scale;  // [k] or null (eval fold)
  const bf16* res;     // NHWC [n][h][w][k] residual (added to the bf16-rounded conv output) or null
  bf16* y;             // NHWC [n][h][w][k]
  float* stats;        // [k][tiles][4] or null
  int n, h, w, c, k, act, accum;  // k = output channels, tiled by 32 over blockIdx.y
};

// ACT >= 0: the activation fixed at compile time (none / ReLU), < 0: P.act (see imgconv.hip)
template <int ACT, int TC>
__global__ void __launch_bounds__(256, 1) hconv_fwd_kernel(const HconvArgs P) {
  using G = HTile<TC>;
  constexpr int kTR = G::TR, kTC = TC, kHC = G::HC, kHaloPix = G::HaloPix, kHaloInstr = G::HaloInstr;
  constexpr int kHaloBytes = G::HaloBytes, kStage = kHaloBytes + kWBytes;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // 2 stages
  __shared__ float red[4][32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tw_n = P.w / kTC, th_n = P.h / kTR;
  int bid;
  {  // XCD-aware bijective remap: each XCD gets a contiguous run of tiles (shared halo rows)
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int img = bid / (th_n * tw_n), rem = bid - img * th_n * tw_n;
  const int trow = rem / tw_n, tcol = rem - trow * tw_n;
  const int oh0 = trow * kTR, ow0 = tcol * kTC;
  const int C = P.c, n0 = blockIdx.y * 32;
  const rsrc_t rx = make_rsrc(P.x, P.n * P.h * P.w * C * 2);
  const rsrc_t rw = make_rsrc(P.wt, P.k * 9 * C * 2);

  // Per-lane DMA pieces (16 B each), fixed for the whole channel walk: wave w issues
  // wave-instructions w, w + 4, ...; each lane's byte offset at channel chunk 0 (chunk q adds
  // q * 64 B as soffset; invalid pieces carry an offset past num_records -> zero-filled).
  int hoff[kHaloInstr / 4], woff[kWInstr / 4];
#pragma unroll
  for (int u = 0; u < kHaloInstr / 4; ++u) {
    const int piece = (wave + 4 * u) * 64 + lane, hp = piece >> 2, slot = piece & 3;
    int v = (int)0x80000000;
    if (hp < kHaloPix) {
      const int hr = hp / kHC, hc = hp - hr * kHC;
      const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
      const int ch = slot ^ ((hp >> 2) & 3);
      if ((unsigned)ih < (unsigned)P.h && (unsigned)iw < (unsigned)P.w)
        v = (((img * P.h + ih) * P.w + iw) * C + ch * 8) * 2;
    }
    hoff[u] = v;
  }
#pragma unroll
  for (int u = 0; u < kWInstr / 4; ++u) {
    const int piece = (wave + 4 * u) * 64 + lane;
    int v = (int)0x80000000;
    if (piece < 9 * 32 * 4) {
      const int tap = piece >> 7, n = (piece >> 2) & 31, slot = piece & 3;
      const int ch = slot ^ ((n >> 2) & 3);
      v = (((n0 + n) * 9 + tap) * C + ch * 8) * 2;  // rows n0 + n >= k fall past num_records
    }
    woff[u] = v;
  }
  auto issue = [&](int q, int buf) {
    unsigned char* hb = lds + buf * kStage;
    unsigned char* wb = hb + kHaloBytes;
    const int qoff = q * kCK * 2;
#pragma unroll
    for (int u = 0; u < kHaloInstr / 4; ++u) buf_lds16(rx, hb + (wave + 4 * u) * 1024, hoff[u], qoff);
#pragma unroll
    for (int u = 0; u < kWInstr / 4; ++u) buf_lds16(rw, wb + (wave + 4 * u) * 1024, woff[u], qoff);
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fc = lane >> 4;  // fragment row, 16-B k-chunk
  int bslot[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 16 * j + fr;
    bslot[j] = (n * 4 + (fc ^ ((n >> 2) & 3))) * 16;
  }

  const int Q = C / kCK;
  issue(0, 0);
  for (int q = 0; q < Q; ++q) {
    if (q + 1 < Q) {
      issue(q + 1, (q + 1) & 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kHaloInstr / 4 + kWInstr / 4) : "memory");  // chunk q landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const unsigned char* hb = lds + (q & 1) * kStage;
    const unsigned char* wb = hb + kHaloBytes;
    // the fragments of tap t + 2 are read before the MFMAs of tap t (the scheduling barriers keep
    // the reads where they are placed): with one wave per SIMD nothing else hides the LDS
    // latency, which the read-then-use order exposed once per tap
    auto rd = [&](int tap, bf16x8* fa, bf16x8* fb) {
      const int r = tap / 3, s = tap - 3 * r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p0 = 64 * wave + 16 * i;  // first pixel of group i (16 | TC: one tile row)
        const int hp = (p0 / kTC + r) * kHC + p0 % kTC + fr + s;
        fa[i] = *(const bf16x8*)(hb + hp * 64 + ((fc ^ ((hp >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = *(const bf16x8*)(wb + tap * 32 * 64 + bslot[j]);
    };
    // two taps of look-ahead (three register sets): one tap's 8 MFMAs (128 cycles) did not
    // cover the read latency where a launch walks a single channel chunk (the FFM data gradient)
    bf16x8 fa_s[3][4], fb_s[3][2];
    rd(0, fa_s[0], fb_s[0]);
    rd(1, fa_s[1], fb_s[1]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      bf16x8* fa = fa_s[tap % 3];
      bf16x8* fb = fb_s[tap % 3];
      if (tap + 2 < 9) rd(tap + 2, fa_s[(tap + 2) % 3], fb_s[(tap + 2) % 3]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // every wave is done with this buffer before it is refilled: its ds_reads retired first
    // (a raw s_barrier does not wait for them; see gl_barrier in conv.hip)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // ---- epilogue: C[pixel = 16 i + 4 (lane >> 4) + e][channel = 16 j + (lane & 15)]
  const int er = (lane >> 4) * 4;
  float v[4][2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + 16 * j + fr;
    const bool ok = n < P.k;
    const float bv = (P.bias && ok) ? P.bias[n] : 0.f;
    const float sv = (P.scale && ok) ? P.scale[n] : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i][j][e] = fmaf(acc[i][j][e], sv, bv);
  }
  if (P.stats) {
    // per-channel (count, mean, M2) over the tile's 256 pixels, exact two-pass
    float mean[2];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float sacc = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float t = pass == 0 ? v[i][j][e] : (v[i][j][e] - mean[j]) * (v[i][j][e] - mean[j]);
            sacc += t;
          }
        sacc += __shfl_xor(sacc, 16, 64);
        sacc += __shfl_xor(sacc, 32, 64);
        if (lane < 16) red[wave][16 * j + lane] = sacc;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = 16 * j + fr;
        const float tot = (red[0][n] + red[1][n]) + (red[2][n] + red[3][n]);
        if (pass == 0) {
          mean[j] = tot / (float)(kTR * kTC);
        } else if (wave == 0 && lane < 16 && n0 + n < P.k) {
          *(f32x4*)(P.stats + ((long)(n0 + n) * gridDim.x + bid) * 4) =  // [channel][tile][4]
              f32x4{(float)(kTR * kTC), mean[j], tot, 0.f};
        }
      }
      __syncthreads();
    }
  }
  auto act_f = [&](float t) {
    const int a = ACT >= 0 ? ACT : P.act;
    if (a == RTSDS_ACT_RELU) return fmaxf(t, 0.f);
    if (a == RTSDS_ACT_LEAKY) return t > 0.f ? t : 0.2f * t;
    if (a == RTSDS_ACT_SIGMOID) return 1.f / (1.f + expf(-t));
    return t;
  };
  if (P.k % 8 == 0) {
    // 16-B stores: the [256 px][32 ch] bf16 tile goes through LDS (the operand buffers are free
    // after the loop's last barrier), then each thread writes 4 row chunks
    bf16* cs = (bf16*)lds;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int px = 64 * wave + 16 * i + er + e;
          cs[px * 32 + 16 * j + fr] = (bf16)((P.accum || P.res) ? v[i][j][e] : act_f(v[i][j][e]));
        }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int cidx = tid + 256 * u, px = cidx >> 2, n = n0 + (cidx & 3) * 8;
      if (n >= P.k) continue;
      const long o = (((long)img * P.h + oh0 + px / kTC) * P.w + ow0 + px % kTC) * P.k + n;
      bf16x8 t = *(const bf16x8*)(cs + px * 32 + (cidx & 3) * 8);
      if (P.accum || P.res) {  // (exclusive: the data gradient accumulates, the forward adds a residual)
        const bf16x8 old = *(const bf16x8*)(P.accum ? (const bf16*)P.y + o : P.res + o);
#pragma unroll
        for (int q = 0; q < 8; ++q) t[q] = (bf16)act_f((float)t[q] + (float)old[q]);
      }
      *(bf16x8*)(P.y + o) = t;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + 16 * j + fr;
    if (n >= P.k) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int px = 64 * wave + 16 * i + er + e;
        const long o = ((long)img * P.h + oh0 + px / kTC) * P.w + ow0 + px % kTC;
        float t = v[i][j][e];
        if (P.accum) t += (float)P.y[o * P.k + n];
        if (P.res) t = (float)(bf16)t + (float)P.res[o * P.k + n];
        P.y[o * P.k + n] = (bf16)act_f(t);
      }
  }
}

// ---- data gradient of the narrow-output conv, persistent over output-channel tiles ------------
// dX = conv(dY_p, W flipped / transposed) with dY_p the 32-channel-padded gradient (ONE channel
// chunk): hconv_fwd_kernel re-stages the dY halo for every 32-wide tile of the Cin outputs (32
// workgroups per spatial tile for the FFM's 1024 channels) and each short workgroup's DMA ->
// 72 MFMAs -> LDS-staged stores run back to back.  Here a workgroup stages the halo ONCE and
// walks nt output-channel tiles with their weights double-buffered (tile j + 1's DMA in flight
// behind tile j's MFMAs and stores); the MFMA computes C^T = W X^T, so a lane ends with 4
// consecutive channels of one pixel and stores 8 B straight from the accumulators (no LDS
// staging: 68 KB of LDS, two workgroups per CU).
template <int TC>
__global__ void __launch_bounds__(256, 2) hconv_dgrad_nt_kernel(const HconvArgs P, int nt) {
  using G = HTile<TC>;
  constexpr int kTR = G::TR, kHC = G::HC, kHaloPix = G::HaloPix, kHaloInstr = G::HaloInstr, kHaloBytes = G::HaloBytes;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // halo | 2 weight stages
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tw_n = P.w / TC, th_n = P.h / kTR;
  int bid;
  {  // XCD-aware bijective remap: each XCD gets a contiguous run of tiles (shared halo rows)
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  }
  const int img = bid / (th_n * tw_n), rem = bid - img * th_n * tw_n;
  const int trow = rem / tw_n, tcol = rem - trow * tw_n;
  const int oh0 = trow * kTR, ow0 = tcol * TC;
  const int C = P.c;  // == kCK: one channel chunk
  const rsrc_t rx = make_rsrc(P.x, P.n * P.h * P.w * C * 2);
  const rsrc_t rw = make_rsrc(P.wt, P.k * 9 * C * 2);
#pragma unroll
  for (int u = 0; u < kHaloInstr / 4; ++u) {
    const int piece = (wave + 4 * u) * 64 + lane, hp = piece >> 2, slot = piece & 3;
    int v = (int)0x80000000;
    if (hp < kHaloPix) {
      const int hr = hp / kHC, hc = hp - hr * kHC;
      const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
      const int ch = slot ^ ((hp >> 2) & 3);
      if ((unsigned)ih < (unsigned)P.h && (unsigned)iw < (unsigned)P.w) v = (((img * P.h + ih) * P.w + iw) * C + ch * 8) * 2;
    }
    buf_lds16(rx, lds + (wave + 4 * u) * 1024, v, 0);
  }
  int woff[kWInstr / 4];
#pragma unroll
  for (int u = 0; u < kWInstr / 4; ++u) {
    const int piece = (wave + 4 * u) * 64 + lane;
    int v = (int)0x80000000;
    if (piece < 9 * 32 * 4) {
      const int tap = piece >> 7, n = (piece >> 2) & 31, slot = piece & 3;
      v = ((n * 9 + tap) * C + (slot ^ ((n >> 2) & 3)) * 8) * 2;  // + the tile's rows as soffset
    }
    woff[u] = v;
  }
  const int j0 = blockIdx.y * nt, j1 = min(P.k / 32, j0 + nt);
  auto issue_w = [&](int j, int st) {
    unsigned char* wb = lds + kHaloBytes + st * kWBytes;
#pragma unroll
    for (int u = 0; u < kWInstr / 4; ++u) buf_lds16(rw, wb + (wave + 4 * u) * 1024, woff[u], j * (32 * 9 * 2) * C);
  };
  if (j0 < j1) issue_w(j0, 0);
  const int fr = lane & 15, fc = lane >> 4;
  int bslot[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 16 * j + fr;
    bslot[j] = (n * 4 + (fc ^ ((n >> 2) & 3))) * 16;
  }
  // vector-memory ops per lane that follow tile j's weight DMA: the 8-B stores of the epilogue
  // below (kFi pixel fragments x kFj channel halves) -- the count the wait at the top of tile
  // j + 1 leaves in flight.  With P.accum the epilogue also loads the old values; the compiler's
  // wait for those drains the prefetched weight DMA as well (vmcnt retires in order), so the
  // accumulate path runs without the weight double-buffer overlap (correct, slower).
  constexpr int kFi = 4, kFj = 2, kSt = kFi * kFj;
  for (int j = j0; j < j1; ++j) {
    const int st = (j - j0) & 1;
    // tile j's weights (and, first, the halo) landed -- all but this wave's stores of tile j - 1 --
    // then everyone's, and every wave is done reading the other weight stage: refill it
    if (j == j0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kSt) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (j + 1 < j1) issue_w(j + 1, st ^ 1);
    const unsigned char* wb = lds + kHaloBytes + st * kWBytes;
    auto rd = [&](int tap, bf16x8* fa, bf16x8* fb) {
      const int r = tap / 3, s = tap - 3 * r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p0 = 64 * wave + 16 * i;
        const int hp = (p0 / TC + r) * kHC + p0 % TC + fr + s;
        fa[i] = *(const bf16x8*)(lds + hp * 64 + ((fc ^ ((hp >> 2) & 3)) << 4));
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) fb[jj] = *(const bf16x8*)(wb + tap * 32 * 64 + bslot[jj]);
    };
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa_s[3][4], fb_s[3][2];
    rd(0, fa_s[0], fb_s[0]);
    rd(1, fa_s[1], fb_s[1]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      bf16x8* fa = fa_s[tap % 3];
      bf16x8* fb = fb_s[tap % 3];
      if (tap + 2 < 9) rd(tap + 2, fa_s[(tap + 2) % 3], fb_s[(tap + 2) % 3]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[jj], fa[i], acc[i][jj], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // C^T: acc[i][jj][e] = dX[pixel 64 wave + 16 i + fr][channel 32 j + 16 jj + 4 fc + e]
    const int px_r = (64 * wave) / TC;
#pragma unroll
    for (int i = 0; i < kFi; ++i) {  // kFi x kFj stores: keep kSt in step with this loop nest
      const int pc = (64 * wave) % TC + 16 * i + fr;
      const long o = (((long)img * P.h + oh0 + px_r + pc / TC) * P.w + ow0 + pc % TC) * P.k + 32 * j + 4 * fc;
#pragma unroll
      for (int jj = 0; jj < kFj; ++jj) {
        bf16x4 t;
        if (P.accum) {
          const bf16x4 old = *(const bf16x4*)(P.y + o + 16 * jj);
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = (bf16)(acc[i][jj][e] + (float)old[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = (bf16)acc[i][jj][e];
        }
        *(bf16x4*)(P.y + o + 16 * jj) = t;
      }
    }
  }
}

// ---- weight gradient of the narrow-output conv ------------------------------------------------
// dW[co][r][s][ci] = sum_px dY[px][co] X[px + (r - 1, s - 1)][ci] for Cout <= 32 (dY channel-padded
// to 32), Cin a multiple of 128.  As a split-K GEMM (M = 32 rows of Cout, N = 9 taps x Cin,
// K = pixels) every input pixel is re-gathered once per tap: 1.2 GB of LDS-DMA for the FFM conv's
// 19 x 9216 weights at bs 8, 121 us.  Here a workgroup owns 128 input channels (blockIdx.y) and
// walks a contiguous run of 2 x 64-pixel output tiles (blockIdx.x); per tile the 4 x 66-pixel
// input halo (its 128 channels) and the dY tile (128 pixels x 32 channels) are staged ONCE by
// LDS-DMA (double-buffered) and all 9 taps read shifted windows of the halo.  Wave w owns input
// channels 16 w .. + 16 x both 16-row blocks of Cout x the 9 taps: 18 accumulator blocks, held
// across the run.  Both MFMA operands are pixel-major in LDS (K = pixels) and read with
// ds_read_b64_tr_b16 (lane 16 g + 4 q + p reads pixel 4 g + q, channels 4 p .. 4 p + 3 of its
// 16-channel block); 16-B chunk c of halo pixel f sits at slot c ^ 2 (f & 7) (256-B rows: the
// 8 pixels of a 32-lane group cover all 64 banks for every tap shift), chunk c of dY pixel q at
// c ^ 2 ((q >> 2) & 1) (64-B rows: pixels q and q + 4 take different halves).  Every read is an
// immediate offset from one of 10 per-lane bases (the halo swizzle of a window depends only on
// (2 row + column) mod 8).  Each workgroup writes its partial dW rows co < Cout as one split-K
// slab [32][9][Cin]; the weight-gradient split reduce sums them in split order (deterministic).
namespace {
constexpr int kNwTH = 2, kNwTW = 64, kNwHC = kNwTW + 2, kNwHalo = (kNwTH + 2) * kNwHC;  // 264 halo pixels
constexpr int kNwCI = 128, kNwWaves = 8;
constexpr int kNwHIns = kNwHalo * kNwCI * 2 / 1024;                   // 66 wave-instructions (4 pixels each)
constexpr int kNwDIns = kNwTH * kNwTW * 64 / 1024;                    // 8 (the dY tile, 16 pixels each)
constexpr int kNwInsW = (kNwHIns + kNwDIns + kNwWaves - 1) / kNwWaves;  // 10 per wave
constexpr int kNwStage = (kNwHIns + kNwDIns) * 1024;                  // 74 KB per stage
constexpr int kNwDOff = kNwHIns * 1024;                               // dY tile offset in a stage
}  // namespace

struct NwArgs {
  const bf16* x;   // NHWC [n][h][w][c]
  const bf16* dy;  // NHWC [n][h][w][32]
  float* slab;     // [gridDim.x][32][9][c] fp32 partial weight gradients (rows co < k written)
  int n, h, w, c, k, tiles, per;
  FastDiv f_tpi, f_tw;  // tiles per image, tile columns per row
};

RT_DEV uint32_t nw_lds_addr(const void* p) { return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p; }
template <int OFF> RT_DEV void nw_rd(s16x4& d, uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(OFF));
}
template <typename F, int... I> RT_DEV void nw_for_i(F&& f, std::integer_sequence<int, I...>) { (f(std::integral_constant<int, I>()), ...); }
template <int N, typename F> RT_DEV void nw_for(F&& f) { nw_for_i(f, std::make_integer_sequence<int, N>()); }

__global__ void __launch_bounds__(512, 1) nwgrad_kernel(const NwArgs P) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * kNwStage];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ci0 = blockIdx.y * kNwCI;
  const int t0 = blockIdx.x * P.per, t1 = min(P.tiles, t0 + P.per);
  const int npix = P.n * P.h * P.w;
  const rsrc_t rx = make_rsrc(P.x, npix * P.c * 2);
  const rsrc_t rdy = make_rsrc(P.dy, npix * 64);
  auto tile_xy = [&](int t, int& img, int& oh0, int& ow0) {
    img = (int)fdiv((uint32_t)t, P.f_tpi);
    const int rem = t - img * (int)P.f_tpi.d, trow = (int)fdiv((uint32_t)rem, P.f_tw);
    oh0 = trow * kNwTH;
    ow0 = (rem - trow * (int)P.f_tw.d) * kNwTW;
  };
  // wave-instruction ins (1 KB) of a stage: halo pixels 4 ins .. 4 ins + 3 (ins < 66; lane l writes
  // slot l & 15 of pixel l >> 4 with source chunk (l & 15) ^ 2 (f & 7)), then the dY tile's pixels
  // (16 per instruction; slot l & 3 of pixel l >> 2, source chunk (l & 3) ^ 2 ((q >> 2) & 1));
  // pixels outside the image get an offset past num_records (zeros)
  auto issue = [&](int t, int b) {
    int img, oh0, ow0;
    tile_xy(t, img, oh0, ow0);
    int lz = lane;
    asm volatile("" : "+v"(lz));
#pragma unroll
    for (int u = 0; u < kNwInsW; ++u) {
      const int ins = wave + kNwWaves * u;
      unsigned char* dst = lds + b * kNwStage + ins * 1024;
      if (ins < kNwHIns) {
        const int f = 4 * ins + (lz >> 4), hr = f / kNwHC, hc = f - hr * kNwHC;
        const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
        const bool ok = (unsigned)ih < (unsigned)P.h && (unsigned)iw < (unsigned)P.w;
        const int ch = (lz & 15) ^ ((f & 7) << 1);
        buf_lds16(rx, dst, ok ? ((img * P.h + ih) * P.w + iw) * (P.c * 2) + ci0 * 2 + (ch << 4) : (int)0x80000000, 0);
      } else if (ins < kNwHIns + kNwDIns) {
        const int q = 16 * (ins - kNwHIns) + (lz >> 2), oh = oh0 + (q >> 6), ow = ow0 + (q & 63);
        const bool ok = oh < P.h && ow < P.w;
        const int ch = (lz & 3) ^ (((q >> 2) & 1) << 1);
        buf_lds16(rdy, dst, ok ? ((img * P.h + oh) * P.w + ow) * 64 + (ch << 4) : (int)0x80000000, 0);
      }
    }
  };
  if (t0 < t1) issue(t0, 0);

  // per-lane read bases: lane 16 g + 4 qq + p reads pixel rows (base + L) and + 16, L = 4 g + qq,
  // channels 4 p .. 4 p + 3 of its 16-channel block
  const int g = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3, L = 4 * g + qq;
  uint32_t abase[2], bbase[8];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)  // dY pixel rows 32 kk + L (+ 16): (row >> 2) & 1 = (L >> 2) & 1
    abase[cb] = nw_lds_addr(lds) + kNwDOff + L * 64 + (((2 * cb + (p >> 1)) ^ (((L >> 2) & 1) << 1)) << 4) + (p & 1) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j)  // halo window with (2 row + column) mod 8 = j: (f & 7) = (j + L) & 7
    bbase[j] = nw_lds_addr(lds) + L * 256 + (((2 * wave + (p >> 1)) ^ (((j + L) & 7) << 1)) << 4) + (p & 1) * 8;
  f32x4 acc[2][9];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) acc[cb][tap] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x4 fa[2][2][2], fb[2][9][2];  // [register set][block or tap][half]
  // reads of K-step KK (32 pixels: tile row KK >> 1, columns 32 (KK & 1) ..) into set S, buffer
  // offset bo; the halo window of tap (r, s) starts at pixel (row + r) * 66 + col + s
  auto rd_a = [&](uint32_t bo, auto kkc, auto sc) {
    constexpr int KK = decltype(kkc)::value, S = decltype(sc)::value;
    nw_for<2>([&](auto cbc) {
      constexpr int CB = decltype(cbc)::value;
      nw_rd<32 * KK * 64>(fa[S][CB][0], abase[CB] + bo);
      nw_rd<(32 * KK + 16) * 64>(fa[S][CB][1], abase[CB] + bo);
    });
  };
  auto rd_b = [&](uint32_t bo, auto kkc, auto sc, auto t0c, auto t1c) {
    constexpr int KK = decltype(kkc)::value, S = decltype(sc)::value;
    constexpr int PR = KK >> 1, PC = 32 * (KK & 1);
    nw_for<decltype(t1c)::value - decltype(t0c)::value>([&](auto ic) {
      constexpr int TAP = decltype(t0c)::value + decltype(ic)::value, R = TAP / 3, SC = TAP % 3;
      constexpr int F0 = (PR + R) * kNwHC + PC + SC, J = (2 * (PR + R) + SC) & 7;
      nw_rd<F0 * 256>(fb[S][TAP][0], bbase[J] + bo);
      nw_rd<(F0 + 16) * 256>(fb[S][TAP][1], bbase[J] + bo);
    });
  };
  auto frag = [](s16x4& u0, s16x4& u1) {
    asm volatile("" : "+v"(u0), "+v"(u1));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 r = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
    return __builtin_bit_cast(bf16x8, r);
  };
  // MFMAs of Cout block CB on register set S.  The halo window is the MFMA's A operand, so a
  // lane's accumulator holds 4 consecutive input channels of one output channel (one 16-B store
  // per block in the epilogue)
  auto mm = [&](auto sc, auto cbc) {
    constexpr int S = decltype(sc)::value, CB = decltype(cbc)::value;
    const bf16x8 a = frag(fa[S][CB][0], fa[S][CB][1]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      asm volatile("" : "+v"(fb[S][tap][0]), "+v"(fb[S][tap][1]));
      acc[CB][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(fb[S][tap][0], fb[S][tap][1]), a, acc[CB][tap], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  for (int t = t0; t < t1; ++t) {
    const int b = (t - t0) & 1;
    const uint32_t bo = b * kNwStage;
    // tile t landed (this wave's DMA, then everyone's) and every wave is done reading the other
    // buffer: refill it with tile t + 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd_a(bo, I0(), I0());
    rd_b(bo, I0(), I0(), I0(), std::integral_constant<int, 9>());
    if (t + 1 < t1) issue(t + 1, b ^ 1);
    // 4 K-steps; the next step's 22 reads are issued in two halves between this step's two MFMA
    // groups, so each group's operands have landed behind the other's MFMAs
    nw_for<4>([&](auto kkc) {
      constexpr int KK = decltype(kkc)::value, S = KK & 1, N = S ^ 1;
      using IS = std::integral_constant<int, S>;
      using IN = std::integral_constant<int, N>;
      using INX = std::integral_constant<int, KK + 1>;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (KK + 1 < 4) {
        rd_a(bo, INX(), IN());
        rd_b(bo, INX(), IN(), I0(), std::integral_constant<int, 4>());
      }
      mm(IS(), I0());
      if constexpr (KK + 1 < 4) rd_b(bo, INX(), IN(), std::integral_constant<int, 4>(), std::integral_constant<int, 9>());
      mm(IS(), I1());
    });
  }
  // partial dW of this workgroup: acc[cb][tap][e] = dW[16 cb + (lane & 15)][tap][ci0 + 16 wave + 4 g + e]
  float* out = P.slab + (long)blockIdx.x * (32 * 9) * P.c;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int co = 16 * cb + (lane & 15);
    if (co >= P.k) continue;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) *(f32x4*)(out + (long)(co * 9 + tap) * P.c + ci0 + 16 * wave + 4 * g) = acc[cb][tap];
  }
}

// ---- host -------------------------------------------------------------------------------
// tile width: 64 columns, or 32 for 32-wide maps
static int hconv_tc(const rtsds_conv_desc* d) {
  if (d->w % 64 == 0 && d->h % 4 == 0) return 64;
  if (d->w % 32 == 0 && d->h % 8 == 0) return 32;
  return 0;
}
static bool hconv_geom(const rtsds_conv_desc* d) {
  return d->dtype == RTSDS_BF16 && d->kh == 3 && d->kw == 3 && d->sh == 1 && d->sw == 1 && d->ph == 1 && d->pw == 1 &&
         d->dh == 1 && d->dw == 1 && hconv_tc(d) > 0;
}
static constexpr auto kHconvKmax = 512;
// forward: narrow outputs (Cout <= 32), or Cout a multiple of 32 up to 512 when the reduction
// is deep enough (Cin >= 256: >= 8 double-buffered channel chunks) -- N-tiled over blockIdx.y,
// each N tile re-staging the halo.  Measured (bs 8, 1024x512): ResNet layer3 3x3 256 -> 256
// at 32 x 64: 34 / 40 us fwd / dgrad vs 38 / 44 us on the implicit GEMM; layer1 / layer2
// (64 / 128 channels, 2-4 chunks) lose to the GEMM (59 vs 41 us, 42 vs 32 us fwd).
static bool hconv_kc_ok(int k, int c) {
  return k <= 32 || (k % 32 == 0 && k <= kHconvKmax && c >= 256);
}
bool hconv_ok(const rtsds_conv_desc* d) {
  if (!hconv_geom(d) || d->c % kCK != 0 || !hconv_kc_ok(d->k, d->c)) return false;
  return (long)d->n * d->h * d->w * d->c * 2 < (1L << 31);
}
// data gradient of a narrow-output conv (the same 3x3 same-padding conv run over dY with the
// flipped, transposed weights): Cout <= 32 padded to 32 input channels, Cin outputs tiled by 32
bool hconv_dgrad_ok(const rtsds_conv_desc* d) {
  if (!hconv_geom(d) || !hconv_kc_ok(d->k, d->k)) return false;  // reduction over Cout here
  return (long)d->n * d->h * d->w * d->c * 2 < (1L << 31);
}
int hconv_tiles(const rtsds_conv_desc* d) {
  const int tc = hconv_tc(d);
  return d->n * (d->h / (256 / tc)) * (d->w / tc);
}
template <int TC>
static void hconv_launch_tc(const HconvArgs& a, int tiles, int ntiles, hipStream_t st) {
  constexpr int stage = HTile<TC>::HaloBytes + kWBytes;
  static const bool lds_ok =
      hipFuncSetAttribute((const void*)hconv_fwd_kernel<0, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * stage) == hipSuccess &&
      hipFuncSetAttribute((const void*)hconv_fwd_kernel<1, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * stage) == hipSuccess &&
      hipFuncSetAttribute((const void*)hconv_fwd_kernel<-1, TC>, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * stage) == hipSuccess;
  (void)lds_ok;
  const int lds = a.c / kCK > 1 ? 2 * stage : stage;  // one channel chunk: a single stage
  const dim3 g(tiles, ntiles), b(256);
  if (a.act == RTSDS_ACT_NONE) hipLaunchKernelGGL((hconv_fwd_kernel<0, TC>), g, b, lds, st, a);
  else if (a.act == RTSDS_ACT_RELU) hipLaunchKernelGGL((hconv_fwd_kernel<1, TC>), g, b, lds, st, a);
  else hipLaunchKernelGGL((hconv_fwd_kernel<-1, TC>), g, b, lds, st, a);
}
static void hconv_launch(const HconvArgs& a, int tc, int tiles, int ntiles, hipStream_t st) {
  if (tc == 64) hconv_launch_tc<64>(a, tiles, ntiles, st);
  else hconv_launch_tc<32>(a, tiles, ntiles, st);
}
void hconv_fwd(const rtsds_conv_desc* d, const void* x, const void* w, const float* bias, const float* scale, const void* res,
               void* y, int act, float* stats, hipStream_t st) {
  HconvArgs a;
  a.x = (const bf16*)x; a.wt = (const bf16*)w; a.bias = bias; a.scale = scale; a.res = (const bf16*)res; a.y = (bf16*)y;
  a.stats = stats;
  a.n = d->n; a.h = d->h; a.w = d->w; a.c = d->c; a.k = d->k; a.act = act; a.accum = 0;
  hconv_launch(a, hconv_tc(d), hconv_tiles(d), (d->k + 31) / 32, st);
}
// dx (+)= conv(dy_p, wt_flipped): dy_p [n][h][w][kp] (kp % 32 == 0), wt [c][3][3][kp]
template <int TC>
static void hconv_dgrad_nt_launch(const HconvArgs& a, int tiles, hipStream_t st) {
  constexpr int lds = HTile<TC>::HaloBytes + 2 * kWBytes;
  static const bool lds_ok =
      hipFuncSetAttribute((const void*)hconv_dgrad_nt_kernel<TC>, hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  (void)lds_ok;
  static int cus = 0;
  if (!cus && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus < 1)) cus = 256;
  // output-channel tiles per workgroup: one round of two workgroups per CU
  const int ntn = a.k / 32;
  const int nt = std::max(1, (int)(((long)ntn * tiles + 2 * cus - 1) / (2 * cus)));
  hipLaunchKernelGGL(hconv_dgrad_nt_kernel<TC>, dim3(tiles, (ntn + nt - 1) / nt), dim3(256), lds, st, a, nt);
}
void hconv_dgrad(const rtsds_conv_desc* d, const void* dyp, int kp, const void* wt, void* dx, int accumulate, hipStream_t st) {
  HconvArgs a;
  a.x = (const bf16*)dyp; a.wt = (const bf16*)wt; a.bias = nullptr; a.scale = nullptr; a.res = nullptr; a.y = (bf16*)dx;
  a.stats = nullptr;
  a.n = d->n; a.h = d->h; a.w = d->w; a.c = kp; a.k = d->c; a.act = 0; a.accum = accumulate ? 1 : 0;
  if (kp == kCK && d->c % 32 == 0) {  // one channel chunk: the halo stays, the weight tiles stream
    if (hconv_tc(d) == 64) hconv_dgrad_nt_launch<64>(a, hconv_tiles(d), st);
    else hconv_dgrad_nt_launch<32>(a, hconv_tiles(d), st);
    return;
  }
  hconv_launch(a, hconv_tc(d), hconv_tiles(d), (d->c + 31) / 32, st);
}

// weight gradient (nwgrad_kernel): Cout <= 32 (dY padded to 32 channels by the caller), Cin a
// multiple of 128, 3x3 same-padding stride 1; any h, w (partial tiles read zeros)
bool nwgrad_ok(const rtsds_conv_desc* d) {
  return d->dtype == RTSDS_BF16 && d->kh == 3 && d->kw == 3 && d->sh == 1 && d->sw == 1 && d->ph == 1 && d->pw == 1 &&
         d->dh == 1 && d->dw == 1 && d->k <= 32 && d->c % kNwCI == 0 && (long)d->n * d->h * d->w * d->c * 2 < (1L << 31);
}
static int nw_tiles(const rtsds_conv_desc* d) { return d->n * ((d->h + kNwTH - 1) / kNwTH) * ((d->w + kNwTW - 1) / kNwTW); }
// one workgroup per CU: the Cin / 128 channel chunks x runs of tiles
static void nw_grid(const rtsds_conv_desc* d, int& runs, int& per) {
  static int cus = 0;
  if (!cus && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus < 1)) cus = 256;
  const int tiles = nw_tiles(d), chunks = d->c / kNwCI;
  const int want = std::max(1, cus / chunks);
  per = (tiles + want - 1) / want;
  runs = (tiles + per - 1) / per;
}
// split-K slabs of the launch (one per run of tiles)
int nwgrad_splits(const rtsds_conv_desc* d) {
  int runs, per;
  nw_grid(d, runs, per);
  return runs;
}
// slab [runs][32][9][c]: the partial dW of every run (rows co < k)
void nwgrad(const rtsds_conv_desc* d, const void* x, const void* dyp, float* slab, hipStream_t st) {
  NwArgs a = {};
  a.x = (const bf16*)x; a.dy = (const bf16*)dyp; a.slab = slab;
  a.n = d->n; a.h = d->h; a.w = d->w; a.c = d->c; a.k = d->k;
  a.tiles = nw_tiles(d);
  const int tw = (d->w + kNwTW - 1) / kNwTW, th = (d->h + kNwTH - 1) / kNwTH;
  a.f_tpi = fastdiv_make(th * tw);
  a.f_tw = fastdiv_make(tw);
  int runs;
  nw_grid(d, runs, a.per);
  hipLaunchKernelGGL(nwgrad_kernel, dim3(runs, d->c / kNwCI), dim3(64 * kNwWaves), 0, st, a);
}
