// Data gradient of narrow-output 1x1 convolutions (Cout <= 32) at full feature-map size: the
// BiSeNet head convs -- supervision1 / supervision2 (256 / 512 -> 19, build_bisenet.py:99-100)
// and the final 19 -> 19 conv (build_bisenet.py:117), run at 1/8 resolution (64 x 128 per
// image at 1024 x 512).  As an implicit GEMM this has a 19-deep reduction: the generic tiles
// need a Cout-pad copy of dY and a weight repack and run a single K-step per output tile.
// Here dx[p][ci..ci+V) (+)= sum_co dy[p][co] * w[co][ci..ci+V) runs as a packed-FMA kernel
// (v_pk_fma_f32, two channels per instruction): a thread owns V input channels and keeps
// their weight column w[0..k)[ci..ci+V) in registers for the whole launch; dY pixel tiles
// are staged in LDS as fp32 and read as broadcasts.  512 -> 19 at 65536 pixels: 28 us vs
// 43 us for the generic GEMM path; 19 -> 19: 7 vs 18 us.  (The weight gradient stays on the
// split-K GEMM, which measured faster than a VALU reduction here: 25 vs 42 us.)
#include "common.h"

namespace {
constexpr int kPwMaxK = 32;
constexpr int kPwTile = 64;         // data gradient: dY pixels staged per tile (large maps)
constexpr int kPwTileSmall = 16;    // ... for maps that would not give kPwDgradBlocks tiles of kPwTile
constexpr int kPwRows = 1;          // data gradient: pixel rows per thread pass
constexpr int kPwDgradBlocks = 1024;
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(float a, f2 b, f2 c) { return __builtin_elementwise_fma(f2{a, a}, b, c); }
__device__ __forceinline__ f2 bf2_to_f2(unsigned int u) { return f2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)}; }
__device__ __forceinline__ unsigned int f2_to_bf2(f2 v) {
  const bf16 lo = (bf16)v[0], hi = (bf16)v[1];
  return (unsigned int)__builtin_bit_cast(unsigned short, lo) | ((unsigned int)__builtin_bit_cast(unsigned short, hi) << 16);
}
}  // namespace

static int pw_kp(int k) { return k <= 20 ? 20 : 32; }
// channels per thread: KP * V weights live in registers
static int pw_dgrad_v(int k, int c) { return c % 2 ? 1 : (pw_kp(k) == 20 && c % 4 == 0 ? 4 : 2); }

bool pw_ok(const rtsds_conv_desc* d) {
  return d->dtype == RTSDS_BF16 && d->kh == 1 && d->kw == 1 && d->sh == 1 && d->sw == 1 && d->ph == 0 && d->pw == 0 &&
         d->k <= kPwMaxK && d->c / pw_dgrad_v(d->k, d->c) <= 256 && (long)d->n * d->h * d->w >= 4096;
}
// ---- data gradient ------------------------------------------------------------------------
// Thread t: lane t % lanes owns channels [lane*V, lane*V + V), pixel slot t / lanes of the
// `slots` pixels a block pass covers.  Per tile of kPwTile pixels: stage dY as fp32 [p][KP]
// (zero beyond k), then each slot walks its pixels.
template <int KP, int V, int TILE, int ROWS>
__global__ void __launch_bounds__(256) pw_dgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ w,
                                                       bf16* __restrict__ dx, long pixels, int c, int k, int accum) {
  __shared__ __attribute__((aligned(16))) float gs[TILE][KP];
  const int lanes = c / V, slots = 256 / lanes;
  const int lane = threadIdx.x % lanes, slot = threadIdx.x / lanes;
  const bool active = slot < slots;
  const int ci = lane * V;
  constexpr int H = V >= 2 ? V / 2 : 1;
  f2 wr[KP][H];
#pragma unroll
  for (int co = 0; co < KP; ++co)
#pragma unroll
    for (int h = 0; h < H; ++h) {
      // clamped, unconditional loads (all in flight together), zeroed past k
      const int cc = min(co, k - 1);
      if constexpr (V == 1) {
        const float v = (float)w[cc * c + ci];
        wr[co][h] = f2{co < k ? v : 0.f, 0.f};
      } else {
        const f2 v = bf2_to_f2(*(const unsigned int*)(w + cc * c + ci + 2 * h));
        wr[co][h] = co < k ? v : f2{0.f, 0.f};
      }
    }
  const long tiles = (pixels + TILE - 1) / TILE;
  for (long tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const long p0 = tile * TILE;
    const int np = (int)min((long)TILE, pixels - p0);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < (TILE * KP + 255) / 256; ++j) {
      const int i = threadIdx.x + j * 256;
      if (TILE * KP % 256 && i >= TILE * KP) break;
      const int r = i / KP, co = i - r * KP;
      const float v = (float)dy[(p0 + min(r, np - 1)) * k + min(co, k - 1)];
      gs[r][co] = (r < np && co < k) ? v : 0.f;
    }
    __syncthreads();
    if (!active) continue;
    // ROWS pixel rows per pass: their accumulate operands loaded first (all in flight with
    // the FMAs), their FMA chains interleaved; each row's sum in the same co order
    for (int r0 = slot; r0 < np; r0 += ROWS * slots) {
      f2 acc[ROWS][H], prev[ROWS][H];
#pragma unroll
      for (int u = 0; u < ROWS; ++u) {
        const int r = min(r0 + u * slots, np - 1);
        const bf16* o = dx + (p0 + r) * c + ci;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          acc[u][h] = f2{0.f, 0.f};
          if (accum) prev[u][h] = V == 1 ? f2{(float)o[0], 0.f} : bf2_to_f2(((const unsigned int*)o)[h]);
        }
      }
#pragma unroll
      for (int co = 0; co < KP; ++co)
#pragma unroll
        for (int u = 0; u < ROWS; ++u) {
          const float g = gs[min(r0 + u * slots, np - 1)][co];
#pragma unroll
          for (int h = 0; h < H; ++h) acc[u][h] = pk_fma(g, wr[co][h], acc[u][h]);
        }
#pragma unroll
      for (int u = 0; u < ROWS; ++u) {
        if (r0 + u * slots >= np) break;
        bf16* o = dx + (p0 + r0 + u * slots) * c + ci;
        // accumulate: the contribution rounded to bf16 first, then added -- bit-identical to
        // storing it and adding the two bf16 gradients (the GEMM epilogue's order)
        if constexpr (V == 1) {
          o[0] = (bf16)(accum ? (float)(bf16)acc[u][0][0] + prev[u][0][0] : acc[u][0][0]);
        } else {
          unsigned int out[H];
#pragma unroll
          for (int h = 0; h < H; ++h) out[h] = f2_to_bf2(accum ? bf2_to_f2(f2_to_bf2(acc[u][h])) + prev[u][h] : acc[u][h]);
          if constexpr (V == 4) *(uint2*)o = make_uint2(out[0], out[1]);
          else *(unsigned int*)o = out[0];
        }
      }
    }
  }
}

// ---- host ---------------------------------------------------------------------------------
template <int KP, int V>
static void pw_dgrad_launch(const rtsds_conv_desc* d, const void* dy, const void* w, void* dx, int accum, hipStream_t st) {
  const long px = (long)d->n * d->h * d->w;
  if (px >= (long)kPwDgradBlocks * kPwTile) {
    hipLaunchKernelGGL((pw_dgrad_kernel<KP, V, kPwTile, kPwRows>), dim3(kPwDgradBlocks), dim3(256), 0, st, (const bf16*)dy,
                       (const bf16*)w, (bf16*)dx, px, d->c, d->k, accum);
  } else {  // small maps (the supervision heads' 1/16 and 1/32 inputs): more, shorter tiles
    const int blocks = (int)std::min<long>(kPwDgradBlocks, (px + kPwTileSmall - 1) / kPwTileSmall);
    hipLaunchKernelGGL((pw_dgrad_kernel<KP, V, kPwTileSmall, kPwRows>), dim3(blocks), dim3(256), 0, st, (const bf16*)dy,
                       (const bf16*)w, (bf16*)dx, px, d->c, d->k, accum);
  }
}
void pw_dgrad(const rtsds_conv_desc* d, const void* dy, const void* w, void* dx, int accum, hipStream_t st) {
  const int v = pw_dgrad_v(d->k, d->c);
  if (pw_kp(d->k) == 20) {
    if (v == 4) pw_dgrad_launch<20, 4>(d, dy, w, dx, accum, st);
    else if (v == 2) pw_dgrad_launch<20, 2>(d, dy, w, dx, accum, st);
    else pw_dgrad_launch<20, 1>(d, dy, w, dx, accum, st);
  } else {
    if (v == 2) pw_dgrad_launch<32, 2>(d, dy, w, dx, accum, st);
    else pw_dgrad_launch<32, 1>(d, dy, w, dx, accum, st);
  }
}
