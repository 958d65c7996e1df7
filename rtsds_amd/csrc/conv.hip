// Convolution host side (C ABI): descriptors, workspace, routing between the implicit GEMM
// (conv_gemm_kernel.h, instantiated in conv_gemm_{fwd,dgrad,wgrad}.hip), the direct kernels
// (hconv / tapconv / imgconv / pw) and the GEMV-sized pooled 1x1 kernels; plus the helper
// kernels (weight repacks, channel padding, split-K reductions, bias column sums).
#include "conv_args.h"
#include <type_traits>
#include <utility>
#include <algorithm>
#include <cstdlib>

template <typename T> RT_DEV typename VecT<T>::v16 vzero() {
  typename VecT<T>::v16 z;
#pragma unroll
  for (int j = 0; j < VecT<T>::N; ++j) z[j] = (T)0.0f;
  return z;
}

// ---- small helper kernels -------------------------------------------------------------
// W[co][r][s][ci] -> Wt[ci][rr][ss][co_p] (DGRAD's B operand) over the taps
// r = r0h + rr*rstep (rr < tkh), s = r0w + ss*rstep (ss < tkw); zero for co >= co_n.
template <typename T>
__global__ void repack_wt_kernel(const T* __restrict__ w, T* __restrict__ wt, int co_n, int co_p, int kh, int kw, int ci_n,
                                 int tkh, int tkw, int r0h, int r0w, int rstep) {
  const int taps = tkh * tkw;
  const long total = (long)co_p * taps * ci_n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % co_p);
    const long rest = i / co_p;
    const int tap = (int)(rest % taps);
    const int ci = (int)(rest / taps);
    const int r = r0h + (tap / tkw) * rstep, sc = r0w + (tap % tkw) * rstep;
    wt[i] = co < co_n ? w[(((long)co * kh + r) * kw + sc) * ci_n + ci] : (T)0.0f;
  }
}

// All stride-2 DGRAD phases in one launch (blockIdx.y = phase): Wt_phase[ci][tap][co_p] at
// element offset boff[phase] (32-bit indexing: a conv's weights are far below 2^31 elements).
struct RepackPhases {
  int tkh[4], tkw[4], r0h[4], r0w[4];
  long boff[4];
};
template <typename T>
__global__ void __launch_bounds__(256) repack_phases_kernel(const T* __restrict__ w, T* __restrict__ wt, int co_n, int co_p, int kh,
                                                            int kw, int ci_n, int rstep, RepackPhases rp) {
  const int ph = blockIdx.y;
  const int tkw = rp.tkw[ph], taps = rp.tkh[ph] * tkw;
  const int total = co_p * taps * ci_n;
  T* out = wt + rp.boff[ph];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int co = i % co_p, rest = i / co_p;
    const int tap = rest % taps, ci = rest / taps;
    const int r = rp.r0h[ph] + (tap / tkw) * rstep, sc = rp.r0w[ph] + (tap % tkw) * rstep;
    out[i] = co < co_n ? w[((co * kh + r) * kw + sc) * ci_n + ci] : (T)0.0f;
  }
}

// dst[r][j] = j < c ? src[r][j] : 0   (channel padding of an NHWC tensor or of [co][tap][ci] weights)
// One thread per 16-byte output vector: dst[r][j0..j0+V) = src[r][j] (j < c) or 0.
template <typename T>
__global__ void __launch_bounds__(256) pad_channels_kernel(const T* __restrict__ src, T* __restrict__ dst, int total, int c,
                                                            int cpv, FastDiv fcpv) {
  constexpr int V = VecT<T>::N;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int r = (int)fdiv((uint32_t)i, fcpv);
    const int j0 = (i - r * cpv) * V;
    const T* s = src + (long)r * c;
    typename VecT<T>::v16 o;
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = j0 + e < c ? s[j0 + e] : (T)0.0f;
    *(typename VecT<T>::v16*)(dst + (long)i * V) = o;
  }
}

// dw[co][tap][ci] = sum_s part[s][co][tap][ci_p]   (split-K reduce + channel unpad).
// V consecutive input channels per thread (16-byte slab reads when c % 4 == 0), splits
// summed in a fixed order -- deterministic, no atomics.
// Block = 64 outputs x 4 split groups (wave g sums splits g, g + 4, ... in order; the four
// group sums are then added in group order): the many-split reductions of small weight
// tensors (ResNet layer1: ~100 splits) get 4x the parallelism of one thread per output.
template <int V>
__global__ void __launch_bounds__(256) split_reduce_kernel(const float* __restrict__ part, float* __restrict__ out, int nv,
                                                            int cv, FastDiv fcv, int cp, long slab, int splits, int accumulate) {
  __shared__ float red[4][64][V];
  const int lane = threadIdx.x & 63, sg = threadIdx.x >> 6;
  for (int i0 = blockIdx.x * 64; i0 < nv; i0 += gridDim.x * 64) {
    const int i = i0 + lane;
    const bool ok = i < nv;
    const int rt = (int)fdiv((uint32_t)(ok ? i : 0), fcv);  // co * taps + tap
    const long src = (long)rt * cp + (long)((ok ? i : 0) - rt * cv) * V;
    float s[V];
#pragma unroll
    for (int e = 0; e < V; ++e) s[e] = 0.f;
    // splits sg, sg + 4, ... summed in order; 8 loads in flight per thread (clamped,
    // unconditional; past-the-end ones contribute nothing)
    for (int q = sg; ok && q < splits; q += 32) {
      float t[8][V];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long off = (long)min(q + 4 * u, splits - 1) * slab + src;
        if constexpr (V == 4) {
          const f32x4 v = *(const f32x4*)(part + off);
#pragma unroll
          for (int e = 0; e < V; ++e) t[u][e] = v[e];
        } else {
          t[u][0] = part[off];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (q + 4 * u < splits)
#pragma unroll
          for (int e = 0; e < V; ++e) s[e] += t[u][e];
    }
#pragma unroll
    for (int e = 0; e < V; ++e) red[sg][lane][e] = s[e];
    __syncthreads();
    if (sg == 0 && ok) {
      float* o = out + (long)i * V;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float t = (red[0][lane][e] + red[1][lane][e]) + (red[2][lane][e] + red[3][lane][e]);
        o[e] = accumulate ? o[e] + t : t;
      }
    }
    __syncthreads();
  }
}

// dbias: two-stage deterministic column sum of dy[rows][c].  Stage 1: grid (RB, channel
// chunks); 256 threads laid out [row group][channel vector] (coalesced whole-row reads);
// block b sums rows b*rpi + rg (+= RB*rpi) -> part[b][c].  Stage 2 sums the RB partials.
template <typename T, int VEC>
__global__ void __launch_bounds__(256) colsum_part_kernel(const T* __restrict__ dy, float* __restrict__ part, long rows, int c) {
  __shared__ float red[256 * VEC];
  const int cbase = blockIdx.y * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const int tpr = (cl + VEC - 1) / VEC, rpi = 256 / tpr;
  const int tid = threadIdx.x, cv = tid % tpr, rg = tid / tpr;
  const int ch0 = cbase + cv * VEC;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  if (rg < rpi) {
    // 4 rows' loads in flight (clamped, unconditional), then the adds in row order
    const long step = (long)gridDim.x * rpi;
    for (long r = (long)blockIdx.x * rpi + rg; r < rows; r += 4 * step) {
      typename VecT<T>::v16 v[4];
      T sv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rr = min(r + u * step, rows - 1);
        if (VEC > 1) v[u] = *(const typename VecT<T>::v16*)(dy + rr * c + ch0);
        else sv[u] = dy[rr * c + ch0];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (r + u * step < rows) {
          if (VEC > 1) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) acc[j] += to_f(v[u][j]);
          } else {
            acc[0] += to_f(sv[u]);
          }
        }
    }
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[tid * VEC + j] = acc[j];
  __syncthreads();
  if (rg == 0) {
    for (int g = 1; g < rpi; ++g)
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += red[(g * tpr + cv) * VEC + j];
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      if (ch0 + j < c) part[(long)blockIdx.x * c + ch0 + j] = acc[j];
  }
}
// colsum_part_kernel<T, 1> (the same layout, loop and reduction: bit-identical partials) that
// also writes the gradient's channel-padded copy [rows][cp] the weight-gradient GEMM reads
// (pad_channels_kernel's job) -- one launch and one read of dY for both (c <= 256).
template <typename T>
__global__ void __launch_bounds__(256) pad_colsum_kernel(const T* __restrict__ dy, T* __restrict__ dyp, float* __restrict__ part,
                                                         long rows, int c, int cp) {
  __shared__ float red[256];
  const int tpr = c, rpi = 256 / tpr;
  const int tid = threadIdx.x, cv = tid % tpr, rg = tid / tpr;
  float acc = 0.f;
  if (rg < rpi) {
    const long step = (long)gridDim.x * rpi;
    for (long r = (long)blockIdx.x * rpi + rg; r < rows; r += 4 * step) {
      T sv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) sv[u] = dy[min(r + u * step, rows - 1) * c + cv];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rr = r + u * step;
        if (rr < rows) {
          acc += to_f(sv[u]);
          T* o = dyp + rr * cp;
          o[cv] = sv[u];
          for (int pc = c + cv; pc < cp; pc += tpr) o[pc] = from_f<T>(0.f);
        }
      }
    }
  }
  red[tid] = acc;
  __syncthreads();
  if (rg == 0) {
    for (int g = 1; g < rpi; ++g) acc += red[g * tpr + cv];
    part[(long)blockIdx.x * c + cv] = acc;
  }
}
__global__ void colsum_final_kernel(const float* __restrict__ part, float* __restrict__ out, int rb, int c, int accumulate) {
  const int cc = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
  for (int i0 = lane; i0 < rb; i0 += 64 * 8) {  // 8 partials in flight (clamped), added in order
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = part[(long)min(i0 + 64 * u, rb - 1) * c + cc];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (i0 + 64 * u < rb) s += t[u];
  }
  s = wave_sum(s);
  if (lane == 0) out[cc] = accumulate ? out[cc] + s : s;
}
static const int kColsumRB = 1024;

// ---- host side ---------------------------------------------------------------------------
static size_t esize(int dtype) { return dtype == RTSDS_BF16 ? 2 : 4; }
static ConvArgs make_args(const rtsds_conv_desc* d) {
  ConvArgs p = {};
  p.n = d->n; p.h = d->h; p.w = d->w; p.c = d->c; p.ho = d->ho; p.wo = d->wo; p.k = d->k;
  p.kh = d->kh; p.kw = d->kw; p.sh = d->sh; p.sw = d->sw; p.ph = d->ph; p.pw = d->pw;
  p.dh = d->dh; p.dw = d->dw;
  p.f_howo = fastdiv_make(d->ho * d->wo);
  p.f_wo = fastdiv_make(d->wo);
  p.f_hw = fastdiv_make(d->h * d->w);
  p.f_w = fastdiv_make(d->w);
  p.f_c = fastdiv_make(d->c);
  p.f_k = fastdiv_make(d->k);
  p.f_kw = fastdiv_make(d->kw);
  p.tkw = d->kw; p.f_tkw = p.f_kw;
  p.r0h = p.r0w = 0; p.rstep = 1; p.psh = 1; p.offh = p.offw = 0;
  p.hp = d->h; p.wp = d->w;
  p.tiles_per_split = 1 << 30;
  const int hw = d->ho * d->wo;
  p.wg_rows = (hw % 64 == 0) && (d->wo % 64 == 0 || 64 % d->wo == 0);
  const long big = std::max((long)d->n * d->h * d->w * d->c, (long)d->n * d->ho * d->wo * d->k) * (long)esize(d->dtype);
  p.gbuf = big < (1L << 31) && (long)d->k * d->kh * d->kw * d->c * (long)esize(d->dtype) < (1L << 31);
  return p;
}

static int check_desc(const rtsds_conv_desc* d) {
  if (d->n <= 0 || d->h <= 0 || d->w <= 0 || d->c <= 0 || d->k <= 0 || d->kh <= 0 || d->kw <= 0 ||
      d->sh <= 0 || d->sw <= 0 || d->dh <= 0 || d->dw <= 0 || d->ph < 0 || d->pw < 0)
    return RTSDS_ERR_SHAPE;
  const int ho = (d->h + 2 * d->ph - d->dh * (d->kh - 1) - 1) / d->sh + 1;
  const int wo = (d->w + 2 * d->pw - d->dw * (d->kw - 1) - 1) / d->sw + 1;
  if (ho != d->ho || wo != d->wo || ho <= 0 || wo <= 0) return RTSDS_ERR_SHAPE;
  if (d->dtype != RTSDS_F32 && d->dtype != RTSDS_BF16) return RTSDS_ERR_UNSUPPORTED;
  if ((long)d->n * d->h * d->w * 32 * ((d->c + 31) / 32) >= (1L << 31) ||
      (long)d->n * d->ho * d->wo * 32 * ((d->k + 31) / 32) >= (1L << 31))
    return RTSDS_ERR_UNSUPPORTED;
  return RTSDS_OK;
}

// Channel padding target so every gather runs on 16-B vectors: channel counts that are not a
// multiple of the vector width (3-channel images, 19-class maps, the 1-channel D logit) are
// zero-padded into workspace -- to a multiple of 32 (one filter tap per K-tile) when that
// costs < 1.7x, else to the vector width.
static int pad_c(int c, int dtype) {
  const int V = dtype == RTSDS_BF16 ? 8 : 4;
  if (c % V == 0) return c;
  const int c32 = (c + 31) / 32 * 32;
  if (c >= 8 && c32 * 10 < c * 17) return c32;
  return (c + V - 1) / V * V;
}
static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

template <typename T>
static void pad_launch(const void* src, void* dst, long rows, int c, int cp, hipStream_t st) {
  const int cpv = cp / VecT<T>::N;
  const long total = rows * cpv;  // < 2^31 (checked by check_desc via the element count)
  const int blocks = (int)std::max<long>(1, std::min<long>(1 << 16, (total + 255) / 256));
  hipLaunchKernelGGL(pad_channels_kernel<T>, dim3(blocks), dim3(256), 0, st, (const T*)src, (T*)dst, (int)total, c, cpv,
                     fastdiv_make(cpv));
}
static void pad_any(int dtype, const void* src, void* dst, long rows, int c, int cp, hipStream_t st) {
  if (dtype == RTSDS_BF16) pad_launch<bf16>(src, dst, rows, c, cp, st);
  else pad_launch<float>(src, dst, rows, c, cp, st);
}

// ---- pooled-vector 1x1 convs (ARM / FFM attention on [N, C, 1, 1], build_bisenet.py:41,
// 67-69): M = N <= 32 rows, a GEMV-sized problem.  One launch per pass, no channel padding,
// fp32 accumulation, BatchNorm partial statistics (one "tile" of M rows) from the exact values.
static const int kPooledMaxRows = 32;
static bool pooled_1x1(const rtsds_conv_desc* d) {
  return d->h == 1 && d->w == 1 && d->kh == 1 && d->kw == 1 && d->sh == 1 && d->sw == 1 && d->ph == 0 &&
         d->pw == 0 && d->n <= kPooledMaxRows;
}

// y[m][k] = act(sum_c x[m][c] w[k][c] + bias[k]); one wave per output channel k.
// scale (optional, [k]): the eval-mode BatchNorm fold, y = act(acc * scale + bias) (as the GEMM
// epilogue of rtsds_conv2d_fwd_bn; fmaf(acc, 1, b) == acc + b without it)
template <typename T, int MR>
__global__ void __launch_bounds__(256) pooled_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                        const float* __restrict__ bias, T* __restrict__ y, int m_n, int c,
                                                        int k_n, int act, int accum, float* __restrict__ stats,
                                                        const float* __restrict__ scale) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= k_n) return;
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
  for (int ci = lane; ci < c; ci += 64) {
    const float wv = to_f(w[(long)k * c + ci]);
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m < m_n) acc[m] = fmaf(to_f(x[(long)m * c + ci]), wv, acc[m]);
  }
#pragma unroll
  for (int m = 0; m < MR; ++m)
    if (m < m_n) acc[m] = wave_sum(acc[m]);
  if (lane != 0) return;
  const float bv = bias ? bias[k] : 0.f, sv = scale ? scale[k] : 1.f;
  float mean = 0.f;
#pragma unroll
  for (int m = 0; m < MR; ++m)
    if (m < m_n) {
      float v = fmaf(acc[m], sv, bv);
      acc[m] = v;
      mean += v;
      if (accum) v += to_f(y[(long)m * k_n + k]);
      if (act == RTSDS_ACT_RELU) v = fmaxf(v, 0.f);
      else if (act == RTSDS_ACT_LEAKY) v = v > 0.f ? v : 0.2f * v;
      else if (act == RTSDS_ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
      y[(long)m * k_n + k] = from_f<T>(v);
    }
  if (stats) {
    mean /= (float)m_n;
    float m2 = 0.f;
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m < m_n) m2 += (acc[m] - mean) * (acc[m] - mean);
    *(f32x4*)(stats + k * 4) = f32x4{(float)m_n, mean, m2, 0.f};
  }
}

// dx[m][c] (+)= sum_k dy[m][k] w[k][c]; one wave per input channel c, lanes over k.
template <typename T, int MR>
__global__ void __launch_bounds__(256) pooled_dgrad_kernel(const T* __restrict__ dy, const T* __restrict__ w, T* __restrict__ dx,
                                                          int m_n, int c, int k_n, int accum) {
  const int ci = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (ci >= c) return;
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
  for (int k = lane; k < k_n; k += 64) {
    const float wv = to_f(w[(long)k * c + ci]);
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m < m_n) acc[m] = fmaf(to_f(dy[(long)m * k_n + k]), wv, acc[m]);
  }
#pragma unroll
  for (int m = 0; m < MR; ++m)
    if (m < m_n) acc[m] = wave_sum(acc[m]);
  if (lane != 0) return;
#pragma unroll
  for (int m = 0; m < MR; ++m)
    if (m < m_n) {
      const long o = (long)m * c + ci;
      dx[o] = from_f<T>(accum ? to_f(from_f<T>(acc[m])) + to_f(dx[o]) : acc[m]);
    }
}

// dw[k][c] (+)= sum_m dy[m][k] x[m][c] (fp32), dbias[k] (+)= sum_m dy[m][k]; one thread per (k, c).
template <typename T>
__global__ void __launch_bounds__(256) pooled_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy, float* __restrict__ dw,
                                                          float* __restrict__ dbias, int m_n, int c, int k_n, int accum) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= k_n * c) return;
  const int k = i / c, ci = i - k * c;
  float acc = 0.f, bsum = 0.f;
  for (int m0 = 0; m0 < m_n; m0 += 8) {  // 8 rows' loads in flight (clamped), then the FMAs in order
    float g[8], xv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int m = min(m0 + u, m_n - 1);
      g[u] = to_f(dy[(long)m * k_n + k]);
      xv[u] = to_f(x[(long)m * c + ci]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (m0 + u < m_n) {
        acc = fmaf(g[u], xv[u], acc);
        bsum += g[u];
      }
  }
  dw[i] = accum ? dw[i] + acc : acc;
  if (dbias && ci == 0) dbias[k] = accum ? dbias[k] + bsum : bsum;
}

// ---- the FFM attention's backward in one launch (build_bisenet.py:67-70: conv1 + ReLU, conv2 +
// sigmoid on the pooled [N, C] vectors).  The unfused chain was six launches of a few hundred
// values each (sigmoid backward, conv2 data / weight gradient, ReLU backward, conv1 data /
// weight gradient).  One workgroup runs the same arithmetic in the same order -- the activation
// gradients rounded to the storage type as act_bwd_kernel stores them, the data gradients as
// pooled_dgrad_kernel forms them (a wave per input channel, lanes over output channels, the
// wave's shuffle sum), the weight gradients as pooled_wgrad_kernel (sums over rows in order) --
// so every result is bit-identical to the chain.
static constexpr int kMlpMaxC = 64, kMlpMaxN = 8, kMlpThreads = 1024;  // 16 waves: a wave per input channel or two
template <typename T>
__global__ void __launch_bounds__(kMlpThreads) pooled_mlp_bwd_kernel(const T* __restrict__ da, const T* __restrict__ a, const T* __restrict__ h,
                                                             const T* __restrict__ p, const T* __restrict__ w1, const T* __restrict__ w2,
                                                             float* __restrict__ dw1, float* __restrict__ db1, float* __restrict__ dw2,
                                                             float* __restrict__ db2, T* __restrict__ dp, int n, int c0, int c1, int c2,
                                                             int accum) {
  __shared__ float sg2[kMlpMaxN][kMlpMaxC], sg1[kMlpMaxN][kMlpMaxC], sh[kMlpMaxN][kMlpMaxC], sp[kMlpMaxN][kMlpMaxC];
  __shared__ float sw1[kMlpMaxC * kMlpMaxC], sw2[kMlpMaxC * kMlpMaxC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // every operand staged in LDS up front, each thread's loads clamped and unconditional (one
  // memory round trip for the launch; a load per loop iteration serialised them)
  {
    constexpr int NW = kMlpMaxC * kMlpMaxC / kMlpThreads, NV = (kMlpMaxN * kMlpMaxC + kMlpThreads - 1) / kMlpThreads;
    const int n1 = c1 * c0, n2 = c2 * c1;
    float v1[NW], v2[NW], vd[NV], va[NV], vh[NV], vp[NV];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int e = tid + kMlpThreads * u;
      v1[u] = to_f(w1[min(e, n1 - 1)]);
      v2[u] = to_f(w2[min(e, n2 - 1)]);
    }
    // (m, ch) = (e / 64, e % 64) of the [kMlpMaxN][kMlpMaxC] arrays, zero outside [n][c]
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int e = tid + kMlpThreads * u, m = min(e >> 6, n - 1), ch = e & 63;
      vd[u] = to_f(da[m * c2 + min(ch, c2 - 1)]);
      va[u] = to_f(a[m * c2 + min(ch, c2 - 1)]);
      vh[u] = to_f(h[m * c1 + min(ch, c1 - 1)]);
      vp[u] = to_f(p[m * c0 + min(ch, c0 - 1)]);
    }
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int e = tid + kMlpThreads * u;
      if (e < n1) sw1[e] = v1[u];
      if (e < n2) sw2[e] = v2[u];
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int e = tid + kMlpThreads * u, m = e >> 6, ch = e & 63;
      if (m >= kMlpMaxN) break;
      // sigmoid backward (act_bwd_kernel, act 3): g * s * (1 - s), stored rounded
      sg2[m][ch] = m < n && ch < c2 ? to_f(from_f<T>(vd[u] * va[u] * (1.f - va[u]))) : 0.f;
      sh[m][ch] = m < n && ch < c1 ? vh[u] : 0.f;
      sp[m][ch] = m < n && ch < c0 ? vp[u] : 0.f;
      sg1[m][ch] = 0.f;
    }
  }
  __syncthreads();
  // conv2 weight / bias gradient (pooled_wgrad_kernel): dw2[k][ci] over the rows in order
  for (int i = tid; i < c2 * c1; i += kMlpThreads) {
    const int k = i / c1, ci = i - k * c1;
    float acc = 0.f, bsum = 0.f;
    for (int m = 0; m < n; ++m) {
      acc = fmaf(sg2[m][k], sh[m][ci], acc);
      bsum += sg2[m][k];
    }
    dw2[i] = accum ? dw2[i] + acc : acc;
    if (db2 && ci == 0) db2[k] = accum ? db2[k] + bsum : bsum;
  }
  // conv2 data gradient (pooled_dgrad_kernel), then the ReLU backward (act_bwd_kernel, act 1)
  for (int ci = wave; ci < c1; ci += kMlpThreads / 64) {
    float acc[kMlpMaxN];
#pragma unroll
    for (int m = 0; m < kMlpMaxN; ++m) acc[m] = 0.f;
    for (int k = lane; k < c2; k += 64) {
      const float wv = sw2[k * c1 + ci];
#pragma unroll
      for (int m = 0; m < kMlpMaxN; ++m) acc[m] = fmaf(sg2[m][k], wv, acc[m]);  // (rows past n: zero)
    }
#pragma unroll
    for (int m = 0; m < kMlpMaxN; ++m) acc[m] = wave_sum(acc[m]);
    if (lane == 0)
#pragma unroll
      for (int m = 0; m < kMlpMaxN; ++m)
        if (m < n) sg1[m][ci] = sh[m][ci] > 0.f ? to_f(from_f<T>(acc[m])) : 0.f;
  }
  __syncthreads();
  // conv1 weight / bias gradient, data gradient into dp (stored, not accumulated)
  for (int i = tid; i < c1 * c0; i += kMlpThreads) {
    const int k = i / c0, ci = i - k * c0;
    float acc = 0.f, bsum = 0.f;
    for (int m = 0; m < n; ++m) {
      acc = fmaf(sg1[m][k], sp[m][ci], acc);
      bsum += sg1[m][k];
    }
    dw1[i] = accum ? dw1[i] + acc : acc;
    if (db1 && ci == 0) db1[k] = accum ? db1[k] + bsum : bsum;
  }
  for (int ci = wave; ci < c0; ci += kMlpThreads / 64) {
    float acc[kMlpMaxN];
#pragma unroll
    for (int m = 0; m < kMlpMaxN; ++m) acc[m] = 0.f;
    for (int k = lane; k < c1; k += 64) {
      const float wv = sw1[k * c0 + ci];
#pragma unroll
      for (int m = 0; m < kMlpMaxN; ++m) acc[m] = fmaf(sg1[m][k], wv, acc[m]);
    }
#pragma unroll
    for (int m = 0; m < kMlpMaxN; ++m) acc[m] = wave_sum(acc[m]);
    if (lane == 0)
#pragma unroll
      for (int m = 0; m < kMlpMaxN; ++m)
        if (m < n) dp[(long)m * c0 + ci] = from_f<T>(acc[m]);
  }
}
// Its forward in one launch: h = relu(conv1(p) + b1), a = sigmoid(conv2(h) + b2) with
// pooled_fwd_kernel's arithmetic per output channel (a wave per channel, lanes over the input
// channels in order, the wave's shuffle sum, then the bias and activation) -- bit-identical to
// its two launches; h is staged (rounded) in LDS between the two layers.
template <typename T>
__global__ void __launch_bounds__(kMlpThreads) pooled_mlp_fwd_kernel(const T* __restrict__ p, const T* __restrict__ w1,
                                                                     const float* __restrict__ b1, const T* __restrict__ w2,
                                                                     const float* __restrict__ b2, T* __restrict__ h, T* __restrict__ a,
                                                                     int n, int c0, int c1, int c2) {
  __shared__ float sx[kMlpMaxN][kMlpMaxC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < kMlpMaxN * kMlpMaxC; e += kMlpThreads) {
    const int m = e >> 6, ch = e & 63;
    sx[m][ch] = m < n && ch < c0 ? to_f(p[m * c0 + ch]) : 0.f;
  }
  __syncthreads();
  auto layer = [&](const T* __restrict__ w, const float* __restrict__ b, T* __restrict__ y, int c, int k_n, int act,
                   float (*keep)[kMlpMaxC]) {
    for (int k = wave; k < k_n; k += kMlpThreads / 64) {
      float acc[kMlpMaxN];
#pragma unroll
      for (int m = 0; m < kMlpMaxN; ++m) acc[m] = 0.f;
      for (int ci = lane; ci < c; ci += 64) {
        const float wv = to_f(w[(long)k * c + ci]);
#pragma unroll
        for (int m = 0; m < kMlpMaxN; ++m) acc[m] = fmaf(sx[m][ci], wv, acc[m]);  // (rows past n: zero)
      }
#pragma unroll
      for (int m = 0; m < kMlpMaxN; ++m) acc[m] = wave_sum(acc[m]);
      if (lane == 0) {
        const float bv = b ? b[k] : 0.f;
#pragma unroll
        for (int m = 0; m < kMlpMaxN; ++m)
          if (m < n) {
            float v = fmaf(acc[m], 1.f, bv);
            if (act == RTSDS_ACT_RELU) v = fmaxf(v, 0.f);
            else v = 1.f / (1.f + expf(-v));
            const T o = from_f<T>(v);
            y[(long)m * k_n + k] = o;
            if (keep) keep[m][k] = to_f(o);
          }
      }
    }
  };
  __shared__ float sh[kMlpMaxN][kMlpMaxC];
  for (int e = tid; e < kMlpMaxN * kMlpMaxC; e += kMlpThreads) sh[e >> 6][e & 63] = 0.f;
  __syncthreads();
  layer(w1, b1, h, c0, c1, RTSDS_ACT_RELU, sh);
  __syncthreads();
  for (int e = tid; e < kMlpMaxN * kMlpMaxC; e += kMlpThreads) sx[e >> 6][e & 63] = sh[e >> 6][e & 63];
  __syncthreads();
  layer(w2, b2, a, c1, c2, RTSDS_ACT_SIGMOID, nullptr);
}
extern "C" int rtsds_pooled_mlp_fwd(const void* p, const void* w1, const float* b1, const void* w2, const float* b2, void* h,
                                    void* a, int n, int c0, int c1, int c2, int dtype, void* stream) {
  if (n <= 0 || n > kMlpMaxN || c0 <= 0 || c1 <= 0 || c2 <= 0 || c0 > kMlpMaxC || c1 > kMlpMaxC || c2 > kMlpMaxC)
    return RTSDS_ERR_UNSUPPORTED;
  if (!p || !w1 || !w2 || !h || !a) return RTSDS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RTSDS_BF16)
    hipLaunchKernelGGL(pooled_mlp_fwd_kernel<bf16>, dim3(1), dim3(kMlpThreads), 0, st, (const bf16*)p, (const bf16*)w1, b1,
                       (const bf16*)w2, b2, (bf16*)h, (bf16*)a, n, c0, c1, c2);
  else if (dtype == RTSDS_F32)
    hipLaunchKernelGGL(pooled_mlp_fwd_kernel<float>, dim3(1), dim3(kMlpThreads), 0, st, (const float*)p, (const float*)w1, b1,
                       (const float*)w2, b2, (float*)h, (float*)a, n, c0, c1, c2);
  else return RTSDS_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
extern "C" int rtsds_pooled_mlp_bwd(const void* da, const void* a, const void* h, const void* p, const void* w1, const void* w2,
                                    float* dw1, float* db1, float* dw2, float* db2, void* dp, int n, int c0, int c1, int c2,
                                    int accumulate, int dtype, void* stream) {
  if (n <= 0 || n > kMlpMaxN || c0 <= 0 || c1 <= 0 || c2 <= 0 || c0 > kMlpMaxC || c1 > kMlpMaxC || c2 > kMlpMaxC)
    return RTSDS_ERR_UNSUPPORTED;
  if (!da || !a || !h || !p || !w1 || !w2 || !dw1 || !dw2 || !dp) return RTSDS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RTSDS_BF16)
    hipLaunchKernelGGL(pooled_mlp_bwd_kernel<bf16>, dim3(1), dim3(kMlpThreads), 0, st, (const bf16*)da, (const bf16*)a, (const bf16*)h,
                       (const bf16*)p, (const bf16*)w1, (const bf16*)w2, dw1, db1, dw2, db2, (bf16*)dp, n, c0, c1, c2,
                       accumulate ? 1 : 0);
  else if (dtype == RTSDS_F32)
    hipLaunchKernelGGL(pooled_mlp_bwd_kernel<float>, dim3(1), dim3(kMlpThreads), 0, st, (const float*)da, (const float*)a, (const float*)h,
                       (const float*)p, (const float*)w1, (const float*)w2, dw1, db1, dw2, db2, (float*)dp, n, c0, c1, c2,
                       accumulate ? 1 : 0);
  else return RTSDS_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// Vector forms (C % V == 0): every lane loads whole 16-B chunks, all loads of a lane issued
// before its FMAs -- one memory round trip per wave instead of one per 64 channels (the scalar
// kernels above walked C in 2-B steps: ~14 us for a 512 x 512 GEMV).
template <typename T, int MR>
__global__ void __launch_bounds__(256) pooled_fwd_vec_kernel(const T* __restrict__ x, const T* __restrict__ w,
                                                            const float* __restrict__ bias, T* __restrict__ y, int m_n, int c,
                                                            int k_n, int act, int accum, float* __restrict__ stats,
                                                            const float* __restrict__ scale) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= k_n) return;
  float acc[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) acc[m] = 0.f;
  for (int cc = lane * V; cc < c; cc += 64 * V) {
    const V16 wv = *(const V16*)(w + (long)k * c + cc);
    V16 xv[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) xv[m] = m < m_n ? *(const V16*)(x + (long)m * c + cc) : vzero<T>();
#pragma unroll
    for (int m = 0; m < MR; ++m)
#pragma unroll
      for (int j = 0; j < V; ++j) acc[m] = fmaf(to_f(xv[m][j]), to_f(wv[j]), acc[m]);
  }
#pragma unroll
  for (int m = 0; m < MR; ++m)
    if (m < m_n) acc[m] = wave_sum(acc[m]);
  if (lane != 0) return;
  const float bv = bias ? bias[k] : 0.f, sv = scale ? scale[k] : 1.f;
  float mean = 0.f;
#pragma unroll
  for (int m = 0; m < MR; ++m)
    if (m < m_n) {
      float v = fmaf(acc[m], sv, bv);
      acc[m] = v;
      mean += v;
      if (accum) v += to_f(y[(long)m * k_n + k]);
      if (act == RTSDS_ACT_RELU) v = fmaxf(v, 0.f);
      else if (act == RTSDS_ACT_LEAKY) v = v > 0.f ? v : 0.2f * v;
      else if (act == RTSDS_ACT_SIGMOID) v = 1.f / (1.f + expf(-v));
      y[(long)m * k_n + k] = from_f<T>(v);
    }
  if (stats) {
    mean /= (float)m_n;
    float m2 = 0.f;
#pragma unroll
    for (int m = 0; m < MR; ++m)
      if (m < m_n) m2 += (acc[m] - mean) * (acc[m] - mean);
    *(f32x4*)(stats + k * 4) = f32x4{(float)m_n, mean, m2, 0.f};
  }
}

// bf16, m_n <= 8, C % 8 == 0: one wave per 8-channel chunk of dx, lanes over k (16-B weight
// chunks); the 8 x 8 per-lane partials are summed by a reduce-scatter butterfly (63 shuffles
// instead of 64 full wave sums), after which lane l holds dx[l / 8][ci0 + l % 8].
__global__ void __launch_bounds__(256) pooled_dgrad_vec_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ w,
                                                              bf16* __restrict__ dx, int m_n, int c, int k_n, int accum) {
  const int ci0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 8, lane = threadIdx.x & 63;
  if (ci0 >= c) return;
  float v[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = 0.f;
  // KI k-rows per lane with every load issued before the FMAs (clamped, unconditional): one
  // memory round trip per 64 KI rows -- the 512-row loop serialised eight of them (18.6 us)
  constexpr int KI = 4;
  for (int k0 = lane; k0 < k_n; k0 += 64 * KI) {
    bf16x8 wv[KI];
    float g[KI][8];
#pragma unroll
    for (int u = 0; u < KI; ++u) {
      const int k = min(k0 + 64 * u, k_n - 1);
      wv[u] = *(const bf16x8*)(w + (long)k * c + ci0);
#pragma unroll
      for (int m = 0; m < 8; ++m) g[u][m] = (float)dy[(long)min(m, m_n - 1) * k_n + k];
    }
#pragma unroll
    for (int u = 0; u < KI; ++u) {
      if (k0 + 64 * u >= k_n) break;
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const float gm = m < m_n ? g[u][m] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[m * 8 + j] = fmaf(gm, (float)wv[u][j], v[m * 8 + j]);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {  // keep the half of v[0, 2o) this lane's bit o selects
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int i = 0; i < o; ++i) {
      const float send = hi ? v[i] : v[i + o];
      const float keep = hi ? v[i + o] : v[i];
      v[i] = keep + __shfl_xor(send, o, 64);
    }
  }
  const int m = lane >> 3;
  if (m < m_n) {
    const long off = (long)m * c + ci0 + (lane & 7);
    // accumulate: rounded first, then added (= storing it and adding the two bf16 gradients)
    dx[off] = (bf16)(accum ? (float)(bf16)v[0] + (float)dx[off] : v[0]);
  }
}

template <typename T>
static void pooled_fwd_launch(const rtsds_conv_desc* d, const void* x, const void* w, const float* bias, void* y, int act,
                              int accum, float* stats, hipStream_t st, const float* scale = nullptr) {
  if (d->c % VecT<T>::N == 0) {
    if (d->n <= 8)
      hipLaunchKernelGGL((pooled_fwd_vec_kernel<T, 8>), dim3(rt_cdiv(d->k, 4)), dim3(256), 0, st, (const T*)x, (const T*)w,
                         bias, (T*)y, d->n, d->c, d->k, act, accum, stats, scale);
    else
      hipLaunchKernelGGL((pooled_fwd_vec_kernel<T, kPooledMaxRows>), dim3(rt_cdiv(d->k, 4)), dim3(256), 0, st, (const T*)x,
                         (const T*)w, bias, (T*)y, d->n, d->c, d->k, act, accum, stats, scale);
    return;
  }
  if (d->n <= 8)
    hipLaunchKernelGGL((pooled_fwd_kernel<T, 8>), dim3(rt_cdiv(d->k, 4)), dim3(256), 0, st, (const T*)x, (const T*)w, bias,
                       (T*)y, d->n, d->c, d->k, act, accum, stats, scale);
  else
    hipLaunchKernelGGL((pooled_fwd_kernel<T, kPooledMaxRows>), dim3(rt_cdiv(d->k, 4)), dim3(256), 0, st, (const T*)x,
                       (const T*)w, bias, (T*)y, d->n, d->c, d->k, act, accum, stats, scale);
}
template <typename T>
static void pooled_dgrad_launch(const rtsds_conv_desc* d, const void* dy, const void* w, void* dx, int accum, hipStream_t st) {
  if (sizeof(T) == 2 && d->n <= 8 && d->c % 8 == 0) {
    hipLaunchKernelGGL(pooled_dgrad_vec_kernel, dim3(rt_cdiv(d->c / 8, 4)), dim3(256), 0, st, (const bf16*)dy, (const bf16*)w,
                       (bf16*)dx, d->n, d->c, d->k, accum);
    return;
  }
  if (d->n <= 8)
    hipLaunchKernelGGL((pooled_dgrad_kernel<T, 8>), dim3(rt_cdiv(d->c, 4)), dim3(256), 0, st, (const T*)dy, (const T*)w,
                       (T*)dx, d->n, d->c, d->k, accum);
  else
    hipLaunchKernelGGL((pooled_dgrad_kernel<T, kPooledMaxRows>), dim3(rt_cdiv(d->c, 4)), dim3(256), 0, st, (const T*)dy,
                       (const T*)w, (T*)dx, d->n, d->c, d->k, accum);
}
template <typename T>
static void pooled_wgrad_launch(const rtsds_conv_desc* d, const void* x, const void* dy, float* dw, float* dbias, int accum,
                                hipStream_t st) {
  hipLaunchKernelGGL(pooled_wgrad_kernel<T>, dim3(rt_cdiv((long)d->k * d->c, 256)), dim3(256), 0, st, (const T*)x,
                     (const T*)dy, dw, dbias, d->n, d->c, d->k, accum);
}

// ---- 3-channel stride-2 convs on the image (ResNet stem 7x7 s2 p3, build_contextpath.py via
// torchvision conv1; spatial-path ConvBlock 3x3 s2 p1, build_bisenet.py:9-14).  Gathering one
// 16-B chunk per tap would carry 3 useful channels of 8 (and 8/3 of the MFMA K): instead the
// image is padded to 4 channels and viewed as "superpixels" of two horizontally adjacent
// pixels (8 bf16 = one 16-B chunk).  With odd padding pw, taps s = 2p - 1 + q (q = 0, 1) of
// output column ow read superpixel ow - (pw + 1) / 2 + p, so the conv becomes an ordinary
// implicit GEMM over (row tap, tap pair, 8 elements) with stride (2, 1): K = kh * (kw + 1) / 2 * 8
// (stem: 224 instead of 392), every chunk 16-B aligned and fully in or out of the padding.
static bool sp_path(const rtsds_conv_desc* d) {
  return d->dtype == RTSDS_BF16 && d->c == 3 && d->sh == 2 && d->sw == 2 && d->dh == 1 && d->dw == 1 &&
         (d->pw & 1) == 1 && (d->kw & 1) == 1 && (d->w & 1) == 0;
}
static rtsds_conv_desc sp_desc(const rtsds_conv_desc* d) {
  rtsds_conv_desc v = *d;
  v.w = d->w / 2;
  v.c = 8;
  v.kw = (d->kw + 1) / 2;
  v.sw = 1;
  v.pw = (d->pw + 1) / 2;
  return v;
}
__global__ void __launch_bounds__(256) sp_pad4_kernel(const bf16* __restrict__ x, bf16* __restrict__ x4, long pixels) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= pixels) return;
  bf16x4 v;
  v[0] = x[i * 3];
  v[1] = x[i * 3 + 1];
  v[2] = x[i * 3 + 2];
  v[3] = (bf16)0.f;
  *(bf16x4*)(x4 + i * 4) = v;
}
// w[k][r][s][3] -> w'[k][r][p][q*4 + ch], s = 2p - 1 + q (zero outside [0, kw), ch == 3).
__global__ void __launch_bounds__(256) sp_repack_w_kernel(const bf16* __restrict__ w, bf16* __restrict__ wp, int k, int kh,
                                                          int kw, int kwp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= k * kh * kwp * 8) return;
  const int e = i & 7, t = i >> 3;
  const int p = t % kwp, kr = t / kwp;  // kr = co * kh + r
  const int s = 2 * p - 1 + (e >> 2), ch = e & 3;
  wp[i] = (s >= 0 && s < kw && ch < 3) ? w[((long)kr * kw + s) * 3 + ch] : (bf16)0.f;
}
// dW'[k][r][p][8] (fp32) -> dw[k][r][s][3] (+=).
__global__ void __launch_bounds__(256) sp_unpack_dw_kernel(const float* __restrict__ dwp, float* __restrict__ dw, int k, int kh,
                                                           int kw, int kwp, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= k * kh * kw * 3) return;
  const int ch = i % 3, t = i / 3;
  const int s = t % kw, kr = t / kw;
  const int p = (s + 1) >> 1, q = (s + 1) & 1;
  const float v = dwp[((long)kr * kwp + p) * 8 + q * 4 + ch];
  dw[i] = accumulate ? dw[i] + v : v;
}
static size_t sp_x4_bytes(const rtsds_conv_desc* d) { return ((size_t)d->n * d->h * d->w * 8 + 255) & ~(size_t)255; }
static size_t sp_w_bytes(const rtsds_conv_desc* d) {
  return ((size_t)d->k * d->kh * ((d->kw + 1) / 2) * 16 + 255) & ~(size_t)255;
}
static void sp_pad4(const rtsds_conv_desc* d, const void* x, void* x4, hipStream_t st) {
  const long px = (long)d->n * d->h * d->w;
  hipLaunchKernelGGL(sp_pad4_kernel, dim3((unsigned)((px + 255) / 256)), dim3(256), 0, st, (const bf16*)x, (bf16*)x4, px);
}

// Halo-resident direct conv for narrow 3x3 outputs (hconv.hip).
bool hconv_ok(const rtsds_conv_desc* d);
int hconv_tiles(const rtsds_conv_desc* d);
void hconv_fwd(const rtsds_conv_desc* d, const void* x, const void* w, const float* bias, const float* scale, const void* res, void* y,
               int act, float* stats, hipStream_t st);
bool hconv_dgrad_ok(const rtsds_conv_desc* d);
bool nwgrad_ok(const rtsds_conv_desc* d);
int nwgrad_splits(const rtsds_conv_desc* d);
void nwgrad(const rtsds_conv_desc* d, const void* x, const void* dyp, float* slab, hipStream_t st);
void hconv_dgrad(const rtsds_conv_desc* d, const void* dyp, int kp, const void* wt, void* dx, int accumulate, hipStream_t st);
bool pw_ok(const rtsds_conv_desc* d);
// Direct MFMA conv for the 3-channel stride-2 image convs (imgconv.hip).
bool imgconv_ok(const rtsds_conv_desc* d);
bool imgconv_pool_ok(const rtsds_conv_desc* d, int hp, int wp);
void imgconv_pool_fwd(const rtsds_conv_desc* d, const void* x4, const void* w, const float* shift, const float* scale, void* y,
                      int act, int hp, int wp, int pp, hipStream_t st);
int imgconv_tiles(const rtsds_conv_desc* d);
void imgconv_fwd(const rtsds_conv_desc* d, const void* x4, const void* w, const float* bias, const float* scale, void* y,
                 int act, float* stats, hipStream_t st);
void pw_dgrad(const rtsds_conv_desc* d, const void* dy, const void* w, void* dx, int accum, hipStream_t st);
// Register-resident-weight direct conv for 3x3 64 -> 64 stride-1 convs (tapconv.hip).
bool tapconv_ok(const rtsds_conv_desc* d);
int tapconv_rows(const rtsds_conv_desc* d, int dgrad);
void tapconv_fwd(const rtsds_conv_desc* d, const void* x, const void* w, const float* bias, const float* scale, const void* res,
                 void* y, int act, float* stats, hipStream_t st);
void tapconv_dgrad(const rtsds_conv_desc* d, const void* dy, const void* wt, void* dx, int accumulate, const void* mask,
                   int mask_act, float* bnb_part, const void* bnb_x, const float* gamma, const float* beta, const float* mean,
                   const float* invstd, int bnb_act, hipStream_t st);

// Number of M tiles (= BatchNorm partial-statistics rows) the forward launch of d uses.
extern "C" int rtsds_conv2d_fwd_stats_tiles(const rtsds_conv_desc* d) {
  if (pooled_1x1(d)) return 1;
  if (tapconv_ok(d)) return tapconv_rows(d, 0);
  if (hconv_ok(d)) return hconv_tiles(d);
  if (imgconv_ok(d)) return imgconv_tiles(d);
  int bm, bn;
  const long M = (long)d->n * d->ho * d->wo;
  const long K = sp_path(d) ? 0 : (long)d->kh * d->kw * pad_c(d->c, d->dtype);  // rtsds_conv2d_fwd's p.K
  pick_tile(M, d->k, d->dtype == RTSDS_BF16, bm, bn, true, K);
  return (int)((M + bm - 1) / bm);
}

// Channel pitch of x the forward / weight-gradient gathers read (RTSDS_INPUT_PADDED: the caller
// hands x with this pitch, zero beyond c): 4 for the superpixel image convs, the vector-padded
// channel count for the implicit GEMM, c itself for the pooled and halo paths.
static int input_pitch(const rtsds_conv_desc* d) {
  if (pooled_1x1(d) || hconv_ok(d)) return d->c;
  if (sp_path(d)) return 4;
  return pad_c(d->c, d->dtype);
}
extern "C" int rtsds_conv2d_input_pitch(const rtsds_conv_desc* d) {
  return check_desc(d) ? 0 : input_pitch(d);
}

// FWD split-K for narrow outputs (<= 32 channels: DeepLab's ASPP branches, 2048 -> 19 classes
// at 65x129, K = 18,432): the 128x32 tiles of M = 33,540 rows make 263 workgroups, one 4-wave
// group per CU walking 288 K-tiles, latency-bound on the operand gathers.  S K-splits (>= 16
// K-tiles each) into fp32 slabs [S][M][N] put ~6 groups on every CU (194 -> 100 us); fwd_split_reduce_kernel
// sums them in split order and adds the bias (and y, for ConvSum's accumulate).  Only without
// BatchNorm-statistics / activation epilogues; BK = 64 (LDS-DMA path: Cin % 32 == 0).
struct FwdSplit {
  int splits, tps;
  size_t slab_bytes;
};
static FwdSplit fwd_split(const rtsds_conv_desc* d) {
  FwdSplit s = {1, 1 << 30, 0};
  if (d->dtype != RTSDS_BF16 || d->k > 32 || d->c % 32 != 0 || pooled_1x1(d) || hconv_ok(d) || sp_path(d)) return s;
  const long M = (long)d->n * d->ho * d->wo;
  const int nk = (d->kh * d->kw * d->c + 63) / 64;
  int bm, bn;
  pick_tile(M, d->k, true, bm, bn, true);
  const long tiles = (M + bm - 1) / bm;
  if (tiles >= 512 || nk < 32) return s;
  const int want = (int)std::min<long>((1536 + tiles - 1) / tiles, nk / 16);
  if (want < 2) return s;
  s.tps = (nk + want - 1) / want;
  s.splits = (nk + s.tps - 1) / s.tps;
  s.slab_bytes = al256((size_t)s.splits * M * d->k * 4);
  return s;
}

// y (+)= bias + sum_s slab[s] -> bf16, the split order fixed (deterministic)
__global__ void __launch_bounds__(256) fwd_split_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ bias,
                                                               bf16* __restrict__ y, long total, int n, long stride,
                                                               int splits, int accum) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    float s = slab[i];
    for (int q = 1; q < splits; ++q) s += slab[q * stride + i];
    if (bias) s += bias[i % n];
    if (accum) s += to_f(y[i]);
    y[i] = from_f<bf16>(s);
  }
}

// FWD workspace: channel-padded copies of x and w when Cin is not a vector multiple, then the
// split-K slabs (fwd_split).
static size_t fwd_operand_ws(const rtsds_conv_desc* d) {
  if (pooled_1x1(d) || hconv_ok(d)) return 0;
  if (sp_path(d)) return sp_x4_bytes(d) + sp_w_bytes(d);
  const int cp = pad_c(d->c, d->dtype);
  if (cp == d->c) return 0;
  const size_t es = esize(d->dtype);
  return al256((size_t)d->n * d->h * d->w * cp * es) + al256((size_t)d->k * d->kh * d->kw * cp * es);
}
extern "C" size_t rtsds_conv2d_fwd_workspace(const rtsds_conv_desc* d) {
  return fwd_operand_ws(d) + fwd_split(d).slab_bytes;
}

// Operands of the forward GEMM: the superpixel view of 3-channel stride-2 convs, or
// channel-padded copies when Cin is not a vector multiple (workspace), else x / w as given.
static void fwd_prepare(const rtsds_conv_desc* d0, const void*& x, const void*& w, void* ws, rtsds_conv_desc& d,
                        hipStream_t st, bool x_padded = false) {
  d = *d0;
  if (sp_path(d0)) {
    void* x4 = ws;
    void* wp = (char*)ws + sp_x4_bytes(d0);
    if (!x_padded) sp_pad4(d0, x, x4, st);
    const int n = d0->k * d0->kh * ((d0->kw + 1) / 2) * 8;
    hipLaunchKernelGGL(sp_repack_w_kernel, dim3(rt_cdiv(n, 256)), dim3(256), 0, st, (const bf16*)w, (bf16*)wp, d0->k,
                       d0->kh, d0->kw, (d0->kw + 1) / 2);
    d = sp_desc(d0);
    if (!x_padded) x = x4;
    w = wp;
    return;
  }
  const int cp = pad_c(d.c, d.dtype);
  if (cp != d.c) {
    const size_t es = esize(d.dtype);
    void* xp = ws;
    void* wp = (char*)ws + al256((size_t)d.n * d.h * d.w * cp * es);
    if (!x_padded) {
      pad_any(d.dtype, x, xp, (long)d.n * d.h * d.w, d.c, cp, st);
      x = xp;
    }
    pad_any(d.dtype, w, wp, (long)d.k * d.kh * d.kw, d.c, cp, st);
    w = wp;
    d.c = cp;
  }
}

extern "C" int rtsds_conv2d_fwd(const rtsds_conv_desc* d0, const void* x, const void* w, const float* bias,
                                void* y, int act, float* bn_stats, void* ws, size_t ws_bytes, void* stream) {
  int e = check_desc(d0);
  if (e) return e;
  if (ws_bytes < rtsds_conv2d_fwd_workspace(d0)) return RTSDS_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  if (pooled_1x1(d0)) {
    const int accum = (act & RTSDS_ACCUMULATE) ? 1 : 0;
    if (bn_stats && ((act & 0xff) || accum)) return RTSDS_ERR_UNSUPPORTED;
    if (d0->dtype == RTSDS_BF16) pooled_fwd_launch<bf16>(d0, x, w, bias, y, act & 0xff, accum, bn_stats, st);
    else pooled_fwd_launch<float>(d0, x, w, bias, y, act & 0xff, accum, bn_stats, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  const bool x_padded = (act & RTSDS_INPUT_PADDED) != 0;
  if (x_padded && input_pitch(d0) == d0->c) return RTSDS_ERR_UNSUPPORTED;
  if (tapconv_ok(d0) && !(act & RTSDS_ACCUMULATE)) {
    if (bn_stats && (act & 0xff)) return RTSDS_ERR_UNSUPPORTED;
    tapconv_fwd(d0, x, w, bias, nullptr, nullptr, y, act & 0xff, bn_stats, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (hconv_ok(d0) && !(act & RTSDS_ACCUMULATE)) {
    if (bn_stats && (act & 0xff)) return RTSDS_ERR_UNSUPPORTED;
    hconv_fwd(d0, x, w, bias, nullptr, nullptr, y, act & 0xff, bn_stats, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (imgconv_ok(d0) && !(act & RTSDS_ACCUMULATE)) {
    if (bn_stats && (act & 0xff)) return RTSDS_ERR_UNSUPPORTED;
    if (!x_padded) sp_pad4(d0, x, ws, st);
    imgconv_fwd(d0, x_padded ? x : ws, w, bias, nullptr, y, act & 0xff, bn_stats, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  rtsds_conv_desc d;
  fwd_prepare(d0, x, w, ws, d, st, x_padded);
  ConvArgs p = make_args(&d);
  p.a = x; p.b = w; p.bias = bias; p.out = y;
  p.act = act & 0xff;
  p.accum = (act & RTSDS_ACCUMULATE) ? 1 : 0;
  if (bn_stats && (p.act || p.accum)) return RTSDS_ERR_UNSUPPORTED;
  p.stats = bn_stats;
  p.M = d.n * d.ho * d.wo;
  p.N = d.k;
  p.K = d.kh * d.kw * d.c;
  const FwdSplit fs = fwd_split(d0);
  if (fs.splits > 1 && !bn_stats && p.act == 0) {
    p.slab = (float*)((char*)ws + fwd_operand_ws(d0));
    p.tiles_per_split = fs.tps;
    p.split_stride = (long)p.M * p.N;
    dispatch_align<bf16, MODE_FWD>(p, d.c, st, fs.splits);
    const long total = (long)p.M * p.N;
    hipLaunchKernelGGL(fwd_split_reduce_kernel, dim3((int)std::min<long>(8192, (total + 255) / 256)), dim3(256), 0, st,
                       (const float*)p.slab, bias, (bf16*)y, total, p.N, p.split_stride, fs.splits, p.accum);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (d.dtype == RTSDS_BF16) dispatch_align<bf16, MODE_FWD>(p, d.c, st);
  else dispatch_align<float, MODE_FWD>(p, d.c, st);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// Eval-mode conv + BatchNorm(running statistics) [+ residual] [+ activation] in one launch:
// y = act(conv(x, w) * scale + shift + res), scale / shift from rtsds_bn_fold.
extern "C" int rtsds_conv2d_fwd_bn(const rtsds_conv_desc* d0, const void* x, const void* w, const float* scale,
                                   const float* shift, const void* res, void* y, int act, void* ws, size_t ws_bytes,
                                   void* stream) {
  if (!scale || !shift || (act & RTSDS_ACCUMULATE)) return RTSDS_ERR_UNSUPPORTED;
  int e = check_desc(d0);
  if (e) return e;
  if (ws_bytes < rtsds_conv2d_fwd_workspace(d0)) return RTSDS_ERR_WORKSPACE;
  const bool x_padded = (act & RTSDS_INPUT_PADDED) != 0;
  if (x_padded && input_pitch(d0) == d0->c) return RTSDS_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  if (pooled_1x1(d0) && !res && !x_padded) {  // the attention refinements' 1x1 convs on pooled vectors
    if (d0->dtype == RTSDS_BF16) pooled_fwd_launch<bf16>(d0, x, w, shift, y, act & 0xff, 0, nullptr, st, scale);
    else pooled_fwd_launch<float>(d0, x, w, shift, y, act & 0xff, 0, nullptr, st, scale);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (tapconv_ok(d0)) {
    tapconv_fwd(d0, x, w, shift, scale, res, y, act & 0xff, nullptr, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (hconv_ok(d0)) {
    hconv_fwd(d0, x, w, shift, scale, res, y, act & 0xff, nullptr, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (imgconv_ok(d0) && !res) {
    if (!x_padded) sp_pad4(d0, x, ws, st);
    imgconv_fwd(d0, x_padded ? x : ws, w, shift, scale, y, act & 0xff, nullptr, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  rtsds_conv_desc d;
  fwd_prepare(d0, x, w, ws, d, st, x_padded);
  ConvArgs p = make_args(&d);
  p.a = x; p.b = w; p.bias = shift; p.scale = scale; p.res = res; p.out = y;
  p.act = act & 0xff;
  p.M = d.n * d.ho * d.wo;
  p.N = d.k;
  p.K = d.kh * d.kw * d.c;
  if (d.dtype == RTSDS_BF16) dispatch_align<bf16, MODE_FWD>(p, d.c, st);
  else dispatch_align<float, MODE_FWD>(p, d.c, st);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

extern "C" int rtsds_conv2d_fwd_bn_ld(const rtsds_conv_desc* d0, const void* x, const void* w, const float* scale,
                                      const float* shift, void* y, long ldy, int act, void* ws, size_t ws_bytes,
                                      void* stream) {
  if (!scale || !shift || (act & RTSDS_ACCUMULATE)) return RTSDS_ERR_UNSUPPORTED;
  int e = check_desc(d0);
  if (e) return e;
  if (ldy == d0->k) return rtsds_conv2d_fwd_bn(d0, x, w, scale, shift, nullptr, y, act, ws, ws_bytes, stream);
  // a channel slice of a wider NHWC tensor: the implicit-GEMM route with 16-B row chunks only
  const int vec = 16 / esize(d0->dtype);
  if (ldy < d0->k || ldy % vec || d0->k % vec || ((uintptr_t)y & 15) || ldy > (1L << 30)) return RTSDS_ERR_UNSUPPORTED;
  if (pooled_1x1(d0) || tapconv_ok(d0) || hconv_ok(d0) || imgconv_ok(d0)) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_conv2d_fwd_workspace(d0)) return RTSDS_ERR_WORKSPACE;
  const bool x_padded = (act & RTSDS_INPUT_PADDED) != 0;
  if (x_padded && input_pitch(d0) == d0->c) return RTSDS_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  rtsds_conv_desc d;
  fwd_prepare(d0, x, w, ws, d, st, x_padded);
  ConvArgs p = make_args(&d);
  p.a = x; p.b = w; p.bias = shift; p.scale = scale; p.res = nullptr; p.out = y;
  p.act = act & 0xff;
  p.ldo = (int)ldy;
  p.M = d.n * d.ho * d.wo;
  p.N = d.k;
  p.K = d.kh * d.kw * d.c;
  if (d.dtype == RTSDS_BF16) dispatch_align<bf16, MODE_FWD>(p, d.c, st);
  else dispatch_align<float, MODE_FWD>(p, d.c, st);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

extern "C" int rtsds_conv2d_fwd_bn_maxpool(const rtsds_conv_desc* d0, const void* x, const void* w, const float* scale,
                                           const float* shift, void* y, int act, int hp, int wp, int pool_pad, void* ws,
                                           size_t ws_bytes, void* stream) {
  if (!scale || !shift || (act & RTSDS_ACCUMULATE)) return RTSDS_ERR_UNSUPPORTED;
  int e = check_desc(d0);
  if (e) return e;
  if (!imgconv_pool_ok(d0, hp, wp) || pool_pad < 0 || pool_pad > 1) return RTSDS_ERR_UNSUPPORTED;
  // the windows must cover the pooled grid: hp <= ceil((ho + 2 pad - 3) / 2) + 1
  if (hp > (d0->ho + 2 * pool_pad - 3 + 1) / 2 + 1 || wp > (d0->wo + 2 * pool_pad - 3 + 1) / 2 + 1) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_conv2d_fwd_workspace(d0)) return RTSDS_ERR_WORKSPACE;
  const bool x_padded = (act & RTSDS_INPUT_PADDED) != 0;
  hipStream_t st = (hipStream_t)stream;
  if (!x_padded) sp_pad4(d0, x, ws, st);
  imgconv_pool_fwd(d0, x_padded ? x : ws, w, shift, scale, y, act & 0xff, hp, wp, pool_pad, st);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// DGRAD split-K for small-M deep stride-1 convs (ResNet layer4: M = 4096 pixels, K = 4608):
// the occupancy rule would fall back to 64x64 tiles (AI 32 flop/B of staged operands); 128x128
// tiles x S K-splits keep the MFMA-dense tile and still put >= 512 workgroups on the chip.
// fp32 slabs [S][M][N] summed in split order (+ accumulate) into the bf16 dx.
struct DgradSplit {
  int splits, tps;
  size_t slab_bytes;
};
static DgradSplit dgrad_split(const rtsds_conv_desc* d, int kp) {
  DgradSplit s = {1, 1 << 30, 0};
  if (d->dtype != RTSDS_BF16 || d->sh != 1 || d->sw != 1 || kp % 64 != 0 || d->c % 8 != 0) return s;
  const long M = (long)d->n * d->h * d->w;
  const int N = d->c, K = d->kh * d->kw * kp;
  int bm, bn;
  pick_tile(M, N, true, bm, bn);
  if (!(bm == 64 && bn == 64)) return s;  // the wide tiles already fill the chip
  const long tiles = ((M + 127) / 128) * ((N + 127) / 128);
  const int nk = (K + 63) / 64;
  int want = (int)std::min<long>(8, (512 + tiles - 1) / tiles);
  want = std::min(want, nk / 16);  // >= 16 K-tiles per split
  if (want < 2) return s;
  s.tps = (nk + want - 1) / want;
  s.splits = (nk + s.tps - 1) / s.tps;
  s.slab_bytes = al256((size_t)s.splits * M * N * 4);
  return s;
}
// dx (+)= sum_s slab[s] -> bf16; 8 channels per thread
__global__ void __launch_bounds__(256) dgrad_split_reduce_kernel(const float* __restrict__ slab, bf16* __restrict__ dx, long nv8,
                                                                long stride, int splits, int accum) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < nv8; i += (long)gridDim.x * 256) {
    float s[8];
    {
      const f32x4 a = *(const f32x4*)(slab + i * 8), b = *(const f32x4*)(slab + i * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { s[e] = a[e]; s[4 + e] = b[e]; }
    }
    for (int q = 1; q < splits; ++q) {
      const f32x4 a = *(const f32x4*)(slab + q * stride + i * 8), b = *(const f32x4*)(slab + q * stride + i * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { s[e] += a[e]; s[4 + e] += b[e]; }
    }
    bf16x8* o = (bf16x8*)(dx + i * 8);
    bf16x8 r;
    if (accum) {
      const bf16x8 old = *o;
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = (bf16)(s[e] + (float)old[e]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = (bf16)s[e];
    }
    *o = r;
  }
}

// The DGRAD route of a descriptor: the halo direct conv for narrow-output 3x3 convs, else
// the implicit GEMM (with split-K slabs when dgrad_split() asks).  One predicate for both the
// workspace query and the launch.
static bool dgrad_hconv(const rtsds_conv_desc* d, int kp) { return kp % 32 == 0 && hconv_dgrad_ok(d); }

// DGRAD workspace: repacked (and Cout-padded) weights + a Cout-padded copy of dy if needed.
extern "C" size_t rtsds_conv2d_dgrad_workspace(const rtsds_conv_desc* d) {
  if (pooled_1x1(d) || pw_ok(d)) return 0;
  const int kp = pad_c(d->k, d->dtype);
  const size_t es = esize(d->dtype);
  size_t b = al256((size_t)kp * d->kh * d->kw * d->c * es);
  if (kp != d->k) b += al256((size_t)d->n * d->ho * d->wo * kp * es);
  if (dgrad_hconv(d, kp) || tapconv_ok(d)) return b;  // the direct convs need no split-K slabs
  return b + dgrad_split(d, kp).slab_bytes;
}

static void repack_launch(int dtype, const void* w, void* wt, int co_n, int co_p, int kh, int kw, int ci_n, int tkh, int tkw,
                          int r0h, int r0w, int rstep, hipStream_t st) {
  const long wn = (long)co_p * tkh * tkw * ci_n;
  if (wn <= 0) return;
  const int blocks = (int)std::min<long>(4096, (wn + 255) / 256);
  if (dtype == RTSDS_BF16)
    hipLaunchKernelGGL(repack_wt_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (const bf16*)w, (bf16*)wt, co_n, co_p, kh, kw, ci_n,
                       tkh, tkw, r0h, r0w, rstep);
  else
    hipLaunchKernelGGL(repack_wt_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)w, (float*)wt, co_n, co_p, kh, kw, ci_n,
                       tkh, tkw, r0h, r0w, rstep);
}

// Taps of one dgrad stride phase along an axis: input index i = t*2 + off receives from
// kernel taps r with (i + pad - r*dil) even.
static void phase_taps(int a, int pad, int dil, int ksz, int size, int& off, int& cnt_pix, int& r0, int& rstep, int& tk) {
  off = ((a - pad) % 2 + 2) % 2;
  cnt_pix = size > off ? (size - off + 1) / 2 : 0;
  if (dil % 2) { r0 = a; rstep = 2; tk = ksz > a ? (ksz - a + 1) / 2 : 0; }
  else { r0 = 0; rstep = 1; tk = a == 0 ? ksz : 0; }
}

// ---- pre-packed DGRAD weights.  Every GEMM / halo DGRAD route reads the weights transposed
// ([ci][tap][co_p], taps flipped for the halo conv, split per parity phase at stride 2).  The
// optimizer re-packs every conv weight it owns right after its update, all of them in one
// launch (rtsds_conv2d_dgrad_pack_many), and the backward passes the packed copy with
// RTSDS_WEIGHT_PACKED instead of repacking per call (one tiny launch per conv and backward).
struct PackSeg {
  const void* w;
  void* wt;  // segment base (phase offset applied)
  int co_n, co_p, kh, kw, ci_n, tkh, tkw, r0h, r0w, rstep, blk0;
};
static const int kPackSegs = 16;
struct PackBatch {
  PackSeg s[kPackSegs];
  int nseg;
};
// One workgroup per (tap, 64 Cout x 64 Cin tile): rows of Cin read coalesced, transposed
// through LDS, rows of Cout written coalesced ([ci][tap][co_p], zero for co >= co_n).
static int pack_tiles(const PackSeg& q) { return q.tkh * q.tkw * rt_cdiv(q.co_p, 64) * rt_cdiv(q.ci_n, 64); }
template <typename T>
__global__ void __launch_bounds__(256) dgrad_pack_kernel(const PackBatch b) {
  __shared__ float tile[64][65];
  int si = 0;
  for (int i = 1; i < b.nseg; ++i)
    if (b.s[i].blk0 <= (int)blockIdx.x) si = i;
  const PackSeg& g = b.s[si];
  const int nco = (g.co_p + 63) / 64, nci = (g.ci_n + 63) / 64, taps = g.tkh * g.tkw;
  int t = (int)blockIdx.x - g.blk0;
  const int ct = t % nci;
  t /= nci;
  const int ot = t % nco, tap = t / nco;
  const int r = g.r0h + (tap / g.tkw) * g.rstep, sc = g.r0w + (tap % g.tkw) * g.rstep;
  const T* __restrict__ w = (const T*)g.w;
  T* __restrict__ wt = (T*)g.wt;
  const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
  // clamped, unconditional loads, all 16 in flight (a guarded load per element serialised them:
  // one memory round trip each), then the zero fill of the padding selected
  T v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int co = min(ot * 64 + ly + 4 * k, g.co_n - 1), ci = min(ct * 64 + lx, g.ci_n - 1);
    v[k] = w[((co * g.kh + r) * g.kw + sc) * g.ci_n + ci];
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int co = ot * 64 + ly + 4 * k, ci = ct * 64 + lx;
    tile[ly + 4 * k][lx] = (co < g.co_n && ci < g.ci_n) ? to_f(v[k]) : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int ci = ct * 64 + ly + 4 * k, co = ot * 64 + lx;
    if (ci < g.ci_n && co < g.co_p) wt[((long)ci * taps + tap) * g.co_p + co] = from_f<T>(tile[lx][ly + 4 * k]);
  }
}
static bool dgrad_hconv(const rtsds_conv_desc* d, int kp);
// Segments of d's DGRAD weight repack (the layout dgrad_impl reads); 0 = no repack on its route.
static int dgrad_pack_plan(const rtsds_conv_desc* d, PackSeg* seg, int& kp) {
  kp = pad_c(d->k, d->dtype);
  if (pooled_1x1(d) || pw_ok(d)) return 0;
  auto one = [&](int tkh, int tkw, int r0h, int r0w, int rstep, long boff) {
    PackSeg q = {};
    q.co_n = d->k; q.co_p = kp; q.kh = d->kh; q.kw = d->kw; q.ci_n = d->c;
    q.tkh = tkh; q.tkw = tkw; q.r0h = r0h; q.r0w = r0w; q.rstep = rstep;
    q.wt = (void*)(intptr_t)boff;  // element offset until the caller adds the base
    return q;
  };
  if (dgrad_hconv(d, kp) || tapconv_ok(d)) {  // flipped taps: the direct convs run over dY
    seg[0] = one(d->kh, d->kw, d->kh - 1, d->kw - 1, -1, 0);
    return 1;
  }
  if (d->sh == 2 && d->sw == 2) {
    int n = 0;
    long boff = 0;
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b) {
        int offh, hp, r0h, rsh, tkh, offw, wp, r0w, rsw, tkw;
        phase_taps(a, d->ph, d->dh, d->kh, d->h, offh, hp, r0h, rsh, tkh);
        phase_taps(b, d->pw, d->dw, d->kw, d->w, offw, wp, r0w, rsw, tkw);
        if (hp == 0 || wp == 0) continue;
        if (tkh * tkw > 0) seg[n++] = one(tkh, tkw, r0h, r0w, rsh, boff);
        boff += (long)tkh * tkw * kp * d->c;
      }
    return n;
  }
  if (d->sh != 1 || d->sw != 1) return 0;
  seg[0] = one(d->kh, d->kw, 0, 0, 1, 0);
  return 1;
}
extern "C" size_t rtsds_conv2d_dgrad_pack_bytes(const rtsds_conv_desc* d) {
  if (check_desc(d)) return 0;
  PackSeg seg[4];
  int kp;
  if (dgrad_pack_plan(d, seg, kp) == 0) return 0;
  return al256((size_t)kp * d->kh * d->kw * d->c * esize(d->dtype));
}
extern "C" int rtsds_conv2d_dgrad_pack_many(int count, const rtsds_conv_desc* descs, const void* const* w, void* const* wt,
                                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  PackBatch b = {};
  int blocks = 0, dtype = -1;
  auto flush = [&]() {
    if (b.nseg == 0) return;
    if (dtype == RTSDS_BF16) hipLaunchKernelGGL(dgrad_pack_kernel<bf16>, dim3(blocks), dim3(256), 0, st, b);
    else hipLaunchKernelGGL(dgrad_pack_kernel<float>, dim3(blocks), dim3(256), 0, st, b);
    b.nseg = 0;
    blocks = 0;
  };
  for (int i = 0; i < count; ++i) {
    const rtsds_conv_desc* d = descs + i;
    if (check_desc(d) || !w[i] || !wt[i]) return RTSDS_ERR_SHAPE;
    PackSeg seg[4];
    int kp;
    const int n = dgrad_pack_plan(d, seg, kp);
    if (n == 0) return RTSDS_ERR_UNSUPPORTED;
    if (d->dtype != dtype || b.nseg + n > kPackSegs) flush();
    dtype = d->dtype;
    for (int j = 0; j < n; ++j) {
      PackSeg q = seg[j];
      q.w = w[i];
      q.wt = (char*)wt[i] + (intptr_t)q.wt * esize(d->dtype);
      q.blk0 = blocks;
      blocks += pack_tiles(q);
      b.s[b.nseg++] = q;
    }
  }
  flush();
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// mask: see ConvArgs::mask.  Paths whose epilogue does not apply it (pooled, narrow 1x1, halo,
// split-K) report false and the caller masks dx in place afterwards.
struct BnbArgs {  // see ConvArgs::bnb_part
  float* part;
  const void* x;
  const float *gamma, *beta, *mean, *invstd;
  int act;
};
static int dgrad_impl(const rtsds_conv_desc* d0, const void* dy, const void* w, void* dx, int accumulate, const void* mask,
                      int mask_act, bool& masked, void* ws, size_t ws_bytes, void* stream, const BnbArgs* bnb = nullptr,
                      bool packed = false);
extern "C" int rtsds_conv2d_dgrad(const rtsds_conv_desc* d0, const void* dy, const void* w, void* dx,
                                  int accumulate, void* ws, size_t ws_bytes, void* stream) {
  bool masked = false;
  const bool packed = (accumulate & RTSDS_WEIGHT_PACKED) != 0;
  return dgrad_impl(d0, dy, w, dx, accumulate & ~RTSDS_WEIGHT_PACKED, nullptr, 0, masked, ws, ws_bytes, stream, nullptr,
                    packed);
}
static bool dgrad_hconv(const rtsds_conv_desc* d, int kp);
static DgradSplit dgrad_split(const rtsds_conv_desc* d, int kp);
// M tiles of the data-gradient GEMM when its epilogue can emit the BatchNorm backward
// statistics (bf16, stride 1, plain GEMM path: not the pooled / narrow-1x1 / halo / split-K
// routes, vector epilogue), else 0.  (The stride-2 parity-phase launch could carry them too:
// measured for the spatial path's BatchNorms, the epilogue cost what the statistics pass saved.)
extern "C" int rtsds_conv2d_dgrad_bnstats_tiles(const rtsds_conv_desc* d) {
  if (check_desc(d) || d->dtype != RTSDS_BF16 || d->sh != 1 || d->sw != 1 || d->c % 8 != 0) return 0;
  if (pooled_1x1(d) || pw_ok(d)) return 0;
  if (tapconv_ok(d)) return tapconv_rows(d, 1);
  const int kp = pad_c(d->k, d->dtype);
  if (dgrad_hconv(d, kp) || dgrad_split(d, kp).splits > 1) return 0;
  int bm, bn;
  const long M = (long)d->n * d->h * d->w;
  pick_tile(M, d->c, true, bm, bn, false, (long)d->kh * d->kw * kp, true);  // dispatch_align's choice
  if (256 % (bn / 8) != 0) return 0;
  return (int)((M + bm - 1) / bm);
}
extern "C" int rtsds_conv2d_dgrad_bnstats(const rtsds_conv_desc* d0, const void* dy, const void* w, void* dx, const void* bn_x,
                                          const float* gamma, const float* beta, const float* save_mean,
                                          const float* save_invstd, int act, float* part, void* ws, size_t ws_bytes,
                                          void* stream) {
  const bool packed = (act & RTSDS_WEIGHT_PACKED) != 0;
  act &= ~RTSDS_WEIGHT_PACKED;
  if (rtsds_conv2d_dgrad_bnstats_tiles(d0) == 0) return RTSDS_ERR_UNSUPPORTED;
  if (!bn_x || !save_mean || !save_invstd || !part || (act != RTSDS_ACT_NONE && act != RTSDS_ACT_RELU && act != RTSDS_ACT_LEAKY))
    return RTSDS_ERR_UNSUPPORTED;
  const BnbArgs b = {part, bn_x, gamma, beta, save_mean, save_invstd, act};
  bool masked = false;
  return dgrad_impl(d0, dy, w, dx, 0, nullptr, 0, masked, ws, ws_bytes, stream, &b, packed);
}
extern "C" int rtsds_act_bwd(const void* dy, const void* y, void* dx, long n, int act, float alpha, int dtype, void* stream);
extern "C" int rtsds_conv2d_dgrad_act(const rtsds_conv_desc* d0, const void* dy, const void* w, void* dx, const void* x_act,
                                      int act, void* ws, size_t ws_bytes, void* stream) {
  const bool packed = (act & RTSDS_WEIGHT_PACKED) != 0;
  act &= ~RTSDS_WEIGHT_PACKED;
  if (!x_act || (act != RTSDS_ACT_RELU && act != RTSDS_ACT_LEAKY)) return RTSDS_ERR_UNSUPPORTED;
  bool masked = false;
  const int e = dgrad_impl(d0, dy, w, dx, 0, x_act, act, masked, ws, ws_bytes, stream, nullptr, packed);
  if (e || masked) return e;
  return rtsds_act_bwd(dx, x_act, dx, (long)d0->n * d0->h * d0->w * d0->c, act, 1.f, d0->dtype, stream);
}
static int dgrad_impl(const rtsds_conv_desc* d0, const void* dy, const void* w, void* dx, int accumulate, const void* mask,
                      int mask_act, bool& masked, void* ws, size_t ws_bytes, void* stream, const BnbArgs* bnb, bool packed) {
  masked = false;
  int e = check_desc(d0);
  if (e) return e;
  if (d0->sh > 2 || d0->sw > 2) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_conv2d_dgrad_workspace(d0)) return RTSDS_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  if (pooled_1x1(d0)) {
    if (d0->dtype == RTSDS_BF16) pooled_dgrad_launch<bf16>(d0, dy, w, dx, accumulate ? 1 : 0, st);
    else pooled_dgrad_launch<float>(d0, dy, w, dx, accumulate ? 1 : 0, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (pw_ok(d0)) {  // narrow-output 1x1: direct FMA over dY rows (pw.hip)
    pw_dgrad(d0, dy, w, dx, accumulate ? 1 : 0, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  rtsds_conv_desc d = *d0;
  const int kp = pad_c(d.k, d.dtype);
  const size_t es = esize(d.dtype);
  // packed: w already is the transposed copy (rtsds_conv2d_dgrad_pack_many); else repack it here
  void* wt = packed ? const_cast<void*>(w) : ws;
  if (kp != d.k) {
    void* dyp = (char*)ws + al256((size_t)kp * d.kh * d.kw * d.c * es);
    pad_any(d.dtype, dy, dyp, (long)d.n * d.ho * d.wo, d.k, kp, st);
    dy = dyp;
  }
  const int k_real = d.k;
  d.k = kp;
  if (tapconv_ok(d0)) {
    // 3x3 64 -> 64 stride 1: the register-resident-weight direct conv over dY with the flipped,
    // transposed weights; mask / accumulate / BatchNorm backward statistics in its epilogue
    if (!packed) repack_launch(d.dtype, w, wt, k_real, kp, d.kh, d.kw, d.c, d.kh, d.kw, d.kh - 1, d.kw - 1, -1, st);
    tapconv_dgrad(d0, dy, wt, dx, accumulate, mask, mask_act, bnb ? bnb->part : nullptr, bnb ? bnb->x : nullptr,
                  bnb ? bnb->gamma : nullptr, bnb ? bnb->beta : nullptr, bnb ? bnb->mean : nullptr,
                  bnb ? bnb->invstd : nullptr, bnb ? bnb->act : 0, st);
    masked = mask != nullptr;
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (dgrad_hconv(d0, kp)) {
    // narrow-output 3x3 conv: halo direct conv over dY with the flipped, transposed weights
    if (!packed) repack_launch(d.dtype, w, wt, k_real, kp, d.kh, d.kw, d.c, d.kh, d.kw, d.kh - 1, d.kw - 1, -1, st);
    hconv_dgrad(d0, dy, kp, wt, dx, accumulate, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (d.sh == 2 && d.sw == 2) {
    // stride-2: the four parity phases, each a dense GEMM over only the taps that reach it,
    // repacked by one launch and computed by one launch (blockIdx.z = phase)
    ConvArgs p = make_args(&d);
    p.a = dy; p.b = wt; p.bias = nullptr; p.out = dx; p.act = 0;
    p.accum = accumulate ? 1 : 0;
    p.mask = mask;
    p.mask_act = mask_act;
    masked = mask != nullptr;
    p.psh = 2;
    p.N = d.c;
    RepackPhases rp = {};
    int nph = 0, rstep = 1, max_m = 0, max_w = 0;
    long boff = 0;
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b) {
        int offh, hp, r0h, rsh, tkh, offw, wp, r0w, rsw, tkw;
        phase_taps(a, d.ph, d.dh, d.kh, d.h, offh, hp, r0h, rsh, tkh);
        phase_taps(b, d.pw, d.dw, d.kw, d.w, offw, wp, r0w, rsw, tkw);
        if (hp == 0 || wp == 0) continue;
        rstep = rsh;
        ConvArgs::Phase& q = p.phs[nph];
        q.hp = hp; q.wp = wp; q.offh = offh; q.offw = offw; q.r0h = r0h; q.r0w = r0w;
        q.tkw = tkw > 0 ? tkw : 1;
        q.f_tkw = fastdiv_make(q.tkw);
        q.f_hw = fastdiv_make(hp * wp);
        q.f_w = fastdiv_make(wp);
        q.M = d.n * hp * wp;
        q.K = tkh * tkw * kp;
        q.boff = boff;
        rp.tkh[nph] = tkh; rp.tkw[nph] = tkw; rp.r0h[nph] = r0h; rp.r0w[nph] = r0w; rp.boff[nph] = boff;
        boff += (long)q.K * d.c;
        max_m = std::max(max_m, q.M);
        max_w = std::max(max_w, q.K * d.c);
        ++nph;
      }
    if (nph == 0) return RTSDS_OK;
    if (max_w > 0 && !packed) {
      const dim3 g(std::min(4096, (max_w + 255) / 256), nph);
      if (d.dtype == RTSDS_BF16)
        hipLaunchKernelGGL(repack_phases_kernel<bf16>, g, dim3(256), 0, st, (const bf16*)w, (bf16*)wt, k_real, kp, d.kh, d.kw,
                           d.c, rstep, rp);
      else
        hipLaunchKernelGGL(repack_phases_kernel<float>, g, dim3(256), 0, st, (const float*)w, (float*)wt, k_real, kp, d.kh, d.kw,
                           d.c, rstep, rp);
    }
    // shared fields: the first phase's (tile choice and alignment class depend only on M, N, kp)
    p.nph = nph;
    p.hp = p.phs[0].hp; p.wp = p.phs[0].wp; p.offh = p.phs[0].offh; p.offw = p.phs[0].offw;
    p.r0h = p.phs[0].r0h; p.r0w = p.phs[0].r0w; p.rstep = rstep; p.tkw = p.phs[0].tkw;
    p.f_tkw = p.phs[0].f_tkw; p.f_hw = p.phs[0].f_hw; p.f_w = p.phs[0].f_w;
    p.M = max_m;
    p.K = p.phs[0].K;
    if (d.dtype == RTSDS_BF16) dispatch_align<bf16, MODE_DGRAD>(p, kp, st);
    else dispatch_align<float, MODE_DGRAD>(p, kp, st);
  } else {
    if (!packed) repack_launch(d.dtype, w, wt, k_real, kp, d.kh, d.kw, d.c, d.kh, d.kw, 0, 0, 1, st);
    ConvArgs p = make_args(&d);
    p.a = dy; p.b = wt; p.bias = nullptr; p.out = dx; p.act = 0;
    p.accum = accumulate ? 1 : 0;
    p.mask = mask;
    p.mask_act = mask_act;
    if (bnb) {  // (rtsds_conv2d_dgrad_bnstats_tiles checked this route)
      p.bnb_part = bnb->part; p.bnb_x = bnb->x; p.bnb_gamma = bnb->gamma; p.bnb_beta = bnb->beta;
      p.bnb_mean = bnb->mean; p.bnb_invstd = bnb->invstd; p.bnb_act = bnb->act;
    }
    p.M = d.n * d.h * d.w;
    p.N = d.c;
    p.K = d.kh * d.kw * kp;
    const DgradSplit sk = dgrad_split(d0, kp);
    if (sk.splits > 1) {
      // slab region: after the repacked weights and the (optional) Cout-padded dy
      size_t off = al256((size_t)kp * d.kh * d.kw * d.c * es);
      if (kp != k_real) off += al256((size_t)d.n * d.ho * d.wo * kp * es);
      p.slab = (float*)((char*)ws + off);
      p.split_stride = (long)p.M * p.N;
      p.tiles_per_split = sk.tps;
      p.accum = 0;
      p.mask = nullptr;  // the split reduce writes dx: masked afterwards by the caller
      launch_al<bf16, MODE_DGRAD, 128, 128, 64, 2, 2>(p, kp, st, sk.splits);
      const long nv8 = (long)p.M * p.N / 8;
      hipLaunchKernelGGL(dgrad_split_reduce_kernel, dim3((int)std::min<long>(8192, (nv8 + 255) / 256)), dim3(256), 0, st,
                         (const float*)p.slab, (bf16*)dx, nv8, p.split_stride, sk.splits, accumulate ? 1 : 0);
    } else {
      masked = mask != nullptr;
      if (d.dtype == RTSDS_BF16) dispatch_align<bf16, MODE_DGRAD>(p, kp, st);
      else dispatch_align<float, MODE_DGRAD>(p, kp, st);
    }
  }
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// WGRAD split-K: enough (M/BM)*(N/BN)*splits workgroups to fill 256 CUs ~2x, each split at
// least 8 K-tiles; fp32 partial slabs summed (and channel-unpadded) by split_reduce_kernel --
// deterministic, no atomics.
// ---- narrow pointwise weight + bias gradient (1x1, stride 1, Cin and Cout <= 32: BiSeNet's final
// 19 -> 19 conv, build_bisenet.py:117).  As a GEMM it needed dY and x padded to 32 channels, a
// split-K launch, its reduce and the bias column sums' two launches -- six launches for 0.05 GFLOP.
// Here: pass 1, one workgroup per run of kPwnRows pixels stages 64-pixel tiles of dY and x in LDS
// and accumulates every (co, ci) product and the dY column sums -> part[block][k*c dW | k db];
// pass 2 (one wave per output) sums the blocks in a fixed order.
static constexpr int kPwnRows = 128;
static bool pwn_wgrad_ok(const rtsds_conv_desc* d) {
  // (k <= 28: 9 threads per output row in a 256-thread workgroup)
  return d->kh == 1 && d->kw == 1 && d->sh == 1 && d->sw == 1 && d->ph == 0 && d->pw == 0 && d->k <= 28 && d->c <= 32;
}
static int pwn_blocks(const rtsds_conv_desc* d) {
  return (int)std::min<long>(4096, ((long)d->n * d->h * d->w + kPwnRows - 1) / kPwnRows);
}
template <typename T>
__global__ void __launch_bounds__(256) pwn_wgrad_part_kernel(const T* __restrict__ dy, const T* __restrict__ x, float* __restrict__ part,
                                                             long P, int k, int c, int ldx, int per) {
  // thread t: output row co = t / 9, column group g = t % 9 -- dW[co][4g .. 4g + 3] for g < 8, the
  // bias sum (x's ones column 32) for g = 8; one dY read and one 16-B x read per pixel, 4 FMAs
  __shared__ float sdy[64][33];
  __shared__ __attribute__((aligned(16))) float sx[64][36];
  const long p0 = (long)blockIdx.x * per, p1 = min(P, p0 + per);
  const int co = threadIdx.x / 9, g = threadIdx.x - co * 9;
  const bool active = co < k && (g == 8 || 4 * g < c);
  const int coc = min(co, 31);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long pb = p0; pb < p1; pb += 64) {
    const int np = (int)min(64L, p1 - pb);
    __syncthreads();
    // 64 x 32 elements of each tensor, 8 per thread: clamped unconditional loads, then the
    // zero fill past the pixels / channels selected
    float vd[8], vx[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = threadIdx.x + 256 * u, r = e >> 5, ch = e & 31;
      const long pr = pb + min(r, np - 1);
      vd[u] = to_f(dy[pr * k + min(ch, k - 1)]);
      vx[u] = to_f(x[pr * ldx + min(ch, c - 1)]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = threadIdx.x + 256 * u, r = e >> 5, ch = e & 31;
      sdy[r][ch] = (r < np && ch < k) ? vd[u] : 0.f;
      sx[r][ch] = (r < np && ch < c) ? vx[u] : 0.f;
    }
    if (threadIdx.x < 64) *(f32x4*)&sx[threadIdx.x][32] = f32x4{threadIdx.x < np ? 1.f : 0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    if (active) {
#pragma unroll 8
      for (int r = 0; r < 64; ++r) {
        const float d = sdy[r][coc];
        const f32x4 v = *(const f32x4*)&sx[r][4 * g];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fmaf(d, v[j], acc[j]);
      }
    }
  }
  if (!active) return;
  const int no = k * c + k;
  float* out = part + (long)blockIdx.x * no;
  if (g == 8) {
    out[k * c + co] = acc[0];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * g + j < c) out[co * c + 4 * g + j] = acc[j];
  }
}
// one wave per output: lane l sums the partials of blocks l, l + 64, ... (8 in flight, in
// order), then the wave's fixed shuffle tree
__global__ void __launch_bounds__(64) pwn_wgrad_final_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                             float* __restrict__ dbias, int nb, int k, int c, int accum) {
  const int no = k * c + k, o = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
  for (int b0 = lane; b0 < nb; b0 += 64 * 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = part[(long)min(b0 + 64 * u, nb - 1) * no + o];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b0 + 64 * u < nb) s += t[u];
  }
  s = wave_sum(s);
  if (lane != 0) return;
  if (o < k * c) dw[o] = accum ? dw[o] + s : s;
  else if (dbias) dbias[o - k * c] = accum ? dbias[o - k * c] + s : s;
}

struct WgradPlan {
  int kp, cp, bm, bn, splits, tps;
  size_t slab_bytes, dyp_bytes, xp_bytes, colsum_bytes;
};
// the halo-direct weight gradient of a narrow-output 3x3 conv (hconv.hip nwgrad): dY padded to 32
// channels, one slab per run of tiles, the same split reduce
static bool nw_path(const rtsds_conv_desc* d) { return pad_c(d->k, d->dtype) == 32 && nwgrad_ok(d); }
static WgradPlan wgrad_plan(const rtsds_conv_desc* d) {
  WgradPlan w;
  const bool b16 = d->dtype == RTSDS_BF16;
  w.kp = pad_c(d->k, d->dtype);
  w.cp = pad_c(d->c, d->dtype);
  const int M = w.kp, N = d->kh * d->kw * w.cp;
  const long R = (long)d->n * d->ho * d->wo;
  if (nw_path(d)) {
    w.bm = w.bn = 0;
    w.splits = nwgrad_splits(d);
    w.tps = 0;
    w.slab_bytes = al256((size_t)w.splits * M * N * 4);
    w.dyp_bytes = w.kp != d->k ? al256((size_t)R * w.kp * 2) : 0;
    w.xp_bytes = 0;
    w.colsum_bytes = al256((size_t)kColsumRB * d->k * 4);
    return w;
  }
  const int BK = b16 ? 64 : 16;
  // Cout <= 32 (the 19-class convs, padded to 32): a 32-row tile (register-staged) instead of
  // half a 64-row one
  w.bm = b16 ? (M <= 32 && N > 64 ? 32 : (M <= 64 ? 64 : 128)) : 64;
  w.bn = b16 ? (N <= 64 ? 64 : 128) : 64;
  const long tiles = (long)rt_cdiv(M, w.bm) * rt_cdiv(N, w.bn);
  const long nk = (R + BK - 1) / BK;
  // narrow outputs (<= 32 rows of Cout: the 19-class convs) stream far more pixels per tile:
  // ~6 groups per CU hide more of the gather latency (DeepLab ASPP 304 -> 226 us, FFM 147 ->
  // 125).  Wide grids that fill only 432 of a round's 512 slots (DeepLab layer4 3x3, 144
  // tiles x 3) take ~2 full rounds of splits instead when every split keeps >= 64 K-tiles
  // (373 -> 325 us); short reductions (BiSeNet layer4, 64 K-tiles) would pay it in slab traffic.
static constexpr auto kWgradWant = 512;
  long want = std::max<long>(1, (w.bm <= 64 && M <= 32 ? 1536 : kWgradWant) / tiles);
  if (!(w.bm <= 64 && M <= 32) && tiles >= 64 && tiles * want < 480) {
    const long w2 = 1024 / tiles;
    if (tiles * w2 >= 922 && nk / w2 >= 64) want = w2;
  }
  want = std::min<long>(want, std::max<long>(1, nk / 8));
  want = std::min<long>(want, 256);
  w.tps = (int)((nk + want - 1) / want);
  w.splits = (int)((nk + w.tps - 1) / w.tps);
  const size_t es = esize(d->dtype);
  w.slab_bytes = al256((size_t)w.splits * M * N * 4);
  w.dyp_bytes = w.kp != d->k ? al256((size_t)R * w.kp * es) : 0;
  w.xp_bytes = w.cp != d->c ? al256((size_t)d->n * d->h * d->w * w.cp * es) : 0;
  w.colsum_bytes = al256((size_t)kColsumRB * d->k * 4);
  return w;
}

extern "C" size_t rtsds_conv2d_wgrad_workspace(const rtsds_conv_desc* d) {
  if (pooled_1x1(d)) return 0;
  if (sp_path(d)) {
    const rtsds_conv_desc v = sp_desc(d);
    const WgradPlan w = wgrad_plan(&v);
    return w.slab_bytes + w.colsum_bytes + sp_x4_bytes(d) + al256((size_t)v.k * v.kh * v.kw * 8 * 4);
  }
  const WgradPlan w = wgrad_plan(d);
  const size_t pwn = pwn_wgrad_ok(d) ? al256((size_t)pwn_blocks(d) * (d->k * d->c + d->k) * 4) : 0;
  return std::max(w.slab_bytes + w.dyp_bytes + w.xp_bytes + w.colsum_bytes, pwn);
}


static int wgrad_impl(const rtsds_conv_desc* d0, const void* x, const void* dy, float* dw, float* dbias, int accumulate,
                      void* ws, size_t ws_bytes, rtsds_split_reduce_desc* pending, void* stream);
extern "C" int rtsds_conv2d_wgrad(const rtsds_conv_desc* d0, const void* x, const void* dy, float* dw,
                                  float* dbias, int accumulate, void* ws, size_t ws_bytes, void* stream) {
  return wgrad_impl(d0, x, dy, dw, dbias, accumulate, ws, ws_bytes, nullptr, stream);
}
extern "C" int rtsds_conv2d_wgrad_deferred(const rtsds_conv_desc* d0, const void* x, const void* dy, float* dw,
                                           float* dbias, int accumulate, void* ws, size_t ws_bytes,
                                           rtsds_split_reduce_desc* pending, void* stream) {
  if (!pending) return RTSDS_ERR_SHAPE;
  pending->nv = 0;
  return wgrad_impl(d0, x, dy, dw, dbias, accumulate, ws, ws_bytes, pending, stream);
}

// Batched split-K reductions (rtsds_split_reduce_many): block b belongs to the descriptor whose
// block range contains it; within it, split_reduce_kernel<4>'s arithmetic (4 split groups per
// 64 outputs, summed in split order) -- bit-identical to the per-wgrad launch.
static const int kReduceBatch = 16;
struct ReduceBatch {
  rtsds_split_reduce_desc d[kReduceBatch];
  int blk0[kReduceBatch];
  int n;
};
__global__ void __launch_bounds__(256) split_reduce_many_kernel(const ReduceBatch b) {
  __shared__ float red[4][64][4];
  int si = 0;
  for (int i = 1; i < b.n; ++i)
    if (b.blk0[i] <= (int)blockIdx.x) si = i;
  const rtsds_split_reduce_desc& q = b.d[si];
  const int lane = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int i = ((int)blockIdx.x - b.blk0[si]) * 64 + lane;
  const bool ok = i < q.nv;
  const int rt = (ok ? i : 0) / q.cv;  // co * taps + tap
  const long src = (long)rt * q.cp + (long)((ok ? i : 0) - rt * q.cv) * 4;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int g = sg; ok && g < q.splits; g += 32) {
    float t[8][4];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const f32x4 v = *(const f32x4*)(q.slab + (long)min(g + 4 * u, q.splits - 1) * q.slab_stride + src);
#pragma unroll
      for (int e = 0; e < 4; ++e) t[u][e] = v[e];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (g + 4 * u < q.splits)
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += t[u][e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[sg][lane][e] = s[e];
  __syncthreads();
  if (sg == 0 && ok) {
    float* o = q.dw + (long)i * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float t = (red[0][lane][e] + red[1][lane][e]) + (red[2][lane][e] + red[3][lane][e]);
      o[e] = q.accumulate ? o[e] + t : t;
    }
  }
}
extern "C" int rtsds_split_reduce_many(int n, const rtsds_split_reduce_desc* descs, void* stream) {
  if (n < 0 || (n && !descs)) return RTSDS_ERR_SHAPE;
  for (int i0 = 0; i0 < n; i0 += kReduceBatch) {
    ReduceBatch b;
    b.n = 0;
    int blocks = 0;
    for (int i = i0; i < n && b.n < kReduceBatch; ++i) {
      if (descs[i].nv <= 0) continue;
      if (descs[i].cv <= 0 || descs[i].splits <= 0 || !descs[i].slab || !descs[i].dw) return RTSDS_ERR_SHAPE;
      b.d[b.n] = descs[i];
      b.blk0[b.n] = blocks;
      blocks += (descs[i].nv + 63) / 64;
      ++b.n;
    }
    if (b.n) hipLaunchKernelGGL(split_reduce_many_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, b);
  }
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

static int wgrad_impl(const rtsds_conv_desc* d0, const void* x, const void* dy, float* dw, float* dbias, int accumulate,
                      void* ws, size_t ws_bytes, rtsds_split_reduce_desc* pending, void* stream) {
  int e = check_desc(d0);
  if (e) return e;
  const bool x_padded = (accumulate & RTSDS_INPUT_PADDED) != 0;
  accumulate &= ~RTSDS_INPUT_PADDED;
  if (x_padded && (pooled_1x1(d0) || (!sp_path(d0) && pad_c(d0->c, d0->dtype) == d0->c))) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_conv2d_wgrad_workspace(d0)) return RTSDS_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  if (pooled_1x1(d0)) {
    if (d0->dtype == RTSDS_BF16) pooled_wgrad_launch<bf16>(d0, x, dy, dw, dbias, accumulate ? 1 : 0, st);
    else pooled_wgrad_launch<float>(d0, x, dy, dw, dbias, accumulate ? 1 : 0, st);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  if (pwn_wgrad_ok(d0)) {
    const long P = (long)d0->n * d0->h * d0->w;
    const int nb = pwn_blocks(d0), per = (int)((P + nb - 1) / nb), no = d0->k * d0->c + d0->k;
    const int ldx = x_padded ? pad_c(d0->c, d0->dtype) : d0->c;
    float* part = (float*)ws;
    if (d0->dtype == RTSDS_BF16)
      hipLaunchKernelGGL(pwn_wgrad_part_kernel<bf16>, dim3(nb), dim3(256), 0, st, (const bf16*)dy, (const bf16*)x, part, P, d0->k,
                         d0->c, ldx, per);
    else
      hipLaunchKernelGGL(pwn_wgrad_part_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)dy, (const float*)x, part, P,
                         d0->k, d0->c, ldx, per);
    hipLaunchKernelGGL(pwn_wgrad_final_kernel, dim3(no), dim3(64), 0, st, (const float*)part, dw, dbias, nb, d0->k, d0->c,
                       accumulate ? 1 : 0);
    return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
  }
  const bool sp = sp_path(d0);
  const rtsds_conv_desc dv = sp ? sp_desc(d0) : *d0;
  const WgradPlan pl = wgrad_plan(&dv);
  char* slab = (char*)ws;
  char* dyp = slab + pl.slab_bytes;
  char* xp = dyp + pl.dyp_bytes;
  float* part = (float*)(xp + pl.xp_bytes);
  const long R = (long)d0->n * d0->ho * d0->wo;
  rtsds_conv_desc d = dv;
  const void* dyk = dy;
  float* dws = nullptr;  // superpixel path: dW' [k][kh][kwp][8] before the unpack
  if (sp) {
    void* x4 = (char*)part + pl.colsum_bytes;
    dws = (float*)((char*)x4 + sp_x4_bytes(d0));
    if (!x_padded) {  // RTSDS_INPUT_PADDED: x already is the 4-channel superpixel image
      sp_pad4(d0, x, x4, st);
      x = x4;
    }
  }
  // bf16 bias gradient of a narrow (k % 8, k <= 256) padded dY: the padded copy and the bias
  // column-sum partials in one pass (pad_colsum_kernel)
  const int crb = (int)std::max<long>(1, std::min<long>(kColsumRB, R / 64));
  const bool fused_colsum = dbias && pl.kp != d.k && d0->dtype == RTSDS_BF16 && d0->k % 8 != 0 && d0->k <= 256;
  if (pl.kp != d.k) {
    if (fused_colsum)
      hipLaunchKernelGGL(pad_colsum_kernel<bf16>, dim3(crb), dim3(256), 0, st, (const bf16*)dy, (bf16*)dyp, part, R, d.k, pl.kp);
    else
      pad_any(d.dtype, dy, dyp, R, d.k, pl.kp, st);
    dyk = dyp;
    d.k = pl.kp;
  }
  if (!sp && pl.cp != d.c) {
    if (!x_padded) {  // RTSDS_INPUT_PADDED: x already has the padded channel pitch
      pad_any(d.dtype, x, xp, (long)d.n * d.h * d.w, d.c, pl.cp, st);
      x = xp;
    }
    d.c = pl.cp;
  }
  ConvArgs p = make_args(&d);
  p.a = dyk; p.b = x; p.bias = nullptr; p.act = 0;
  p.M = d.k;
  p.N = d.kh * d.kw * d.c;
  p.K = (int)R;
  p.tiles_per_split = pl.tps;
  p.split_stride = (long)p.M * p.N;
  p.out = slab;
  if (!sp && nw_path(d0)) {  // (dyk: 32-channel pitch; the slab rows co >= k stay unwritten)
    rtsds_conv_desc dn = d;
    dn.k = d0->k;
    nwgrad(&dn, x, dyk, (float*)slab, st);
  } else if (d.dtype == RTSDS_BF16) wgrad_launch<bf16>(p, pl.bm, pl.bn, pl.splits, st);
  else wgrad_launch<float>(p, pl.bm, pl.bn, pl.splits, st);
  if (sp) {
    const int nv = dv.k * dv.kh * dv.kw * 2;
    hipLaunchKernelGGL(split_reduce_kernel<4>, dim3(std::min(8192, (nv + 63) / 64)), dim3(256), 0, st, (const float*)slab, dws,
                       nv, 2, fastdiv_make(2), 8, p.split_stride, pl.splits, 0);
    const int n = d0->k * d0->kh * d0->kw * 3;
    hipLaunchKernelGGL(sp_unpack_dw_kernel, dim3(rt_cdiv(n, 256)), dim3(256), 0, st, (const float*)dws, dw, d0->k, d0->kh,
                       d0->kw, dv.kw, accumulate);
  } else {
    const int V = d0->c % 4 == 0 ? 4 : 1, cv = d0->c / V;
    const int nv = d0->k * d0->kh * d0->kw * cv;
    const int blocks = std::min(8192, (nv + 63) / 64);
    if (pending && V == 4) {  // the caller reduces it later, batched (rtsds_split_reduce_many)
      pending->slab = (const float*)slab;
      pending->dw = dw;
      pending->slab_stride = p.split_stride;
      pending->nv = nv;
      pending->cv = cv;
      pending->cp = pl.cp;
      pending->splits = pl.splits;
      pending->accumulate = accumulate ? 1 : 0;
    } else if (V == 4)
      hipLaunchKernelGGL(split_reduce_kernel<4>, dim3(blocks), dim3(256), 0, st, (const float*)slab, dw, nv, cv, fastdiv_make(cv),
                         pl.cp, p.split_stride, pl.splits, accumulate);
    else
      hipLaunchKernelGGL(split_reduce_kernel<1>, dim3(blocks), dim3(256), 0, st, (const float*)slab, dw, nv, cv, fastdiv_make(cv),
                         pl.cp, p.split_stride, pl.splits, accumulate);
  }
  if (dbias) {
    const int k = d0->k;
    const int rb = crb;
    const bool b16 = d0->dtype == RTSDS_BF16;
    if (fused_colsum)
      ;  // partials already written by pad_colsum_kernel
    else if (b16 && k % 8 == 0)
      hipLaunchKernelGGL((colsum_part_kernel<bf16, 8>), dim3(rb, rt_cdiv(k, 2048)), dim3(256), 0, st, (const bf16*)dy, part, R, k);
    else if (b16)
      hipLaunchKernelGGL((colsum_part_kernel<bf16, 1>), dim3(rb, rt_cdiv(k, 256)), dim3(256), 0, st, (const bf16*)dy, part, R, k);
    else if (k % 4 == 0)
      hipLaunchKernelGGL((colsum_part_kernel<float, 4>), dim3(rb, rt_cdiv(k, 1024)), dim3(256), 0, st, (const float*)dy, part, R, k);
    else
      hipLaunchKernelGGL((colsum_part_kernel<float, 1>), dim3(rb, rt_cdiv(k, 256)), dim3(256), 0, st, (const float*)dy, part, R, k);
    hipLaunchKernelGGL(colsum_final_kernel, dim3(k), dim3(64), 0, st, (const float*)part, dbias, rb, k, accumulate);
  }
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
