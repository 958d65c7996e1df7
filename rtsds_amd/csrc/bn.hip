// BatchNorm2d (train: batch statistics; eval: running statistics) over NHWC [rows][c],
// fused with an optional residual add and ReLU / LeakyReLU, plus its backward.
//
// Statistics are single-pass: each thread keeps shifted sums (shift = its first sample) for
// its channels, which are merged across threads / blocks with Chan's parallel formula, so
// large-mean conv outputs (the reference feeds 0-255-scale normalised images,
// main.py:69-72) do not cancel catastrophically.  Three launches per direction:
// partial statistics (grid over row chunks) -> per-channel finalize -> vectorised apply.
#include "common.h"
#include <type_traits>
#include <algorithm>

static const int kBnMaxRB = 2048;  // row blocks of the partial-statistics pass
static const int kBnTinyRows = 64;  // up to this many rows: one block per channel finalizes and applies

// Threads of a 256-block are laid out [row group][channel vector]; TPR = threads per row.
template <int VEC> struct BnLayout {
  int tpr, rpi;  // threads per row, rows per block iteration
  RT_DEV BnLayout(int c) {
    tpr = (c + VEC - 1) / VEC;
    if (tpr > 256) tpr = 256;
    rpi = 256 / tpr;
  }
};

// VEC is either the 16-B vector width (dispatched only when c % VEC == 0, so an active thread's
// channel vector is always complete) or 1.
template <typename T, int VEC>
RT_DEV void load_vec(const T* p, float* v, int cvalid) {
  static_assert(VEC == 1 || VEC == VecT<T>::N, "VEC");
  if constexpr (VEC == VecT<T>::N) {
    typename VecT<T>::v16 t = *(const typename VecT<T>::v16*)p;
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = to_f(t[j]);
  } else {
    v[0] = cvalid > 0 ? to_f(p[0]) : 0.f;
  }
}
template <typename T, int VEC>
RT_DEV void store_vec(T* p, const float* v, int cvalid) {
  if constexpr (VEC == VecT<T>::N) {
    typename VecT<T>::v16 t;
#pragma unroll
    for (int j = 0; j < VEC; ++j) t[j] = from_f<T>(v[j]);
    *(typename VecT<T>::v16*)p = t;
  } else {
    if (cvalid > 0) p[0] = from_f<T>(v[0]);
  }
}

// scale/shift of y = x*scale + shift.  Written with explicit fma so the backward can
// recompute exactly the forward's pre-activation (ReLU mask without reading y).
RT_DEV void bn_coef(float g, float b, float m, float inv, float& sc, float& sh) {
  sc = g * inv;
  sh = fmaf(-m, sc, b);
}

RT_DEV void chan_merge(float& na, float& ma, float& Ma, float nb, float mb, float Mb) {
  if (nb == 0.f) return;
  if (na == 0.f) { na = nb; ma = mb; Ma = Mb; return; }
  const float n = na + nb, d = mb - ma;
  ma += d * (nb / n);
  Ma += Mb + d * d * (na * nb / n);
  na = n;
}

// Pass 1 (forward): part[(ch * RB + rb) * 4 + {0,1,2}] = (count, mean, M2) of block rb (16-B
// records: one vector store / load each)
// (channel-major: the finalize reads one contiguous run per channel).
template <typename T, int VEC>
__global__ void __launch_bounds__(256) bn_stats_kernel(const T* __restrict__ x, float* __restrict__ part, long rows, int c) {
  __shared__ float sh[3][256][VEC];
  const int cbase = blockIdx.y * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const BnLayout<VEC> L(cl);
  const int tid = threadIdx.x, cv = tid % L.tpr, rg = tid / L.tpr;
  const int ch0 = cbase + cv * VEC;
  const bool active = rg < L.rpi && cv * VEC < cl;
  float cnt = 0.f, shift[VEC], s1[VEC], s2[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { shift[j] = 0.f; s1[j] = 0.f; s2[j] = 0.f; }
  if (active) {
    long r = (long)blockIdx.x * L.rpi + rg;
    const long step = (long)gridDim.x * L.rpi;
    if (r < rows) {
      load_vec<T, VEC>(x + r * c + ch0, shift, c - ch0);
      cnt = 1.f;
      r += step;
    }
    for (; r < rows; r += step) {
      float v[VEC];
      load_vec<T, VEC>(x + r * c + ch0, v, c - ch0);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float d = v[j] - shift[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
      cnt += 1.f;
    }
  }
  // thread-level (count, mean, M2)
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const float mean = cnt > 0.f ? shift[j] + s1[j] / cnt : 0.f;
    const float m2 = cnt > 0.f ? s2[j] - s1[j] * s1[j] / cnt : 0.f;
    sh[0][tid][j] = cnt;
    sh[1][tid][j] = mean;
    sh[2][tid][j] = fmaxf(m2, 0.f);
  }
  __syncthreads();
  if (rg == 0 && cv * VEC < cl) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float n = sh[0][tid][j], m = sh[1][tid][j], M = sh[2][tid][j];
      for (int g = 1; g < L.rpi; ++g) {
        const int t = g * L.tpr + cv;
        chan_merge(n, m, M, sh[0][t][j], sh[1][t][j], sh[2][t][j]);
      }
      if (ch0 + j < c) {
        *(f32x4*)(part + ((long)(ch0 + j) * gridDim.x + blockIdx.x) * 4) = f32x4{n, m, M, 0.f};
      }
    }
  }
}


// Pass 2 (forward): one wave per channel merges the row-block partials (Chan, lane-strided,
// then a shuffle tree), updates running stats and emits scale/shift.
RT_DEV void chan_merge_shfl(float& n, float& m, float& M) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float nb = __shfl_xor(n, o, 64), mb = __shfl_xor(m, o, 64), Mb = __shfl_xor(M, o, 64);
    chan_merge(n, m, M, nb, mb, Mb);
  }
}
// 4 waves per channel: wave w merges partials b = w*64 + lane (+ 256 k), then the four wave
// results are merged in wave order -- up to kBnMaxRB partials without a pre-merge launch.
// (returns true in thread 0, which then holds the channel's scale / shift in sc_out / sh_out)
RT_DEV bool bn_finalize_body(const float* __restrict__ part, int nrb, int c, long rows, const float* gamma, const float* beta,
                             float* rmean, float* rvar, float* smean, float* sinv, float* scale, float* shift, float momentum,
                             float eps, long long* nbt, float (*wr)[3], float& sc_out, float& sh_out) {
  const int ch = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (nbt && ch == 0 && threadIdx.x == 0) *nbt += 1;  // num_batches_tracked.add_(1)
  // the per-channel operands of the tail, loaded up front (in flight with the partials: the
  // tail then pays no extra memory round trip; thread 0 alone reads and writes them)
  float g0 = 1.f, b0 = 0.f, rm0 = 0.f, rv0 = 0.f;
  if (threadIdx.x == 0) {
    if (gamma) g0 = gamma[ch];
    if (beta) b0 = beta[ch];
    if (rmean) rm0 = rmean[ch];
    if (rvar) rv0 = rvar[ch];
  }
  float n = 0.f, m = 0.f, M = 0.f;
  // up to 8 partials per thread loaded before any merge (one L2 round trip instead of eight);
  // merge order b = tid, tid + 256, ... as before
  for (int b0 = threadIdx.x; b0 < nrb; b0 += 256 * 8) {
    float pn[8], pm[8], pM[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = min(b0 + 256 * u, nrb - 1);
      const f32x4 p = *(const f32x4*)(part + ((long)ch * nrb + b) * 4);  // clamped: unconditional
      pn[u] = b0 + 256 * u < nrb ? p[0] : 0.f;                             // zero count past nrb
      pm[u] = p[1];
      pM[u] = p[2];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) chan_merge(n, m, M, pn[u], pm[u], pM[u]);
  }
  chan_merge_shfl(n, m, M);
  if (lane == 0) { wr[wave][0] = n; wr[wave][1] = m; wr[wave][2] = M; }
  __syncthreads();
  if (threadIdx.x != 0) return false;
  n = wr[0][0]; m = wr[0][1]; M = wr[0][2];
  for (int w = 1; w < 4; ++w) chan_merge(n, m, M, wr[w][0], wr[w][1], wr[w][2]);
  const float var = M / (float)rows;
  const float inv = 1.0f / sqrtf(var + eps);
  smean[ch] = m;
  sinv[ch] = inv;
  if (rmean) rmean[ch] = (1.f - momentum) * rm0 + momentum * m;
  if (rvar) {
    const float unb = rows > 1 ? M / (float)(rows - 1) : var;
    rvar[ch] = (1.f - momentum) * rv0 + momentum * unb;
  }
  bn_coef(g0, b0, m, inv, sc_out, sh_out);
  scale[ch] = sc_out;
  shift[ch] = sh_out;
  return true;
}
__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ part, int nrb, int c, long rows, const float* gamma,
                                   const float* beta, float* rmean, float* rvar, float* smean, float* sinv,
                                   float* scale, float* shift, float momentum, float eps, long long* nbt) {
  __shared__ float wr[4][3];
  float sc, sh;
  bn_finalize_body(part, nrb, c, rows, gamma, beta, rmean, rvar, smean, sinv, scale, shift, momentum, eps, nbt, wr, sc, sh);
}
__global__ void bn_eval_coef_kernel(int c, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                    float* scale, float* shift, float* smean, float* sinv, float eps) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float inv = 1.0f / sqrtf(rvar[ch] + eps);
  if (smean) smean[ch] = rmean[ch];
  if (sinv) sinv[ch] = inv;
  const float g = gamma ? gamma[ch] : 1.f, b = beta ? beta[ch] : 0.f;
  bn_coef(g, b, rmean[ch], inv, scale[ch], shift[ch]);
}

RT_DEV float act_f(float v, int act) {
  if (act == RTSDS_ACT_RELU) return fmaxf(v, 0.f);
  if (act == RTSDS_ACT_LEAKY) return v > 0.f ? v : 0.2f * v;
  if (act == RTSDS_ACT_SIGMOID) return 1.f / (1.f + expf(-v));
  return v;
}
RT_DEV float act_grad(float y, int act) {
  if (act == RTSDS_ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == RTSDS_ACT_LEAKY) return y > 0.f ? 1.f : 0.2f;
  if (act == RTSDS_ACT_SIGMOID) return y * (1.f - y);
  return 1.f;
}

// Per-channel coefficients for a thread's VEC channels.  Coefficient arrays live in the
// 256-B aligned workspace and VEC > 1 only when c % VEC == 0, so VEC % 4 == 0 loads are 16 B.
template <int VEC>
RT_DEV void load_coef(const float* __restrict__ p, int ch0, int c, float* v) {
  if constexpr (VEC % 4 == 0) {
#pragma unroll
    for (int q = 0; q < VEC / 4; ++q) {
      const f32x4 t = *(const f32x4*)(p + ch0 + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = t[e];
    }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = p[min(ch0 + j, c - 1)];
  }
}

// Few rows (the attention modules' BatchNorms on [N, C] pooled rows): the finalize's block also
// applies y = act(x * scale + shift [+ res]) to its channel's rows (bn_apply_kernel's expression)
// -- one launch instead of two, bit-identical.
template <typename T>
__global__ void __launch_bounds__(256) bn_finalize_apply_kernel(const float* __restrict__ part, int nrb, int c, long rows,
                                                                 const float* gamma, const float* beta, float* rmean, float* rvar,
                                                                 float* smean, float* sinv, float* scale, float* shift,
                                                                 float momentum, float eps, long long* nbt, const T* __restrict__ x,
                                                                 const T* __restrict__ res, T* __restrict__ y, long ldy, int act) {
  __shared__ float wr[4][3];
  __shared__ float cs[2];
  float sc, sh;
  if (bn_finalize_body(part, nrb, c, rows, gamma, beta, rmean, rvar, smean, sinv, scale, shift, momentum, eps, nbt, wr, sc, sh)) {
    cs[0] = sc;
    cs[1] = sh;
  }
  __syncthreads();
  const int ch = blockIdx.x;
  for (long r = threadIdx.x; r < rows; r += 256) {
    float a = fmaf(to_f(x[r * c + ch]), cs[0], cs[1]);
    if (res) a += to_f(res[r * c + ch]);
    y[r * ldy + ch] = from_f<T>(act_f(a, act));
  }
}

// Pass 3 (forward): y = act(x * scale + shift [+ res]).  Same [row group][channel vector]
// layout as the statistics pass: each thread owns one channel vector for its whole row
// sweep, so the coefficients sit in registers and there is no per-element index division.
// ACT (here and in the backward passes): the activation fixed at compile time for the ones the
// networks use (RTSDS_ACT_NONE / RTSDS_ACT_RELU), < 0 = the runtime argument; with a runtime
// activation every element paid act_f's uniform compare-and-branch chain.
template <typename T, int VEC, int ACT>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        long rows, int c, int act_rt, long ldy) {
  const int act = ACT >= 0 ? ACT : act_rt;
  const int cbase = blockIdx.y * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const BnLayout<VEC> L(cl);
  const int tid = threadIdx.x, cv = tid % L.tpr, rg = tid / L.tpr;
  if (rg >= L.rpi || cv * VEC >= cl) return;
  const int ch0 = cbase + cv * VEC, cvalid = c - ch0;
  float sc[VEC], sh[VEC];
  load_coef<VEC>(scale, ch0, c, sc);
  load_coef<VEC>(shift, ch0, c, sh);
  const long step = (long)gridDim.x * L.rpi;
  long r = (long)blockIdx.x * L.rpi + rg;
  for (; r + step < rows; r += 2 * step) {  // two independent rows in flight per thread
    float v0[VEC], v1[VEC], r0[VEC], r1[VEC];
    load_vec<T, VEC>(x + r * c + ch0, v0, cvalid);
    load_vec<T, VEC>(x + (r + step) * c + ch0, v1, cvalid);
    if (res) {
      load_vec<T, VEC>(res + r * c + ch0, r0, cvalid);
      load_vec<T, VEC>(res + (r + step) * c + ch0, r1, cvalid);
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float a = fmaf(v0[j], sc[j], sh[j]), b = fmaf(v1[j], sc[j], sh[j]);
      if (res) { a += r0[j]; b += r1[j]; }
      v0[j] = act_f(a, act);
      v1[j] = act_f(b, act);
    }
    store_vec<T, VEC>(y + r * ldy + ch0, v0, cvalid);
    store_vec<T, VEC>(y + (r + step) * ldy + ch0, v1, cvalid);
  }
  if (r < rows) {
    float v0[VEC], r0[VEC];
    load_vec<T, VEC>(x + r * c + ch0, v0, cvalid);
    if (res) load_vec<T, VEC>(res + r * c + ch0, r0, cvalid);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float a = fmaf(v0[j], sc[j], sh[j]);
      if (res) a += r0[j];
      v0[j] = act_f(a, act);
    }
    store_vec<T, VEC>(y + r * ldy + ch0, v0, cvalid);
  }
}

// Activation derivative from either the saved output y, or -- when y is not kept (no
// residual, monotone activation with act'(v) determined by sign(v)) -- from the recomputed
// pre-activation x*scale+shift, which is bit-identical to the forward's.
template <typename T, int VEC>
RT_DEV void bn_act_grad(float* g, const T* y, const float* xv, const float* sc, const float* sh, int act, int cvalid) {
  if (!act) return;
  if (y) {
    float yv[VEC];
    load_vec<T, VEC>(y, yv, cvalid);
#pragma unroll
    for (int j = 0; j < VEC; ++j) g[j] *= act_grad(yv[j], act);
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const bool pos = fmaf(xv[j], sc[j], sh[j]) > 0.f;
      g[j] = pos ? g[j] : (act == RTSDS_ACT_LEAKY ? 0.2f * g[j] : 0.f);
    }
  }
}

// Where the backward passes read g (before the activation mask): the stored dY, or -- for a
// BatchNorm + ReLU feeding a 3x3 stride-2 max pool (the ResNet stem, fused forward in
// bn_relu_pool_fwd_kernel) -- a gather of the pooled gradient: input pixel r of channel vector
// ch0 receives dY_pool[o] from each of the <= 2 x 2 windows o covering it whose argmax byte
// names r.  The dY of the BatchNorm never exists in memory.
template <typename T>
struct GradDirect {
  static constexpr bool kDirect = true;
  const T* dy;
  int c;
  template <int VEC> RT_DEV void load(long r, int ch0, float* g, int cvalid) const { load_vec<T, VEC>(dy + r * c + ch0, g, cvalid); }
};
template <typename T>
struct GradPool {
  static constexpr bool kDirect = false;
  const T* dyp;
  const uint8_t* idx;
  int c, h, w, ho, wo, p;
  FastDiv f_w, f_h;
  template <int VEC> RT_DEV void load(long r, int ch0, float* g, int cvalid) const {
    static_assert(VEC == 8 && sizeof(T) == 2, "pooled gradient source: bf16 vectors of 8 channels");
    typedef typename VecT<T>::v16 V16;
    const uint32_t q = fdiv((uint32_t)r, f_w), img = fdiv(q, f_h);
    const int iw = (int)((uint32_t)r - q * w), ih = (int)(q - img * h);
    const int oh_lo = max(0, (ih + p - 1) / 2), ow_lo = max(0, (iw + p - 1) / 2);
    V16 gv[4];
    unsigned long long ib[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {  // clamped, unconditional (all in flight together)
      const int oh = min(oh_lo + (t >> 1), ho - 1), ow = min(ow_lo + (t & 1), wo - 1);
      const long o = (((long)img * ho + oh) * wo + ow) * c + ch0;
      gv[t] = *(const V16*)(dyp + o);
      ib[t] = *(const unsigned long long*)(idx + o);
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) g[j] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int oh = oh_lo + (t >> 1), ow = ow_lo + (t & 1);
      const int a = ih - (oh * 2 - p), b = iw - (ow * 2 - p);
      if (oh >= ho || ow >= wo || a < 0 || a >= 3 || b < 0 || b >= 3) continue;
      const unsigned want = (unsigned)(a * 3 + b);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (((ib[t] >> (8 * j)) & 0xff) == want) g[j] += to_f(gv[t][j]);
    }
  }
};

template <int VEC>
RT_DEV void bn_bwd_coef(int ch0, int c, const float* gamma, const float* beta, const float* mean, const float* sinv,
                        float* mu, float* sc, float* sh) {
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const int ch = min(ch0 + j, c - 1);
    mu[j] = mean[ch];
    bn_coef(gamma ? gamma[ch] : 1.f, beta ? beta[ch] : 0.f, mu[j], sinv[ch], sc[j], sh[j]);
  }
}

// Backward pass 1: part[(rb*c+ch)*2 + {0,1}] = (sum g, sum g*(x-mean)) with g = dy*act'(y) --
// row-block-major, so each block's partials leave as contiguous stores (channel-major rows
// scattered 8-B stores RB*c*8 bytes apart: 16 MB of them for 1024 channels).  Merged by
// bn_bwd_finalize_rb_kernel.
// HAS_Y: the activation mask comes from y (residual BNs); otherwise from x (no y registers).
// gout (HAS_Y): g = dy * act'(y) is also stored (the residual branch's gradient, and the apply
// pass's input instead of dy and y).
template <typename T, int VEC, bool HAS_Y, class GS, int ACT>
__global__ void __launch_bounds__(256) bn_bwd_stats_kernel(const GS gs, const T* __restrict__ x,
                                                            const T* __restrict__ y, const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, const float* __restrict__ mean,
                                                            const float* __restrict__ sinv, float* __restrict__ part,
                                                            long rows, int c, int act_rt, T* __restrict__ gout) {
  const int act = ACT >= 0 ? ACT : act_rt;
  __shared__ float red[2][256][VEC];
  const int cbase = blockIdx.y * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const BnLayout<VEC> L(cl);
  const int tid = threadIdx.x, cv = tid % L.tpr, rg = tid / L.tpr;
  const int ch0 = cbase + cv * VEC;
  const bool active = rg < L.rpi && cv * VEC < cl;
  float sg[VEC], sgx[VEC], mu[VEC], sc[VEC], sh[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { sg[j] = 0.f; sgx[j] = 0.f; }
  if (active) {
    bn_bwd_coef<VEC>(ch0, c, gamma, beta, mean, sinv, mu, sc, sh);
    const long step = (long)gridDim.x * L.rpi;
    constexpr int U = 2;  // rows in flight per thread (loads issued before any use)
    for (long r = (long)blockIdx.x * L.rpi + rg; r < rows; r += U * step) {
      float g[U][VEC], xv[U][VEC], yv[HAS_Y ? U : 1][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        // clamped, unconditional loads (all U rows in flight together); rows past the end
        // contribute g = 0
        const long rr = min(r + u * step, rows - 1);
        gs.template load<VEC>(rr, ch0, g[u], c - ch0);
        load_vec<T, VEC>(x + rr * c + ch0, xv[u], c - ch0);
        if constexpr (HAS_Y) load_vec<T, VEC>(y + rr * c + ch0, yv[u], c - ch0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (r + u * step >= rows) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) g[u][j] = 0.f;
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (act) {
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            g[u][j] *= HAS_Y ? act_grad(yv[HAS_Y ? u : 0][j], act)
                             : (fmaf(xv[u][j], sc[j], sh[j]) > 0.f ? 1.f : (act == RTSDS_ACT_LEAKY ? 0.2f : 0.f));
        }
        if (HAS_Y && gout && r + u * step < rows) store_vec<T, VEC>(gout + (r + u * step) * c + ch0, g[u], c - ch0);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          sg[j] += g[u][j];
          sgx[j] = fmaf(g[u][j], xv[u][j] - mu[j], sgx[j]);
        }
      }
    }
  }
  if ((L.tpr & (L.tpr - 1)) == 0 && L.tpr <= 64) {
    // power-of-two row width: sum the wave's rows with xor shuffles (lanes l and l ^ (tpr << i)
    // hold the same channel vector), then the four wave sums through LDS -- a per-block tail of
    // a few hundred cycles instead of a serial LDS loop over all rpi rows.
    const int lane = tid & 63, wave = tid >> 6;
    for (int o = L.tpr; o < 64; o <<= 1) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        sg[j] += __shfl_xor(sg[j], o, 64);
        sgx[j] += __shfl_xor(sgx[j], o, 64);
      }
    }
    if (lane < L.tpr) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) { red[0][wave * 64 + lane][j] = sg[j]; red[1][wave * 64 + lane][j] = sgx[j]; }
    }
    __syncthreads();
    if (tid < L.tpr && tid * VEC < cl) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float a = (red[0][tid][j] + red[0][64 + tid][j]) + (red[0][128 + tid][j] + red[0][192 + tid][j]);
        const float b = (red[1][tid][j] + red[1][64 + tid][j]) + (red[1][128 + tid][j] + red[1][192 + tid][j]);
        if (ch0 + j < c) {
          *(float2*)(part + ((long)blockIdx.x * c + ch0 + j) * 2) = make_float2(a, b);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) { red[0][tid][j] = sg[j]; red[1][tid][j] = sgx[j]; }
  __syncthreads();
  if (rg == 0 && cv * VEC < cl) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float a = red[0][tid][j], b = red[1][tid][j];
      for (int gi = 1; gi < L.rpi; ++gi) {
        a += red[0][gi * L.tpr + cv][j];
        b += red[1][gi * L.tpr + cv][j];
      }
      if (ch0 + j < c) {
        *(float2*)(part + ((long)blockIdx.x * c + ch0 + j) * 2) = make_float2(a, b);
      }
    }
  }
}

// All three backward passes in one launch when the statistics pass has a single row block
// (bn_bwd_rb == 1: the attention modules' BatchNorms on [N, C] pooled rows): the same statistics
// loop and reduction as bn_bwd_stats_kernel (grid (1, channel blocks)), the finalize of a single
// partial (bn_bwd_finalize_rb_kernel's 0 + p), the apply of bn_bwd_apply_kernel -- so the results
// are bit-identical to the three launches.
template <typename T, int VEC, bool HAS_Y, class GS, int ACT>
__global__ void __launch_bounds__(256) bn_bwd_tiny_kernel(const GS gs, const T* __restrict__ x, const T* __restrict__ y,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           const float* __restrict__ mean, const float* __restrict__ sinv,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta, T* __restrict__ dx,
                                                           T* __restrict__ dres, long rows, int c, int act_rt, int training,
                                                           int accumulate) {
  const int act = ACT >= 0 ? ACT : act_rt;
  __shared__ float red[2][256][VEC];
  __shared__ float cf[3][256 * VEC];
  const int cbase = blockIdx.y * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const BnLayout<VEC> L(cl);
  const int tid = threadIdx.x, cv = tid % L.tpr, rg = tid / L.tpr;
  const int ch0 = cbase + cv * VEC;
  const bool active = rg < L.rpi && cv * VEC < cl;
  float sg[VEC], sgx[VEC], mu[VEC], sc[VEC], sh[VEC];
  constexpr int U = 2;
  // rows <= U * rpi: the statistics loop runs once and its (masked) g and x stay in registers
  // for the apply -- one memory round trip fewer
  const bool one_pass = rows <= U * (long)L.rpi;
  float g[U][VEC], xv[U][VEC];
  // the accumulated parameter gradients and the finalize's operands, loaded up front
  float dg0[VEC], db0[VEC], inv0[VEC], gm0[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    sg[j] = 0.f;
    sgx[j] = 0.f;
    const int ch = min(ch0 + j, c - 1);
    inv0[j] = sinv[ch];
    gm0[j] = gamma ? gamma[ch] : 1.f;
    dg0[j] = accumulate && dgamma ? dgamma[ch] : 0.f;
    db0[j] = accumulate && dbeta ? dbeta[ch] : 0.f;
  }
  if (active) {
    bn_bwd_coef<VEC>(ch0, c, gamma, beta, mean, sinv, mu, sc, sh);
    const long step = L.rpi;  // (one row block)
    for (long r = rg; r < rows; r += U * step) {
      float yv[HAS_Y ? U : 1][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long rr = min(r + u * step, rows - 1);
        gs.template load<VEC>(rr, ch0, g[u], c - ch0);
        load_vec<T, VEC>(x + rr * c + ch0, xv[u], c - ch0);
        if constexpr (HAS_Y) load_vec<T, VEC>(y + rr * c + ch0, yv[u], c - ch0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (r + u * step >= rows) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) g[u][j] = 0.f;
        }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (act) {
#pragma unroll
          for (int j = 0; j < VEC; ++j)
            g[u][j] *= HAS_Y ? act_grad(yv[HAS_Y ? u : 0][j], act)
                             : (fmaf(xv[u][j], sc[j], sh[j]) > 0.f ? 1.f : (act == RTSDS_ACT_LEAKY ? 0.2f : 0.f));
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          sg[j] += g[u][j];
          sgx[j] = fmaf(g[u][j], xv[u][j] - mu[j], sgx[j]);
        }
      }
    }
  }
  // the block sums (bn_bwd_stats_kernel's two reduction forms), then the single partial's finalize
  float tg[VEC], tgx[VEC];
  bool have = false;
  if ((L.tpr & (L.tpr - 1)) == 0 && L.tpr <= 64) {
    const int lane = tid & 63, wave = tid >> 6;
    for (int o = L.tpr; o < 64; o <<= 1) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        sg[j] += __shfl_xor(sg[j], o, 64);
        sgx[j] += __shfl_xor(sgx[j], o, 64);
      }
    }
    if (lane < L.tpr) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) { red[0][wave * 64 + lane][j] = sg[j]; red[1][wave * 64 + lane][j] = sgx[j]; }
    }
    __syncthreads();
    if (tid < L.tpr && tid * VEC < cl) {
      have = true;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        tg[j] = (red[0][tid][j] + red[0][64 + tid][j]) + (red[0][128 + tid][j] + red[0][192 + tid][j]);
        tgx[j] = (red[1][tid][j] + red[1][64 + tid][j]) + (red[1][128 + tid][j] + red[1][192 + tid][j]);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) { red[0][tid][j] = sg[j]; red[1][tid][j] = sgx[j]; }
    __syncthreads();
    if (rg == 0 && cv * VEC < cl) {
      have = true;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float a = red[0][tid][j], b = red[1][tid][j];
        for (int gi = 1; gi < L.rpi; ++gi) {
          a += red[0][gi * L.tpr + cv][j];
          b += red[1][gi * L.tpr + cv][j];
        }
        tg[j] = a;
        tgx[j] = b;
      }
    }
  }
  if (have) {  // (tid == cv here: the first row group holds the channel vector)
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const int ch = ch0 + j;
      if (ch >= c) continue;
      const float sgv = 0.f + tg[j], sgxv = 0.f + tgx[j];  // bn_bwd_finalize_rb_kernel: one partial
      const float inv = inv0[j], gm = gm0[j];
      if (dgamma) dgamma[ch] = accumulate ? dg0[j] + sgxv * inv : sgxv * inv;
      if (dbeta) dbeta[ch] = accumulate ? db0[j] + sgv : sgv;
      const float a = gm * inv;
      const float invn = 1.f / (float)rows;
      cf[0][cv * VEC + j] = a;
      cf[1][cv * VEC + j] = training ? -a * inv * inv * sgxv * invn : 0.f;
      cf[2][cv * VEC + j] = training ? -a * sgv * invn : 0.f;
    }
  }
  __syncthreads();
  if (!active || (!dx && !dres)) return;
  const int cvalid = c - ch0;
  float ca[VEC], cb[VEC], ck[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    ca[j] = cf[0][cv * VEC + j];
    cb[j] = cf[1][cv * VEC + j];
    ck[j] = cf[2][cv * VEC + j];
  }
  if (one_pass) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = rg + u * (long)L.rpi;
      if (r >= rows) break;
      const long off = r * c + ch0;
      float o[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = fmaf(ca[j], g[u][j], fmaf(cb[j], xv[u][j] - mu[j], ck[j]));
      if (dx) store_vec<T, VEC>(dx + off, o, cvalid);
      if (dres) store_vec<T, VEC>(dres + off, g[u], cvalid);
    }
    return;
  }
  for (long r = rg; r < rows; r += L.rpi) {
    const long off = r * c + ch0;
    float gr[VEC], xr[VEC];
    gs.template load<VEC>(r, ch0, gr, cvalid);
    load_vec<T, VEC>(x + off, xr, cvalid);
    bn_act_grad<T, VEC>(gr, HAS_Y ? y + off : nullptr, xr, sc, sh, act, cvalid);
#pragma unroll
    for (int j = 0; j < VEC; ++j) xr[j] = fmaf(ca[j], gr[j], fmaf(cb[j], xr[j] - mu[j], ck[j]));
    if (dx) store_vec<T, VEC>(dx + off, xr, cvalid);
    if (dres) store_vec<T, VEC>(dres + off, gr, cvalid);
  }
}

// Backward pass 2: coefficients  dx = A*g + B*(x-mean) + C  per channel (one wave each).
// coef = [A | B | C | mean | scale | shift] x c  (the last three for the mask recompute).
__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* __restrict__ part, int nrb, int c, long rows, const float* gamma,
                                       const float* beta, const float* smean, const float* sinv, float* dgamma, float* dbeta,
                                       float* coef, int training, int accumulate) {
  __shared__ float wr[4][2];
  const int ch = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the tail's per-channel operands up front (see bn_finalize_kernel)
  float inv = 0.f, g = 1.f, bt = 0.f, mu = 0.f, dg0 = 0.f, db0 = 0.f;
  if (threadIdx.x == 0) {
    inv = sinv[ch];
    mu = smean[ch];
    if (gamma) g = gamma[ch];
    if (beta) bt = beta[ch];
    if (accumulate && dgamma) dg0 = dgamma[ch];
    if (accumulate && dbeta) db0 = dbeta[ch];
  }
  float sg = 0.f, sgx = 0.f;
  for (int b0 = threadIdx.x; b0 < nrb; b0 += 256 * 8) {  // 8 partials in flight per thread
    float pg[8], px[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = min(b0 + 256 * u, nrb - 1);
      const bool ok = b0 + 256 * u < nrb;
      const float2 pr = *(const float2*)(part + ((long)ch * nrb + b) * 2);
      const float g = pr.x, gx = pr.y;
      pg[u] = ok ? g : 0.f;
      px[u] = ok ? gx : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) { sg += pg[u]; sgx += px[u]; }
  }
  sg = wave_sum(sg);
  sgx = wave_sum(sgx);
  if (lane == 0) { wr[wave][0] = sg; wr[wave][1] = sgx; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  sg = (wr[0][0] + wr[1][0]) + (wr[2][0] + wr[3][0]);
  sgx = (wr[0][1] + wr[1][1]) + (wr[2][1] + wr[3][1]);
  if (dgamma) dgamma[ch] = accumulate ? dg0 + sgx * inv : sgx * inv;
  if (dbeta) dbeta[ch] = accumulate ? db0 + sg : sg;
  const float a = g * inv;
  const float invn = 1.f / (float)rows;
  coef[ch] = a;
  coef[c + ch] = training ? -a * inv * inv * sgx * invn : 0.f;
  coef[2 * c + ch] = training ? -a * sg * invn : 0.f;
  coef[3 * c + ch] = mu;
  bn_coef(g, bt, mu, inv, coef[4 * c + ch], coef[5 * c + ch]);
}

// Backward pass 2 for the row-block-major partials of bn_bwd_stats_kernel: 16 channels per
// block, lane q (0..15) of a channel sums row blocks q, q + 16, ... (8 in flight, 128-B rows of
// 16 channels per load group), the 16 lane sums added in a fixed tree order; coefficients as
// bn_bwd_finalize_kernel.
__global__ void __launch_bounds__(256) bn_bwd_finalize_rb_kernel(const float* __restrict__ part, int nrb, int c, long rows,
                                                                  const float* gamma, const float* beta, const float* smean,
                                                                  const float* sinv, float* dgamma, float* dbeta, float* coef,
                                                                  int training, int accumulate) {
  __shared__ float wr[16][16][2];
  const int cl = threadIdx.x & 15, q = threadIdx.x >> 4, ch = blockIdx.x * 16 + cl;
  const int chc = min(ch, c - 1);
  // the tail's per-channel operands up front (see bn_finalize_kernel)
  float inv = 0.f, g = 1.f, bt = 0.f, mu = 0.f, dg0 = 0.f, db0 = 0.f;
  if (q == 0) {
    inv = sinv[chc];
    mu = smean[chc];
    if (gamma) g = gamma[chc];
    if (beta) bt = beta[chc];
    if (accumulate && dgamma) dg0 = dgamma[chc];
    if (accumulate && dbeta) db0 = dbeta[chc];
  }
  float sg = 0.f, sgx = 0.f;
  for (int b0 = q; b0 < nrb; b0 += 16 * 8) {
    float2 pv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = min(b0 + 16 * u, nrb - 1);  // clamped: unconditional
      pv[u] = *(const float2*)(part + ((long)b * c + chc) * 2);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b0 + 16 * u < nrb) { sg += pv[u].x; sgx += pv[u].y; }
  }
  wr[q][cl][0] = sg;
  wr[q][cl][1] = sgx;
  __syncthreads();
  if (q != 0 || ch >= c) return;
  float t0[8], t1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { t0[i] = wr[2 * i][cl][0] + wr[2 * i + 1][cl][0]; t1[i] = wr[2 * i][cl][1] + wr[2 * i + 1][cl][1]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) { t0[i] = t0[2 * i] + t0[2 * i + 1]; t1[i] = t1[2 * i] + t1[2 * i + 1]; }
  sg = (t0[0] + t0[1]) + (t0[2] + t0[3]);
  sgx = (t1[0] + t1[1]) + (t1[2] + t1[3]);
  if (dgamma) dgamma[ch] = accumulate ? dg0 + sgx * inv : sgx * inv;
  if (dbeta) dbeta[ch] = accumulate ? db0 + sg : sg;
  const float a = g * inv;
  const float invn = 1.f / (float)rows;
  coef[ch] = a;
  coef[c + ch] = training ? -a * inv * inv * sgx * invn : 0.f;
  coef[2 * c + ch] = training ? -a * sg * invn : 0.f;
  coef[3 * c + ch] = mu;
  bn_coef(g, bt, mu, inv, coef[4 * c + ch], coef[5 * c + ch]);
}

// Backward pass 3: dx = A*g + B*(x - mean) + C;  dres = g.  Layout as bn_apply_kernel.
template <typename T, int VEC, class GS, int ACT>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const GS gs, const T* __restrict__ x,
                                                            const T* __restrict__ y, T* __restrict__ dx, T* __restrict__ dres,
                                                            const float* __restrict__ coef, long rows, int c, int act_rt) {
  const int act = ACT >= 0 ? ACT : act_rt;
  const int cbase = blockIdx.y * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const BnLayout<VEC> L(cl);
  const int tid = threadIdx.x, cv = tid % L.tpr, rg = tid / L.tpr;
  if (rg >= L.rpi || cv * VEC >= cl) return;
  const int ch0 = cbase + cv * VEC, cvalid = c - ch0;
  float a[VEC], b[VEC], k[VEC], mu[VEC], sc[VEC], sh[VEC];
  load_coef<VEC>(coef, ch0, c, a);
  load_coef<VEC>(coef + c, ch0, c, b);
  load_coef<VEC>(coef + 2 * c, ch0, c, k);
  load_coef<VEC>(coef + 3 * c, ch0, c, mu);
  if (act && !y) {
    load_coef<VEC>(coef + 4 * c, ch0, c, sc);
    load_coef<VEC>(coef + 5 * c, ch0, c, sh);
  }
  const long step = (long)gridDim.x * L.rpi;
  long r = (long)blockIdx.x * L.rpi + rg;
  for (; r + step < rows; r += 2 * step) {  // two independent rows in flight per thread
    const long o0 = r * c + ch0, o1 = o0 + step * c;
    float g0[VEC], x0[VEC], g1[VEC], x1[VEC];
    gs.template load<VEC>(r, ch0, g0, cvalid);
    load_vec<T, VEC>(x + o0, x0, cvalid);
    gs.template load<VEC>(r + step, ch0, g1, cvalid);
    load_vec<T, VEC>(x + o1, x1, cvalid);
    bn_act_grad<T, VEC>(g0, y ? y + o0 : nullptr, x0, sc, sh, act, cvalid);
    bn_act_grad<T, VEC>(g1, y ? y + o1 : nullptr, x1, sc, sh, act, cvalid);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      x0[j] = fmaf(a[j], g0[j], fmaf(b[j], x0[j] - mu[j], k[j]));
      x1[j] = fmaf(a[j], g1[j], fmaf(b[j], x1[j] - mu[j], k[j]));
    }
    if (dx) {
      store_vec<T, VEC>(dx + o0, x0, cvalid);
      store_vec<T, VEC>(dx + o1, x1, cvalid);
    }
    if (dres) {
      store_vec<T, VEC>(dres + o0, g0, cvalid);
      store_vec<T, VEC>(dres + o1, g1, cvalid);
    }
  }
  if (r < rows) {
    const long off = r * c + ch0;
    float g[VEC], xv[VEC];
    gs.template load<VEC>(r, ch0, g, cvalid);
    load_vec<T, VEC>(x + off, xv, cvalid);
    bn_act_grad<T, VEC>(g, y ? y + off : nullptr, xv, sc, sh, act, cvalid);
#pragma unroll
    for (int j = 0; j < VEC; ++j) xv[j] = fmaf(a[j], g[j], fmaf(b[j], xv[j] - mu[j], k[j]));
    if (dx) store_vec<T, VEC>(dx + off, xv, cvalid);
    if (dres) store_vec<T, VEC>(dres + off, g, cvalid);
  }
}

// ------------------------------------------------------------------ host
// f(std::integral_constant<int, A>) with A the compile-time activation variant of the kernels above
template <typename F>
static void with_act(int act, F f) {
  if (act == RTSDS_ACT_NONE) f(std::integral_constant<int, RTSDS_ACT_NONE>());
  else if (act == RTSDS_ACT_RELU) f(std::integral_constant<int, RTSDS_ACT_RELU>());
  else f(std::integral_constant<int, -1>());
}
static long bn_need(long rows, int c, int vec) {
  int tpr = (c + vec - 1) / vec;
  if (tpr > 256) tpr = 256;
  const int rpi = 256 / tpr;
  return (rows + rpi - 1) / rpi;
}
// Row blocks of the reduction passes: enough to fill the chip (8+ waves per CU), at least
// 4 row-iterations per thread, at most kBnMaxRB partials to merge.
static int bn_rb(long rows, int c, int vec) {
  const long need = bn_need(rows, c, vec);
  long rb = std::min<long>(need, kBnMaxRB);
  rb = std::max<long>(1, std::min<long>(rb, (need + 7) / 8));
  return (int)rb;
}
// Row blocks of the elementwise passes: ~2 rows per thread.
static constexpr auto kBnApplyMaxRB = (1L << 24);
static int bn_apply_rb(long rows, int c, int vec) {
  const long need = bn_need(rows, c, vec);
  return (int)std::max<long>(1, std::min<long>((need + 1) / 2, kBnApplyMaxRB));
}

static size_t bn_part_floats(long rows, int c) { return (size_t)bn_rb(rows, c, 1) * c * 4; }

// Workspace: [row-block partials | 8 coefficient arrays], each part
// 256-B aligned (coefficient arrays are read with 16-B vector loads).
static size_t al64f(size_t n) { return (n + 63) & ~(size_t)63; }
struct BnWs {
  float *part, *coef;
};
static BnWs bn_ws(void* ws, long rows, int c) {
  BnWs w;
  w.part = (float*)ws;
  w.coef = w.part + al64f(bn_part_floats(rows, c));
  return w;
}
extern "C" size_t rtsds_bn_workspace(long rows, int c) {
  if (rows <= 0 || c <= 0) return 256;
  // partials (3 floats x RB x c; VEC=1 gives the most row blocks) + 8 x c
  return (al64f(bn_part_floats(rows, c)) + al64f((size_t)c * 8)) * 4 + 256;
}


template <typename T, int VEC>
static void bn_fwd_launch(const void* x, const void* res, void* y, long rows, int c, const float* gamma, const float* beta,
                          float* rm, float* rv, float* sm, float* si, float mom, float eps, int training, int act,
                          const float* pre, int pre_nrb, long long* nbt, const BnWs& w, hipStream_t st, long ldy) {
  float* scale = w.coef;
  float* shift = w.coef + c;
  if (training) {
    int rb = pre_nrb;
    const float* part = pre;  // statistics already produced by the conv epilogue, or:
    if (!pre) {
      rb = bn_rb(rows, c, VEC);
      hipLaunchKernelGGL((bn_stats_kernel<T, VEC>), dim3(rb, rt_cdiv(c, 256 * VEC)), dim3(256), 0, st, (const T*)x, w.part, rows, c);
      part = w.part;
    }
    if (rows <= kBnTinyRows) {  // finalize + apply in one launch
      hipLaunchKernelGGL(bn_finalize_apply_kernel<T>, dim3(c), dim3(256), 0, st, part, rb, c, rows, gamma, beta, rm, rv, sm, si,
                         scale, shift, mom, eps, nbt, (const T*)x, (const T*)res, (T*)y, ldy, act);
      return;
    }
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(c), dim3(256), 0, st, part, rb, c, rows, gamma, beta, rm, rv,
                       sm, si, scale, shift, mom, eps, nbt);
  } else {
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3(rt_cdiv(c, 256)), dim3(256), 0, st, c, gamma, beta, rm, rv, scale, shift, sm, si, eps);
  }
  with_act(act, [&](auto a) {
    hipLaunchKernelGGL((bn_apply_kernel<T, VEC, decltype(a)::value>), dim3(bn_apply_rb(rows, c, VEC), rt_cdiv(c, 256 * VEC)),
                       dim3(256), 0, st, (const T*)x, (const T*)res, (T*)y, scale, shift, rows, c, act, ldy);
  });
}

extern "C" int rtsds_bn_fwd_ld(const void* x, const void* res, void* y, long ldy, long rows, int c, const float* gamma,
                               const float* beta, float* running_mean, float* running_var, long long* num_batches_tracked,
                               float* save_mean, float* save_invstd, float momentum, float eps, int training, int act,
                               const float* stats_part, int stats_nrb, int dtype, void* ws, size_t ws_bytes, void* stream) {
  if (rows <= 0 || c <= 0 || ldy < c) return RTSDS_ERR_SHAPE;
  if (ldy != c && !(dtype == RTSDS_BF16 && c % 8 == 0 && ldy % 8 == 0)) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_bn_workspace(rows, c)) return RTSDS_ERR_WORKSPACE;
  if (!training && (!running_mean || !running_var)) return RTSDS_ERR_UNSUPPORTED;
  if (training && (!save_mean || !save_invstd)) return RTSDS_ERR_UNSUPPORTED;
  if (c > 65535 * 256) return RTSDS_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const BnWs w = bn_ws(ws, rows, c);
  long long* nbt = training ? num_batches_tracked : nullptr;
  if (dtype == RTSDS_BF16) {
    if (c % 8 == 0) bn_fwd_launch<bf16, 8>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, nbt, w, st, ldy);
    else bn_fwd_launch<bf16, 1>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, nbt, w, st, ldy);
  } else if (dtype == RTSDS_F32) {
    if (c % 4 == 0) bn_fwd_launch<float, 4>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, nbt, w, st, ldy);
    else bn_fwd_launch<float, 1>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, nbt, w, st, ldy);
  } else return RTSDS_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

extern "C" int rtsds_bn_fwd(const void* x, const void* res, void* y, long rows, int c, const float* gamma, const float* beta,
                            float* running_mean, float* running_var, long long* num_batches_tracked, float* save_mean,
                            float* save_invstd, float momentum,
                            float eps, int training, int act, const float* stats_part, int stats_nrb, int dtype, void* ws,
                            size_t ws_bytes, void* stream) {
  return rtsds_bn_fwd_ld(x, res, y, c, rows, c, gamma, beta, running_mean, running_var, num_batches_tracked, save_mean,
                         save_invstd, momentum, eps, training, act, stats_part, stats_nrb, dtype, ws, ws_bytes, stream);
}

static constexpr auto kBnBwdRBMax = 512;
static constexpr auto kBnBwdRBDiv = 8;
// Row blocks of the backward statistics pass (row-block-major partials, merged 16 lanes per
// channel by bn_bwd_finalize_rb_kernel).  At most 512 (tools/ab_bn2.sh, stats pass: 33,540 x
// 1024 58.8 -> 29.2 us, 262,144 x 128 41.3 -> 27.7 us, 262,144 x 64 17.6 -> 15.6 us against 2048
// channel-major row blocks; finalize unchanged at ~5 us).
static int bn_bwd_rb(long rows, int c, int vec) {
  const long need = bn_need(rows, c, vec);
  long rb = std::min<long>(need, kBnBwdRBMax);
  rb = std::max<long>(1, std::min<long>(rb, (need + kBnBwdRBDiv - 1) / kBnBwdRBDiv));
  return (int)rb;
}
template <typename T, int VEC, class GS>
static void bn_bwd_launch(const GS& gs, const void* x, const void* y, void* dx, void* dres, float* dgamma, float* dbeta,
                          long rows, int c, const float* gamma, const float* beta, const float* smean, const float* sinv, int training,
                          int act, int accumulate, const BnWs& w, hipStream_t st, const float* pre = nullptr, int pre_nrb = 0) {
  int rb = bn_bwd_rb(rows, c, VEC);
  const float* part = w.part;
  // residual BatchNorm + ReLU with both gradients wanted: the statistics pass stores
  // g = dy * relu'(y) as dres, and the apply pass reads g and x (not dy, y) -- one full read
  // less; g is exactly dy or 0, so the arithmetic is unchanged
  const bool g_out = !pre && y && act == RTSDS_ACT_RELU && dres && dx && GS::kDirect;
  if (!pre && rb == 1 && GS::kDirect && !g_out) {  // one row block: the three passes in one launch
    const dim3 grid(1, rt_cdiv(c, 256 * VEC));
    if (y && act)
      with_act(act, [&](auto a) {
        hipLaunchKernelGGL((bn_bwd_tiny_kernel<T, VEC, true, GS, decltype(a)::value>), grid, dim3(256), 0, st, gs, (const T*)x,
                           (const T*)y, gamma, beta, smean, sinv, dgamma, dbeta, (T*)dx, (T*)dres, rows, c, act, training,
                           accumulate);
      });
    else
      with_act(act, [&](auto a) {
        hipLaunchKernelGGL((bn_bwd_tiny_kernel<T, VEC, false, GS, decltype(a)::value>), grid, dim3(256), 0, st, gs, (const T*)x,
                           (const T*)y, gamma, beta, smean, sinv, dgamma, dbeta, (T*)dx, (T*)dres, rows, c, act, training,
                           accumulate);
      });
    return;
  }
  if (pre) {  // statistics already produced by the consumer conv's data-gradient epilogue
    part = pre;
    rb = pre_nrb;
  } else if (y && act)
    with_act(act, [&](auto a) {
      hipLaunchKernelGGL((bn_bwd_stats_kernel<T, VEC, true, GS, decltype(a)::value>), dim3(rb, rt_cdiv(c, 256 * VEC)), dim3(256), 0,
                         st, gs, (const T*)x, (const T*)y, gamma, beta, smean, sinv, w.part, rows, c, act,
                         g_out ? (T*)dres : (T*)nullptr);
    });
  else
    with_act(act, [&](auto a) {
      hipLaunchKernelGGL((bn_bwd_stats_kernel<T, VEC, false, GS, decltype(a)::value>), dim3(rb, rt_cdiv(c, 256 * VEC)), dim3(256),
                         0, st, gs, (const T*)x, (const T*)y, gamma, beta, smean, sinv, w.part, rows, c, act, (T*)nullptr);
    });
  if (pre)  // channel-major [c][tile][2] partials of the data-gradient epilogue
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(c), dim3(256), 0, st, part, rb, c, rows, gamma, beta, smean, sinv,
                       dgamma, dbeta, w.coef, training, accumulate);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_rb_kernel, dim3(rt_cdiv(c, 16)), dim3(256), 0, st, part, rb, c, rows, gamma, beta, smean,
                       sinv, dgamma, dbeta, w.coef, training, accumulate);
  if (g_out) {
    const GradDirect<T> gg{(const T*)dres, c};
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, VEC, GradDirect<T>, RTSDS_ACT_NONE>), dim3(bn_apply_rb(rows, c, VEC), rt_cdiv(c, 256 * VEC)),
                       dim3(256), 0, st, gg, (const T*)x, (const T*)nullptr, (T*)dx, (T*)nullptr, w.coef, rows, c, 0);
  } else if (dx || dres) {
    with_act(act, [&](auto a) {
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, VEC, GS, decltype(a)::value>), dim3(bn_apply_rb(rows, c, VEC), rt_cdiv(c, 256 * VEC)),
                         dim3(256), 0, st, gs, (const T*)x, (const T*)y, (T*)dx, (T*)dres, w.coef, rows, c, act);
    });
  }
}
template <typename T, int VEC>
static void bn_bwd_launch(const void* dy, const void* x, const void* y, void* dx, void* dres, float* dgamma, float* dbeta,
                          long rows, int c, const float* gamma, const float* beta, const float* smean, const float* sinv, int training,
                          int act, int accumulate, const BnWs& w, hipStream_t st, const float* pre = nullptr, int pre_nrb = 0,
                          long ldy = 0) {
  const GradDirect<T> gs{(const T*)dy, (int)(ldy ? ldy : c)};
  bn_bwd_launch<T, VEC, GradDirect<T>>(gs, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, beta, smean, sinv, training, act,
                                       accumulate, w, st, pre, pre_nrb);
}

extern "C" int rtsds_bn_bwd_part(const void* dy, const void* x, void* dx, float* dgamma, float* dbeta, long rows, int c,
                                 const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                                 int training, int act, int accumulate_params, const float* part, int nrb, int dtype, void* ws,
                                 size_t ws_bytes, void* stream) {
  if (rows <= 0 || c <= 0 || nrb <= 0 || !part) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_bn_workspace(rows, c)) return RTSDS_ERR_WORKSPACE;
  if (dtype != RTSDS_BF16 || c % 8 != 0) return RTSDS_ERR_UNSUPPORTED;
  if (!(act == RTSDS_ACT_NONE || act == RTSDS_ACT_RELU || act == RTSDS_ACT_LEAKY)) return RTSDS_ERR_UNSUPPORTED;
  bn_bwd_launch<bf16, 8>(dy, x, nullptr, dx, nullptr, dgamma, dbeta, rows, c, gamma, beta, save_mean, save_invstd, training, act,
                         accumulate_params, bn_ws(ws, rows, c), (hipStream_t)stream, part, nrb);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

extern "C" int rtsds_bn_bwd_ld(const void* dy, long ldy, const void* x, const void* y, void* dx, void* dres, float* dgamma,
                               float* dbeta, long rows, int c, const float* gamma, const float* beta, const float* save_mean,
                               const float* save_invstd, int training, int act, int accumulate_params, int dtype, void* ws,
                               size_t ws_bytes, void* stream) {
  if (rows <= 0 || c <= 0 || ldy < c || ldy > (1L << 30)) return RTSDS_ERR_SHAPE;
  if (ldy != c && !(dtype == RTSDS_BF16 && c % 8 == 0 && ldy % 8 == 0)) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_bn_workspace(rows, c)) return RTSDS_ERR_WORKSPACE;
  if (!y && !(act == RTSDS_ACT_NONE || act == RTSDS_ACT_RELU || act == RTSDS_ACT_LEAKY)) return RTSDS_ERR_UNSUPPORTED;
  if (!y && act && dres) return RTSDS_ERR_UNSUPPORTED;  // residual: the mask needs y
  hipStream_t st = (hipStream_t)stream;
  const BnWs w = bn_ws(ws, rows, c);
  if (dtype == RTSDS_BF16) {
    if (c % 8 == 0) bn_bwd_launch<bf16, 8>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, beta, save_mean, save_invstd, training, act, accumulate_params, w, st, nullptr, 0, ldy);
    else bn_bwd_launch<bf16, 1>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, beta, save_mean, save_invstd, training, act, accumulate_params, w, st, nullptr, 0, ldy);
  } else if (dtype == RTSDS_F32) {
    if (c % 4 == 0) bn_bwd_launch<float, 4>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, beta, save_mean, save_invstd, training, act, accumulate_params, w, st, nullptr, 0, ldy);
    else bn_bwd_launch<float, 1>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, beta, save_mean, save_invstd, training, act, accumulate_params, w, st, nullptr, 0, ldy);
  } else return RTSDS_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
extern "C" int rtsds_bn_bwd(const void* dy, const void* x, const void* y, void* dx, void* dres, float* dgamma, float* dbeta,
                            long rows, int c, const float* gamma, const float* beta, const float* save_mean,
                            const float* save_invstd, int training, int act, int accumulate_params, int dtype, void* ws,
                            size_t ws_bytes, void* stream) {
  return rtsds_bn_bwd_ld(dy, c, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, beta, save_mean, save_invstd, training, act,
                         accumulate_params, dtype, ws, ws_bytes, stream);
}

// ---- BatchNorm + ReLU + MaxPool2d(3, 2, p) (the ResNet stem: bn1 -> relu -> maxpool,
// build_contextpath.py:15-18 / torchvision resnet.py; deeplabv2.py:106-110 with ceil mode).
// Forward: the pool reads the conv output and applies the BatchNorm scale / shift + ReLU to
// each window value (rounded to the storage dtype, exactly the value the separate bn_apply
// would have stored), so the full-resolution activation is never written; the window argmax
// bytes are stored for the backward, which gathers the pooled gradient inside the BatchNorm
// backward passes (GradPool) -- the full-resolution gradient is never written either.
template <typename T>
__global__ void __launch_bounds__(256) bn_relu_pool_fwd_kernel(const T* __restrict__ x, const float* __restrict__ scale,
                                                              const float* __restrict__ shift, T* __restrict__ y,
                                                              uint8_t* __restrict__ idx, int h, int w, int c, int ho, int wo, int p,
                                                              long total, FastDiv f_cv, FastDiv f_wo, FastDiv f_ho) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = c / V;
  const int nwg = gridDim.x, bx = blockIdx.x, xcd = bx & 7, qq = nwg >> 3, rr = nwg & 7;  // XCD-contiguous blocks
  const long lb = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bx >> 3);
  for (long i = lb * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const uint32_t ii = (uint32_t)i, q0 = fdiv(ii, f_cv), q1 = fdiv(q0, f_wo), img = fdiv(q1, f_ho);
    const int ch = (int)(ii - q0 * cv) * V;
    const int ow = (int)(q0 - q1 * wo), oh = (int)(q1 - img * ho);
    const int h0 = oh * 2 - p, w0 = ow * 2 - p;
    V16 v[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int hh = min(max(h0 + t / 3, 0), h - 1), ww = min(max(w0 + t % 3, 0), w - 1);
      v[t] = *(const V16*)(x + (((long)img * h + hh) * w + ww) * c + ch);
    }
    float sc[V], sh[V];
    load_coef<V>(scale, ch, c, sc);
    load_coef<V>(shift, ch, c, sh);
    float best[V];
    int bi[V];
#pragma unroll
    for (int j = 0; j < V; ++j) { best[j] = -INFINITY; bi[j] = -1; }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int hh = h0 + t / 3, ww = w0 + t % 3;
      if ((unsigned)hh >= (unsigned)h || (unsigned)ww >= (unsigned)w) continue;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float f = to_f(from_f<T>(fmaxf(fmaf(to_f(v[t][j]), sc[j], sh[j]), 0.f)));
        if (bi[j] < 0 || f > best[j] || (f != f && best[j] == best[j])) { best[j] = f; bi[j] = t; }
      }
    }
    V16 o;
    const long oi = (((long)img * ho + oh) * wo + ow) * c + ch;
    unsigned long long ib = 0;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      o[j] = from_f<T>(best[j]);
      ib |= (unsigned long long)(bi[j] < 0 ? 0 : bi[j]) << (8 * j);
    }
    *(V16*)(y + oi) = o;
    *(unsigned long long*)(idx + oi) = ib;
  }
}
static bool bn_pool_ok(int n, int h, int w, int c, int ho, int wo, int p, int dtype) {
  return dtype == RTSDS_BF16 && c % 8 == 0 && n > 0 && ho > 0 && wo > 0 && (p == 0 || p == 1) &&
         (long)n * h * w * c < (1L << 31) && (long)n * ho * wo * c < (1L << 31);
}
extern "C" int rtsds_bn_relu_maxpool_fwd(const void* x, void* y, uint8_t* idx, int n, int h, int w, int c, int ho, int wo, int p,
                                         const float* gamma, const float* beta, float* running_mean, float* running_var,
                                         long long* num_batches_tracked, float* save_mean, float* save_invstd, float momentum,
                                         float eps, int training, const float* stats_part, int stats_nrb, int dtype, void* ws,
                                         size_t ws_bytes, void* stream) {
  const long rows = (long)n * h * w;
  if (!bn_pool_ok(n, h, w, c, ho, wo, p, dtype)) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_bn_workspace(rows, c)) return RTSDS_ERR_WORKSPACE;
  if (!training && (!running_mean || !running_var)) return RTSDS_ERR_UNSUPPORTED;
  if (training && (!save_mean || !save_invstd)) return RTSDS_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  const BnWs wsb = bn_ws(ws, rows, c);
  float* scale = wsb.coef;
  float* shift = wsb.coef + c;
  long long* nbt = training ? num_batches_tracked : nullptr;
  if (training) {
    int rb = stats_nrb;
    const float* part = stats_part;
    if (!part) {
      rb = bn_rb(rows, c, 8);
      hipLaunchKernelGGL((bn_stats_kernel<bf16, 8>), dim3(rb, rt_cdiv(c, 256 * 8)), dim3(256), 0, st, (const bf16*)x, wsb.part, rows, c);
      part = wsb.part;
    }
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(c), dim3(256), 0, st, part, rb, c, rows, gamma, beta, running_mean, running_var,
                       save_mean, save_invstd, scale, shift, momentum, eps, nbt);
  } else {
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3(rt_cdiv(c, 256)), dim3(256), 0, st, c, gamma, beta, running_mean, running_var,
                       scale, shift, save_mean, save_invstd, eps);
  }
  const long total = (long)n * ho * wo * (c / 8);
  const int blocks = (int)std::max<long>(1, std::min<long>((total + 255) / 256, 1L << 20));
  hipLaunchKernelGGL(bn_relu_pool_fwd_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (const bf16*)x, (const float*)scale,
                     (const float*)shift, (bf16*)y, idx, h, w, c, ho, wo, p, total, fastdiv_make(c / 8), fastdiv_make(wo),
                     fastdiv_make(ho));
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
extern "C" int rtsds_bn_relu_maxpool_bwd(const void* dy_pool, const uint8_t* idx, const void* x, void* dx, float* dgamma,
                                         float* dbeta, int n, int h, int w, int c, int ho, int wo, int p, const float* gamma,
                                         const float* beta, const float* save_mean, const float* save_invstd, int training,
                                         int accumulate_params, int dtype, void* ws, size_t ws_bytes, void* stream) {
  const long rows = (long)n * h * w;
  if (!bn_pool_ok(n, h, w, c, ho, wo, p, dtype)) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_bn_workspace(rows, c)) return RTSDS_ERR_WORKSPACE;
  const GradPool<bf16> gs{(const bf16*)dy_pool, idx, c, h, w, ho, wo, p, fastdiv_make(w), fastdiv_make(h)};
  bn_bwd_launch<bf16, 8, GradPool<bf16>>(gs, x, nullptr, dx, nullptr, dgamma, dbeta, rows, c, gamma, beta, save_mean, save_invstd,
                                         training, RTSDS_ACT_RELU, accumulate_params, bn_ws(ws, rows, c), (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// Eval-mode BatchNorm folded into the producing conv (rtsds_conv2d_fwd_bn):
// scale = gamma / sqrt(running_var + eps), shift = beta + (bias - running_mean) * scale.
__global__ void bn_fold_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                               const float* __restrict__ rm, const float* __restrict__ rv,
                               const float* __restrict__ bias, float eps, int c, float* __restrict__ scale,
                               float* __restrict__ shift) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  const float s = (gamma ? gamma[i] : 1.f) / sqrtf(rv[i] + eps);
  scale[i] = s;
  shift[i] = fmaf((bias ? bias[i] : 0.f) - rm[i], s, beta ? beta[i] : 0.f);
}

extern "C" int rtsds_bn_fold(const float* gamma, const float* beta, const float* running_mean,
                             const float* running_var, const float* conv_bias, float eps, int c, float* scale,
                             float* shift, void* stream) {
  if (c <= 0) return RTSDS_ERR_SHAPE;
  if (!running_mean || !running_var || !scale || !shift) return RTSDS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(bn_fold_kernel, dim3(rt_cdiv(c, 256)), dim3(256), 0, (hipStream_t)stream, gamma, beta, running_mean,
                     running_var, conv_bias, eps, c, scale, shift);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
