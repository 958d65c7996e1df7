// BatchNorm2d (train: batch statistics; eval: running statistics) over NHWC [rows][c],
// fused with an optional residual add and ReLU / LeakyReLU, plus its backward.
//
// Statistics are single-pass: each thread keeps shifted sums (shift = its first sample) for
// its channels, which are merged across threads / blocks with Chan's parallel formula, so
// large-mean conv outputs (the reference feeds 0-255-scale normalised images,
// main.py:69-72) do not cancel catastrophically.  Three launches per direction:
// partial statistics (grid over row chunks) -> per-channel finalize -> vectorised apply.
#include "common.h"
#include <algorithm>

static const int kBnMaxRB = 512;  // row blocks of the partial-statistics pass

// Threads of a 256-block are laid out [row group][channel vector]; TPR = threads per row.
template <int VEC> struct BnLayout {
  int tpr, rpi;  // threads per row, rows per block iteration
  RT_DEV BnLayout(int c) {
    tpr = (c + VEC - 1) / VEC;
    if (tpr > 256) tpr = 256;
    rpi = 256 / tpr;
  }
};

template <typename T, int VEC>
RT_DEV void load_vec(const T* p, float* v, int cvalid) {
  if (VEC == VecT<T>::N && cvalid >= VEC) {
    typename VecT<T>::v16 t = *(const typename VecT<T>::v16*)p;
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = to_f(t[j]);
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = j < cvalid ? to_f(p[j]) : 0.f;
  }
}
template <typename T, int VEC>
RT_DEV void store_vec(T* p, const float* v, int cvalid) {
  if (VEC == VecT<T>::N && cvalid >= VEC) {
    typename VecT<T>::v16 t;
#pragma unroll
    for (int j = 0; j < VEC; ++j) t[j] = from_f<T>(v[j]);
    *(typename VecT<T>::v16*)p = t;
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      if (j < cvalid) p[j] = from_f<T>(v[j]);
  }
}

RT_DEV void chan_merge(float& na, float& ma, float& Ma, float nb, float mb, float Mb) {
  if (nb == 0.f) return;
  if (na == 0.f) { na = nb; ma = mb; Ma = Mb; return; }
  const float n = na + nb, d = mb - ma;
  ma += d * (nb / n);
  Ma += Mb + d * d * (na * nb / n);
  na = n;
}

// Pass 1 (forward): part[(rb * c + ch) * 3 + {0,1,2}] = (count, mean, M2) of block rb.
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
        float* o = part + ((long)blockIdx.x * c + ch0 + j) * 3;
        o[0] = n; o[1] = m; o[2] = M;
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
__global__ void __launch_bounds__(64) bn_finalize_kernel(const float* __restrict__ part, int nrb, int c, long rows, const float* gamma,
                                   const float* beta, float* rmean, float* rvar, float* smean, float* sinv,
                                   float* scale, float* shift, float momentum, float eps) {
  const int ch = blockIdx.x, lane = threadIdx.x;
  float n = 0.f, m = 0.f, M = 0.f;
  for (int b = lane; b < nrb; b += 64) {
    const float* p = part + ((long)b * c + ch) * 3;
    chan_merge(n, m, M, p[0], p[1], p[2]);
  }
  chan_merge_shfl(n, m, M);
  if (lane != 0) return;
  const float var = M / (float)rows;
  const float inv = 1.0f / sqrtf(var + eps);
  smean[ch] = m;
  sinv[ch] = inv;
  if (rmean) rmean[ch] = (1.f - momentum) * rmean[ch] + momentum * m;
  if (rvar) {
    const float unb = rows > 1 ? M / (float)(rows - 1) : var;
    rvar[ch] = (1.f - momentum) * rvar[ch] + momentum * unb;
  }
  const float g = gamma ? gamma[ch] : 1.f, b = beta ? beta[ch] : 0.f;
  scale[ch] = g * inv;
  shift[ch] = b - m * g * inv;
}

__global__ void bn_eval_coef_kernel(int c, const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                    float* scale, float* shift, float* smean, float* sinv, float eps) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= c) return;
  const float inv = 1.0f / sqrtf(rvar[ch] + eps);
  if (smean) smean[ch] = rmean[ch];
  if (sinv) sinv[ch] = inv;
  const float g = gamma ? gamma[ch] : 1.f, b = beta ? beta[ch] : 0.f;
  scale[ch] = g * inv;
  shift[ch] = b - rmean[ch] * g * inv;
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

// Pass 3 (forward): y = act(x * scale + shift [+ res]).
template <typename T, int VEC>
__global__ void __launch_bounds__(256) bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ y,
                                                        const float* __restrict__ scale, const float* __restrict__ shift,
                                                        long rows, int c, int act) {
  const int cvn = (c + VEC - 1) / VEC;
  const long total = rows * cvn;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cvn;
    const int ch0 = (int)(i - r * cvn) * VEC;
    const long off = r * c + ch0;
    float v[VEC], rv[VEC];
    load_vec<T, VEC>(x + off, v, c - ch0);
    if (res) load_vec<T, VEC>(res + off, rv, c - ch0);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const int ch = min(ch0 + j, c - 1);
      float o = fmaf(v[j], scale[ch], shift[ch]);
      if (res) o += rv[j];
      v[j] = act_f(o, act);
    }
    store_vec<T, VEC>(y + off, v, c - ch0);
  }
}

// Backward pass 1: part[(rb*c+ch)*2 + {0,1}] = (sum g, sum g*(x-mean)) with g = dy*act'(y).
template <typename T, int VEC>
__global__ void __launch_bounds__(256) bn_bwd_stats_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const T* __restrict__ y, const float* __restrict__ mean,
                                                            float* __restrict__ part, long rows, int c, int act) {
  __shared__ float sh[2][256][VEC];
  const int cbase = blockIdx.y * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const BnLayout<VEC> L(cl);
  const int tid = threadIdx.x, cv = tid % L.tpr, rg = tid / L.tpr;
  const int ch0 = cbase + cv * VEC;
  const bool active = rg < L.rpi && cv * VEC < cl;
  float sg[VEC], sgx[VEC], mu[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { sg[j] = 0.f; sgx[j] = 0.f; mu[j] = active ? mean[min(ch0 + j, c - 1)] : 0.f; }
  if (active) {
    for (long r = (long)blockIdx.x * L.rpi + rg; r < rows; r += (long)gridDim.x * L.rpi) {
      float g[VEC], xv[VEC], yv[VEC];
      load_vec<T, VEC>(dy + r * c + ch0, g, c - ch0);
      load_vec<T, VEC>(x + r * c + ch0, xv, c - ch0);
      if (act) load_vec<T, VEC>(y + r * c + ch0, yv, c - ch0);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float gg = act ? g[j] * act_grad(yv[j], act) : g[j];
        sg[j] += gg;
        sgx[j] = fmaf(gg, xv[j] - mu[j], sgx[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) { sh[0][tid][j] = sg[j]; sh[1][tid][j] = sgx[j]; }
  __syncthreads();
  if (rg == 0 && cv * VEC < cl) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float a = sh[0][tid][j], b = sh[1][tid][j];
      for (int gi = 1; gi < L.rpi; ++gi) {
        a += sh[0][gi * L.tpr + cv][j];
        b += sh[1][gi * L.tpr + cv][j];
      }
      if (ch0 + j < c) {
        float* o = part + ((long)blockIdx.x * c + ch0 + j) * 2;
        o[0] = a; o[1] = b;
      }
    }
  }
}

// Backward pass 2: coefficients  dx = A*g + B*(x-mean) + C  per channel (one wave each).
__global__ void __launch_bounds__(64) bn_bwd_finalize_kernel(const float* __restrict__ part, int nrb, int c, long rows, const float* gamma,
                                       const float* smean, const float* sinv, float* dgamma, float* dbeta,
                                       float* coefA, float* coefB, float* coefC, int training, int accumulate) {
  const int ch = blockIdx.x, lane = threadIdx.x;
  float sg = 0.f, sgx = 0.f;
  for (int b = lane; b < nrb; b += 64) {
    sg += part[((long)b * c + ch) * 2];
    sgx += part[((long)b * c + ch) * 2 + 1];
  }
  sg = wave_sum(sg);
  sgx = wave_sum(sgx);
  if (lane != 0) return;
  const float inv = sinv[ch], g = gamma ? gamma[ch] : 1.f;
  if (dgamma) dgamma[ch] = accumulate ? dgamma[ch] + sgx * inv : sgx * inv;
  if (dbeta) dbeta[ch] = accumulate ? dbeta[ch] + sg : sg;
  const float a = g * inv;
  const float invn = 1.f / (float)rows;
  coefA[ch] = a;
  coefB[ch] = training ? -a * inv * inv * sgx * invn : 0.f;
  coefC[ch] = training ? -a * sg * invn : 0.f;
  (void)smean;
}

// Backward pass 3: dx = A*g + B*(x - mean) + C;  dres = g.
template <typename T, int VEC>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                            const T* __restrict__ y, T* __restrict__ dx, T* __restrict__ dres,
                                                            const float* __restrict__ mean, const float* __restrict__ A,
                                                            const float* __restrict__ B, const float* __restrict__ C,
                                                            long rows, int c, int act) {
  const int cvn = (c + VEC - 1) / VEC;
  const long total = rows * cvn;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cvn;
    const int ch0 = (int)(i - r * cvn) * VEC;
    const long off = r * c + ch0;
    float g[VEC], xv[VEC], yv[VEC], o[VEC];
    load_vec<T, VEC>(dy + off, g, c - ch0);
    load_vec<T, VEC>(x + off, xv, c - ch0);
    if (act) load_vec<T, VEC>(y + off, yv, c - ch0);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const int ch = min(ch0 + j, c - 1);
      if (act) g[j] *= act_grad(yv[j], act);
      o[j] = fmaf(A[ch], g[j], fmaf(B[ch], xv[j] - mean[ch], C[ch]));
    }
    if (dx) store_vec<T, VEC>(dx + off, o, c - ch0);
    if (dres) store_vec<T, VEC>(dres + off, g, c - ch0);
  }
}

// ------------------------------------------------------------------ host
static int bn_rb(long rows, int c, int vec) {
  int tpr = (c + vec - 1) / vec;
  if (tpr > 256) tpr = 256;
  const int rpi = 256 / tpr;
  long need = (rows + rpi - 1) / rpi;
  // ~1-2k blocks overall, at least 4 row-iterations per thread when rows are large
  long rb = std::min<long>(need, kBnMaxRB);
  rb = std::max<long>(1, std::min<long>(rb, (need + 3) / 4));
  return (int)rb;
}

extern "C" size_t rtsds_bn_workspace(long rows, int c) {
  (void)rows;
  // partials (3 floats x RB x c) + 5 per-channel coefficient arrays
  return (size_t)kBnMaxRB * c * 3 * 4 + (size_t)c * 5 * 4 + 256;
}

template <typename T, int VEC>
static void bn_fwd_launch(const void* x, const void* res, void* y, long rows, int c, const float* gamma, const float* beta,
                          float* rm, float* rv, float* sm, float* si, float mom, float eps, int training, int act,
                          const float* pre, int pre_nrb, float* part, float* scale, float* shift, hipStream_t st) {
  if (training) {
    int rb = pre_nrb;
    if (pre) {
      part = (float*)pre;  // statistics already produced by the conv epilogue
    } else {
      rb = bn_rb(rows, c, VEC);
      hipLaunchKernelGGL((bn_stats_kernel<T, VEC>), dim3(rb, rt_cdiv(c, 256 * VEC)), dim3(256), 0, st, (const T*)x, part, rows, c);
    }
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(c), dim3(64), 0, st, part, rb, c, rows, gamma, beta, rm, rv,
                       sm, si, scale, shift, mom, eps);
  } else {
    hipLaunchKernelGGL(bn_eval_coef_kernel, dim3(rt_cdiv(c, 256)), dim3(256), 0, st, c, gamma, beta, rm, rv, scale, shift, sm, si, eps);
  }
  const long total = rows * ((c + VEC - 1) / VEC);
  const int blocks = (int)std::min<long>(8192, (total + 255) / 256);
  hipLaunchKernelGGL((bn_apply_kernel<T, VEC>), dim3(blocks), dim3(256), 0, st, (const T*)x, (const T*)res, (T*)y, scale, shift,
                     rows, c, act);
}

extern "C" int rtsds_bn_fwd(const void* x, const void* res, void* y, long rows, int c, const float* gamma, const float* beta,
                            float* running_mean, float* running_var, float* save_mean, float* save_invstd, float momentum,
                            float eps, int training, int act, const float* stats_part, int stats_nrb, int dtype, void* ws,
                            size_t ws_bytes, void* stream) {
  if (rows <= 0 || c <= 0) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_bn_workspace(rows, c)) return RTSDS_ERR_WORKSPACE;
  if (!training && (!running_mean || !running_var)) return RTSDS_ERR_UNSUPPORTED;
  if (training && (!save_mean || !save_invstd)) return RTSDS_ERR_UNSUPPORTED;
  if (c > 65535 * 256) return RTSDS_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  float* scale = part + (size_t)kBnMaxRB * c * 3;
  float* shift = scale + c;
  if (dtype == RTSDS_BF16) {
    if (c % 8 == 0) bn_fwd_launch<bf16, 8>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, part, scale, shift, st);
    else bn_fwd_launch<bf16, 1>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, part, scale, shift, st);
  } else if (dtype == RTSDS_F32) {
    if (c % 4 == 0) bn_fwd_launch<float, 4>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, part, scale, shift, st);
    else bn_fwd_launch<float, 1>(x, res, y, rows, c, gamma, beta, running_mean, running_var, save_mean, save_invstd, momentum, eps, training, act, stats_part, stats_nrb, part, scale, shift, st);
  } else return RTSDS_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

template <typename T, int VEC>
static void bn_bwd_launch(const void* dy, const void* x, const void* y, void* dx, void* dres, float* dgamma, float* dbeta,
                          long rows, int c, const float* gamma, const float* smean, const float* sinv, int training,
                          int act, int accumulate, float* part, float* A, float* B, float* C, hipStream_t st) {
  const int rb = bn_rb(rows, c, VEC);
  hipLaunchKernelGGL((bn_bwd_stats_kernel<T, VEC>), dim3(rb, rt_cdiv(c, 256 * VEC)), dim3(256), 0, st, (const T*)dy, (const T*)x, (const T*)y, smean,
                     part, rows, c, act);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(c), dim3(64), 0, st, part, rb, c, rows, gamma, smean, sinv,
                     dgamma, dbeta, A, B, C, training, accumulate);
  if (dx || dres) {
    const long total = rows * ((c + VEC - 1) / VEC);
    const int blocks = (int)std::min<long>(8192, (total + 255) / 256);
    hipLaunchKernelGGL((bn_bwd_apply_kernel<T, VEC>), dim3(blocks), dim3(256), 0, st, (const T*)dy, (const T*)x, (const T*)y,
                       (T*)dx, (T*)dres, smean, A, B, C, rows, c, act);
  }
}

extern "C" int rtsds_bn_bwd(const void* dy, const void* x, const void* y, void* dx, void* dres, float* dgamma, float* dbeta,
                            long rows, int c, const float* gamma, const float* save_mean, const float* save_invstd,
                            int training, int act, int accumulate_params, int dtype, void* ws, size_t ws_bytes, void* stream) {
  if (rows <= 0 || c <= 0) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_bn_workspace(rows, c)) return RTSDS_ERR_WORKSPACE;
  if (act && !y) return RTSDS_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  float* A = part + (size_t)kBnMaxRB * c * 3;
  float* B = A + c;
  float* C = B + c;
  if (dtype == RTSDS_BF16) {
    if (c % 8 == 0) bn_bwd_launch<bf16, 8>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, save_mean, save_invstd, training, act, accumulate_params, part, A, B, C, st);
    else bn_bwd_launch<bf16, 1>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, save_mean, save_invstd, training, act, accumulate_params, part, A, B, C, st);
  } else if (dtype == RTSDS_F32) {
    if (c % 4 == 0) bn_bwd_launch<float, 4>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, save_mean, save_invstd, training, act, accumulate_params, part, A, B, C, st);
    else bn_bwd_launch<float, 1>(dy, x, y, dx, dres, dgamma, dbeta, rows, c, gamma, save_mean, save_invstd, training, act, accumulate_params, part, A, B, C, st);
  } else return RTSDS_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
