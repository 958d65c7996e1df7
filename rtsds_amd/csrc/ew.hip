// Memory-bound kernels of the RTSDS hot path (gfx950): layout/dtype conversion, max-pool,
// global average pool, channel attention scaling, bilinear resize, channel softmax,
// cross-entropy with ignore_index, BCE-with-logits, fused Adam, argmax / pixel accuracy.
// All activations are NHWC; per-pixel channel vectors are contiguous.
#include "common.h"
#include <algorithm>
#include <climits>
#include <cmath>

static inline int ew_blocks(long work, int per_block = 256, int cap = 8192) {
  return (int)std::max<long>(1, std::min<long>(cap, (work + per_block - 1) / per_block));
}
#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)
// XCD-aware variant: workgroups b and b + 8 run on one XCD, so logical block = the XCD's
// contiguous run (bijective) -- neighbouring output rows (which share input rows) stay in one
// XCD's L2.
RT_DEV long xcd_block() {
  const int nwg = gridDim.x, b = blockIdx.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}
#define GRID_STRIDE_XCD(i, n) for (long i = xcd_block() * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)
#define DISPATCH_T(dtype, ...)                                \
  do {                                                        \
    if ((dtype) == RTSDS_BF16) { typedef bf16 T; __VA_ARGS__; } \
    else if ((dtype) == RTSDS_F32) { typedef float T; __VA_ARGS__; } \
    else return RTSDS_ERR_UNSUPPORTED;                        \
  } while (0)
#define RET_LAUNCH() return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH

// ------------------------------------------------------------------ layout / dtype
// NCHW fp32 (the reference's input tensors) -> NHWC T.
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int n, int c, long hw) {
  const long total = (long)n * c * hw;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    const long p = i / c;
    const long img = p / hw, s = p - img * hw;
    y[i] = from_f<T>(x[(img * c + ch) * hw + s]);
  }
}
extern "C" int rtsds_nchw_to_nhwc(const float* x, void* y, int n, int c, int h, int w, int dtype, void* stream) {
  const long total = (long)n * c * h * w;
  if (total <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, hipLaunchKernelGGL(nchw_to_nhwc_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, (hipStream_t)stream, x, (T*)y, n, c, (long)h * w));
  RET_LAUNCH();
}

// NCHW fp32 -> NHWC T with channel pitch cp >= c, channels c..cp-1 zero: the image batch in
// the layout its convs gather (3 -> 4 channels: the superpixel view of the stem / spatial-path
// convs, conv.hip sp_path), so they skip their own pad pass.  One thread per pixel.
template <typename T, int CP>
__global__ void nchw_to_nhwc_pad_kernel(const float* __restrict__ x, T* __restrict__ y, int c, long hw, long pixels) {
  GRID_STRIDE(p, pixels) {
    const long img = p / hw, s = p - img * hw;
    T v[CP];
#pragma unroll
    for (int ch = 0; ch < CP; ++ch) v[ch] = from_f<T>(ch < c ? x[(img * c + ch) * hw + s] : 0.f);
    if constexpr (CP * sizeof(T) == 8) {
      typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
      *(u32x2*)(y + p * CP) = __builtin_bit_cast(u32x2, v);
    } else {
#pragma unroll
      for (int ch = 0; ch < CP; ++ch) y[p * CP + ch] = v[ch];
    }
  }
}
// Same for planes of a multiple of 4 pixels: 4 pixels per thread, one 16-B load per channel
// plane and 16-B stores, the image index from the grid (no 64-bit divisions).
template <typename T>
__global__ void nchw_to_nhwc_pad4_x4_kernel(const float* __restrict__ x, T* __restrict__ y, int c, int hw4) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  typedef __attribute__((ext_vector_type(4))) float f32x4;
  const int img = blockIdx.y;
  const float* xi = x + (long)img * c * hw4 * 4;
  T* yi = y + (long)img * hw4 * 16;
  for (int q = blockIdx.x * 256 + threadIdx.x; q < hw4; q += gridDim.x * 256) {
    f32x4 v[4];
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) v[ch] = ch < c ? ((const f32x4*)(xi + (long)ch * hw4 * 4))[q] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 16 / V; ++k) {
      V16 r;
#pragma unroll
      for (int j = 0; j < V; ++j) r[j] = from_f<T>(v[(k * V + j) & 3][(k * V + j) >> 2]);
      ((V16*)(yi + (long)q * 16))[k] = r;
    }
  }
}
extern "C" int rtsds_nchw_to_nhwc_pad(const float* x, void* y, int n, int c, int h, int w, int pitch, int dtype, void* stream) {
  const long px = (long)n * h * w;
  if (px <= 0 || c <= 0 || pitch != 4 || c > pitch) return RTSDS_ERR_UNSUPPORTED;
  const long hw = (long)h * w;
  // 16-B vector loads / stores: only for 16-B aligned bases (a view with a storage offset
  // that is not a multiple of 4 floats takes the per-pixel kernel)
  if (hw % 4 == 0 && hw / 4 < INT_MAX && n <= 65535 && (((uintptr_t)x | (uintptr_t)y) & 15) == 0) {
    const int hw4 = (int)(hw / 4);
    DISPATCH_T(dtype, hipLaunchKernelGGL((nchw_to_nhwc_pad4_x4_kernel<T>), dim3(std::min(rt_cdiv(hw4, 256), 4096), n), dim3(256), 0,
                                         (hipStream_t)stream, x, (T*)y, c, hw4));
  } else {
    DISPATCH_T(dtype, hipLaunchKernelGGL((nchw_to_nhwc_pad_kernel<T, 4>), dim3(ew_blocks(px)), dim3(256), 0, (hipStream_t)stream, x,
                                         (T*)y, c, hw, px));
  }
  RET_LAUNCH();
}

// dst (dtype_dst) = src (dtype_src), elementwise.
template <typename S, typename D>
__global__ void cast_kernel(const S* __restrict__ s, D* __restrict__ d, long n) {
  GRID_STRIDE(i, n) d[i] = from_f<D>(to_f(s[i]));
}
extern "C" int rtsds_cast(const void* src, int src_dtype, void* dst, int dst_dtype, long n, void* stream) {
  if (n <= 0) return n == 0 ? RTSDS_OK : RTSDS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  const int b = ew_blocks(n);
  if (src_dtype == RTSDS_F32 && dst_dtype == RTSDS_BF16) hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(b), dim3(256), 0, st, (const float*)src, (bf16*)dst, n);
  else if (src_dtype == RTSDS_BF16 && dst_dtype == RTSDS_F32) hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(b), dim3(256), 0, st, (const bf16*)src, (float*)dst, n);
  else if (src_dtype == RTSDS_F32 && dst_dtype == RTSDS_F32) hipLaunchKernelGGL((cast_kernel<float, float>), dim3(b), dim3(256), 0, st, (const float*)src, (float*)dst, n);
  else if (src_dtype == RTSDS_BF16 && dst_dtype == RTSDS_BF16) hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(b), dim3(256), 0, st, (const bf16*)src, (bf16*)dst, n);
  else if (src_dtype == RTSDS_F32 && dst_dtype == RTSDS_F16) hipLaunchKernelGGL((cast_kernel<float, f16>), dim3(b), dim3(256), 0, st, (const float*)src, (f16*)dst, n);
  else if (src_dtype == RTSDS_F16 && dst_dtype == RTSDS_F32) hipLaunchKernelGGL((cast_kernel<f16, float>), dim3(b), dim3(256), 0, st, (const f16*)src, (float*)dst, n);
  else return RTSDS_ERR_UNSUPPORTED;
  RET_LAUNCH();
}

// Channel-slice copy: dst[r][doff + j] = src[r][soff + j], j < cnt  (torch.cat / its backward
// split along channels, build_bisenet.py:72,153).
template <typename T>
__global__ void copy_channels_kernel(const T* __restrict__ s, int sld, int soff, T* __restrict__ d, int dld, int doff, long rows, int cnt,
                                     int acc) {
  const long total = rows * cnt;
  GRID_STRIDE(i, total) {
    const long r = i / cnt;
    const int j = (int)(i - r * cnt);
    T* o = d + r * dld + doff + j;
    const T v = s[r * sld + soff + j];
    *o = acc ? from_f<T>(to_f(*o) + to_f(v)) : v;
  }
}
template <typename T>
__global__ void copy_channels_vec_kernel(const T* __restrict__ s, int sld, int soff, T* __restrict__ d, int dld, int doff, long rows, int cnt,
                                         int acc) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = cnt / V;
  const long total = rows * cv;
  GRID_STRIDE(i, total) {
    const long r = i / cv;
    const int j = (int)(i - r * cv) * V;
    V16* o = (V16*)(d + r * dld + doff + j);
    V16 v = *(const V16*)(s + r * sld + soff + j);
    if (acc) {
      const V16 a = *o;
#pragma unroll
      for (int q = 0; q < V; ++q) v[q] = from_f<T>(to_f(a[q]) + to_f(v[q]));
    }
    *o = v;
  }
}
extern "C" int rtsds_copy_channels(const void* src, int src_ld, int src_off, void* dst, int dst_ld, int dst_off, long rows,
                                   int cnt, int accumulate, int dtype, void* stream) {
  if (rows <= 0 || cnt <= 0) return RTSDS_ERR_SHAPE;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    constexpr int V = VecT<T>::N;
    if (cnt % V == 0 && src_ld % V == 0 && dst_ld % V == 0 && src_off % V == 0 && dst_off % V == 0)
      hipLaunchKernelGGL(copy_channels_vec_kernel<T>, dim3(ew_blocks(rows * cnt / V)), dim3(256), 0, st, (const T*)src, src_ld, src_off, (T*)dst, dst_ld, dst_off, rows, cnt,
                         accumulate ? 1 : 0);
    else
      hipLaunchKernelGGL(copy_channels_kernel<T>, dim3(ew_blocks(rows * cnt)), dim3(256), 0, st, (const T*)src, src_ld, src_off, (T*)dst, dst_ld, dst_off, rows, cnt,
                         accumulate ? 1 : 0);
  });
  RET_LAUNCH();
}

// ------------------------------------------------------------------ activations (pointwise)
// act: 1 relu, 2 leaky(0.2), 3 sigmoid.  Backward uses the forward OUTPUT y.
template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long n, int act) {
  GRID_STRIDE(i, n) {
    float v = to_f(x[i]);
    if (act == 1) v = fmaxf(v, 0.f);
    else if (act == 2) v = v > 0.f ? v : 0.2f * v;
    else if (act == 3) v = 1.f / (1.f + expf(-v));
    y[i] = from_f<T>(v);
  }
}
template <typename T>
__global__ void act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx, long n, int act, float alpha) {
  GRID_STRIDE(i, n) {
    const float g = to_f(dy[i]);
    float r;
    if (act == 1) r = to_f(y[i]) > 0.f ? g : 0.f;
    else if (act == 2) r = to_f(y[i]) > 0.f ? g : 0.2f * g;
    else if (act == 3) { const float s = to_f(y[i]); r = g * s * (1.f - s); }
    else r = alpha * g;  // act 0: scale (gradient reversal, model.py:9-17)
    dx[i] = from_f<T>(r);
  }
}
extern "C" int rtsds_act_fwd(const void* x, void* y, long n, int act, int dtype, void* stream) {
  if (n <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, hipLaunchKernelGGL(act_fwd_kernel<T>, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, n, act));
  RET_LAUNCH();
}
extern "C" int rtsds_act_bwd(const void* dy, const void* y, void* dx, long n, int act, float alpha, int dtype, void* stream) {
  if (n <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, hipLaunchKernelGGL(act_bwd_kernel<T>, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, (const T*)dy, (const T*)y, (T*)dx, n, act, alpha));
  RET_LAUNCH();
}

// ------------------------------------------------------------------ max pool
// torchvision / deeplab max pool (build_contextpath.py:21, deeplabv2.py:79): padded taps are
// skipped, first maximum wins (ATen CPU scan order), NaN propagates.  idx = tap index.
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int n, int h, int w,
                                   int c, int ho, int wo, int k, int s, int p) {
  const long total = (long)n * ho * wo * c;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    long q = i / c;
    const int ow = (int)(q % wo); q /= wo;
    const int oh = (int)(q % ho);
    const int img = (int)(q / ho);
    const int h0 = oh * s - p, w0 = ow * s - p;
    float best = -INFINITY;
    int bi = -1;
    for (int a = 0; a < k; ++a) {
      const int hh = h0 + a;
      if (hh < 0 || hh >= h) continue;
      for (int b = 0; b < k; ++b) {
        const int ww = w0 + b;
        if (ww < 0 || ww >= w) continue;
        const float v = to_f(x[(((long)img * h + hh) * w + ww) * c + ch]);
        if (bi < 0 || v > best || v != v) { best = v; bi = a * k + b; if (v != v) goto done; }
      }
    }
  done:
    y[i] = from_f<T>(best);
    idx[i] = (uint8_t)(bi < 0 ? 0 : bi);
  }
}
// Gather backward (deterministic): each input element sums the windows that chose it.
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx, int n, int h,
                                   int w, int c, int ho, int wo, int k, int s, int p) {
  const long total = (long)n * h * w * c;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    long q = i / c;
    const int iw = (int)(q % w); q /= w;
    const int ih = (int)(q % h);
    const int img = (int)(q / h);
    const int oh_lo = max(0, (ih + p - k + s) / s), oh_hi = min(ho - 1, (ih + p) / s);
    const int ow_lo = max(0, (iw + p - k + s) / s), ow_hi = min(wo - 1, (iw + p) / s);
    float acc = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int a = ih - (oh * s - p);
      if (a < 0 || a >= k) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int b = iw - (ow * s - p);
        if (b < 0 || b >= k) continue;
        const long o = (((long)img * ho + oh) * wo + ow) * c + ch;
        if (idx[o] == a * k + b) acc += to_f(dy[o]);
      }
    }
    dx[i] = from_f<T>(acc);
  }
}

// Vector variants (c % V == 0): one thread per (pixel, 16-B channel vector).
template <typename T>
__global__ void maxpool_fwd_vec(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int n, int h, int w,
                                int c, int ho, int wo, int k, int s, int p) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = c / V;
  const long total = (long)n * ho * wo * cv;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % cv) * V;
    long q = i / cv;
    const int ow = (int)(q % wo); q /= wo;
    const int oh = (int)(q % ho);
    const int img = (int)(q / ho);
    const int h0 = oh * s - p, w0 = ow * s - p;
    float best[V];
    int bi[V];
#pragma unroll
    for (int j = 0; j < V; ++j) { best[j] = -INFINITY; bi[j] = -1; }
    for (int a = 0; a < k; ++a) {
      const int hh = h0 + a;
      if (hh < 0 || hh >= h) continue;
      for (int b = 0; b < k; ++b) {
        const int ww = w0 + b;
        if (ww < 0 || ww >= w) continue;
        const V16 v = *(const V16*)(x + (((long)img * h + hh) * w + ww) * c + ch);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float f = to_f(v[j]);
          if (bi[j] < 0 || f > best[j] || (f != f && best[j] == best[j])) { best[j] = f; bi[j] = a * k + b; }
        }
      }
    }
    V16 o;
    const long oi = (((long)img * ho + oh) * wo + ow) * c + ch;
#pragma unroll
    for (int j = 0; j < V; ++j) { o[j] = from_f<T>(best[j]); idx[oi + j] = (uint8_t)(bi[j] < 0 ? 0 : bi[j]); }
    *(V16*)(y + oi) = o;
  }
}
template <typename T>
__global__ void maxpool_bwd_vec(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx, int n, int h, int w,
                                int c, int ho, int wo, int k, int s, int p) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = c / V;
  const long total = (long)n * h * w * cv;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % cv) * V;
    long q = i / cv;
    const int iw = (int)(q % w); q /= w;
    const int ih = (int)(q % h);
    const int img = (int)(q / h);
    const int oh_lo = max(0, (ih + p - k + s) / s), oh_hi = min(ho - 1, (ih + p) / s);
    const int ow_lo = max(0, (iw + p - k + s) / s), ow_hi = min(wo - 1, (iw + p) / s);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int a = ih - (oh * s - p);
      if (a < 0 || a >= k) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int b = iw - (ow * s - p);
        if (b < 0 || b >= k) continue;
        const long o = (((long)img * ho + oh) * wo + ow) * c + ch;
        const V16 g = *(const V16*)(dy + o);
        const int want = a * k + b;
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (idx[o + j] == want) acc[j] += to_f(g[j]);
      }
    }
    V16 r;
#pragma unroll
    for (int j = 0; j < V; ++j) r[j] = from_f<T>(acc[j]);
    *(V16*)(dx + (((long)img * h + ih) * w + iw) * c + ch) = r;
  }
}

// 3x3 windows (the ResNet stem pool, build_contextpath.py via torchvision resnet.py:
// MaxPool2d(3, 2, 1)): all nine 16-B window loads issued unconditionally from clamped
// coordinates before any compare (the generic loop's bounds branches serialised them), the
// out-of-image taps masked afterwards in the same a-major order; the argmax bytes of a
// channel vector leave as one 8-B store.
template <typename T>
__global__ void __launch_bounds__(256) maxpool_fwd_k3(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int n,
                                                     int h, int w, int c, int ho, int wo, int s, int p, FastDiv f_cv, FastDiv f_wo,
                                                     FastDiv f_ho) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = c / V;
  const long total = (long)n * ho * wo * cv;  // < 2^31 (host-checked): 32-bit index math
  GRID_STRIDE_XCD(i, total) {
    const uint32_t ii = (uint32_t)i, q0 = fdiv(ii, f_cv), q1 = fdiv(q0, f_wo), img = fdiv(q1, f_ho);
    const int ch = (int)(ii - q0 * cv) * V;
    const int ow = (int)(q0 - q1 * wo), oh = (int)(q1 - img * ho);
    const int h0 = oh * s - p, w0 = ow * s - p;
    V16 v[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int hh = min(max(h0 + t / 3, 0), h - 1), ww = min(max(w0 + t % 3, 0), w - 1);
      v[t] = *(const V16*)(x + (((long)img * h + hh) * w + ww) * c + ch);
    }
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
        const float f = to_f(v[t][j]);
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
    if (idx == nullptr) continue;  // inference: no backward reads the argmax bytes
    if constexpr (V == 8) {
      *(unsigned long long*)(idx + oi) = ib;
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) idx[oi + j] = (uint8_t)(ib >> (8 * j));
    }
  }
}
// Backward of the 3x3 stride-2 pool: an input pixel is covered by at most 2 x 2 windows; their
// dY vectors and argmax bytes are loaded unconditionally (clamped), then matched.
template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_k3s2(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx,
                                                       int n, int h, int w, int c, int ho, int wo, int p, FastDiv f_cv, FastDiv f_w,
                                                       FastDiv f_h) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = c / V;
  const long total = (long)n * h * w * cv;  // < 2^31 (host-checked)
  GRID_STRIDE_XCD(i, total) {
    const uint32_t ii = (uint32_t)i, q0 = fdiv(ii, f_cv), q1 = fdiv(q0, f_w), img = fdiv(q1, f_h);
    const int ch = (int)(ii - q0 * cv) * V;
    const int iw = (int)(q0 - q1 * w), ih = (int)(q1 - img * h);
    const int oh_lo = max(0, (ih + p - 1) / 2), ow_lo = max(0, (iw + p - 1) / 2);  // (ih + p - k + s) / s
    V16 g[4];
    unsigned long long ib[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int oh = min(oh_lo + (t >> 1), ho - 1), ow = min(ow_lo + (t & 1), wo - 1);
      const long o = (((long)img * ho + oh) * wo + ow) * c + ch;
      g[t] = *(const V16*)(dy + o);
      if constexpr (V == 8) {
        ib[t] = *(const unsigned long long*)(idx + o);
      } else {
        ib[t] = 0;
#pragma unroll
        for (int j = 0; j < V; ++j) ib[t] |= (unsigned long long)idx[o + j] << (8 * j);
      }
    }
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int oh = oh_lo + (t >> 1), ow = ow_lo + (t & 1);
      const int a = ih - (oh * 2 - p), b = iw - (ow * 2 - p);
      if (oh >= ho || ow >= wo || a < 0 || a >= 3 || b < 0 || b >= 3) continue;
      const unsigned want = (unsigned)(a * 3 + b);
#pragma unroll
      for (int j = 0; j < V; ++j)
        if (((ib[t] >> (8 * j)) & 0xff) == want) acc[j] += to_f(g[t][j]);
    }
    V16 r;
#pragma unroll
    for (int j = 0; j < V; ++j) r[j] = from_f<T>(acc[j]);
    *(V16*)(dx + (((long)img * h + ih) * w + iw) * c + ch) = r;
  }
}

// The same gather for 2 x 2 input pixels per thread (padding 0 or 1): the four pixels of the quad
// (2m + {0, 1}, 2k + {0, 1}) are covered only by the windows (m - 1 + p + {0, 1}, k - 1 + p + {0, 1}),
// so one set of four dY vectors + argmax loads serves four outputs (the per-pixel kernel loaded
// 16 for them).  Each pixel adds its matching windows in the same (oh, ow) order: bit-identical.
template <typename T>
__global__ void __launch_bounds__(256) maxpool_bwd_k3s2_quad(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                            T* __restrict__ dx, int n, int h, int w, int c, int ho, int wo, int p,
                                                            FastDiv f_cv, FastDiv f_w2, FastDiv f_h2) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = c / V, w2 = (w + 1) >> 1, h2 = (h + 1) >> 1;
  const long total = (long)n * h2 * w2 * cv;  // < 2^31 (host-checked)
  GRID_STRIDE_XCD(i, total) {
    const uint32_t ii = (uint32_t)i, q0 = fdiv(ii, f_cv), q1 = fdiv(q0, f_w2), img = fdiv(q1, f_h2);
    const int ch = (int)(ii - q0 * cv) * V;
    const int kq = (int)(q0 - q1 * w2), mq = (int)(q1 - img * h2);
    const int oh0 = mq - 1 + p, ow0 = kq - 1 + p;
    V16 g[4];
    unsigned long long ib[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int oh = min(max(oh0 + (t >> 1), 0), ho - 1), ow = min(max(ow0 + (t & 1), 0), wo - 1);
      const long o = (((long)img * ho + oh) * wo + ow) * c + ch;
      g[t] = *(const V16*)(dy + o);
      if constexpr (V == 8) {
        ib[t] = *(const unsigned long long*)(idx + o);
      } else {
        ib[t] = 0;
#pragma unroll
        for (int j = 0; j < V; ++j) ib[t] |= (unsigned long long)idx[o + j] << (8 * j);
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ih = 2 * mq + (e >> 1), iw = 2 * kq + (e & 1);
      if (ih >= h || iw >= w) continue;
      float acc[V];
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int oh = oh0 + (t >> 1), ow = ow0 + (t & 1);
        const int a = ih - (oh * 2 - p), b = iw - (ow * 2 - p);
        if (oh < 0 || ow < 0 || oh >= ho || ow >= wo || a < 0 || a >= 3 || b < 0 || b >= 3) continue;
        const unsigned want = (unsigned)(a * 3 + b);
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (((ib[t] >> (8 * j)) & 0xff) == want) acc[j] += to_f(g[t][j]);
      }
      V16 r;
#pragma unroll
      for (int j = 0; j < V; ++j) r[j] = from_f<T>(acc[j]);
      *(V16*)(dx + (((long)img * h + ih) * w + iw) * c + ch) = r;
    }
  }
}

extern "C" int rtsds_maxpool_fwd(const void* x, void* y, uint8_t* idx, int n, int h, int w, int c, int ho, int wo, int k, int s,
                                 int p, int dtype, void* stream) {
  if (k * k > 255 || n <= 0 || ho <= 0 || wo <= 0) return RTSDS_ERR_SHAPE;
  const long total = (long)n * ho * wo * c;
  DISPATCH_T(dtype, {
    if (c % VecT<T>::N == 0 && k == 3 && total < (1L << 31))
      hipLaunchKernelGGL(maxpool_fwd_k3<T>, dim3(ew_blocks(total / VecT<T>::N, 256, 1 << 20)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, idx,
                         n, h, w, c, ho, wo, s, p, fastdiv_make(c / VecT<T>::N), fastdiv_make(wo), fastdiv_make(ho));
    else if (idx == nullptr)
      return RTSDS_ERR_UNSUPPORTED;
    else if (c % VecT<T>::N == 0)
      hipLaunchKernelGGL(maxpool_fwd_vec<T>, dim3(ew_blocks(total / VecT<T>::N)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, idx, n, h, w, c, ho, wo, k, s, p);
    else
      hipLaunchKernelGGL(maxpool_fwd_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, idx, n, h, w, c, ho, wo, k, s, p);
  });
  RET_LAUNCH();
}
extern "C" int rtsds_maxpool_bwd(const void* dy, const uint8_t* idx, void* dx, int n, int h, int w, int c, int ho, int wo, int k,
                                 int s, int p, int dtype, void* stream) {
  const long total = (long)n * h * w * c;
  if (total <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, {
    if (c % VecT<T>::N == 0 && k == 3 && s == 2 && (p == 0 || p == 1) && total < (1L << 31)) {
      const long quads = (long)n * ((h + 1) / 2) * ((w + 1) / 2) * (c / VecT<T>::N);
      hipLaunchKernelGGL(maxpool_bwd_k3s2_quad<T>, dim3(ew_blocks(quads, 256, 1 << 20)), dim3(256), 0, (hipStream_t)stream, (const T*)dy,
                         idx, (T*)dx, n, h, w, c, ho, wo, p, fastdiv_make(c / VecT<T>::N), fastdiv_make((w + 1) / 2),
                         fastdiv_make((h + 1) / 2));
    } else if (c % VecT<T>::N == 0 && k == 3 && s == 2 && total < (1L << 31))
      hipLaunchKernelGGL(maxpool_bwd_k3s2<T>, dim3(ew_blocks(total / VecT<T>::N, 256, 1 << 20)), dim3(256), 0, (hipStream_t)stream, (const T*)dy, idx, (T*)dx,
                         n, h, w, c, ho, wo, p, fastdiv_make(c / VecT<T>::N), fastdiv_make(w), fastdiv_make(h));
    else if (c % VecT<T>::N == 0)
      hipLaunchKernelGGL(maxpool_bwd_vec<T>, dim3(ew_blocks(total / VecT<T>::N)), dim3(256), 0, (hipStream_t)stream, (const T*)dy, idx, (T*)dx, n, h, w, c, ho, wo, k, s, p);
    else
      hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, (hipStream_t)stream, (const T*)dy, idx, (T*)dx, n, h, w, c, ho, wo, k, s, p);
  });
  RET_LAUNCH();
}

// ------------------------------------------------------------------ global average pool
// y[img][c] = mean_hw x[img][hw][c]   (AdaptiveAvgPool2d(1) / torch.mean over H,W:
// build_bisenet.py:46,75, build_contextpath.py:27-28, model.py:63,82).
//
// Shared per-image channel reduction: out[img][c] = scale * sum_hw a (* b if DOT), in two
// deterministic stages.  Stage 1: grid (S row slices, img, channel chunk) of 256-thread blocks
// laid out [row group][16-B channel vector] (VEC = 8 bf16 / 4 f32 when c allows, else 1) ->
// part[img][s][c] fp32.  Stage 2 sums the S slices in order.  (One block per image would
// leave all but n CUs idle: the ARM / FFM / tail pools have n = 8 images.)
static int chan_slices(int n, long hw) {
  return (int)std::max<long>(1, std::min<long>(hw / 32, std::max(1, 1024 / std::max(1, n))));
}
template <typename T, int VEC, bool DOT>
__global__ void __launch_bounds__(256) chan_part_kernel(const T* __restrict__ a, const T* __restrict__ b, float* __restrict__ part,
                                                        long hw, int c) {
  __shared__ float red[256 * VEC];
  const int s = blockIdx.x, S = gridDim.x, img = blockIdx.y;
  const int cbase = blockIdx.z * 256 * VEC;
  const int cl = min(c - cbase, 256 * VEC);
  const int tpr = (cl + VEC - 1) / VEC, rpi = 256 / tpr;
  const int tid = threadIdx.x, cv = tid % tpr, rg = tid / tpr;
  const int ch0 = cbase + cv * VEC;
  const long per = (hw + S - 1) / S, r0 = s * per, r1 = min(hw, r0 + per);
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  if (rg < rpi) {
    const long base = (long)img * hw * c + ch0;
    long r = r0 + rg;
    for (; r + rpi < r1; r += 2 * rpi) {  // two rows in flight
      const long o0 = base + r * c, o1 = o0 + (long)rpi * c;
      if (VEC > 1) {
        typedef typename VecT<T>::v16 V16;
        const V16 a0 = *(const V16*)(a + o0), a1 = *(const V16*)(a + o1);
        if (DOT) {
          const V16 b0 = *(const V16*)(b + o0), b1 = *(const V16*)(b + o1);
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] = fmaf(to_f(a1[j]), to_f(b1[j]), fmaf(to_f(a0[j]), to_f(b0[j]), acc[j]));
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] += to_f(a0[j]) + to_f(a1[j]);
        }
      } else {
        acc[0] = DOT ? fmaf(to_f(a[o1]), to_f(b[o1]), fmaf(to_f(a[o0]), to_f(b[o0]), acc[0])) : acc[0] + (to_f(a[o0]) + to_f(a[o1]));
      }
    }
    for (; r < r1; r += rpi) {
      const long o = base + r * c;
      if (VEC > 1) {
        typedef typename VecT<T>::v16 V16;
        const V16 va = *(const V16*)(a + o);
        if (DOT) {
          const V16 vb = *(const V16*)(b + o);
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] = fmaf(to_f(va[j]), to_f(vb[j]), acc[j]);
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] += to_f(va[j]);
        }
      } else {
        acc[0] = DOT ? fmaf(to_f(a[o]), to_f(b[o]), acc[0]) : acc[0] + to_f(a[o]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[tid * VEC + j] = acc[j];
  __syncthreads();
  if (rg == 0 && cv * VEC < cl) {
    for (int g = 1; g < rpi; ++g)
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += red[(g * tpr + cv) * VEC + j];
#pragma unroll
    for (int j = 0; j < VEC; ++j)
      if (ch0 + j < c) part[((long)img * S + s) * c + ch0 + j] = acc[j];
  }
}
template <typename T>
__global__ void __launch_bounds__(256) chan_final_kernel(const float* __restrict__ part, T* __restrict__ out, int S, int c, float scale) {
  const int img = blockIdx.y, ch = blockIdx.x * 256 + threadIdx.x;
  if (ch >= c) return;
  const float* p = part + (long)img * S * c + ch;
  float s = 0.f;
  int q = 0;
  for (; q + 8 <= S; q += 8) {  // 8 slices in flight, summed in order
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = p[(long)(q + u) * c];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += t[u];
  }
  for (; q < S; ++q) s += p[(long)q * c];
  out[(long)img * c + ch] = from_f<T>(s * scale);
}
extern "C" size_t rtsds_gap_workspace(int n, long hw, int c) {
  if (n <= 0 || hw <= 0 || c <= 0) return 256;
  return (size_t)n * chan_slices(n, hw) * c * 4 + 256;
}
template <typename T, bool DOT>
static void chan_reduce(const T* a, const T* b, T* out, int n, long hw, int c, float scale, float* part, hipStream_t st) {
  constexpr int V = VecT<T>::N;
  const int S = chan_slices(n, hw);
  if (c % V == 0)
    hipLaunchKernelGGL((chan_part_kernel<T, V, DOT>), dim3(S, n, rt_cdiv(c, 256 * V)), dim3(256), 0, st, a, b, part, hw, c);
  else
    hipLaunchKernelGGL((chan_part_kernel<T, 1, DOT>), dim3(S, n, rt_cdiv(c, 256)), dim3(256), 0, st, a, b, part, hw, c);
  hipLaunchKernelGGL(chan_final_kernel<T>, dim3(rt_cdiv(c, 256), n), dim3(256), 0, st, (const float*)part, out, S, c, scale);
}
// accum: dx += the (rounded) gradient -- the other reader's contribution already in dx
// (functional.GradJoin), the same two roundings as autograd's separate elementwise add
template <typename T>
__global__ void gap_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int n, long hw, int c, int accum) {
  const long total = (long)n * hw * c;
  const float inv = 1.f / (float)hw;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    const long img = i / c / hw;
    const T g = from_f<T>(to_f(dy[img * c + ch]) * inv);
    dx[i] = accum ? from_f<T>(to_f(dx[i]) + to_f(g)) : g;
  }
}
extern "C" int rtsds_gap_fwd(const void* x, void* y, int n, long hw, int c, int dtype, void* ws, size_t ws_bytes, void* stream) {
  if (n <= 0 || hw <= 0 || c <= 0) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_gap_workspace(n, hw, c)) return RTSDS_ERR_WORKSPACE;
  DISPATCH_T(dtype, (chan_reduce<T, false>((const T*)x, nullptr, (T*)y, n, hw, c, 1.f / (float)hw, (float*)ws, (hipStream_t)stream)));
  RET_LAUNCH();
}
// 16-B channel vectors (c % 8 == 0, bf16): one division per 8 elements instead of two per element
__global__ void gap_bwd_vec_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dx, long pixels, long hw, int cv, int accum,
                                   float inv) {
  const long total = pixels * cv;
  GRID_STRIDE(i, total) {
    const long p = i / cv;
    const int q = (int)(i - p * cv);
    const long img = p / hw;
    const bf16x8 g = *(const bf16x8*)(dy + (img * cv + q) * 8);
    bf16x8 o;
    if (accum) o = *(const bf16x8*)(dx + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bf16 v = from_f<bf16>(to_f(g[j]) * inv);
      o[j] = accum ? from_f<bf16>(to_f(o[j]) + to_f(v)) : v;
    }
    *(bf16x8*)(dx + i * 8) = o;
  }
}
extern "C" int rtsds_gap_bwd(const void* dy, void* dx, int n, long hw, int c, int accumulate, int dtype, void* stream) {
  if (n <= 0 || hw <= 0 || c <= 0) return RTSDS_ERR_SHAPE;
  if (dtype == RTSDS_BF16 && c % 8 == 0) {
    const long pixels = (long)n * hw;
    hipLaunchKernelGGL(gap_bwd_vec_kernel, dim3(ew_blocks(pixels * (c / 8))), dim3(256), 0, (hipStream_t)stream, (const bf16*)dy,
                       (bf16*)dx, pixels, hw, c / 8, accumulate ? 1 : 0, 1.f / (float)hw);
    RET_LAUNCH();
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(gap_bwd_kernel<T>, dim3(ew_blocks((long)n * hw * c)), dim3(256), 0, (hipStream_t)stream, (const T*)dy, (T*)dx, n, hw, c, accumulate ? 1 : 0));
  RET_LAUNCH();
}

// ------------------------------------------------------------------ channel attention scale
// mode 0: y = x * a[img][c]           (ARM x*sigmoid, cx2*tail: build_bisenet.py:52,149)
// mode 1: y = x * a[img][c] + x       (FFM: build_bisenet.py:79-80)
template <typename T>
__global__ void chscale_fwd_kernel(const T* __restrict__ x, const T* __restrict__ a, T* __restrict__ y, int n, long hw, int c, int mode) {
  const long total = (long)n * hw * c;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    const long img = i / c / hw;
    const float xv = to_f(x[i]), av = to_f(a[img * c + ch]);
    y[i] = from_f<T>(mode ? fmaf(xv, av, xv) : xv * av);
  }
}
template <typename T>
__global__ void chscale_bwd_dx_kernel(const T* __restrict__ dy, const T* __restrict__ a, T* __restrict__ dx, int n, long hw, int c, int mode) {
  const long total = (long)n * hw * c;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    const long img = i / c / hw;
    const float av = to_f(a[img * c + ch]) + (mode ? 1.f : 0.f);
    dx[i] = from_f<T>(to_f(dy[i]) * av);
  }
}
extern "C" int rtsds_chscale_fwd(const void* x, const void* a, void* y, int n, long hw, int c, int mode, int dtype, void* stream) {
  const long total = (long)n * hw * c;
  if (total <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, hipLaunchKernelGGL(chscale_fwd_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (const T*)a, (T*)y, n, hw, c, mode));
  RET_LAUNCH();
}
// Inference tail of the FeatureFusionModule plus BiSeNet's final 1x1 conv (build_bisenet.py:75-80,
// 167): a = sigmoid(conv2(relu(conv1(GAP(f))))), r = f * a + f, out = conv(r) + bias, for a
// narrow class map f [N][hw][C] (C <= 32).  Unfused these are 8 launches (two-stage GAP, two
// pooled 1x1 convs, the channel scale, two channel pads and the padded GEMM: ~54 us at bs 8,
// all launch-bound).  Two launches here: (1) chan_part_kernel's GAP partials over FFM_CHUNK-pixel
// slices of each image; (2) grid (slices, N): every workgroup sums its image's partials in slice
// order, evaluates the two pooled convs in LDS, stages its slice of pixels in LDS (coalesced 16-B
// loads), maps each pixel in place (one pixel per thread, the C x C head weights in LDS) and writes
// the slice back with 16-B stores.  (One launch whose 64 workgroups each re-read their whole image
// for the GAP ran one wave per CU through the 19 x 19 per-pixel maps: 21.7 us.)  Each intermediate
// is rounded to T where the unfused chain stores it.
static constexpr int kFfmChunk = 256;  // pixels per slice / workgroup
template <typename T, int C>
__global__ void __launch_bounds__(256) ffm_head_apply_kernel(const float* __restrict__ part, const T* __restrict__ f,
                                                             const T* __restrict__ w1, const float* __restrict__ b1,
                                                             const T* __restrict__ w2, const float* __restrict__ b2,
                                                             const T* __restrict__ w3, const float* __restrict__ b3,
                                                             T* __restrict__ out, int hw) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  __shared__ float wl[3][C][C + 1];
  __shared__ float gap[C], hid[C], att[C], bias3[C];
  __shared__ __attribute__((aligned(16))) T stage[kFfmChunk * C];
  const int tid = threadIdx.x, img = blockIdx.y, S = gridDim.x;
  const T* fi = f + (long)img * hw * C;
  for (int e = tid; e < C * C; e += 256) {
    const int o = e / C, i = e - o * C;
    wl[0][o][i] = to_f(w1[e]);
    wl[1][o][i] = to_f(w2[e]);
    wl[2][o][i] = to_f(w3[e]);
  }
  // this slice's pixels, in flight while the attention vector is formed
  const int p0 = blockIdx.x * kFfmChunk, np = min(kFfmChunk, hw - p0);  // np % V == 0 (host: hw % V == 0)
  const int nvec = np * C / V;
  const V16* src = (const V16*)(fi + (long)p0 * C);
  for (int e = tid; e < nvec; e += 256) ((V16*)stage)[e] = src[e];
  if (tid < C) {  // GAP: the slices' partials summed in order (chan_final_kernel's order)
    const float* pp = part + (long)img * S * C + tid;
    float t = 0.f;
    int q = 0;
    for (; q + 8 <= S; q += 8) {
      float u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = pp[(long)(q + k) * C];
#pragma unroll
      for (int k = 0; k < 8; ++k) t += u[k];
    }
    for (; q < S; ++q) t += pp[(long)q * C];
    gap[tid] = to_f(from_f<T>(t * (1.f / (float)hw)));
    bias3[tid] = b3 ? b3[tid] : 0.f;
  }
  __syncthreads();
  if (tid < C) {
    float v = b1 ? b1[tid] : 0.f;
    for (int i = 0; i < C; ++i) v = fmaf(wl[0][tid][i], gap[i], v);
    hid[tid] = to_f(from_f<T>(fmaxf(v, 0.f)));
  }
  __syncthreads();
  if (tid < C) {
    float v = b2 ? b2[tid] : 0.f;
    for (int i = 0; i < C; ++i) v = fmaf(wl[1][tid][i], hid[i], v);
    att[tid] = to_f(from_f<T>(1.f / (1.f + expf(-v))));
  }
  __syncthreads();
  for (int p = tid; p < np; p += 256) {
    T* q = stage + p * C;
    float r[C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const float x = to_f(q[i]);
      r[i] = to_f(from_f<T>(fmaf(x, att[i], x)));
    }
#pragma unroll
    for (int k = 0; k < C; ++k) {
      float v = bias3[k];
#pragma unroll
      for (int i = 0; i < C; ++i) v = fmaf(wl[2][k][i], r[i], v);
      q[k] = from_f<T>(v);
    }
  }
  __syncthreads();
  V16* dst = (V16*)(out + ((long)img * hw + p0) * C);
  for (int e = tid; e < nvec; e += 256) dst[e] = ((const V16*)stage)[e];
}
extern "C" size_t rtsds_ffm_head_eval_workspace(int n, long hw, int c) {
  if (n <= 0 || hw <= 0 || c <= 0) return 256;
  return (size_t)n * ((hw + kFfmChunk - 1) / kFfmChunk) * c * 4 + 256;
}
extern "C" int rtsds_ffm_head_eval(const void* f, const void* w1, const float* b1, const void* w2, const float* b2,
                                   const void* w3, const float* b3, void* out, int n, long hw, int c, int dtype, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (n <= 0 || n > 65535 || hw <= 0 || hw >= (1L << 31)) return RTSDS_ERR_SHAPE;
  if (c != 19) return RTSDS_ERR_UNSUPPORTED;  // instantiated for the 19-class maps
  const int V = dtype == RTSDS_BF16 ? 8 : 4;
  if (hw % V) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_ffm_head_eval_workspace(n, hw, c)) return RTSDS_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int S = (int)((hw + kFfmChunk - 1) / kFfmChunk);
  float* part = (float*)ws;
  DISPATCH_T(dtype, {
    hipLaunchKernelGGL((chan_part_kernel<T, 1, false>), dim3(S, n, 1), dim3(256), 0, st, (const T*)f, (const T*)nullptr, part,
                       hw, c);
    hipLaunchKernelGGL((ffm_head_apply_kernel<T, 19>), dim3(S, n), dim3(256), 0, st, (const float*)part, (const T*)f, (const T*)w1,
                       b1, (const T*)w2, b2, (const T*)w3, b3, (T*)out, (int)hw);
  });
  RET_LAUNCH();
}
extern "C" int rtsds_chscale_bwd(const void* dy, const void* x, const void* a, void* dx, void* da, int n, long hw, int c, int mode,
                                 int dtype, void* ws, size_t ws_bytes, void* stream) {
  const long total = (long)n * hw * c;
  if (total <= 0) return RTSDS_ERR_SHAPE;
  if (da && ws_bytes < rtsds_gap_workspace(n, hw, c)) return RTSDS_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (dx) hipLaunchKernelGGL(chscale_bwd_dx_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, st, (const T*)dy, (const T*)a, (T*)dx, n, hw, c, mode);
    if (da) chan_reduce<T, true>((const T*)dy, (const T*)x, (T*)da, n, hw, c, 1.f, (float*)ws, st);
  });
  RET_LAUNCH();
}

// ------------------------------------------------------------------ adaptive average pool
// ATen start/end indices: [floor(o*in/out), ceil((o+1)*in/out)).
RT_DEV int ap_start(int o, int out, int in) { return (int)(((long)o * in) / out); }
RT_DEV int ap_end(int o, int out, int in) { return (int)(((long)(o + 1) * in + out - 1) / out); }

// One thread per (output pixel, channel); channels fastest -> coalesced NHWC access.
template <typename T>
__global__ void adaptive_avgpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int n, int hi, int wi, int c,
                                            int ho, int wo) {
  const long total = (long)n * ho * wo * c;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    long q = i / c;
    const int ow = (int)(q % wo);
    q /= wo;
    const int oh = (int)(q % ho);
    const int img = (int)(q / ho);
    const int h0 = ap_start(oh, ho, hi), h1 = ap_end(oh, ho, hi);
    const int w0 = ap_start(ow, wo, wi), w1 = ap_end(ow, wo, wi);
    const T* b = x + (long)img * hi * wi * c + ch;
    float s = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) s += to_f(b[((long)h * wi + w) * c]);
    y[i] = from_f<T>(s / (float)((h1 - h0) * (w1 - w0)));
  }
}
// dx[i] = sum over windows o containing i of dy[o] / area(o).  Window o covers input index i
// iff start(o) <= i < end(o); every such o lies in [floor(i*out/in) - 1, ceil((i+1)*out/in)],
// and each candidate is tested exactly.
template <typename T>
__global__ void adaptive_avgpool_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int n, int hi, int wi, int c,
                                            int ho, int wo) {
  const long total = (long)n * hi * wi * c;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    long q = i / c;
    const int iw = (int)(q % wi);
    q /= wi;
    const int ih = (int)(q % hi);
    const int img = (int)(q / hi);
    // candidate output rows: o with start(o) <= ih < end(o)
    const int oh_lo = max(0, (int)(((long)ih * ho) / hi) - 1), oh_hi = min(ho - 1, (int)(((long)(ih + 1) * ho + hi - 1) / hi));
    const int ow_lo = max(0, (int)(((long)iw * wo) / wi) - 1), ow_hi = min(wo - 1, (int)(((long)(iw + 1) * wo + wi - 1) / wi));
    const T* b = dy + (long)img * ho * wo * c + ch;
    float s = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int h0 = ap_start(oh, ho, hi), h1 = ap_end(oh, ho, hi);
      if (ih < h0 || ih >= h1) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int w0 = ap_start(ow, wo, wi), w1 = ap_end(ow, wo, wi);
        if (iw < w0 || iw >= w1) continue;
        s += to_f(b[((long)oh * wo + ow) * c]) / (float)((h1 - h0) * (w1 - w0));
      }
    }
    dx[i] = from_f<T>(s);
  }
}
extern "C" int rtsds_adaptive_avgpool_fwd(const void* x, void* y, int n, int hi, int wi, int c, int ho, int wo, int dtype,
                                          void* stream) {
  if (n <= 0 || hi <= 0 || wi <= 0 || c <= 0 || ho <= 0 || wo <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, hipLaunchKernelGGL(adaptive_avgpool_fwd_kernel<T>, dim3(ew_blocks((long)n * ho * wo * c)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)x, (T*)y, n, hi, wi, c, ho, wo));
  RET_LAUNCH();
}
extern "C" int rtsds_adaptive_avgpool_bwd(const void* dy, void* dx, int n, int hi, int wi, int c, int ho, int wo, int dtype,
                                          void* stream) {
  if (n <= 0 || hi <= 0 || wi <= 0 || c <= 0 || ho <= 0 || wo <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, hipLaunchKernelGGL(adaptive_avgpool_bwd_kernel<T>, dim3(ew_blocks((long)n * hi * wi * c)), dim3(256), 0,
                                       (hipStream_t)stream, (const T*)dy, (T*)dx, n, hi, wi, c, ho, wo));
  RET_LAUNCH();
}

// ------------------------------------------------------------------ bilinear (align_corners=False)
// bil_src (ATen source index, align_corners=False): common.h
// Forward: one thread per (output pixel, channel chunk of CH); the 4 taps and weights are
// computed once per chunk.  CH = 16-B vector when the channel layout allows it, else the whole
// pixel (c <= 64, e.g. the 19-class heads) or single channels.
template <typename T, int MODE>  // MODE 0: 16-B vectors, 1: whole pixel loop, 2: per channel
__global__ void bilinear_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int n, int hi, int wi, int c, int ho, int wo,
                                    float sh, float sw, int yld, int yoff) {
  constexpr int V = VecT<T>::N;
  const int cpp = MODE == 0 ? c / V : (MODE == 1 ? 1 : c);  // chunks per pixel
  const long total = (long)n * ho * wo * cpp;
  GRID_STRIDE(i, total) {
    const int chunk = (int)(i % cpp);
    long q = i / cpp;
    const int ow = (int)(q % wo); q /= wo;
    const int oh = (int)(q % ho);
    const int img = (int)(q / ho);
    int h0, h1, w0, w1;
    float lh0, lh1, lw0, lw1;
    bil_src(oh, sh, hi, h0, h1, lh0, lh1);
    bil_src(ow, sw, wi, w0, w1, lw0, lw1);
    const T* b = x + (long)img * hi * wi * c;
    const T* p00 = b + ((long)h0 * wi + w0) * c;
    const T* p01 = b + ((long)h0 * wi + w1) * c;
    const T* p10 = b + ((long)h1 * wi + w0) * c;
    const T* p11 = b + ((long)h1 * wi + w1) * c;
    T* o = y + ((((long)img * ho + oh) * wo) + ow) * yld + yoff;
    if (MODE == 0) {
      typedef typename VecT<T>::v16 V16;
      const int c0 = chunk * V;
      const V16 a = *(const V16*)(p00 + c0), bb = *(const V16*)(p01 + c0);
      const V16 cc = *(const V16*)(p10 + c0), dd = *(const V16*)(p11 + c0);
      V16 r;
#pragma unroll
      for (int j = 0; j < V; ++j)
        r[j] = from_f<T>(bil_mix(to_f(a[j]), to_f(bb[j]), to_f(cc[j]), to_f(dd[j]), lh0, lh1, lw0, lw1));
      *(V16*)(o + c0) = r;
    } else {
      const int cs = MODE == 1 ? 0 : chunk, ce = MODE == 1 ? c : chunk + 1;
      for (int ch = cs; ch < ce; ++ch)
        o[ch] = from_f<T>(bil_mix(to_f(p00[ch]), to_f(p01[ch]), to_f(p10[ch]), to_f(p11[ch]), lh0, lh1, lw0, lw1));
    }
  }
}

// Upsampling with 16-B channel vectors (the context-path resizes into the FFM concat): one thread
// per (image, source row h0, output column, channel vector) loads the 4 taps once, forms bil_mix's
// two horizontal blends and writes every output row whose top tap is h0 (bit-identical to MODE 0;
// the taps are gathered once per source row instead of once per output row).  s1 / s2 (optional,
// [n][c]): channel scales applied to each tap first, rounded to T after each as the stored
// rtsds_chscale_fwd outputs would be (BiSeNet's attention refinement, build_bisenet.py:42-53,
// 157-159, folded into the eval forward's resize: bit-identical to scale, scale, resize).
template <typename T, int U>
__global__ void __launch_bounds__(256) bilinear_fwd_group_vec_kernel(const T* __restrict__ x, T* __restrict__ y, int n, int hi,
                                                                     int wi, int c, int ho, int wo, float sh, float sw, int yld,
                                                                     int yoff, const T* __restrict__ s1, const T* __restrict__ s2) {
  constexpr int V = VecT<T>::N;
  typedef typename VecT<T>::v16 V16;
  // grid (column-vector blocks, n * hi): the source row and its output rows are block-uniform.
  // A thread takes U column vectors gridDim.x * 256 apart and issues all their tap loads before
  // any arithmetic (U x 4 loads in flight instead of 4 per thread-lifetime).
  const int cpp = c / V, nv = wo * cpp;
  const int img = blockIdx.y / hi, h0 = blockIdx.y - img * hi;
  const int oa = bil_first_ge(h0, sh, hi, ho), ob = bil_first_ge(h0 + 1, sh, hi, ho);
  const int h1 = h0 + (h0 < hi - 1 ? 1 : 0);
  if (oa >= ob) return;
  const int i0 = blockIdx.x * 256 + threadIdx.x, step = gridDim.x * 256;
  const T* xb = x + (long)img * hi * wi * c;
  V16 a[U], bb[U], cc[U], dd[U], k1[U], k2[U];
  float lw0[U], lw1[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = min(i0 + u * step, nv - 1);  // clamped: unconditional loads
    const int ow = i / cpp, chunk = i - ow * cpp;
    int w0, w1;
    bil_src(ow, sw, wi, w0, w1, lw0[u], lw1[u]);
    const T* b = xb + chunk * V;
    a[u] = *(const V16*)(b + ((long)h0 * wi + w0) * c);
    bb[u] = *(const V16*)(b + ((long)h0 * wi + w1) * c);
    cc[u] = *(const V16*)(b + ((long)h1 * wi + w0) * c);
    dd[u] = *(const V16*)(b + ((long)h1 * wi + w1) * c);
    if (s1) k1[u] = *(const V16*)(s1 + (long)img * c + chunk * V);
    if (s2) k2[u] = *(const V16*)(s2 + (long)img * c + chunk * V);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = i0 + u * step;
    if (i >= nv) break;
    const int ow = i / cpp, chunk = i - ow * cpp;
    auto tap = [&](T v, int j) {
      float f = to_f(v);
      if (s1) f = to_f(from_f<T>(f * to_f(k1[u][j])));
      if (s2) f = to_f(from_f<T>(f * to_f(k2[u][j])));
      return f;
    };
    float t0[V], t1[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      t0[j] = fmaf(lw1[u], tap(bb[u][j], j), lw0[u] * tap(a[u][j], j));
      t1[j] = fmaf(lw1[u], tap(dd[u][j], j), lw0[u] * tap(cc[u][j], j));
    }
    for (int oh = oa; oh < ob; ++oh) {
      int i0_, i1_;
      float lh0, lh1;
      bil_src(oh, sh, hi, i0_, i1_, lh0, lh1);
      V16 r;
#pragma unroll
      for (int j = 0; j < V; ++j) r[j] = from_f<T>(fmaf(lh1, t1[j], lh0 * t0[j]));
      *(V16*)(y + (((long)img * ho + oh) * wo + ow) * yld + yoff + chunk * V) = r;
    }
  }
}

// Narrow channel counts that are not a 16-B multiple (the 19-class logits of the eval forward's
// final x8 resize, build_bisenet.py:165-166): one workgroup per output row.  The row's two source
// rows are staged in LDS as fp32 (coalesced), then every thread writes whole 16-B vectors of the
// dense output row (a wave writes 1 KB contiguously; the whole-pixel loop wrote 38-B runs at a
// 38-B lane stride, 1.8 TB/s) from 4 LDS taps per element.  Same taps, weights and bil_mix
// expression as the other modes.
template <typename T>
__global__ void __launch_bounds__(256) bilinear_fwd_rows_kernel(const T* __restrict__ x, T* __restrict__ y, int hi, int wi, int c,
                                                                 int ho, int wo, float sh, float sw, FastDiv f_c) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  extern __shared__ float rows[];  // [2][wi * c]
  const int row = blockIdx.x, img = row / ho, oh = row - img * ho;
  int h0, h1;
  float lh0, lh1;
  bil_src(oh, sh, hi, h0, h1, lh0, lh1);
  const int rl = wi * c;
  const T* r0 = x + ((long)img * hi + h0) * rl;
  const T* r1 = x + ((long)img * hi + h1) * rl;
  for (int e = threadIdx.x; e < rl; e += 256) {
    rows[e] = to_f(r0[e]);
    rows[rl + e] = to_f(r1[e]);
  }
  __syncthreads();
  const int nv = wo * c / V;  // (wo * c) % V == 0 (host)
  T* yo = y + (long)row * wo * c;
  for (int v = threadIdx.x; v < nv; v += 256) {
    const int e = v * V;
    int ow = (int)fdiv((uint32_t)e, f_c), ch = e - ow * c;
    int w0, w1;
    float lw0, lw1;
    bil_src(ow, sw, wi, w0, w1, lw0, lw1);
    V16 r;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if (ch == c) {
        ch = 0;
        ++ow;
        bil_src(ow, sw, wi, w0, w1, lw0, lw1);
      }
      const float* a = rows + w0 * c + ch;
      const float* b = rows + w1 * c + ch;
      r[k] = from_f<T>(bil_mix(a[0], b[0], a[rl], b[rl], lh0, lh1, lw0, lw1));
      ++ch;
    }
    *(V16*)(yo + e) = r;
  }
}

// The same resize for upsampling, one workgroup per (image, source row h0, column chunk): every
// output row whose top tap is h0 blends the same two horizontal blends t0 / t1 (bil_mix's inner
// terms), so each thread computes them once for its J output vectors of the chunk, keeps them in
// registers and writes all of the group's rows (~ the scale factor of them) as
// fmaf(lh1, t1, lh0 * t0) -- bil_mix bit for bit, at 2 VALU ops per element instead of ~12 and
// 4 LDS reads per element per group instead of per row.
template <typename T, int J>
__global__ void __launch_bounds__(256) bilinear_fwd_rowgroup_kernel(const T* __restrict__ x, T* __restrict__ y, int hi, int wi, int c,
                                                                     int ho, int wo, float sh, float sw, int nchunk, FastDiv f_c) {
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  extern __shared__ float rows[];  // [2][wi * c]
  const int grp = blockIdx.x / nchunk, chunk = blockIdx.x - grp * nchunk;
  const int img = grp / hi, h0 = grp - img * hi;
  const int oa = bil_first_ge(h0, sh, hi, ho), ob = bil_first_ge(h0 + 1, sh, hi, ho);
  if (oa >= ob) return;  // no output row starts at h0 (downsampling): whole workgroup
  const int h1 = h0 + (h0 < hi - 1 ? 1 : 0);
  const int rl = wi * c;
  const T* r0 = x + ((long)img * hi + h0) * rl;
  const T* r1 = x + ((long)img * hi + h1) * rl;
  for (int e = threadIdx.x; e < rl; e += 256) {
    rows[e] = to_f(r0[e]);
    rows[rl + e] = to_f(r1[e]);
  }
  __syncthreads();
  const int nv = wo * c / V;  // (wo * c) % V == 0 (host)
  const int v0 = (int)((long)nv * chunk / nchunk), v1 = (int)((long)nv * (chunk + 1) / nchunk);
  float t0[J][V], t1[J][V];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int v = v0 + threadIdx.x + 256 * j;
    if (v >= v1) break;
    const int e = v * V;
    int ow = (int)fdiv((uint32_t)e, f_c), ch = e - ow * c;
    int w0, w1;
    float lw0, lw1;
    bil_src(ow, sw, wi, w0, w1, lw0, lw1);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if (ch == c) {
        ch = 0;
        ++ow;
        bil_src(ow, sw, wi, w0, w1, lw0, lw1);
      }
      const float* a = rows + w0 * c + ch;
      const float* b = rows + w1 * c + ch;
      t0[j][k] = fmaf(lw1, b[0], lw0 * a[0]);
      t1[j][k] = fmaf(lw1, b[rl], lw0 * a[rl]);
      ++ch;
    }
  }
  for (int oh = oa; oh < ob; ++oh) {
    int i0, i1;
    float lh0, lh1;
    bil_src(oh, sh, hi, i0, i1, lh0, lh1);
    T* yo = y + ((long)img * ho + oh) * wo * c;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int v = v0 + threadIdx.x + 256 * j;
      if (v >= v1) break;
      V16 r;
#pragma unroll
      for (int k = 0; k < V; ++k) r[k] = from_f<T>(fmaf(lh1, t1[j][k], lh0 * t0[j][k]));
      *(V16*)(yo + (long)v * V) = r;
    }
  }
}

static const bool kBilRowGroup = true;
static constexpr auto kBilGroupU = 4;  // column vectors per thread of bilinear_fwd_group_vec_kernel (1 / 2 / 4: 48 / 43 / 41 us, profiles/r6f)
static constexpr auto kBilJ = 2;  // output vectors per thread and column chunk (2, 3, 4, 6 measured: 2 best)

// Backward, separable gather (deterministic, no atomics): input index i along one axis
// receives from outputs o with i0(o) == i (weight l0) or i1(o) == i (weight l1); those o lie
// in [(i-0.5)/s - 0.5, (i+1.5)/s - 0.5], widened by one and tested exactly with bil_src.
RT_DEV float bil_wsum_range(int i, float s, int in, int out, int& lo, int& hi) {
  lo = max(0, (int)floorf(((float)i - 0.5f) / s - 0.5f) - 1);
  hi = min(out - 1, (int)ceilf(((float)i + 1.5f) / s - 0.5f) + 1);
  return 0.f;
}
RT_DEV float bil_weight(int o, int i, float s, int in) {
  int a0, a1;
  float l0, l1;
  bil_src(o, s, in, a0, a1, l0, l1);
  return (a0 == i ? l0 : 0.f) + (a1 == i ? l1 : 0.f);
}
// pass 1 (W): tmp[img][oh][iw][c] = sum_ow w(ow->iw) dy[img][oh][ow][c]   (fp32)
template <typename T>
__global__ void bilinear_bwd_w_kernel(const T* __restrict__ dy, float* __restrict__ tmp, int n, int wi, int c, int ho, int wo, float sw,
                                      int dyld, int dyoff) {
  const long total = (long)n * ho * wi * c;
  GRID_STRIDE(i, total) {
    const int ch = (int)(i % c);
    long q = i / c;
    const int iw = (int)(q % wi);
    const long row = q / wi;  // img * ho + oh
    int lo, hi;
    bil_wsum_range(iw, sw, wi, wo, lo, hi);
    const T* src = dy + row * wo * dyld + dyoff + ch;
    float acc = 0.f;
    for (int ow = lo; ow <= hi; ++ow) {
      const float wt = bil_weight(ow, iw, sw, wi);
      if (wt != 0.f) acc = fmaf(wt, to_f(src[(long)ow * dyld]), acc);
    }
    tmp[i] = acc;
  }
}
// pass 2 (H): dx[img][ih][iw][c] = sum_oh w(oh->ih) tmp[img][oh][iw][c]
template <typename T>
__global__ void bilinear_bwd_h_kernel(const float* __restrict__ tmp, T* __restrict__ dx, int n, int hi, int wi, int c, int ho, float sh) {
  const long total = (long)n * hi * wi * c;
  const long plane = (long)wi * c;
  GRID_STRIDE(i, total) {
    const long inner = i % plane;  // iw * c + ch
    long q = i / plane;
    const int ih = (int)(q % hi);
    const int img = (int)(q / hi);
    int lo, hh;
    bil_wsum_range(ih, sh, hi, ho, lo, hh);
    const float* src = tmp + (long)img * ho * plane + inner;
    float acc = 0.f;
    for (int oh = lo; oh <= hh; ++oh) {
      const float wt = bil_weight(oh, ih, sh, hi);
      if (wt != 0.f) acc = fmaf(wt, src[(long)oh * plane], acc);
    }
    dx[i] = from_f<T>(acc);
  }
}
// Table-driven variants of the two passes: the weights of one axis (per input index i: lo(i)
// and w(lo + j -> i), zero past hi(i)) are tabulated once per block in LDS instead of being
// re-derived (two bil_src evaluations) for every element and tap; same taps, same order, same
// zero skipping, so the sums are bit-identical to the kernels above.
static const int kBilTabLds = 48 * 1024;
RT_DEV void bil_table_build(float* tab, int* tlo, int in, int out, float s, int maxw) {
  for (int e = threadIdx.x; e < in * maxw; e += blockDim.x) {
    const int i = e / maxw, j = e - i * maxw;
    int lo, hi;
    bil_wsum_range(i, s, in, out, lo, hi);
    tab[e] = lo + j <= hi ? bil_weight(lo + j, i, s, in) : 0.f;
    if (j == 0) tlo[i] = lo;
  }
  __syncthreads();
}
template <typename T>
__global__ void bilinear_bwd_w_tab_kernel(const T* __restrict__ dy, float* __restrict__ tmp, int n, int wi, int c, int ho, int wo,
                                          float sw, int dyld, int dyoff, int maxw, FastDiv f_c, FastDiv f_wi) {
  extern __shared__ float tab[];
  int* tlo = (int*)(tab + wi * maxw);
  bil_table_build(tab, tlo, wi, wo, sw, maxw);
  const long total = (long)n * ho * wi * c;  // < 2^31 (host)
  GRID_STRIDE(i, total) {
    const uint32_t q = fdiv((uint32_t)i, f_c), row = fdiv(q, f_wi);
    const int ch = (int)((uint32_t)i - q * c), iw = (int)(q - row * wi);
    const float* w = tab + iw * maxw;
    const T* src = dy + ((long)row * wo + tlo[iw]) * dyld + dyoff + ch;
    float acc = 0.f;
    for (int j = 0; j < maxw; ++j) {
      const float wt = w[j];
      if (wt != 0.f) acc = fmaf(wt, to_f(src[(long)j * dyld]), acc);
    }
    tmp[i] = acc;
  }
}
template <typename T>
__global__ void bilinear_bwd_h_tab_kernel(const float* __restrict__ tmp, T* __restrict__ dx, int n, int hi, int wi, int c, int ho,
                                          float sh, int maxh, FastDiv f_plane, FastDiv f_hi) {
  extern __shared__ float tab[];
  int* tlo = (int*)(tab + hi * maxh);
  bil_table_build(tab, tlo, hi, ho, sh, maxh);
  const uint32_t plane = (uint32_t)wi * c;
  const long total = (long)n * hi * plane;  // < 2^31 (host)
  GRID_STRIDE(i, total) {
    const uint32_t q = fdiv((uint32_t)i, f_plane), img = fdiv(q, f_hi);
    const uint32_t inner = (uint32_t)i - q * plane;
    const int ih = (int)(q - img * hi);
    const float* w = tab + ih * maxh;
    const float* src = tmp + ((long)img * ho + tlo[ih]) * plane + inner;
    float acc = 0.f;
    for (int j = 0; j < maxh; ++j) {
      const float wt = w[j];
      if (wt != 0.f) acc = fmaf(wt, src[(long)j * plane], acc);
    }
    dx[i] = from_f<T>(acc);
  }
}
// [first, last] nonzero entry of each table row, packed first | (last + 1) << 16 (the tables
// carry a one-entry margin either side, so a plain loop over maxw wastes taps)
RT_DEV void bil_table_span(const float* tab, int* span, int in, int maxw) {
  for (int i = threadIdx.x; i < in; i += blockDim.x) {
    int f = maxw, l = -1;
    for (int j = 0; j < maxw; ++j)
      if (tab[i * maxw + j] != 0.f) {
        f = min(f, j);
        l = j;
      }
    span[i] = f | (l + 1) << 16;
  }
  __syncthreads();
}
// Both passes in one kernel for 16-B channel vectors: a thread owns V channels of one input
// pixel and forms each output row's W-pass sum t (the W kernel's taps, order and zero skipping,
// fp32) right before the H-pass FMA that consumes it -- the same two fp32 FMA chains, so dx is
// bit-identical to the two-pass kernels, without the fp32 [ho][wi] intermediate's write and
// re-read.  Neighbouring input pixels re-read dY rows through L2 (XCD-aware block order).
// Only each row's nonzero span is visited, and its column taps go four at a time: the four
// loads issued (clamped into the span) before their FMAs, a zero weight leaving t unchanged
// exactly as the skipped tap of the two-pass kernel.
template <typename T, int G>
__global__ void __launch_bounds__(256) bilinear_bwd_fused_vec_kernel(const T* __restrict__ dy, T* __restrict__ dx, int hi, int wi,
                                                                     int c, int ho, int wo, float sh, float sw, int dyld, int dyoff,
                                                                     int maxh, int maxw, long total, FastDiv f_cv, FastDiv f_wi,
                                                                     FastDiv f_hi) {
  extern __shared__ float tab[];
  float* wtab = tab;
  int* wlo = (int*)(wtab + wi * maxw);
  float* htab = (float*)(wlo + wi);
  int* hlo = (int*)(htab + hi * maxh);
  int* wspan = hlo + hi;
  int* hspan = wspan + wi;
  bil_table_build(wtab, wlo, wi, wo, sw, maxw);
  bil_table_build(htab, hlo, hi, ho, sh, maxh);
  bil_table_span(wtab, wspan, wi, maxw);
  bil_table_span(htab, hspan, hi, maxh);
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  const int cv = c / V;
  GRID_STRIDE_XCD(i, total) {  // total < 2^31 (host)
    const uint32_t q = fdiv((uint32_t)i, f_cv), r = fdiv(q, f_wi);
    const int ch = ((int)((uint32_t)i - q * cv)) * V, iw = (int)(q - r * wi);
    const uint32_t img = fdiv(r, f_hi);
    const int ih = (int)(r - img * hi);
    const float* wx = wtab + iw * maxw;
    const float* wy = htab + ih * maxh;
    const T* base = dy + ((long)img * ho + hlo[ih]) * wo * dyld + (long)wlo[iw] * dyld + dyoff + ch;
    const int jx0 = wspan[iw] & 0xffff, jx1 = wspan[iw] >> 16;
    const int ky0 = hspan[ih] & 0xffff, ky1 = hspan[ih] >> 16;
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    for (int k = ky0; k < ky1; ++k) {
      const float yk = wy[k];
      if (yk == 0.f) continue;
      const T* row = base + (long)k * wo * dyld;
      float t[V];
#pragma unroll
      for (int e = 0; e < V; ++e) t[e] = 0.f;
      for (int j0 = jx0; j0 < jx1; j0 += G) {
        V16 v[G];
        float xw[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int j = j0 + u;
          xw[u] = j < jx1 ? wx[j] : 0.f;
          v[u] = *(const V16*)(row + (long)min(j, jx1 - 1) * dyld);
        }
#pragma unroll
        for (int u = 0; u < G; ++u)
#pragma unroll
          for (int e = 0; e < V; ++e) t[e] = xw[u] != 0.f ? fmaf(xw[u], to_f(v[u][e]), t[e]) : t[e];
      }
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = fmaf(yk, t[e], acc[e]);
    }
    V16 o;
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = from_f<T>(acc[e]);
    *(V16*)(dx + (((long)img * hi + ih) * wi + iw) * c + ch) = o;
  }
}
// The same one-pass form for channel counts off the vector width (the supervision heads'
// 19-class logits): a thread per (input pixel, channel), dY dense (pitch c).  Adjacent lanes
// read adjacent channels, so each tap's loads stay contiguous across the wave.
template <typename T, int G>
__global__ void __launch_bounds__(256) bilinear_bwd_fused_kernel(const T* __restrict__ dy, T* __restrict__ dx, int hi, int wi, int c,
                                                                 int ho, int wo, float sh, float sw, int maxh, int maxw, long total,
                                                                 FastDiv f_c, FastDiv f_wi, FastDiv f_hi) {
  extern __shared__ float tab[];
  float* wtab = tab;
  int* wlo = (int*)(wtab + wi * maxw);
  float* htab = (float*)(wlo + wi);
  int* hlo = (int*)(htab + hi * maxh);
  int* wspan = hlo + hi;
  int* hspan = wspan + wi;
  bil_table_build(wtab, wlo, wi, wo, sw, maxw);
  bil_table_build(htab, hlo, hi, ho, sh, maxh);
  bil_table_span(wtab, wspan, wi, maxw);
  bil_table_span(htab, hspan, hi, maxh);
  GRID_STRIDE_XCD(i, total) {  // total < 2^31 (host)
    const uint32_t q = fdiv((uint32_t)i, f_c), r = fdiv(q, f_wi);
    const int ch = (int)((uint32_t)i - q * c), iw = (int)(q - r * wi);
    const uint32_t img = fdiv(r, f_hi);
    const int ih = (int)(r - img * hi);
    const float* wx = wtab + iw * maxw;
    const float* wy = htab + ih * maxh;
    const T* base = dy + (((long)img * ho + hlo[ih]) * wo + wlo[iw]) * c + ch;
    const int jx0 = wspan[iw] & 0xffff, jx1 = wspan[iw] >> 16;
    const int ky0 = hspan[ih] & 0xffff, ky1 = hspan[ih] >> 16;
    float acc = 0.f;
    for (int k = ky0; k < ky1; ++k) {
      const float yk = wy[k];
      if (yk == 0.f) continue;
      const T* row = base + (long)k * wo * c;
      float t = 0.f;
      for (int j0 = jx0; j0 < jx1; j0 += G) {
        T v[G];
        float xw[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
          const int j = j0 + u;
          xw[u] = j < jx1 ? wx[j] : 0.f;
          v[u] = row[(long)min(j, jx1 - 1) * c];
        }
#pragma unroll
        for (int u = 0; u < G; ++u) t = xw[u] != 0.f ? fmaf(xw[u], to_f(v[u]), t) : t;
      }
      acc = fmaf(yk, t, acc);
    }
    dx[i] = from_f<T>(acc);
  }
}
// most outputs any input index of an axis receives from (bil_wsum_range, host float math)
static int bil_maxw(int in, int out, float s) {
  int m = 0;
  for (int i = 0; i < in; ++i) {
    int lo = (int)std::floor(((float)i - 0.5f) / s - 0.5f) - 1;
    int hi = (int)std::ceil(((float)i + 1.5f) / s - 0.5f) + 1;
    lo = std::max(lo, 0);
    hi = std::min(hi, out - 1);
    m = std::max(m, hi - lo + 1);
  }
  return m + 1;  // margin for the device's own rounding of the same range (zero entries)
}
static size_t bil_tab_bytes(int in, int maxw) { return ((size_t)in * maxw + in) * 4; }
// launch both passes table-driven when the tables fit and the index math fits 32 bits, else the
// per-element kernels; w pass reads dy with row pitch dyld at channel offset dyoff
template <typename T>
static void bilinear_bwd_launch(const T* dy, float* tmp, T* dx, int n, int hi, int wi, int c, int ho, int wo, float sh, float sw,
                                int dyld, int dyoff, hipStream_t st) {
  const long tw = (long)n * ho * wi * c, th = (long)n * hi * wi * c;
  const int mw = bil_maxw(wi, wo, sw), mh = bil_maxw(hi, ho, sh);
  const size_t bw = bil_tab_bytes(wi, mw), bh = bil_tab_bytes(hi, mh);
  constexpr int V = VecT<T>::N;
  if (c % V == 0 && dyld % V == 0 && dyoff % V == 0 && th < (1L << 31) && bw + bh + (wi + hi) * 4 <= (size_t)kBilTabLds &&
      (long)n * ho * wo * dyld < (1L << 40)) {
    const long tv = th / V;
    // taps per load batch: 8 when an input column reaches ~8 output columns (x4), else 4 (x2)
    auto kern = mw >= 10 ? bilinear_bwd_fused_vec_kernel<T, 8> : bilinear_bwd_fused_vec_kernel<T, 4>;
    hipLaunchKernelGGL(kern, dim3(ew_blocks(tv)), dim3(256), bw + bh + (wi + hi) * 4, st, dy, dx, hi, wi, c, ho, wo, sh, sw, dyld,
                       dyoff, mh, mw, tv, fastdiv_make(c / V), fastdiv_make(wi), fastdiv_make(hi));
    return;
  }
  if (c % V != 0 && dyld == c && dyoff == 0 && th < (1L << 31) && bw + bh + (wi + hi) * 4 <= (size_t)kBilTabLds &&
      (long)n * ho * wo * c < (1L << 40)) {
    auto kern = mw >= 10 ? bilinear_bwd_fused_kernel<T, 8> : bilinear_bwd_fused_kernel<T, 4>;
    hipLaunchKernelGGL(kern, dim3(ew_blocks(th)), dim3(256), bw + bh + (wi + hi) * 4, st, dy, dx, hi, wi, c, ho, wo, sh, sw, mh, mw,
                       th, fastdiv_make(c), fastdiv_make(wi), fastdiv_make(hi));
    return;
  }
  if (tw < (1L << 31) && bw <= (size_t)kBilTabLds)
    hipLaunchKernelGGL(bilinear_bwd_w_tab_kernel<T>, dim3(ew_blocks(tw)), dim3(256), bw, st, dy, tmp, n, wi, c, ho, wo, sw, dyld,
                       dyoff, mw, fastdiv_make(c), fastdiv_make(wi));
  else
    hipLaunchKernelGGL(bilinear_bwd_w_kernel<T>, dim3(ew_blocks(tw)), dim3(256), 0, st, dy, tmp, n, wi, c, ho, wo, sw, dyld, dyoff);
  if (th < (1L << 31) && bh <= (size_t)kBilTabLds)
    hipLaunchKernelGGL(bilinear_bwd_h_tab_kernel<T>, dim3(ew_blocks(th)), dim3(256), bh, st, (const float*)tmp, dx, n, hi, wi, c, ho,
                       sh, mh, fastdiv_make((uint32_t)wi * c), fastdiv_make(hi));
  else
    hipLaunchKernelGGL(bilinear_bwd_h_kernel<T>, dim3(ew_blocks(th)), dim3(256), 0, st, (const float*)tmp, dx, n, hi, wi, c, ho, sh);
}
extern "C" int rtsds_bilinear_fwd(const void* x, void* y, int n, int hi, int wi, int c, int ho, int wo, float scale_h, float scale_w,
                                  int y_ld, int y_off, int dtype, void* stream) {
  const long total = (long)n * ho * wo * c;
  if (total <= 0 || hi <= 0 || wi <= 0) return RTSDS_ERR_SHAPE;
  if (y_ld <= 0) y_ld = c;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    constexpr int V = VecT<T>::N;
    const long pix = (long)n * ho * wo;
    // grouped taps pay off from ~3 output rows per source row (x2: 24 vs 17 us at 256 ch, x4:
    // 26 vs 28 us, tools/ab_bilinear.sh)
    if (c % V == 0 && y_ld % V == 0 && y_off % V == 0 && ho >= 3 * hi && kBilRowGroup)
      hipLaunchKernelGGL((bilinear_fwd_group_vec_kernel<T, kBilGroupU>), dim3(rt_cdiv(wo * (c / V), 256 * kBilGroupU), n * hi),
                         dim3(256), 0, st, (const T*)x, (T*)y, n, hi, wi, c, ho, wo, scale_h, scale_w, y_ld, y_off, nullptr, nullptr);
    else if (c % V == 0 && y_ld % V == 0 && y_off % V == 0)
      hipLaunchKernelGGL((bilinear_fwd_kernel<T, 0>), dim3(ew_blocks(pix * (c / V))), dim3(256), 0, st, (const T*)x, (T*)y, n, hi, wi, c, ho, wo, scale_h, scale_w, y_ld, y_off);
    else if (c >= V && y_ld == c && y_off == 0 && (wo * c) % V == 0 && 2L * wi * c * 4 <= 64 * 1024 && ho >= hi && kBilRowGroup) {
      // column chunks: <= 256 * kJ vectors each, and enough workgroups to fill the chip
      constexpr int kJ = kBilJ;
      const int nv = wo * c / V;
      int nchunk = std::max((nv + 256 * kJ - 1) / (256 * kJ), (1024 + n * hi - 1) / (n * hi));
      nchunk = std::min(nchunk, std::max(1, nv / 64));
      nchunk = std::max(nchunk, (nv + 256 * kJ - 1) / (256 * kJ));
      hipLaunchKernelGGL((bilinear_fwd_rowgroup_kernel<T, kJ>), dim3(n * hi * nchunk), dim3(256), 2 * wi * c * 4, st, (const T*)x,
                         (T*)y, hi, wi, c, ho, wo, scale_h, scale_w, nchunk, fastdiv_make(c));
    } else if (c >= V && y_ld == c && y_off == 0 && (wo * c) % V == 0 && 2L * wi * c * 4 <= 64 * 1024)
      hipLaunchKernelGGL((bilinear_fwd_rows_kernel<T>), dim3(n * ho), dim3(256), 2 * wi * c * 4, st, (const T*)x, (T*)y, hi, wi, c, ho,
                         wo, scale_h, scale_w, fastdiv_make(c));
    else if (c <= 64)
      hipLaunchKernelGGL((bilinear_fwd_kernel<T, 1>), dim3(ew_blocks(pix)), dim3(256), 0, st, (const T*)x, (T*)y, n, hi, wi, c, ho, wo, scale_h, scale_w, y_ld, y_off);
    else
      hipLaunchKernelGGL((bilinear_fwd_kernel<T, 2>), dim3(ew_blocks(pix * c)), dim3(256), 0, st, (const T*)x, (T*)y, n, hi, wi, c, ho, wo, scale_h, scale_w, y_ld, y_off);
  });
  RET_LAUNCH();
}
extern "C" int rtsds_bilinear_fwd_scaled(const void* x, const void* s1, const void* s2, void* y, int n, int hi, int wi, int c, int ho,
                                         int wo, float scale_h, float scale_w, int y_ld, int y_off, int dtype, void* stream) {
  const long total = (long)n * ho * wo * c;
  if (total <= 0 || hi <= 0 || wi <= 0) return RTSDS_ERR_SHAPE;
  if (y_ld <= 0) y_ld = c;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    constexpr int V = VecT<T>::N;
    if (!(c % V == 0 && y_ld % V == 0 && y_off % V == 0 && ho >= hi)) return RTSDS_ERR_UNSUPPORTED;
    hipLaunchKernelGGL((bilinear_fwd_group_vec_kernel<T, kBilGroupU>), dim3(rt_cdiv(wo * (c / V), 256 * kBilGroupU), n * hi),
                       dim3(256), 0, st, (const T*)x, (T*)y, n, hi, wi, c, ho, wo, scale_h, scale_w, y_ld, y_off, (const T*)s1,
                       (const T*)s2);
  });
  RET_LAUNCH();
}
extern "C" size_t rtsds_bilinear_bwd_workspace(int n, int hi, int wi, int c, int ho, int wo) {
  (void)hi; (void)wo;
  return (size_t)n * ho * wi * c * sizeof(float) + 256;
}
extern "C" int rtsds_bilinear_bwd(const void* dy, void* dx, int n, int hi, int wi, int c, int ho, int wo, float scale_h, float scale_w,
                                  int dy_ld, int dy_off, int dtype, void* ws, size_t ws_bytes, void* stream) {
  const long total = (long)n * hi * wi * c;
  if (total <= 0 || ho <= 0 || wo <= 0) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_bilinear_bwd_workspace(n, hi, wi, c, ho, wo)) return RTSDS_ERR_WORKSPACE;
  if (dy_ld <= 0) dy_ld = c;
  hipStream_t st = (hipStream_t)stream;
  float* tmp = (float*)ws;
  DISPATCH_T(dtype, bilinear_bwd_launch<T>((const T*)dy, tmp, (T*)dx, n, hi, wi, c, ho, wo, scale_h, scale_w, dy_ld, dy_off, st));
  RET_LAUNCH();
}


// ------------------------------------------------------------------ LDS-staged per-pixel kernels
// The per-pixel channel loops (C = 19 classes) read/write rows of C*sizeof(T) bytes (38 B for
// bf16) that are not 16-B aligned per pixel.  These variants move a block's 256 pixels
// (256*C elements, contiguous in NHWC) between HBM and LDS with 16-B vector accesses and
// run the per-pixel math out of LDS, so global traffic is fully coalesced.
static const int kStagePix = 256;
template <typename T>
RT_DEV void stage_in(const T* __restrict__ g, T* s, int nel) {
  const int nb = nel * (int)sizeof(T);
  const char* gb = (const char*)g;
  char* sb = (char*)s;
  if ((((uintptr_t)gb) & 15) == 0) {
    const int nv = nb >> 4;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) ((uint4*)sb)[i] = ((const uint4*)gb)[i];
    for (int i = (nv << 4) / (int)sizeof(T) + threadIdx.x; i < nel; i += blockDim.x) s[i] = g[i];
  } else {
    for (int i = threadIdx.x; i < nel; i += blockDim.x) s[i] = g[i];
  }
}
template <typename T>
RT_DEV void stage_out(T* __restrict__ g, const T* s, int nel) {
  const int nb = nel * (int)sizeof(T);
  char* gb = (char*)g;
  const char* sb = (const char*)s;
  if ((((uintptr_t)gb) & 15) == 0) {
    const int nv = nb >> 4;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) ((uint4*)gb)[i] = ((const uint4*)sb)[i];
    for (int i = (nv << 4) / (int)sizeof(T) + threadIdx.x; i < nel; i += blockDim.x) g[i] = s[i];
  } else {
    for (int i = threadIdx.x; i < nel; i += blockDim.x) g[i] = s[i];
  }
}
// ------------------------------------------------------------------ fused resize + softmax
// The discriminator input of the DA iteration (train.py:225,245,256): softmax over classes of
// the bilinearly resized head, zero-padded to y_ld channels so the discriminator's first conv
// reads it without a separate pad pass.  The logits are the bilinear_fwd values rounded to T
// and the softmax is softmax_fwd_staged's arithmetic (two expf passes, sequential sum), so the
// probabilities are bit-identical to the unfused resize -> softmax -> pad chain; the resized
// logits and the unpadded probabilities never exist in memory.
//   forward:  one block per 256 output pixels of a row.  The two low-res source rows the tile
//             reads (a few dozen pixels for x8) are staged once in LDS as fp32 (coalesced), each
//             thread blends its pixel's 4 taps from LDS, and the tile's padded rows leave through
//             LDS as lane-consecutive 16-B chunks (HBM-bound on the padded output).
//   backward: one block per (row, tile of up to 64 input columns): the dy segment the tile's
//             width adjoint reads is staged in LDS (coalesced), then thread per output pixel
//             forms the softmax backward T(p_k (dp_k - sum_j p_j dp_j)) in place (its p row by
//             16-B loads); the tile's bilinear
//             weights are tabulated once in LDS; thread per (input column, class) accumulates
//             the width adjoint in bilinear_bwd_w_kernel's order (ascending output column,
//             zero weights skipped).  The vertical pass is bilinear_bwd_h_kernel.
static const int kUpsmMaxC = 32;
static const int kUpsmPix = 256;
static const int kUpsmLds = 48 * 1024;
// one output pixel of upsoftmax_fwd_kernel: blend, softmax, padded row into the LDS tile
template <typename T, bool STAGED, int CC>
RT_DEV void upsm_pixel(const T* __restrict__ r0, const T* __restrict__ r1, const float* src, T* o, int wlo, int n1, int c_, int ow,
                       float sw, int wi, float lh0, float lh1, int yld) {
  const int c = CC > 0 ? CC : c_;
  int w0, w1;
  float lw0, lw1;
  bil_src(ow, sw, wi, w0, w1, lw0, lw1);
  float z[kUpsmMaxC];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < kUpsmMaxC; ++k) {
    if (k < c) {
      float p00, p01, p10, p11;
      if (STAGED) {
        p00 = src[(w0 - wlo) * c + k];
        p01 = src[(w1 - wlo) * c + k];
        p10 = src[n1 + (w0 - wlo) * c + k];
        p11 = src[n1 + (w1 - wlo) * c + k];
      } else {
        p00 = to_f(r0[(long)w0 * c + k]);
        p01 = to_f(r0[(long)w1 * c + k]);
        p10 = to_f(r1[(long)w0 * c + k]);
        p11 = to_f(r1[(long)w1 * c + k]);
      }
      z[k] = to_f(from_f<T>(bil_mix(p00, p01, p10, p11, lh0, lh1, lw0, lw1)));
      m = fmaxf(m, z[k]);
    }
  }
  float sum = 0.f;  // exp(z - m) evaluated once per class (softmax_fwd_staged evaluates the same
                    // expf twice: identical values)
#pragma unroll
  for (int k = 0; k < kUpsmMaxC; ++k)
    if (k < c) {
      z[k] = expf(z[k] - m);
      sum += z[k];
    }
  const float iz = 1.f / sum;
  // the padded row goes through LDS so the tile leaves as lane-consecutive 16-B chunks (the
  // tile's rows are contiguous in y): full-line writes instead of 64-B-strided partial ones
  if (sizeof(T) == 2 && yld == 32) {  // 4 x 16-B LDS writes, chunk q at slot q ^ (pixel & 3)
    typedef typename VecT<T>::v16 V16;
    const int sw4 = ow & 3;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      V16 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = from_f<T>(q * 8 + j < c ? z[q * 8 + j] * iz : 0.f);
      *(V16*)(o + (q ^ sw4) * 8) = v;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kUpsmMaxC; ++k)
      if (k < yld) o[k] = from_f<T>(k < c ? z[k] * iz : 0.f);
  }
}
template <typename T, bool STAGED, int CC>  // CC > 0: compile-time class count (19), 0: runtime c
__global__ void __launch_bounds__(256) upsoftmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int hi, int wi, int c_,
                                                            int ho, int wo, float sh, float sw, int yld, int tiles) {
  const int c = CC > 0 ? CC : c_;
  extern __shared__ __attribute__((aligned(16))) float src[];  // STAGED: [2][ncols][c]
  const int tile = blockIdx.x % tiles;
  const long row = blockIdx.x / tiles;  // img * ho + oh
  const int oh = (int)(row % ho), img = (int)(row / ho);
  const int ow0 = tile * kUpsmPix, np = min(kUpsmPix, wo - ow0);
  const int tid = threadIdx.x;
  int h0, h1;
  float lh0, lh1;
  bil_src(oh, sh, hi, h0, h1, lh0, lh1);
  const T* r0 = x + ((long)img * hi + h0) * wi * c;
  const T* r1 = x + ((long)img * hi + h1) * wi * c;
  int wlo = 0, n1 = 0;
  if (STAGED) {  // taps are monotone in ow: columns [w0(ow0), w1(last)] cover the tile
    int a0, a1, b0, b1;
    float t0, t1;
    bil_src(ow0, sw, wi, a0, a1, t0, t1);
    bil_src(ow0 + np - 1, sw, wi, b0, b1, t0, t1);
    wlo = a0;
    n1 = (b1 - a0 + 1) * c;
    for (int e = tid; e < n1; e += 256) {
      src[e] = to_f(r0[(long)wlo * c + e]);
      src[n1 + e] = to_f(r1[(long)wlo * c + e]);
    }
    __syncthreads();
  }
  T* outbuf = (T*)(src + ((2 * n1 + 3) & ~3));  // [256][yld], 16-B aligned
  if (tid < np) upsm_pixel<T, STAGED, CC>(r0, r1, src, outbuf + tid * yld, wlo, n1, c, ow0 + tid, sw, wi, lh0, lh1, yld);
  __syncthreads();  // every lane reaches the same barrier (no early exit)
  T* dst = y + (row * wo + ow0) * yld;
  if (sizeof(T) == 2 && yld == 32) {  // un-swizzle: LDS read linear, global chunk q = slot ^ (pixel & 3)
    typedef typename VecT<T>::v16 V16;
    for (int i = tid; i < np * 4; i += 256) {
      const int t = i >> 2, q = (i & 3) ^ ((ow0 + t) & 3);
      *(V16*)(dst + t * 32 + q * 8) = *(const V16*)(outbuf + i * 8);
    }
  } else {
    stage_out(dst, outbuf, np * yld);
  }
}
// exact output-pixel span [lo, hi] read by input columns [iw0, iw1] (bil_wsum_range bounds)
__host__ __device__ inline void upsm_span(int iw0, int iw1, float sw, int wi, int wo, int& lo, int& hi) {
  lo = (int)floorf(((float)iw0 - 0.5f) / sw - 0.5f) - 1;
  hi = (int)ceilf(((float)iw1 + 1.5f) / sw - 0.5f) + 1;
  lo = lo < 0 ? 0 : lo;
  hi = hi > wo - 1 ? wo - 1 : hi;
}
template <typename T, int CC>  // CC > 0: compile-time class count (19), 0: runtime c
__global__ void __launch_bounds__(256) upsoftmax_bwd_w_kernel(const T* __restrict__ dy, int dyld, const T* __restrict__ y,
                                                              int yld, float* __restrict__ tmp, int wi, int c_, int wo, float sw,
                                                              int tw, int tiles, int cap, int maxw) {
  const int c = CC > 0 ? CC : c_;
  extern __shared__ __attribute__((aligned(16))) float smf[];
  float* wt = smf;                       // [tw][maxw]: weights of output columns lo(iw) + j
  int* wlo = (int*)(wt + tw * maxw);     // [tw]
  T* sgt = (T*)(wlo + tw);               // [cap][c]: dy, then the softmax backward in place
  const int tid = threadIdx.x;
  const int tile = blockIdx.x % tiles;
  const long row = blockIdx.x / tiles;  // img * ho + oh
  const int iw0 = tile * tw, iw1 = min(wi, iw0 + tw) - 1, nw = iw1 - iw0 + 1;
  int olo, ohi;
  upsm_span(iw0, iw1, sw, wi, wo, olo, ohi);
  const int cnt = ohi - olo + 1;  // <= cap (host: exact maximum over the tiles)
  // dy segment -> LDS as T, coalesced (rows of pitch c; contiguous in memory when dyld == c)
  const T* gseg = dy + (row * wo + olo) * dyld;
  if (dyld == c) {
    for (int e = tid; e < cnt * c; e += 256) sgt[e] = gseg[e];
  } else {
    for (int e = tid; e < cnt * c; e += 256) {
      const int q = e / c;
      sgt[e] = gseg[(long)q * dyld + (e - q * c)];
    }
  }
  __syncthreads();
  // thread per output pixel: p row (16-B vectors when the pitch allows), softmax backward in place
  for (int q = tid; q < cnt; q += 256) {
    const T* pr = y + (row * wo + olo + q) * yld;
    float pv[kUpsmMaxC];
    if (sizeof(T) == 2 && (yld & 7) == 0) {
      typedef typename VecT<T>::v16 V16;
#pragma unroll
      for (int v = 0; v < kUpsmMaxC / 8; ++v)
        if (v * 8 < c) {
          const V16 t = *(const V16*)(pr + v * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) pv[v * 8 + j] = to_f(t[j]);
        }
    } else {
#pragma unroll
      for (int k = 0; k < kUpsmMaxC; ++k)
        if (k < c) pv[k] = to_f(pr[k]);
    }
    T* g = sgt + q * c;
    float gv[kUpsmMaxC];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < kUpsmMaxC; ++k)
      if (k < c) {
        gv[k] = to_f(g[k]);
        dot = fmaf(gv[k], pv[k], dot);
      }
#pragma unroll
    for (int k = 0; k < kUpsmMaxC; ++k)
      if (k < c) g[k] = from_f<T>(pv[k] * (gv[k] - dot));
  }
  for (int e = tid; e < nw * maxw; e += 256) {
    const int il = e / maxw, j = e - il * maxw, iw = iw0 + il;
    int lo, hi;
    bil_wsum_range(iw, sw, wi, wo, lo, hi);
    wt[e] = lo + j <= hi ? bil_weight(lo + j, iw, sw, wi) : 0.f;
    if (j == 0) wlo[il] = lo - olo;
  }
  __syncthreads();
  for (int e = tid; e < nw * c; e += 256) {  // (input column, class) items, classes inner
    const int il = e / c, k = e - il * c;
    const float* w = wt + il * maxw;
    const T* s = sgt + wlo[il] * c + k;
    float acc = 0.f;
    for (int j = 0; j < maxw; ++j) {
      const float wv = w[j];
      if (wv != 0.f) acc = fmaf(wv, to_f(s[j * c]), acc);
    }
    tmp[(row * wi + iw0) * c + e] = acc;
  }
}
// columns of the low-res rows one forward tile stages (taps monotone in ow)
static int upsm_fwd_cols(int wi, int wo, float sw) {
  int cols = 0;
  for (int ow0 = 0; ow0 < wo; ow0 += kUpsmPix) {
    const int ow1 = std::min(wo, ow0 + kUpsmPix) - 1;
    float src0 = sw * ((float)ow0 + 0.5f) - 0.5f, src1 = sw * ((float)ow1 + 0.5f) - 0.5f;
    int a = src0 < 0.f ? 0 : (int)src0, b = src1 < 0.f ? 0 : (int)src1;
    a = std::min(a, wi - 1);
    b = std::min(b, wi - 1);
    b = b + (b < wi - 1 ? 1 : 0);
    cols = std::max(cols, b - a + 1);
  }
  return cols + 2;  // margin: the device computes the tap columns with its own float rounding
}
extern "C" int rtsds_upsoftmax_fwd(const void* x, void* y, int n, int hi, int wi, int c, int ho, int wo, float scale_h,
                                   float scale_w, int y_ld, int dtype, void* stream) {
  if (n <= 0 || ho <= 0 || wo <= 0 || hi <= 0 || wi <= 0 || c <= 0 || c > kUpsmMaxC || y_ld < c || y_ld > kUpsmMaxC)
    return RTSDS_ERR_SHAPE;
  const int tiles = rt_cdiv(wo, kUpsmPix);
  const long blocks = (long)n * ho * tiles;
  if (blocks > INT_MAX) return RTSDS_ERR_UNSUPPORTED;
  const size_t taps = (size_t)2 * upsm_fwd_cols(wi, wo, scale_w) * c * sizeof(float);
  const bool staged = taps <= (size_t)kUpsmLds;
  const size_t outb = (size_t)kUpsmPix * y_ld * (dtype == RTSDS_BF16 ? 2 : 4);
  const size_t lds = (staged ? taps + 16 : 0) + outb;
  hipStream_t st = (hipStream_t)stream;
  DISPATCH_T(dtype, {
    if (staged && c == 19)
      hipLaunchKernelGGL((upsoftmax_fwd_kernel<T, true, 19>), dim3((unsigned)blocks), dim3(256), lds, st, (const T*)x, (T*)y, hi,
                         wi, c, ho, wo, scale_h, scale_w, y_ld, tiles);
    else if (staged)
      hipLaunchKernelGGL((upsoftmax_fwd_kernel<T, true, 0>), dim3((unsigned)blocks), dim3(256), lds, st, (const T*)x, (T*)y, hi,
                         wi, c, ho, wo, scale_h, scale_w, y_ld, tiles);
    else
      hipLaunchKernelGGL((upsoftmax_fwd_kernel<T, false, 0>), dim3((unsigned)blocks), dim3(256), lds, st, (const T*)x, (T*)y, hi,
                         wi, c, ho, wo, scale_h, scale_w, y_ld, tiles);
  });
  RET_LAUNCH();
}
extern "C" size_t rtsds_upsoftmax_bwd_workspace(int n, int hi, int wi, int c, int ho, int wo) {
  return rtsds_bilinear_bwd_workspace(n, hi, wi, c, ho, wo);
}
// widest tile (<= 64 input columns) whose staged segment + weight table fit kUpsmLds; cap =
// its exact largest segment, maxw = the most output columns any input column reads
static bool upsm_tiling(int wi, int wo, int c, float sw, size_t esz, int& tw, int& cap, int& maxw) {
  maxw = 0;
  for (int iw = 0; iw < wi; ++iw) {
    int lo, hi;
    upsm_span(iw, iw, sw, wi, wo, lo, hi);
    maxw = std::max(maxw, hi - lo + 1);
  }
  for (tw = 64; tw >= 1; tw /= 2) {
    cap = 0;
    for (int iw0 = 0; iw0 < wi; iw0 += tw) {
      int lo, hi;
      upsm_span(iw0, std::min(wi, iw0 + tw) - 1, sw, wi, wo, lo, hi);
      cap = std::max(cap, hi - lo + 1);
    }
    if ((size_t)cap * c * esz + (size_t)tw * (maxw + 1) * 4 <= (size_t)kUpsmLds) return true;
  }
  return false;
}
extern "C" int rtsds_upsoftmax_bwd(const void* dy, int dy_ld, const void* y, int y_ld, void* dx, int n, int hi, int wi, int c,
                                   int ho, int wo, float scale_h, float scale_w, int dtype, void* ws, size_t ws_bytes,
                                   void* stream) {
  const long total = (long)n * hi * wi * c;
  if (total <= 0 || ho <= 0 || wo <= 0 || c > kUpsmMaxC || dy_ld < c || y_ld < c) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_upsoftmax_bwd_workspace(n, hi, wi, c, ho, wo)) return RTSDS_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  float* tmp = (float*)ws;
  DISPATCH_T(dtype, {
    int tw, cap, maxw;
    if (!upsm_tiling(wi, wo, c, scale_w, sizeof(T), tw, cap, maxw)) return RTSDS_ERR_UNSUPPORTED;
    const int tiles = rt_cdiv(wi, tw);
    const long blocks = (long)n * ho * tiles;
    if (blocks > INT_MAX) return RTSDS_ERR_UNSUPPORTED;
    const size_t lds = (size_t)tw * (maxw + 1) * 4 + (size_t)cap * c * sizeof(T);
    if (c == 19)
      hipLaunchKernelGGL((upsoftmax_bwd_w_kernel<T, 19>), dim3((unsigned)blocks), dim3(256), lds, st, (const T*)dy, dy_ld,
                         (const T*)y, y_ld, tmp, wi, c, wo, scale_w, tw, tiles, cap, maxw);
    else
      hipLaunchKernelGGL((upsoftmax_bwd_w_kernel<T, 0>), dim3((unsigned)blocks), dim3(256), lds, st, (const T*)dy, dy_ld,
                         (const T*)y, y_ld, tmp, wi, c, wo, scale_w, tw, tiles, cap, maxw);
    const int mh = bil_maxw(hi, ho, scale_h);
    const size_t bh = bil_tab_bytes(hi, mh);
    if (total < (1L << 31) && bh <= (size_t)kBilTabLds)
      hipLaunchKernelGGL(bilinear_bwd_h_tab_kernel<T>, dim3(ew_blocks(total)), dim3(256), bh, st, (const float*)tmp, (T*)dx, n,
                         hi, wi, c, ho, scale_h, mh, fastdiv_make((uint32_t)wi * c), fastdiv_make(hi));
    else
      hipLaunchKernelGGL(bilinear_bwd_h_kernel<T>, dim3(ew_blocks(total)), dim3(256), 0, st, (const float*)tmp, (T*)dx, n, hi,
                         wi, c, ho, scale_h);
  });
  RET_LAUNCH();
}

// Staged variants need NHWC-contiguous logits with c <= kStageMaxC.
static const int kStageMaxC = 64;
static inline bool stage_ok(long sn, long sc, long shw, long hw, int c) {
  return sc == 1 && shw == c && sn == hw * c && c <= kStageMaxC;
}

template <typename T>
__global__ void __launch_bounds__(256) softmax_fwd_staged(const T* __restrict__ x, T* __restrict__ y, long total, int c) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* buf = (T*)smem_raw;
  for (long p0 = (long)blockIdx.x * kStagePix; p0 < total; p0 += (long)gridDim.x * kStagePix) {
    const int np = (int)min<long>(kStagePix, total - p0);
    __syncthreads();
    stage_in(x + p0 * c, buf, np * c);
    __syncthreads();
    if ((int)threadIdx.x < np) {
      T* r = buf + threadIdx.x * c;
      float m = -INFINITY;
      for (int k = 0; k < c; ++k) m = fmaxf(m, to_f(r[k]));
      float z = 0.f;
      for (int k = 0; k < c; ++k) z += expf(to_f(r[k]) - m);
      const float iz = 1.f / z;
      for (int k = 0; k < c; ++k) r[k] = from_f<T>(expf(to_f(r[k]) - m) * iz);
    }
    __syncthreads();
    stage_out(y + p0 * c, buf, np * c);
  }
}
template <typename T>
__global__ void __launch_bounds__(256) softmax_bwd_staged(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx, long total, int c) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* bg = (T*)smem_raw;
  T* by = bg + kStagePix * c;
  for (long p0 = (long)blockIdx.x * kStagePix; p0 < total; p0 += (long)gridDim.x * kStagePix) {
    const int np = (int)min<long>(kStagePix, total - p0);
    __syncthreads();
    stage_in(dy + p0 * c, bg, np * c);
    stage_in(y + p0 * c, by, np * c);
    __syncthreads();
    if ((int)threadIdx.x < np) {
      T* g = bg + threadIdx.x * c;
      const T* yy = by + threadIdx.x * c;
      float dot = 0.f;
      for (int k = 0; k < c; ++k) dot = fmaf(to_f(g[k]), to_f(yy[k]), dot);
      for (int k = 0; k < c; ++k) g[k] = from_f<T>(to_f(yy[k]) * (to_f(g[k]) - dot));
    }
    __syncthreads();
    stage_out(dx + p0 * c, bg, np * c);
  }
}

// ------------------------------------------------------------------ channel softmax (dim=1)
// train.py:225,245,256.  One thread per pixel; logits addressed by (sn, sc, shw) strides so
// NHWC and NCHW tensors both work.  Output NHWC contiguous with row pitch yld (zero-padded
// channels c..yld-1 so a padded discriminator input can be produced directly).
template <typename T, typename O>
__global__ void softmax_fwd_kernel(const T* __restrict__ x, O* __restrict__ y, int n, long hw, int c, long sn, long sc, long shw, int yld) {
  const long total = (long)n * hw;
  GRID_STRIDE(p, total) {
    const long img = p / hw, s = p - img * hw;
    const T* b = x + img * sn + s * shw;
    float m = -INFINITY;
    for (int k = 0; k < c; ++k) m = fmaxf(m, to_f(b[k * sc]));
    float z = 0.f;
    for (int k = 0; k < c; ++k) z += expf(to_f(b[k * sc]) - m);
    const float iz = 1.f / z;
    O* o = y + p * yld;
    for (int k = 0; k < c; ++k) o[k] = from_f<O>(expf(to_f(b[k * sc]) - m) * iz);
    for (int k = c; k < yld; ++k) o[k] = from_f<O>(0.f);
  }
}
// dx = y * (dy - sum_k dy_k y_k); dy/y have row pitch ld (>= c), dx strided like the logits.
template <typename T, typename O>
__global__ void softmax_bwd_kernel(const O* __restrict__ dy, const O* __restrict__ y, T* __restrict__ dx, int n, long hw, int c, int ld,
                                   long sn, long sc, long shw) {
  const long total = (long)n * hw;
  GRID_STRIDE(p, total) {
    const long img = p / hw, s = p - img * hw;
    const O* g = dy + p * ld;
    const O* yy = y + p * ld;
    float dot = 0.f;
    for (int k = 0; k < c; ++k) dot = fmaf(to_f(g[k]), to_f(yy[k]), dot);
    T* o = dx + img * sn + s * shw;
    for (int k = 0; k < c; ++k) o[k * sc] = from_f<T>(to_f(yy[k]) * (to_f(g[k]) - dot));
  }
}
extern "C" int rtsds_softmax_fwd(const void* x, long sn, long sc, long shw, void* y, int y_ld, int n, long hw, int c, int dtype,
                                 void* stream) {
  if (n <= 0 || hw <= 0 || c <= 0 || y_ld < c) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, {
    if (y_ld == c && stage_ok(sn, sc, shw, hw, c))
      hipLaunchKernelGGL(softmax_fwd_staged<T>, dim3(ew_blocks((long)n * hw, kStagePix, 4096)), dim3(256), kStagePix * c * sizeof(T),
                         (hipStream_t)stream, (const T*)x, (T*)y, (long)n * hw, c);
    else
      hipLaunchKernelGGL((softmax_fwd_kernel<T, T>), dim3(ew_blocks((long)n * hw)), dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y, n, hw, c, sn, sc, shw, y_ld);
  });
  RET_LAUNCH();
}
extern "C" int rtsds_softmax_bwd(const void* dy, const void* y, int ld, void* dx, long sn, long sc, long shw, int n, long hw, int c,
                                 int dtype, void* stream) {
  if (n <= 0 || hw <= 0 || c <= 0 || ld < c) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, {
    if (ld == c && stage_ok(sn, sc, shw, hw, c))
      hipLaunchKernelGGL(softmax_bwd_staged<T>, dim3(ew_blocks((long)n * hw, kStagePix, 4096)), dim3(256), 2 * kStagePix * c * sizeof(T),
                         (hipStream_t)stream, (const T*)dy, (const T*)y, (T*)dx, (long)n * hw, c);
    else
      hipLaunchKernelGGL((softmax_bwd_kernel<T, T>), dim3(ew_blocks((long)n * hw)), dim3(256), 0, (hipStream_t)stream, (const T*)dy, (const T*)y, (T*)dx, n, hw, c, ld, sn, sc, shw);
  });
  RET_LAUNCH();
}

// ------------------------------------------------------------------ cross entropy (ignore_index)
// nn.CrossEntropyLoss(ignore_index=19) (main.py:124-130, train.py:86-92,202-204): mean over
// non-ignored pixels of logsumexp(x) - x[t].  Two passes for the forward (per-block partial
// (sum, count) -> final), one fused pass for the backward.
// ws layout: [0, RB) partial sums, [RB, 2RB) partial counts, [2RB] total count.
static const int kCeRB = 1024;
template <typename T>
__global__ void ce_fwd_part_kernel(const T* __restrict__ x, const int64_t* __restrict__ tgt, float* __restrict__ part, int n, long hw, int c,
                                   long sn, long sc, long shw, int ignore) {
  __shared__ float rs[4], rc[4];
  const long total = (long)n * hw;
  float ls = 0.f, lc = 0.f;
  GRID_STRIDE(p, total) {
    const long t = tgt[p];
    if (t == ignore) continue;
    const long img = p / hw, s = p - img * hw;
    const T* b = x + img * sn + s * shw;
    float m = -INFINITY;
    for (int k = 0; k < c; ++k) m = fmaxf(m, to_f(b[k * sc]));
    float z = 0.f;
    for (int k = 0; k < c; ++k) z += expf(to_f(b[k * sc]) - m);
    const float xt = (t >= 0 && t < c) ? to_f(b[t * sc]) : NAN;
    ls += logf(z) + m - xt;
    lc += 1.f;
  }
  ls = wave_sum(ls);
  lc = wave_sum(lc);
  if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = ls; rc[threadIdx.x >> 6] = lc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = rs[0] + rs[1] + rs[2] + rs[3];
    part[kCeRB + blockIdx.x] = rc[0] + rc[1] + rc[2] + rc[3];
  }
}
__global__ void ce_fwd_final_kernel(float* __restrict__ part, int nb, float* __restrict__ loss) {
  __shared__ float rs[4], rc[4];
  float s = 0.f, cn = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) { s += part[i]; cn += part[kCeRB + i]; }
  s = wave_sum(s);
  cn = wave_sum(cn);
  if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = s; rc[threadIdx.x >> 6] = cn; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float S = rs[0] + rs[1] + rs[2] + rs[3], C = rc[0] + rc[1] + rc[2] + rc[3];
    part[2 * kCeRB] = C;
    part[2 * kCeRB + 1] = S;
    loss[0] = S / C;
  }
}
__global__ void ce_finish_kernel(const float* __restrict__ part, float* __restrict__ loss) {
  if (threadIdx.x == 0) loss[0] = part[2 * kCeRB + 1] / part[2 * kCeRB];
}
template <typename T>
__global__ void ce_bwd_kernel(const T* __restrict__ x, const int64_t* __restrict__ tgt, const float* __restrict__ gout,
                              const float* __restrict__ count, T* __restrict__ dx, int n, long hw, int c, long sn, long sc, long shw,
                              int ignore) {
  const long total = (long)n * hw;
  const float g = gout[0] / count[0];
  GRID_STRIDE(p, total) {
    const long t = tgt[p];
    const long img = p / hw, s = p - img * hw;
    const T* b = x + img * sn + s * shw;
    T* o = dx + img * sn + s * shw;
    if (t == ignore) {
      for (int k = 0; k < c; ++k) o[k * sc] = from_f<T>(0.f);
      continue;
    }
    float m = -INFINITY;
    for (int k = 0; k < c; ++k) m = fmaxf(m, to_f(b[k * sc]));
    float z = 0.f;
    for (int k = 0; k < c; ++k) z += expf(to_f(b[k * sc]) - m);
    const float iz = 1.f / z;
    for (int k = 0; k < c; ++k) {
      const float pr = expf(to_f(b[k * sc]) - m) * iz;
      o[k * sc] = from_f<T>(g * (pr - (k == t ? 1.f : 0.f)));
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) ce_fwd_part_staged(const T* __restrict__ x, const int64_t* __restrict__ tgt, float* __restrict__ part,
                                                          long total, int c, int ignore) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* buf = (T*)smem_raw;
  __shared__ float rs[4], rc[4];
  float ls = 0.f, lc = 0.f;
  for (long p0 = (long)blockIdx.x * kStagePix; p0 < total; p0 += (long)gridDim.x * kStagePix) {
    const int np = (int)min<long>(kStagePix, total - p0);
    __syncthreads();
    stage_in(x + p0 * c, buf, np * c);
    __syncthreads();
    if ((int)threadIdx.x < np) {
      const long t = tgt[p0 + threadIdx.x];
      if (t != ignore) {
        const T* r = buf + threadIdx.x * c;
        float m = -INFINITY;
        for (int k = 0; k < c; ++k) m = fmaxf(m, to_f(r[k]));
        float z = 0.f;
        for (int k = 0; k < c; ++k) z += expf(to_f(r[k]) - m);
        const float xt = (t >= 0 && t < c) ? to_f(r[t]) : NAN;
        ls += logf(z) + m - xt;
        lc += 1.f;
      }
    }
  }
  ls = wave_sum(ls);
  lc = wave_sum(lc);
  if ((threadIdx.x & 63) == 0) { rs[threadIdx.x >> 6] = ls; rc[threadIdx.x >> 6] = lc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = rs[0] + rs[1] + rs[2] + rs[3];
    part[kCeRB + blockIdx.x] = rc[0] + rc[1] + rc[2] + rc[3];
  }
}
template <typename T>
__global__ void __launch_bounds__(256) ce_bwd_staged(const T* __restrict__ x, const int64_t* __restrict__ tgt, const float* __restrict__ gout,
                                                     const float* __restrict__ count, T* __restrict__ dx, long total, int c, int ignore) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* buf = (T*)smem_raw;
  const float g = gout[0] / count[0];
  for (long p0 = (long)blockIdx.x * kStagePix; p0 < total; p0 += (long)gridDim.x * kStagePix) {
    const int np = (int)min<long>(kStagePix, total - p0);
    __syncthreads();
    stage_in(x + p0 * c, buf, np * c);
    __syncthreads();
    if ((int)threadIdx.x < np) {
      const long t = tgt[p0 + threadIdx.x];
      T* r = buf + threadIdx.x * c;
      if (t == ignore) {
        for (int k = 0; k < c; ++k) r[k] = from_f<T>(0.f);
      } else {
        float m = -INFINITY;
        for (int k = 0; k < c; ++k) m = fmaxf(m, to_f(r[k]));
        float z = 0.f;
        for (int k = 0; k < c; ++k) z += expf(to_f(r[k]) - m);
        const float gz = g / z;
        for (int k = 0; k < c; ++k) r[k] = from_f<T>(gz * expf(to_f(r[k]) - m) - (k == t ? g : 0.f));
      }
    }
    __syncthreads();
    stage_out(dx + p0 * c, buf, np * c);
  }
}

extern "C" size_t rtsds_ce_workspace(void) { return (2 * kCeRB + 64) * sizeof(float); }
extern "C" int rtsds_ce_fwd(const void* x, long sn, long sc, long shw, const int64_t* tgt, float* loss, int n, long hw, int c,
                            int ignore_index, int dtype, void* ws, size_t ws_bytes, void* stream) {
  if (n <= 0 || hw <= 0 || c <= 0) return RTSDS_ERR_SHAPE;
  if (ws_bytes < rtsds_ce_workspace()) return RTSDS_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int nb = std::min<int>(kCeRB, ew_blocks((long)n * hw, kStagePix, kCeRB));
  DISPATCH_T(dtype, {
    if (stage_ok(sn, sc, shw, hw, c))
      hipLaunchKernelGGL(ce_fwd_part_staged<T>, dim3(nb), dim3(256), kStagePix * c * sizeof(T), st, (const T*)x, tgt, (float*)ws,
                         (long)n * hw, c, ignore_index);
    else
      hipLaunchKernelGGL(ce_fwd_part_kernel<T>, dim3(nb), dim3(256), 0, st, (const T*)x, tgt, (float*)ws, n, hw, c, sn, sc, shw, ignore_index);
  });
  hipLaunchKernelGGL(ce_fwd_final_kernel, dim3(1), dim3(256), 0, st, (float*)ws, nb, loss);
  RET_LAUNCH();
}
// loss = S / C with C summed by the caller over data-parallel ranks (ws + 2*1024 floats: C, S).
extern "C" int rtsds_ce_finish(const void* ws, float* loss, void* stream) {
  hipLaunchKernelGGL(ce_finish_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)ws, loss);
  RET_LAUNCH();
}
// count = the valid-pixel count written by rtsds_ce_fwd into its workspace (ws + 2*1024 floats).
extern "C" int rtsds_ce_bwd(const void* x, long sn, long sc, long shw, const int64_t* tgt, const float* grad_loss, const float* count,
                            void* dx, int n, long hw, int c, int ignore_index, int dtype, void* stream) {
  if (n <= 0 || hw <= 0 || c <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, {
    if (stage_ok(sn, sc, shw, hw, c))
      hipLaunchKernelGGL(ce_bwd_staged<T>, dim3(ew_blocks((long)n * hw, kStagePix, 4096)), dim3(256), kStagePix * c * sizeof(T),
                         (hipStream_t)stream, (const T*)x, tgt, grad_loss, count, (T*)dx, (long)n * hw, c, ignore_index);
    else
      hipLaunchKernelGGL(ce_bwd_kernel<T>, dim3(ew_blocks((long)n * hw)), dim3(256), 0, (hipStream_t)stream, (const T*)x, tgt, grad_loss, count, (T*)dx, n, hw, c, sn, sc, shw, ignore_index);
  });
  RET_LAUNCH();
}

// ------------------------------------------------------------------ BCE with logits
// nn.BCEWithLogitsLoss() (main.py:131-132, train.py:229,247,258): mean of
// max(x,0) - x*t + log1p(exp(-|x|)).  Tiny (one logit per image): one block.
__global__ void bce_fwd_kernel(const float* __restrict__ x, const float* __restrict__ t, float* __restrict__ loss, int n) {
  __shared__ float r[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float v = x[i];
    s += fmaxf(v, 0.f) - v * t[i] + log1pf(expf(-fabsf(v)));
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = (r[0] + r[1] + r[2] + r[3]) / (float)n;
}
__global__ void bce_bwd_kernel(const float* __restrict__ x, const float* __restrict__ t, const float* __restrict__ gout, float* __restrict__ dx, int n) {
  const float g = gout[0] / (float)n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float s = 1.f / (1.f + expf(-x[i]));
    dx[i] = g * (s - t[i]);
  }
}
extern "C" int rtsds_bce_fwd(const float* x, const float* target, float* loss, int n, void* stream) {
  if (n <= 0) return RTSDS_ERR_SHAPE;
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, x, target, loss, n);
  RET_LAUNCH();
}
extern "C" int rtsds_bce_bwd(const float* x, const float* target, const float* grad_loss, float* dx, int n, void* stream) {
  if (n <= 0) return RTSDS_ERR_SHAPE;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, (hipStream_t)stream, x, target, grad_loss, dx, n);
  RET_LAUNCH();
}

// ------------------------------------------------------------------ Adam (flat, fused)
// torch.optim.Adam (main.py:116-117; L2 weight decay folded into the gradient, as torch does
// for weight_decay != 0 without decoupling).  One launch over the flat parameter arena;
// optionally refreshes the bf16 shadow weights in the same pass.
template <typename GT>
__global__ void adam_kernel(float* __restrict__ p, const GT* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                            bf16* __restrict__ shadow, long n, float lr, float b1, float b2, float eps, float wd, float bc1,
                            float bc2_sqrt, float gscale) {
  const float step = lr / bc1;
  GRID_STRIDE(i, n) {
    float gi = to_f(g[i]) * gscale;
    float pi = p[i];
    if (wd != 0.f) gi = fmaf(wd, pi, gi);
    float mi = m[i], vi = v[i];
    mi = fmaf(1.f - b1, gi - mi, mi);
    vi = fmaf(b2, vi, (1.f - b2) * gi * gi);
    const float den = sqrtf(vi) / bc2_sqrt + eps;
    pi -= step * (mi / den);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (shadow) shadow[i] = (bf16)pi;
  }
}
// Same update with (lr, bias_correction1, sqrt(bias_correction2)) read from device memory, so
// a captured hipGraph replays correct steps as the host advances lr / step counts between
// replays (runtime.GraphedStep).
template <typename GT>
__global__ void adam_dev_kernel(float* __restrict__ p, const GT* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                                bf16* __restrict__ shadow, long n, const float* __restrict__ hyper, float b1, float b2, float eps,
                                float wd, float gscale) {
  const float lr = hyper[0], bc1 = hyper[1], bc2_sqrt = hyper[2];
  const float step = lr / bc1;
  GRID_STRIDE(i, n) {
    float gi = to_f(g[i]) * gscale;
    float pi = p[i];
    if (wd != 0.f) gi = fmaf(wd, pi, gi);
    float mi = m[i], vi = v[i];
    mi = fmaf(1.f - b1, gi - mi, mi);
    vi = fmaf(b2, vi, (1.f - b2) * gi * gi);
    const float den = sqrtf(vi) / bc2_sqrt + eps;
    pi -= step * (mi / den);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (shadow) shadow[i] = (bf16)pi;
  }
}
// the gradient in fp32 (the arena), or the all-reduced fp16 / bf16 wire copy read directly
#define DISPATCH_GRAD(gd, ...)                                               \
  do {                                                                       \
    if ((gd) == RTSDS_F32) { typedef float GT; __VA_ARGS__; }                \
    else if ((gd) == RTSDS_BF16) { typedef bf16 GT; __VA_ARGS__; }           \
    else if ((gd) == RTSDS_F16) { typedef f16 GT; __VA_ARGS__; }             \
    else return RTSDS_ERR_UNSUPPORTED;                                       \
  } while (0)
extern "C" int rtsds_adam_step_dev(float* param, const void* grad, float* exp_avg, float* exp_avg_sq, void* bf16_shadow,
                                   long n, const float* hyper, float beta1, float beta2, float eps, float weight_decay,
                                   float grad_scale, int grad_dtype, void* stream) {
  if (n <= 0 || !hyper) return RTSDS_ERR_SHAPE;
  DISPATCH_GRAD(grad_dtype, hipLaunchKernelGGL(adam_dev_kernel<GT>, dim3(ew_blocks(n, 256, 4096)), dim3(256), 0,
                                               (hipStream_t)stream, param, (const GT*)grad, exp_avg, exp_avg_sq,
                                               (bf16*)bf16_shadow, n, hyper, beta1, beta2, eps, weight_decay, grad_scale));
  RET_LAUNCH();
}

extern "C" int rtsds_adam_step(float* param, const void* grad, float* exp_avg, float* exp_avg_sq, void* bf16_shadow, long n, float lr,
                               float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale, int grad_dtype,
                               void* stream) {
  if (n <= 0 || step <= 0) return RTSDS_ERR_SHAPE;
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  DISPATCH_GRAD(grad_dtype, hipLaunchKernelGGL(adam_kernel<GT>, dim3(ew_blocks(n, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                                               param, (const GT*)grad, exp_avg, exp_avg_sq, (bf16*)bf16_shadow, n, lr, beta1, beta2,
                                               eps, weight_decay, (float)bc1, (float)sqrt(bc2), grad_scale));
  RET_LAUNCH();
}

// ------------------------------------------------------------------ argmax / pixel accuracy
// argmax over channels, first maximum wins (torch.argmax / max(1), train.py:102-106,272-275,
// validation.py:51).  out_idx may be NULL; correct += #(argmax == target) (ignored pixels
// count as wrong, exactly like the reference).
template <typename T>
__global__ void argmax_kernel(const T* __restrict__ x, int64_t* __restrict__ out, const int64_t* __restrict__ tgt,
                              unsigned long long* __restrict__ correct, int n, long hw, int c, long sn, long sc, long shw) {
  const long total = (long)n * hw;
  unsigned long long cnt = 0;
  GRID_STRIDE(p, total) {
    const long img = p / hw, s = p - img * hw;
    const T* b = x + img * sn + s * shw;
    float best = to_f(b[0]);
    int bi = 0;
    for (int k = 1; k < c; ++k) {
      const float v = to_f(b[k * sc]);
      if (v > best || (v != v && best == best)) { best = v; bi = k; }
    }
    if (out) out[p] = bi;
    if (tgt && tgt[p] == bi) ++cnt;
  }
  if (correct) {
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(correct, cnt);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) argmax_staged(const T* __restrict__ x, int64_t* __restrict__ out, const int64_t* __restrict__ tgt,
                                                     unsigned long long* __restrict__ correct, long total, int c) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  T* buf = (T*)smem_raw;
  unsigned long long cnt = 0;
  for (long p0 = (long)blockIdx.x * kStagePix; p0 < total; p0 += (long)gridDim.x * kStagePix) {
    const int np = (int)min<long>(kStagePix, total - p0);
    __syncthreads();
    stage_in(x + p0 * c, buf, np * c);
    __syncthreads();
    if ((int)threadIdx.x < np) {
      const T* r = buf + threadIdx.x * c;
      float best = to_f(r[0]);
      int bi = 0;
      for (int k = 1; k < c; ++k) {
        const float v = to_f(r[k]);
        if (v > best || (v != v && best == best)) { best = v; bi = k; }
      }
      const long p = p0 + threadIdx.x;
      if (out) out[p] = bi;
      if (tgt && tgt[p] == bi) ++cnt;
    }
  }
  if (correct) {
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(correct, cnt);
  }
}

extern "C" int rtsds_argmax(const void* x, long sn, long sc, long shw, int64_t* out, const int64_t* target, unsigned long long* correct,
                            int n, long hw, int c, int dtype, void* stream) {
  if (n <= 0 || hw <= 0 || c <= 0) return RTSDS_ERR_SHAPE;
  DISPATCH_T(dtype, {
    if (stage_ok(sn, sc, shw, hw, c))
      hipLaunchKernelGGL(argmax_staged<T>, dim3(ew_blocks((long)n * hw, kStagePix, 4096)), dim3(256), kStagePix * c * sizeof(T),
                         (hipStream_t)stream, (const T*)x, out, target, correct, (long)n * hw, c);
    else
      hipLaunchKernelGGL(argmax_kernel<T>, dim3(ew_blocks((long)n * hw, 256, 4096)), dim3(256), 0, (hipStream_t)stream, (const T*)x, out, target, correct, n, hw, c, sn, sc, shw);
  });
  RET_LAUNCH();
}

// 19x19 confusion histogram (utils.fast_hist, utils.py:52-58): labels outside [0, nc) dropped.
__global__ void confusion_kernel(const int64_t* __restrict__ label, const int64_t* __restrict__ pred, unsigned long long* __restrict__ hist,
                                 long total, int nc) {
  extern __shared__ unsigned int lh[];
  for (int i = threadIdx.x; i < nc * nc; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  GRID_STRIDE(p, total) {
    const long a = label[p];
    if (a >= 0 && a < nc) atomicAdd(&lh[a * nc + pred[p]], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nc * nc; i += blockDim.x)
    if (lh[i]) atomicAdd(&hist[i], (unsigned long long)lh[i]);
}
extern "C" int rtsds_confusion(const int64_t* label, const int64_t* pred, unsigned long long* hist, long total, int nc, void* stream) {
  if (total <= 0 || nc <= 0 || nc > 64) return RTSDS_ERR_SHAPE;
  hipLaunchKernelGGL(confusion_kernel, dim3(ew_blocks(total, 256, 1024)), dim3(256), nc * nc * 4, (hipStream_t)stream, label, pred, hist, total, nc);
  RET_LAUNCH();
}

// ------------------------------------------------------------------ SGD (flat, fused)
// torch.optim.SGD (main.py:118-120): d = g (+ wd p); with momentum, buf = d on a parameter's
// first step, else buf = momentum buf + (1 - dampening) d; d = nesterov ? d + momentum buf :
// buf; p -= lr d.  hyper (device, may be NULL) = {lr, first-step flag}: the hipGraph-replay
// variant (runtime.GraphedStep) reads them per replay.
template <typename GT>
__global__ void sgd_kernel(float* __restrict__ p, const GT* __restrict__ g, float* __restrict__ buf,
                           bf16* __restrict__ shadow, long n, const float* __restrict__ hyper, float lr, float momentum,
                           float dampening, float wd, int nesterov, int first, float gscale) {
  if (hyper) {
    lr = hyper[0];
    first = hyper[1] != 0.f;
  }
  GRID_STRIDE(i, n) {
    float pi = p[i];
    float d = to_f(g[i]) * gscale;
    if (wd != 0.f) d = d + wd * pi;
    if (momentum != 0.f) {
      const float b = first ? d : buf[i] * momentum + (1.f - dampening) * d;
      buf[i] = b;
      d = nesterov ? d + momentum * b : b;
    }
    pi = pi + (-lr) * d;
    p[i] = pi;
    if (shadow) shadow[i] = (bf16)pi;
  }
}

extern "C" int rtsds_sgd_step(float* param, const void* grad, float* momentum_buf, void* bf16_shadow, long n,
                              const float* hyper, float lr, float momentum, float dampening, float weight_decay,
                              int nesterov, int first, float grad_scale, int grad_dtype, void* stream) {
  if (n <= 0 || (momentum != 0.f && !momentum_buf)) return RTSDS_ERR_SHAPE;
  DISPATCH_GRAD(grad_dtype, hipLaunchKernelGGL(sgd_kernel<GT>, dim3(ew_blocks(n, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                                               param, (const GT*)grad, momentum_buf, (bf16*)bf16_shadow, n, hyper, lr, momentum,
                                               dampening, weight_decay, nesterov, first, grad_scale));
  RET_LAUNCH();
}
