// Input pipeline on the device (reference main.py:60-108, datasets/cityscapes.py:56-68,
// datasets/gta5.py:69-118): the per-sample torchvision transforms the reference runs on CPU
// DataLoader workers, here on a decoded uint8 image already in HBM.
//
//   resize   torchvision Resize(size) on a tensor = F.interpolate(bilinear, align_corners=False,
//            antialias=True) on the float image (integer tensors -- labels -- are interpolated
//            in float, rounded half-to-even and cast back).  ATen's separable antialias
//            resampler: triangle filter of support scale (scale = in/out when downscaling, 1
//            otherwise), horizontal pass first into an fp32 [H][Wo][C] intermediate, then the
//            vertical pass; weights normalised per output index.  Fused into the passes:
//            horizontal flip (RandomHorizontalFlip: the source is read mirrored), Normalize
//            ((v - mean) / std, on the reference's 0-255 scale), IntRangeTransformer clamp
//            (utils.py:67-75), and the NHWC compute-dtype store the network reads.
//   blur     GaussianBlur(kernel_size, sigma): the separable Gaussian of torchvision applied as
//            its 2-D outer-product kernel with reflect padding.
//   decode   GTA5 RGB label -> train id (gta5.py:111-118: every pixel whose colour equals the
//            colour of train id i gets i, others 0).
//
// Images arrive as decoded HWC uint8 (PIL's layout); every kernel is HBM-bound elementwise /
// small-stencil work (one thread per output element, coalesced over the channel-inner layout).
#include "common.h"
#include <algorithm>
#include <cmath>

static const int kAaMaxTaps = 64;  // support up to a 31x downscale

// Antialias weights of one axis (ATen _compute_weights_aa, bilinear filter): xmin / xsize of
// output index o and its normalised weights.
__global__ void aa_weights_kernel(int in, int out, int ktaps, int* __restrict__ xmin, int* __restrict__ xsize,
                                  float* __restrict__ wt) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= out) return;
  // the float / double mix of ATen's expressions, kept exactly (weights identical to the CPU's)
  const float scale = (float)in / (float)out;
  const float support = scale >= 1.f ? (float)(1.0 * (double)scale) : 1.f;
  const float invscale = scale >= 1.f ? (float)(1.0 / (double)scale) : 1.f;
  const float center = (float)((double)scale * ((double)o + 0.5));
  const int lo = std::max((int)((double)center - (double)support + 0.5), 0);
  const int sz = std::min((int)((double)center + (double)support + 0.5), in) - lo;
  float w[kAaMaxTaps];
  float total = 0.f;
  for (int j = 0; j < ktaps; ++j) {
    float v = 0.f;
    if (j < sz) {
      float x = (float)(((double)(j + lo) - (double)center + 0.5) * (double)invscale);
      x = fabsf(x);
      v = x < 1.f ? 1.f - x : 0.f;
    }
    w[j] = v;
    total += v;
  }
  for (int j = 0; j < ktaps; ++j) wt[(long)o * ktaps + j] = total != 0.f && j < sz ? w[j] / total : 0.f;
  xmin[o] = lo;
  xsize[o] = sz;
}

// horizontal pass: tmp[y][xo][c] = sum_j w[xo][j] src[y][x(xmin + j)][c], x mirrored when flip
template <typename S>
__global__ void aa_h_kernel(const S* __restrict__ src, float* __restrict__ tmp, int h, int w, int c, int wo, int ktaps,
                            const int* __restrict__ xmin, const int* __restrict__ xsize, const float* __restrict__ wt,
                            int flip) {
  const long total = (long)h * wo * c;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    const long r = e / c;
    const int xo = (int)(r % wo), y = (int)(r / wo);
    const int lo = xmin[xo], sz = xsize[xo];
    const float* ww = wt + (long)xo * ktaps;
    const S* row = src + (long)y * w * c + ch;
    float acc = 0.f;
    for (int j = 0; j < sz; ++j) {
      const int x = flip ? w - 1 - (lo + j) : lo + j;
      acc = j == 0 ? (float)row[(long)x * c] * ww[0] : fmaf((float)row[(long)x * c], ww[j], acc);
    }
    tmp[e] = acc;
  }
}

// vertical pass + epilogue.  kind 0: f32 NHWC, 1: bf16 NHWC (normalised when mean/std given);
// 2: int64 label (round half-to-even, clamp to [lo, hi] when lo <= hi)
__global__ void aa_v_kernel(const float* __restrict__ tmp, void* __restrict__ dst, int h, int wo, int c, int ho, int ktaps,
                            const int* __restrict__ ymin, const int* __restrict__ ysize, const float* __restrict__ wt,
                            int kind, const float* __restrict__ mean, const float* __restrict__ stdv, int clamp_lo,
                            int clamp_hi) {
  const long total = (long)ho * wo * c;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    const long r = e / c;
    const int xo = (int)(r % wo), yo = (int)(r / wo);
    const int lo = ymin[yo], sz = ysize[yo];
    const float* ww = wt + (long)yo * ktaps;
    const float* col = tmp + (long)xo * c + ch;
    float acc = 0.f;
    for (int i = 0; i < sz; ++i) {
      const float t = col[(long)(lo + i) * wo * c];
      acc = i == 0 ? t * ww[0] : fmaf(t, ww[i], acc);
    }
    if (kind == 2) {
      long v = (long)rintf(acc);
      if (clamp_lo <= clamp_hi) v = std::min<long>(std::max<long>(v, clamp_lo), clamp_hi);
      ((int64_t*)dst)[e] = v;
    } else {
      if (mean) acc = (acc - mean[ch]) / stdv[ch];
      if (kind == 1) ((bf16*)dst)[e] = (bf16)acc;
      else ((float*)dst)[e] = acc;
    }
  }
}

static int aa_taps(int in, int out) {
  const float scale = (float)in / (float)out;
  const float support = scale >= 1.f ? (float)(1.0 * (double)scale) : 1.f;
  return (int)std::ceil(support) * 2 + 1;
}

static size_t al256(size_t b) { return (b + 255) / 256 * 256; }

extern "C" size_t rtsds_resize_aa_workspace(int c, int h, int w, int ho, int wo) {
  if (c <= 0 || h <= 0 || w <= 0 || ho <= 0 || wo <= 0) return 0;
  const int kx = aa_taps(w, wo), ky = aa_taps(h, ho);
  return al256((size_t)h * wo * c * 4) + al256((size_t)(wo + ho) * 8) + al256((size_t)(wo * kx + ho * ky) * 4);
}

extern "C" int rtsds_resize_aa(const void* src, int src_u8, int c, int h, int w, void* dst, int kind, int ho, int wo,
                               int flip, const float* mean, const float* stdv, int clamp_lo, int clamp_hi, void* ws,
                               size_t ws_bytes, void* stream) {
  if (c <= 0 || h <= 0 || w <= 0 || ho <= 0 || wo <= 0 || kind < 0 || kind > 2 || !src || !dst) return RTSDS_ERR_SHAPE;
  if ((mean == nullptr) != (stdv == nullptr)) return RTSDS_ERR_SHAPE;
  const int kx = aa_taps(w, wo), ky = aa_taps(h, ho);
  if (kx > kAaMaxTaps || ky > kAaMaxTaps) return RTSDS_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < rtsds_resize_aa_workspace(c, h, w, ho, wo)) return RTSDS_ERR_WORKSPACE;
  char* p = (char*)ws;
  float* tmp = (float*)p;
  p += al256((size_t)h * wo * c * 4);
  int* xmin = (int*)p;
  int* xsz = xmin + wo;
  int* ymin = xsz + wo;
  int* ysz = ymin + ho;
  p += al256((size_t)(wo + ho) * 8);
  float* wx = (float*)p;
  float* wy = wx + (size_t)wo * kx;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(aa_weights_kernel, dim3(rt_cdiv(wo, 256)), dim3(256), 0, st, w, wo, kx, xmin, xsz, wx);
  hipLaunchKernelGGL(aa_weights_kernel, dim3(rt_cdiv(ho, 256)), dim3(256), 0, st, h, ho, ky, ymin, ysz, wy);
  const long nh = (long)h * wo * c, nv = (long)ho * wo * c;
  const int bh = (int)std::min<long>(8192, (nh + 255) / 256), bv = (int)std::min<long>(8192, (nv + 255) / 256);
  if (src_u8)
    hipLaunchKernelGGL(aa_h_kernel<uint8_t>, dim3(bh), dim3(256), 0, st, (const uint8_t*)src, tmp, h, w, c, wo, kx, xmin,
                       xsz, wx, flip);
  else
    hipLaunchKernelGGL(aa_h_kernel<float>, dim3(bh), dim3(256), 0, st, (const float*)src, tmp, h, w, c, wo, kx, xmin, xsz,
                       wx, flip);
  hipLaunchKernelGGL(aa_v_kernel, dim3(bv), dim3(256), 0, st, tmp, dst, h, wo, c, ho, ky, ymin, ysz, wy, kind, mean, stdv,
                     clamp_lo, clamp_hi);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// ---- GaussianBlur: dst = conv2d(reflect_pad(src), outer(ky, kx)) per channel, HWC fp32 ----
// (torchvision gaussian_blur: 1-D kernels pdf(x) = exp(-0.5 (x / sigma)^2) over
// x = -(k-1)/2 .. (k-1)/2, normalised; 2-D kernel = ky^T kx; reflect padding k // 2)
__global__ void gblur_kernel(const void* __restrict__ src, int src_u8, float* __restrict__ dst, int h, int w, int c, int kx,
                             int ky, float sx, float sy) {
  __shared__ float kxw[32], kyw[32];
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < kx; ++i) {
      const float x = -(float)(kx - 1) * 0.5f + (float)i;
      kxw[i] = expf(-0.5f * (x / sx) * (x / sx));
      t += kxw[i];
    }
    for (int i = 0; i < kx; ++i) kxw[i] /= t;
    t = 0.f;
    for (int i = 0; i < ky; ++i) {
      const float y = -(float)(ky - 1) * 0.5f + (float)i;
      kyw[i] = expf(-0.5f * (y / sy) * (y / sy));
      t += kyw[i];
    }
    for (int i = 0; i < ky; ++i) kyw[i] /= t;
  }
  __syncthreads();
  const int px = kx / 2, py = ky / 2;
  const long total = (long)h * w * c;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    const long r = e / c;
    const int x = (int)(r % w), y = (int)(r / w);
    float acc = 0.f;
    for (int i = 0; i < ky; ++i) {
      int yy = y - py + i;
      yy = yy < 0 ? -yy : (yy >= h ? 2 * h - 2 - yy : yy);
      for (int j = 0; j < kx; ++j) {
        int xx = x - px + j;
        xx = xx < 0 ? -xx : (xx >= w ? 2 * w - 2 - xx : xx);
        const long o = ((long)yy * w + xx) * c + ch;
        const float v = src_u8 ? (float)((const uint8_t*)src)[o] : ((const float*)src)[o];
        acc = fmaf(v, kyw[i] * kxw[j], acc);
      }
    }
    dst[e] = acc;
  }
}

extern "C" int rtsds_gaussian_blur(const void* src, int src_u8, float* dst, int c, int h, int w, int kx, int ky, float sigma_x,
                                   float sigma_y, void* stream) {
  if (c <= 0 || h <= 0 || w <= 0 || kx <= 0 || ky <= 0 || kx % 2 == 0 || ky % 2 == 0 || kx > 31 || ky > 31) return RTSDS_ERR_SHAPE;
  if (kx / 2 >= w || ky / 2 >= h || !(sigma_x > 0.f) || !(sigma_y > 0.f)) return RTSDS_ERR_SHAPE;
  const long n = (long)h * w * c;
  hipLaunchKernelGGL(gblur_kernel, dim3((int)std::min<long>(8192, (n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, src,
                     src_u8, dst, h, w, c, kx, ky, sigma_x, sigma_y);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

// ---- GTA5 RGB label -> train id (gta5.py:111-118), HWC uint8 -> int64 ----
__constant__ unsigned char kTrainColors[19][3] = {
    {128, 64, 128}, {244, 35, 232}, {70, 70, 70},   {102, 102, 156}, {190, 153, 153}, {153, 153, 153}, {250, 170, 30},
    {220, 220, 0},  {107, 142, 35}, {152, 251, 152}, {70, 130, 180},  {220, 20, 60},   {255, 0, 0},     {0, 0, 142},
    {0, 0, 70},     {0, 60, 100},   {0, 80, 100},   {0, 0, 230},     {119, 11, 32}};
__global__ void gta5_decode_kernel(const uint8_t* __restrict__ rgb, int64_t* __restrict__ out, long npix) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const uint8_t r = rgb[p * 3], g = rgb[p * 3 + 1], b = rgb[p * 3 + 2];
    int64_t v = 0;
    for (int i = 0; i < 19; ++i)
      if (r == kTrainColors[i][0] && g == kTrainColors[i][1] && b == kTrainColors[i][2]) v = i;
    out[p] = v;
  }
}
extern "C" int rtsds_gta5_decode(const uint8_t* rgb, int64_t* out, int h, int w, void* stream) {
  if (h <= 0 || w <= 0 || !rgb || !out) return RTSDS_ERR_SHAPE;
  const long n = (long)h * w;
  hipLaunchKernelGGL(gta5_decode_kernel, dim3((int)std::min<long>(8192, (n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     rgb, out, n);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
