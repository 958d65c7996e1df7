// Shared device helpers for the RTSDS MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtsds_hip.h"

typedef __bf16 bf16;
typedef _Float16 f16;  // the fp16 gradient wire only (rtsds_cast, optimizer gradients)
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

#define RT_DEV __device__ __forceinline__

// Element-type traits: storage type T, 16-byte vector of T, elements per 16 B.
template <typename T> struct VecT;
template <> struct VecT<float> { typedef f32x4 v16; static constexpr int N = 4; };
template <> struct VecT<bf16> { typedef bf16x8 v16; static constexpr int N = 8; };

RT_DEV float to_f(float x) { return x; }
RT_DEV float to_f(bf16 x) { return (float)x; }
RT_DEV float to_f(f16 x) { return (float)x; }
template <typename T> RT_DEV T from_f(float x);
template <> RT_DEV float from_f<float>(float x) { return x; }
template <> RT_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> RT_DEV f16 from_f<f16>(float x) { return (f16)x; }

// Exact unsigned division by a runtime-invariant divisor (Granlund-Montgomery), valid
// for n < 2^31.  Built on the host by fastdiv_make(), carried in kernel arguments.
struct FastDiv {
  uint32_t d, m, s;
};
static inline FastDiv fastdiv_make(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)((((1ull << s) - d) << 32) / d + 1);
  return f;
}
RT_DEV uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t hi = __umulhi(n, f.m);
  return (uint32_t)(((uint64_t)hi + n) >> f.s);
}

RT_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
RT_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bilinear (align_corners=False) source index, ATen semantics: src = scale*(dst+0.5)-0.5
// clamped at 0; i0 = floor, i1 = min(i0+1, in-1); l0/l1 the weights of i0/i1.  scale = in/out
// for size=..., 1/scale_factor for scale_factor=... (computed by the host in fp32 exactly as
// ATen's area_pixel_compute_scale does).  Shared by the resize kernels and the fused
// upsample+cross-entropy so both see identical taps and weights.
RT_DEV void bil_src(int o, float scale, int in, int& i0, int& i1, float& l0, float& l1) {
  float src = scale * ((float)o + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = src - (float)i0;
  l0 = 1.f - l1;
}

// Smallest output index o in [0, out] whose top tap i0(o) >= target (i0 is non-decreasing in o).
RT_DEV int bil_first_ge(int target, float s, int in, int out) {
  if (target <= 0) return 0;
  if (target >= in) return out;
  int o = (int)floorf(((float)target + 0.5f) / s - 0.5f);
  o = max(0, min(out, o));
  int i0, i1;
  float l0, l1;
  while (o > 0) {
    bil_src(o - 1, s, in, i0, i1, l0, l1);
    if (i0 < target) break;
    --o;
  }
  while (o < out) {
    bil_src(o, s, in, i0, i1, l0, l1);
    if (i0 >= target) break;
    ++o;
  }
  return o;
}

// Blend of the 4 taps (p00 = (h0,w0), p01 = (h0,w1), p10 = (h1,w0), p11 = (h1,w1)): width
// inner, height outer (the association of ATen's separable upsample_bilinear2d), explicit fma
// order -- the fused upsample+CE computes the identical expression from per-column
// horizontal blends, so both paths produce the same logits bit for bit.
RT_DEV float bil_mix(float p00, float p01, float p10, float p11, float lh0, float lh1, float lw0, float lw1) {
  const float t0 = fmaf(lw1, p01, lw0 * p00);
  const float t1 = fmaf(lw1, p11, lw0 * p10);
  return fmaf(lh1, t1, lh0 * t0);
}

// Buffer-resource LDS-DMA (buffer_load_dwordx4 ... offen lds): 32-bit byte offsets, and an
// offset past num_records zero-fills the LDS destination.  The host compilation pass of the
// kernel templates only needs the signatures.
#if defined(__HIP_DEVICE_COMPILE__)
typedef __amdgpu_buffer_rsrc_t rsrc_t;
RT_DEV rsrc_t make_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, bytes, 0x00020000);
}
RT_DEV void buf_lds16(rsrc_t r, void* lds, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}
#else
struct rsrc_t { int w[4]; };
RT_DEV rsrc_t make_rsrc(const void*, int) { return rsrc_t{}; }
RT_DEV void buf_lds16(rsrc_t, void*, int, int) {}
#endif

#define RT_CHECK_LAUNCH()                                      \
  do {                                                          \
    if (hipPeekAtLastError() != hipSuccess) return RTSDS_ERR_LAUNCH; \
  } while (0)

static inline int rt_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
