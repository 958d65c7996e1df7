// Shared device helpers for the RTSDS MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rtsds_hip.h"

typedef __bf16 bf16;
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
template <typename T> RT_DEV T from_f(float x);
template <> RT_DEV float from_f<float>(float x) { return x; }
template <> RT_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

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

#define RT_CHECK_LAUNCH()                                      \
  do {                                                          \
    if (hipPeekAtLastError() != hipSuccess) return RTSDS_ERR_LAUNCH; \
  } while (0)

static inline int rt_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
