// Probe: gfx950 permlane16/32 swap semantics as used by conv.hip's statistics epilogue.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* in, float* out) {
  const int l = threadIdx.x;
  float x = in[l];
  auto a = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x), __builtin_bit_cast(unsigned, x), false, false);
  auto b = __builtin_amdgcn_permlane32_swap(a[0], a[0], false, false);
  out[l] = __builtin_bit_cast(float, a[0]);
  out[64 + l] = __builtin_bit_cast(float, a[1]);
  out[128 + l] = __builtin_bit_cast(float, b[0]);
  out[192 + l] = __builtin_bit_cast(float, b[1]);
}
int main() {
  float h[64], *din, *dout, r[256];
  for (int i = 0; i < 64; ++i) h[i] = (float)i;
  hipMalloc(&din, 256); hipMalloc(&dout, 1024);
  hipMemcpy(din, h, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(din, dout);
  hipMemcpy(r, dout, 1024, hipMemcpyDeviceToHost);
  const char* nm[4] = {"p16[0]", "p16[1]", "p32(p16[0])[0]", "p32(p16[0])[1]"};
  for (int q = 0; q < 4; ++q) {
    printf("%s:", nm[q]);
    for (int i = 0; i < 64; i += 4) printf(" %g", r[q * 64 + i]);
    printf("\n");
  }
  return 0;
}
