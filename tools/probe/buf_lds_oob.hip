// Probe: does buffer_load_dwordx4 ... lds write zeros to LDS for an out-of-range offset?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const int* src, int nbytes, int* out) {
  __shared__ __attribute__((aligned(16))) int lds[256 * 4];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0x77777777;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nbytes, 0x00020000);
  const int lane = threadIdx.x;
  // lanes 0-31 in range, 32-47 just past the end, 48-63 at 0x80000000
  int voff = lane < 32 ? lane * 16 : (lane < 48 ? nbytes + (lane - 32) * 16 : (int)0x80000000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}
int main() {
  int *src, *out;
  hipMalloc(&src, 1 << 20);
  hipMalloc(&out, 4096);
  int h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = i + 1;
  hipMemcpy(src, h, 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, src, 512, out);
  hipMemcpy(h, out, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) {
    const int want = i < 128 ? i + 1 : 0;
    if (h[i] != want) { if (bad < 8) printf("lds[%d] = %#x want %#x\n", i, h[i], want); ++bad; }
  }
  printf("oob probe: %s (%d mismatches)\n", bad ? "NOT zero-filled" : "zero-filled", bad);
  return 0;
}
