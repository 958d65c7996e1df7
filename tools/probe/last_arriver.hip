// Probe: cost and correctness of a "last-arriving workgroup" reduction on gfx950 (the pattern a
// fused BatchNorm-statistics finalize would use in a conv epilogue).  Each of G workgroups
// writes a 64 KB tile (the conv output, normal stores) and a 1 KB partial, then bumps a counter;
// the last arriver sums every workgroup's partial in index order.  Variants:
//   0: no counter / no reduction (baseline)
//   1: agent-scope release / acquire fences around the counter (compiler: buffer_wbl2 / buffer_inv)
//   2: partials stored as agent-scope relaxed atomics, s_waitcnt vmcnt(0), relaxed counter,
//      last arriver reads the partials with agent-scope relaxed atomic loads (no L2 writeback)
// Prints time per launch and whether the reduced value matches the expected sum.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int MODE>
__global__ void __launch_bounds__(256) k(float* tile, float* part, unsigned* cnt, float* result, int it) {
  const int b = blockIdx.x, t = threadIdx.x;
  float4 v = make_float4(b + it, t, 1.f, 2.f);
  float4* tp = (float4*)(tile + (size_t)b * 16384);
#pragma unroll
  for (int i = 0; i < 16; ++i) tp[i * 256 + t] = v;
  const float pv = (float)(b % 7) + 0.25f * it;
  if (MODE == 0) {
    part[b * 256 + t] = pv;
    return;
  }
  if (MODE == 1) {
    part[b * 256 + t] = pv;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  } else {
    __hip_atomic_store(part + b * 256 + t, pv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);  // all counters: the partial stores are acknowledged
  }
  __shared__ unsigned ticket;
  __syncthreads();
  if (t == 0) ticket = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (ticket != gridDim.x - 1) return;
  if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  float s = 0.f;
  for (int w = (int)gridDim.x - 8; w < (int)gridDim.x; ++w)  // a short final merge: the fence cost is measured
    s += MODE == 1 ? part[w * 256 + t] : __hip_atomic_load(part + w * 256 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  result[t] = s;
  if (t == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // self-reset
}

int main() {
  const int G = 2048, iters = 200;
  float *tile, *part, *res;
  unsigned* cnt;
  (void)hipMalloc(&tile, (size_t)G * 16384 * 4);
  (void)hipMalloc(&part, (size_t)G * 256 * 4);
  (void)hipMalloc(&res, 256 * 4);
  (void)hipMalloc(&cnt, 4);
  (void)hipMemset(cnt, 0, 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode) {
    int bad = 0;
    float ms = 0.f;
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      for (int it = 0; it < iters; ++it) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(G), dim3(256), 0, 0, tile, part, cnt, res, it);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(G), dim3(256), 0, 0, tile, part, cnt, res, it);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(G), dim3(256), 0, 0, tile, part, cnt, res, it);
        if (mode > 0 && rep == 1 && it % 20 == 0) {
          float h[256];
          (void)hipMemcpy(h, res, sizeof(h), hipMemcpyDeviceToHost);
          double want = 0;
          for (int w = G - 8; w < G; ++w) want += (float)(w % 7) + 0.25f * it;
          if (h[0] != (float)want && fabs(h[0] - want) > 1e-3 * want) ++bad;
        }
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
    }
    printf("mode %d: %.2f us per launch (%d workgroups x 64 KB), mismatches %d\n", mode, 1000.f * ms / iters, G, bad);
  }
  return 0;
}
