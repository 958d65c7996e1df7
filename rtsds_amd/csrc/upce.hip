// Fused bilinear upsample + cross-entropy (+ pixel accuracy) for the segmentation heads.
//
// The reference upsamples every head's 19-class logits to full resolution
// (build_bisenet.py:151-152,158-159,166; deeplabv2.py:126 -- F.interpolate, bilinear,
// align_corners=False) and then applies nn.CrossEntropyLoss(ignore_index=19) to each
// (train.py:86-92) and argmax for the pixel accuracy (train.py:102-106).  At 1024x512 the
// full-resolution logits are 8 x 512 x 1024 x 19 values per head; materialising them costs
// an upsample write, a CE forward read, a CE backward read+write and a resize-backward read
// per head.  Here the full-resolution logits exist only in registers:
//
//   forward  (one workgroup per TH x TW low-resolution cell tile, all heads in turn):
//     stage the (TH+1) x (TW+1) x C low-res tile in LDS (fp32), then for every full-res
//     pixel whose top-left source tap lies in the tile: interpolate z (same taps, weights and
//     expression as rtsds_bilinear_fwd), softmax, loss = lse - z[t], argmax (head 0), and
//     g = softmax - onehot(t).  g goes to LDS in 4-row chunks and is folded back onto the
//     low-res grid (the adjoint of the interpolation): first along x with a per-block weight
//     table (four rows at once, independent FMA chains), then along y into two running
//     register accumulators per owned (low-res column, class) pair, written out as the
//     full-res rows move past each low-res row -- no atomics, fixed summation order,
//     deterministic.  Labels of the next chunk are prefetched while the current one runs.
//   final    per-head loss = sum(lse - z_t) / count(valid) (deterministic two-stage).
//   backward dlogits[i][j] = (gout / count) * (sum of the <= 4 tile partials covering (i,j)).
//
// Traffic per head: the low-res logits once, the int64 labels once (L2-resident across the
// heads of one tile), the low-res gradient partials once; nothing at full resolution is
// written.
#include "common.h"
#include <algorithm>
#include <cmath>

static const int kUpceCMax = 32;
static const int kUpceMaxHeads = 4;

struct UpceGeo {
  int n, hl, wl, c, H, W;
  float sh, sw;
  int th, tw, ntr, ntc, wmax, nblocks;
};

struct UpceArgs {
  const void* x[kUpceMaxHeads];
  float* gpart[kUpceMaxHeads];
  float* lpart;  // [heads][nblocks]
  float* cpart;  // [nblocks]
  const int64_t* tgt;
  unsigned long long* correct;
  UpceGeo g;
  int nheads, ignore, want_grad;
};

// Smallest o in [0, out] with i0(o) >= target (i0 is non-decreasing in o).
RT_DEV int upce_first_ge(int target, float s, int in, int out) {
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

RT_DEV float upce_block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// CP: channel count padded to a multiple of 4 (compile time, so every per-class loop is
// fully unrolled without guards); padding classes hold -1e30 logits (softmax weight 0).
template <typename T, int CP>
__global__ void __launch_bounds__(256) upce_fwd_kernel(UpceArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float red[4];
  const UpceGeo& q = a.g;
  const int TH = q.th, TW = q.tw, C = q.c, TW1 = TW + 1, tid = threadIdx.x;
  const int tiles = q.ntr * q.ntc;
  const int img = blockIdx.x / tiles, tt = blockIdx.x - img * tiles;
  const int tr = tt / q.ntc, tc = tt - tr * q.ntc;
  const int r0 = tr * TH, c0 = tc * TW;
  const int rows_l = min(TH + 1, q.hl - r0), cols_l = min(TW1, q.wl - c0);
  const int y_lo = upce_first_ge(r0, q.sh, q.hl, q.H), y_hi = upce_first_ge(r0 + TH, q.sh, q.hl, q.H);
  const int x_lo = upce_first_ge(c0, q.sw, q.wl, q.W);
  const int x_hi = upce_first_ge(c0 + TW, q.sw, q.wl, q.W);
  const int Wt = min(x_hi - x_lo, q.wmax);
  const int tile_el = (TH + 1) * TW1 * C;  // gradient-partial layout (compact classes)
  const int rowp = TW1 * CP, ltile = (TH + 1) * rowp;

  // LDS (class stride CP): lt[TH+1][TW1] | vb[4][TW1] | gb[4][wmax] | wcol[TW1][wmax] |
  //                        xj0 | xj1 | xm0 | xm1 | xs | xe
  float* lt = smem;
  float* vb = lt + ltile;
  float* gb = vb + 4 * rowp;
  float* wcol = gb + 4 * q.wmax * CP;
  int* xj0 = (int*)(wcol + TW1 * q.wmax);
  int* xj1 = xj0 + q.wmax;
  float* xm0 = (float*)(xj1 + q.wmax);
  float* xm1 = xm0 + q.wmax;
  int* xs = (int*)(xm1 + q.wmax);
  int* xe = xs + TW1;

  for (int xx = tid; xx < Wt; xx += 256) {
    int j0, j1;
    float m0, m1;
    bil_src(x_lo + xx, q.sw, q.wl, j0, j1, m0, m1);
    xj0[xx] = j0 - c0;
    xj1[xx] = j1 - c0;
    xm0[xx] = m0;
    xm1[xx] = m1;
  }
  __syncthreads();
  // x-adjoint weights: wcol[jl][xx] = weight of full-res column xx on low-res column jl
  for (int e = tid; e < TW1 * Wt; e += 256) {
    const int jl = e / Wt, xx = e - jl * Wt;
    wcol[jl * q.wmax + xx] = (xj0[xx] == jl ? xm0[xx] : 0.f) + (xj1[xx] == jl ? xm1[xx] : 0.f);
  }
  // contiguous full-res column range feeding low-res column jl (taps are monotone in x)
  for (int jl = tid; jl < TW1; jl += 256) {
    int lo = Wt, hi = -1;
    for (int xx = 0; xx < Wt; ++xx)
      if (xj0[xx] == jl || xj1[xx] == jl) { lo = min(lo, xx); hi = xx; }
    xs[jl] = lo;
    xe[jl] = hi;
  }

  float cnt = 0.f;
  unsigned long long corr = 0;
  const int ry = tid >> 6, rx = tid & 63;
  const int npair = TW1 * C;  // <= 512: each thread owns pairs tid and tid + 256
  int pj[2], pc[2];
#pragma unroll
  for (int q2 = 0; q2 < 2; ++q2) {
    const int p = tid + q2 * 256;
    pj[q2] = p / C;
    pc[q2] = p - pj[q2] * C;
  }
  // labels of this thread's pixel(s) in a 4-row chunk (column groups 0 / 64; Wt <= 128)
  auto tload = [&](int yb, int xb) -> long {
    const int y = yb + ry, xx = xb + rx;
    return (y < y_hi && xx < Wt) ? a.tgt[((long)img * q.H + y) * q.W + x_lo + xx] : -1;
  };
  for (int h = 0; h < a.nheads; ++h) {
    const T* X = (const T*)a.x[h] + (long)img * q.hl * q.wl * C;
    __syncthreads();
    for (int e = tid; e < ltile; e += 256) {
      const int cc = e % CP, cell = e / CP;
      const int il = cell / TW1, jl = cell - il * TW1;
      float v = cc < C ? 0.f : -1e30f;
      if (cc < C && il < rows_l && jl < cols_l) v = to_f(X[((long)(r0 + il) * q.wl + (c0 + jl)) * C + cc]);
      lt[e] = v;
    }
    __syncthreads();
    float lsum = 0.f;
    // y-fold accumulators of the owned (jl, c) pairs for low-res rows cur and cur + 1;
    // rows are finalised (written to gpart) as the full-res rows advance past them.
    float Aa[2] = {0.f, 0.f}, Ab[2] = {0.f, 0.f};
    int cur = 0;
    float* gdst = a.want_grad ? a.gpart[h] + (long)blockIdx.x * tile_el : nullptr;
    long tn0 = tload(y_lo, 0), tn1 = Wt > 64 ? tload(y_lo, 64) : -1;
    for (int yb = y_lo; yb < y_hi; yb += 4) {
      const long tc0 = tn0, tc1 = tn1;
      if (yb + 4 < y_hi) {  // prefetch the next chunk's labels
        tn0 = tload(yb + 4, 0);
        if (Wt > 64) tn1 = tload(yb + 4, 64);
      }
      const int y = yb + ry;
      // vertical interpolation of this wave's full-res row on the tile's low-res columns
      // (vrow[jl][c]); each pixel then only blends its two columns:
      //   z = m1 * vrow[j1] + m0 * vrow[j0],  vrow[j] = l1 * L[i1][j] + l0 * L[i0][j]
      // (the same fma order as rtsds_bilinear_fwd, so both give identical logits).
      float* vrow = vb + ry * rowp;
      if (y < y_hi) {
        int i0, i1;
        float l0, l1;
        bil_src(y, q.sh, q.hl, i0, i1, l0, l1);
        const float* L0 = lt + (i0 - r0) * rowp;
        const float* L1 = lt + (i1 - r0) * rowp;
        for (int e = rx; e < rowp; e += 64) vrow[e] = fmaf(l1, L1[e], l0 * L0[e]);
      }
      __syncthreads();
      for (int xb = 0; xb < Wt; xb += 64) {
        const int xx = xb + rx;
        if (y >= y_hi || xx >= Wt) continue;
        const long t = xb == 0 ? tc0 : tc1;
        const float m0 = xm0[xx], m1 = xm1[xx];
        const float* v0 = vrow + xj0[xx] * CP;
        const float* v1 = vrow + xj1[xx] * CP;
        float z[CP];
        float mx = -INFINITY;
#pragma unroll
        for (int k = 0; k < CP; ++k) {
          z[k] = fmaf(m1, v1[k], m0 * v0[k]);
          mx = fmaxf(mx, z[k]);
        }
        const bool in_range = t >= 0 && t < C;
        const float zt = in_range ? fmaf(m1, v1[t], m0 * v0[t]) : NAN;
        if (h == 0 && a.correct) {  // first maximum wins (torch argmax)
          float best = z[0];
          int bi = 0;
#pragma unroll
          for (int k = 1; k < CP; ++k)
            if (z[k] > best || (z[k] != z[k] && best == best)) { best = z[k]; bi = k; }
          corr += (t == bi) ? 1ull : 0ull;
        }
        const bool valid = t != a.ignore;
        // softmax with the hardware exp2 / log2 / rcp (v_exp_f32, v_log_f32, v_rcp_f32)
        const float kL2E = 1.4426950408889634f, kLN2 = 0.6931471805599453f;
        const float mxs = mx * kL2E;
        float se = 0.f;
#pragma unroll
        for (int k = 0; k < CP; ++k) {
          z[k] = __builtin_amdgcn_exp2f(fmaf(z[k], kL2E, -mxs));
          se += z[k];
        }
        if (valid) {
          lsum += fmaf(__builtin_amdgcn_logf(se), kLN2, mx) - zt;
          if (h == 0) cnt += 1.f;
        }
        if (a.want_grad) {
          float* gp = gb + (ry * q.wmax + xx) * CP;
          const float is = valid ? __builtin_amdgcn_rcpf(se) : 0.f;
#pragma unroll
          for (int k = 0; k < CP; ++k) gp[k] = z[k] * is;
          if (valid && in_range) gp[t] -= 1.f;
        }
      }
      if (!a.want_grad) continue;
      __syncthreads();
      // adjoint, x-fold: R[r][jl][c] = sum_x wcol[jl][x] g[r][x][c] for the 4 chunk rows at once
      float R[2][4];
#pragma unroll
      for (int q2 = 0; q2 < 2; ++q2) {
        R[q2][0] = R[q2][1] = R[q2][2] = R[q2][3] = 0.f;
        const int p = tid + q2 * 256;
        if (p < npair) {
          const int jl = pj[q2];
          const float* wr = wcol + jl * q.wmax;
          const float* gq = gb + pc[q2];
          const int rs = q.wmax * CP;
          const int xhi = xe[jl];
          for (int xx = xs[jl]; xx <= xhi; ++xx) {
            const float w = wr[xx];
            const float* g0 = gq + xx * CP;
            R[q2][0] = fmaf(w, g0[0], R[q2][0]);
            R[q2][1] = fmaf(w, g0[rs], R[q2][1]);
            R[q2][2] = fmaf(w, g0[2 * rs], R[q2][2]);
            R[q2][3] = fmaf(w, g0[3 * rs], R[q2][3]);
          }
        }
      }
      // y-fold into the running row accumulators
#pragma unroll
      for (int r2 = 0; r2 < 4; ++r2) {
        const int y2 = yb + r2;
        if (y2 >= y_hi) break;
        int k0, k1;
        float h0, h1;
        bil_src(y2, q.sh, q.hl, k0, k1, h0, h1);
        k0 -= r0;
        k1 -= r0;
        while (k0 > cur) {
#pragma unroll
          for (int q2 = 0; q2 < 2; ++q2) {
            const int p = tid + q2 * 256;
            if (p < npair) gdst[cur * npair + p] = Aa[q2];
            Aa[q2] = Ab[q2];
            Ab[q2] = 0.f;
          }
          ++cur;
        }
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
          Aa[q2] = fmaf(h0, R[q2][r2], Aa[q2]);
          if (k1 == k0) Aa[q2] = fmaf(h1, R[q2][r2], Aa[q2]);
          else Ab[q2] = fmaf(h1, R[q2][r2], Ab[q2]);
        }
      }
      __syncthreads();
    }
    if (a.want_grad) {  // flush rows cur, cur + 1; rows never reached are zero
#pragma unroll
      for (int q2 = 0; q2 < 2; ++q2) {
        const int p = tid + q2 * 256;
        if (p >= npair) continue;
        for (int il = cur; il <= TH; ++il) gdst[il * npair + p] = il == cur ? Aa[q2] : (il == cur + 1 ? Ab[q2] : 0.f);
      }
    }
    const float s = upce_block_sum(lsum, red);
    if (tid == 0) a.lpart[(long)h * q.nblocks + blockIdx.x] = s;
  }
  const float cs = upce_block_sum(cnt, red);
  if (tid == 0) a.cpart[blockIdx.x] = cs;
  if (a.correct) {
    for (int o = 32; o > 0; o >>= 1) corr += __shfl_xor(corr, o, 64);
    if ((tid & 63) == 0 && corr) atomicAdd(a.correct, corr);
  }
}

// stat[0] = valid-pixel count, stat[1 + h] = head h's loss sum (deterministic block sums);
// then loss[h] = stat[1 + h] / stat[0], *loss_sum = ((loss[0] + loss[1]) + ...) in head order
// (the reference's left-to-right sum of the head losses).  rtsds_upce_finish re-runs the
// second half after the caller has summed the count stat[0] over data-parallel ranks.
RT_DEV void upce_losses(const float* stat, int nheads, float* loss, float* loss_sum) {
  float total = 0.f;
  for (int h = 0; h < nheads; ++h) {
    const float l = stat[1 + h] / stat[0];
    total = h == 0 ? l : total + l;
    if (loss) loss[h] = l;
  }
  if (loss_sum) loss_sum[0] = total;
}
__global__ void __launch_bounds__(256) upce_final_kernel(const float* __restrict__ lpart, const float* __restrict__ cpart, int nblocks,
                                                         int nheads, float* __restrict__ loss, float* __restrict__ loss_sum,
                                                         float* __restrict__ stat) {
  __shared__ float red[4];
  float c = 0.f;
  for (int b = threadIdx.x; b < nblocks; b += 256) c += cpart[b];
  c = upce_block_sum(c, red);
  if (threadIdx.x == 0) stat[0] = c;
  for (int h = 0; h < nheads; ++h) {
    float s = 0.f;
    for (int b = threadIdx.x; b < nblocks; b += 256) s += lpart[(long)h * nblocks + b];
    s = upce_block_sum(s, red);
    if (threadIdx.x == 0) stat[1 + h] = s;
  }
  if (threadIdx.x == 0) upce_losses(stat, nheads, loss, loss_sum);
}
__global__ void upce_finish_kernel(const float* __restrict__ stat, int nheads, float* __restrict__ loss,
                                   float* __restrict__ loss_sum) {
  if (threadIdx.x == 0) upce_losses(stat, nheads, loss, loss_sum);
}

struct UpceBwdArgs {
  const float* gpart[kUpceMaxHeads];
  void* dx[kUpceMaxHeads];
  const float* gout;  // gout[h * gstride]
  int gstride;
  const float* count;
  UpceGeo g;
  int nheads;
};

// dx[h][img][i][j][c] = gout[h] / count * (tile partial sums covering (i, j)), fixed order.
template <typename T>
__global__ void __launch_bounds__(256) upce_bwd_kernel(UpceBwdArgs a) {
  const UpceGeo& q = a.g;
  const int C = q.c, TW1 = q.tw + 1;
  const int tile_el = (q.th + 1) * TW1 * C;
  const long per_head = (long)q.n * q.hl * q.wl * C;
  const long total = per_head * a.nheads;
  const float inv = 1.f / a.count[0];
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int h = (int)(e / per_head);
    const long off = e - h * per_head;
    long r = off;
    const int cc = (int)(r % C);
    r /= C;
    const int j = (int)(r % q.wl);
    r /= q.wl;
    const int i = (int)(r % q.hl);
    const int img = (int)(r / q.hl);
    const int tr = i / q.th, il = i - tr * q.th, tc = j / q.tw, jl = j - tc * q.tw;
    const float* P = a.gpart[h] + (long)img * q.ntr * q.ntc * tile_el;
    auto at = [&](int rr, int cc2, int li, int lj) { return P[((long)rr * q.ntc + cc2) * tile_el + (li * TW1 + lj) * C + cc]; };
    float s = at(tr, tc, il, jl);
    if (il == 0 && tr > 0) s += at(tr - 1, tc, q.th, jl);
    if (jl == 0 && tc > 0) s += at(tr, tc - 1, il, q.tw);
    if (il == 0 && tr > 0 && jl == 0 && tc > 0) s += at(tr - 1, tc - 1, q.th, q.tw);
    ((T*)a.dx[h])[off] = from_f<T>(s * a.gout[h * a.gstride] * inv);
  }
}

// ------------------------------------------------------------------ host
static bool upce_plan(int n, int hl, int wl, int c, int H, int W, float sh, float sw, UpceGeo& g) {
  if (n <= 0 || hl <= 0 || wl <= 0 || c <= 0 || H <= 0 || W <= 0) return false;
  if (c > kUpceCMax || !(sh > 0.f) || !(sw > 0.f) || sh > 1.f || sw > 1.f) return false;
  const float fy = 1.f / sh, fx = 1.f / sw;
  g.n = n; g.hl = hl; g.wl = wl; g.c = c; g.H = H; g.W = W; g.sh = sh; g.sw = sw;
  g.tw = std::max(1, std::min(32, (int)(64.f / std::ceil(fx))));
  g.th = std::max(1, std::min(32, (int)(64.f / std::ceil(fy))));
  g.ntr = (hl + g.th - 1) / g.th;
  g.ntc = (wl + g.tw - 1) / g.tw;
  g.wmax = (int)std::ceil((g.tw + 1) * fx) + 4;
  // kernel limits: two 64-column groups per row, <= 512 owned (column, class) pairs
  while (g.tw > 1 && (g.wmax > 128 || (g.tw + 1) * c > 512)) {
    --g.tw;
    g.wmax = (int)std::ceil((g.tw + 1) * fx) + 4;
  }
  if (g.wmax > 128 || (g.tw + 1) * c > 512) return false;
  g.nblocks = n * g.ntr * g.ntc;
  return (long)g.nblocks * g.ntr < (1L << 31);
}
static int upce_cp(int c) { return (c + 3) / 4 * 4; }
static size_t upce_lds(const UpceGeo& g) {
  const size_t cp = upce_cp(g.c), tile_el = (size_t)(g.th + 1) * (g.tw + 1) * cp;
  return (tile_el + 4 * (size_t)(g.tw + 1) * cp + 4 * (size_t)g.wmax * cp + (size_t)(g.tw + 1) * g.wmax + 4 * (size_t)g.wmax + 2 * (size_t)(g.tw + 1)) * 4;
}
static size_t upce_tile_el(const UpceGeo& g) { return (size_t)(g.th + 1) * (g.tw + 1) * g.c; }
// ws: stat[64] (count, per-head loss sums; offset 0, see the header) | [heads][nblocks][tile_el]
//     gradient partials | [heads][nblocks] loss partials | [nblocks] counts
static const size_t kUpceStat = 64;
static size_t upce_ws_floats(const UpceGeo& g, int heads) {
  return kUpceStat + (size_t)heads * g.nblocks * upce_tile_el(g) + (size_t)heads * g.nblocks + g.nblocks;
}

extern "C" size_t rtsds_upce_workspace(int nheads, int n, int hl, int wl, int c, int H, int W, float scale_h, float scale_w) {
  UpceGeo g;
  if (nheads <= 0 || nheads > kUpceMaxHeads || !upce_plan(n, hl, wl, c, H, W, scale_h, scale_w, g)) return 0;
  if (upce_lds(g) > 64 * 1024) return 0;
  return upce_ws_floats(g, nheads) * 4 + 256;
}

extern "C" int rtsds_upce_fwd(int nheads, const void* const* logits, const int64_t* target, int n, int hl, int wl, int c, int H, int W,
                              float scale_h, float scale_w, int ignore_index, float* loss, float* loss_sum,
                              unsigned long long* correct, int want_grad,
                              int dtype, void* ws, size_t ws_bytes, void* stream) {
  UpceGeo g;
  if (nheads <= 0 || nheads > kUpceMaxHeads) return RTSDS_ERR_UNSUPPORTED;
  if (!upce_plan(n, hl, wl, c, H, W, scale_h, scale_w, g)) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_upce_workspace(nheads, n, hl, wl, c, H, W, scale_h, scale_w) || !ws) return RTSDS_ERR_WORKSPACE;
  UpceArgs a;
  float* stat = (float*)ws;
  float* f = stat + kUpceStat;
  const size_t te = upce_tile_el(g);
  for (int h = 0; h < kUpceMaxHeads; ++h) {
    a.x[h] = h < nheads ? logits[h] : nullptr;
    a.gpart[h] = h < nheads ? f + (size_t)h * g.nblocks * te : nullptr;
  }
  a.lpart = f + (size_t)nheads * g.nblocks * te;
  a.cpart = a.lpart + (size_t)nheads * g.nblocks;
  a.tgt = target;
  a.correct = correct;
  a.g = g;
  a.nheads = nheads;
  a.ignore = ignore_index;
  a.want_grad = want_grad;
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = upce_lds(g);
  if (dtype != RTSDS_BF16 && dtype != RTSDS_F32) return RTSDS_ERR_UNSUPPORTED;
  switch (upce_cp(c)) {
#define UPCE_CASE(CPV)                                                                                      \
  case CPV:                                                                                                 \
    if (dtype == RTSDS_BF16) hipLaunchKernelGGL((upce_fwd_kernel<bf16, CPV>), dim3(g.nblocks), dim3(256), lds, st, a); \
    else hipLaunchKernelGGL((upce_fwd_kernel<float, CPV>), dim3(g.nblocks), dim3(256), lds, st, a);          \
    break;
    UPCE_CASE(4) UPCE_CASE(8) UPCE_CASE(12) UPCE_CASE(16) UPCE_CASE(20) UPCE_CASE(24) UPCE_CASE(28) UPCE_CASE(32)
#undef UPCE_CASE
    default: return RTSDS_ERR_UNSUPPORTED;
  }
  hipLaunchKernelGGL(upce_final_kernel, dim3(1), dim3(256), 0, st, a.lpart, a.cpart, g.nblocks, nheads, loss, loss_sum, stat);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

extern "C" int rtsds_upce_bwd(int nheads, const float* grad_loss, int grad_stride, void* const* dlogits, int n, int hl, int wl, int c, int H, int W,
                              float scale_h, float scale_w, int dtype, const void* ws, size_t ws_bytes, void* stream) {
  UpceGeo g;
  if (nheads <= 0 || nheads > kUpceMaxHeads) return RTSDS_ERR_UNSUPPORTED;
  if (!upce_plan(n, hl, wl, c, H, W, scale_h, scale_w, g)) return RTSDS_ERR_UNSUPPORTED;
  if (ws_bytes < rtsds_upce_workspace(nheads, n, hl, wl, c, H, W, scale_h, scale_w) || !ws) return RTSDS_ERR_WORKSPACE;
  UpceBwdArgs a;
  const float* f = (const float*)ws + kUpceStat;
  const size_t te = upce_tile_el(g);
  for (int h = 0; h < kUpceMaxHeads; ++h) {
    a.gpart[h] = h < nheads ? f + (size_t)h * g.nblocks * te : nullptr;
    a.dx[h] = h < nheads ? dlogits[h] : nullptr;
  }
  a.gout = grad_loss;
  a.gstride = grad_stride;
  a.count = (const float*)ws;  // stat[0]
  a.g = g;
  a.nheads = nheads;
  const long total = (long)nheads * n * hl * wl * c;
  const int blocks = (int)std::min<long>(8192, (total + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == RTSDS_BF16) hipLaunchKernelGGL(upce_bwd_kernel<bf16>, dim3(blocks), dim3(256), 0, st, a);
  else if (dtype == RTSDS_F32) hipLaunchKernelGGL(upce_bwd_kernel<float>, dim3(blocks), dim3(256), 0, st, a);
  else return RTSDS_ERR_UNSUPPORTED;
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}

extern "C" int rtsds_upce_finish(int nheads, const void* ws, float* loss, float* loss_sum, void* stream) {
  if (nheads <= 0 || nheads > kUpceMaxHeads || !ws) return RTSDS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(upce_finish_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)ws, nheads, loss, loss_sum);
  return hipGetLastError() == hipSuccess ? RTSDS_OK : RTSDS_ERR_LAUNCH;
}
