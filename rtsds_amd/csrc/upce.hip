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
#include <type_traits>

static const int kUpceCMax = 32;
typedef float f2 __attribute__((ext_vector_type(2)));
static constexpr auto kUpceRows = 32.f;  // full-res rows per tile (one wave walks them)
static const int kUpceMaxHeads = 4;

struct UpceGeo {
  int n, hl, wl, c, H, W;
  float sh, sw;
  int th, tw, ntr, ntc, wmax, hmax, nblocks;
};

struct UpceArgs {
  const void* x[kUpceMaxHeads];
  float* gpart[kUpceMaxHeads];
  float* gcorr;  // [nblocks][tile_el]: the auxiliary wave's one-hot partials (null: no auxiliary wave)
  float* lpart;  // [heads][nblocks]
  float* cpart;  // [nblocks]
  float* kpart;  // [nblocks]: head 0's argmax matches per block (exact: <= the block's pixels)
  const int64_t* tgt;
  unsigned long long* correct;
  UpceGeo g;
  int nheads, ignore, want_grad;
};

RT_DEV float upce_block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// CP: channel count padded to a multiple of 4 (compile time, so every per-class loop is
// fully unrolled without guards); padding classes hold -1e30 logits (softmax weight 0).
//
// One wave per (tile, head): lane l owns the full-res column x = x_lo + xb + l of the tile
// (xb = 0, then 64 for the rare tiles wider than 64 columns) and walks down the tile's rows.
// Per row the logits are z = l0*H0 + l1*H1, H0 / H1 the horizontal blends of the two
// low-res rows at this column (width inner, as ATen's separable upsample_bilinear2d; the
// same expression as bil_mix, so rtsds_bilinear_fwd gives identical logits), recomputed only
// when the low-res row pair advances.  g = softmax - onehot is folded vertically in registers
// into the two low-res rows the pixel feeds (Rlo, Rhi); when the pair advances, the finished
// low-res row goes through the x-fold once (wave-private LDS row x the tile's weight table),
// i.e. once per scale-factor rows instead of once per row, and no workgroup barrier runs
// inside the row loop.
//
// With fewer than kUpceMaxHeads heads one more wave joins the workgroup (the auxiliary wave):
// it takes the label-only work off the head waves -- head 0's argmax / accuracy count and the
// one-hot term of every head's gradient (the same for all heads: -onehot(t) folded with the
// same bilinear weights), folded into one shared partial that the backward adds to each head's.
// The head waves then run softmax, loss and the z-part of the gradient only; head 0's wave no
// longer carries the 20-class argmax on top (a workgroup lasts as long as its slowest wave).
static constexpr int kUpceOcc = 3;  // workgroups per CU
enum { UPCE_ALL = 0, UPCE_HEAD = 1, UPCE_AUX = 2 };  // wave roles
template <typename T, int CP, bool AX>
__global__ void __launch_bounds__(256, kUpceOcc) upce_fwd_kernel(UpceArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const UpceGeo& q = a.g;
  const int TH = q.th, TW = q.tw, C = q.c, TW1 = TW + 1, tid = threadIdx.x, nthr = blockDim.x;
  const int lane = tid & 63, h = tid >> 6;  // wave = head (h == nheads: the auxiliary wave)
  constexpr bool has_aux = AX;  // (a.gcorr != nullptr)
  const int tiles = q.ntr * q.ntc;
  const int img = blockIdx.x / tiles, tt = blockIdx.x - img * tiles;
  const int tr = tt / q.ntc, tc = tt - tr * q.ntc;
  const int r0 = tr * TH, c0 = tc * TW;
  const int rows_l = min(TH + 1, q.hl - r0), cols_l = min(TW1, q.wl - c0);
  const int y_lo = bil_first_ge(r0, q.sh, q.hl, q.H), y_hi = bil_first_ge(r0 + TH, q.sh, q.hl, q.H);
  const int x_lo = bil_first_ge(c0, q.sw, q.wl, q.W);
  const int x_hi = bil_first_ge(c0 + TW, q.sw, q.wl, q.W);
  const int Wt = min(x_hi - x_lo, q.wmax);
  const int tile_el = (TH + 1) * TW1 * C;  // gradient-partial layout (compact classes)
  const int rowp = TW1 * CP, ltile = (TH + 1) * rowp;
  const int npair = TW1 * C;

  // LDS: wcol[TW1][wmax] | xj0 | xj1 | xm0 | xm1 [wmax] | xs | xe [TW1] |
  //      per head: lt[TH+1][TW1][CP] (low-res tile) | xrow[64][CP] (x-fold staging) |
  //      auxiliary wave: two one-hot fold rows [2][64][CP] | labels
  float* wcol = smem;
  int* xj0 = (int*)(wcol + TW1 * q.wmax);
  int* xj1 = xj0 + q.wmax;
  float* xm0 = (float*)(xj1 + q.wmax);
  float* xm1 = xm0 + q.wmax;
  int* xs = (int*)(xm1 + q.wmax);
  int* xe = xs + TW1;
  // per-head buffers 16-B aligned (packed 8-B LDS accesses)
  float* hbase = smem + ((TW1 * q.wmax + 4 * q.wmax + 2 * TW1 + 3) & ~3);
  const int per_head = ltile + 64 * CP;
  // labels of the tile's pixels as bytes (class, 254 = ignore_index, 253 = out of range),
  // staged once for all heads: the row loop then never waits on a global load
  unsigned char* lab = (unsigned char*)(hbase + a.nheads * per_head + (has_aux ? 2 * 64 * CP : 0));
  const int Ht = min(y_hi - y_lo, q.hmax);
  // 8 label loads in flight per thread before any LDS store (the loads are the prologue's
  // latency, not its bandwidth)
  for (int e0 = tid; e0 < Ht * Wt; e0 += 8 * nthr) {
    long tv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * nthr;
      const int yy = e / Wt, xx = e - yy * Wt;
      tv[u] = e < Ht * Wt ? a.tgt[((long)img * q.H + y_lo + yy) * q.W + x_lo + xx] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * nthr;
      const long t = tv[u];
      if (e < Ht * Wt) lab[e] = t == a.ignore ? 254 : ((t >= 0 && t < C) ? (unsigned char)t : 253);
    }
  }

  for (int xx = tid; xx < Wt; xx += nthr) {
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
  for (int e = tid; e < TW1 * Wt; e += nthr) {
    const int jl = e / Wt, xx = e - jl * Wt;
    wcol[jl * q.wmax + xx] = (xj0[xx] == jl ? xm0[xx] : 0.f) + (xj1[xx] == jl ? xm1[xx] : 0.f);
  }
  // contiguous full-res column range feeding low-res column jl (taps are monotone in x)
  for (int jl = tid; jl < TW1; jl += nthr) {
    int lo = Wt, hi = -1;
    for (int xx = 0; xx < Wt; ++xx)
      if (xj0[xx] == jl || xj1[xx] == jl) { lo = min(lo, xx); hi = xx; }
    xs[jl] = lo;
    xe[jl] = hi;
  }
  for (int hh = 0; hh < a.nheads; ++hh) {
    const T* X = (const T*)a.x[hh] + (long)img * q.hl * q.wl * C;
    float* lt = hbase + hh * per_head;
    for (int e0 = tid; e0 < ltile; e0 += 8 * nthr) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * nthr;
        const int cc = e % CP, cell = e / CP;
        const int il = cell / TW1, jl = cell - il * TW1;
        v[u] = cc < C ? 0.f : -1e30f;
        if (e < ltile && cc < C && il < rows_l && jl < cols_l) v[u] = to_f(X[((long)(r0 + il) * q.wl + (c0 + jl)) * C + cc]);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (e0 + u * nthr < ltile) lt[e0 + u * nthr] = v[u];
    }
  }
  __syncthreads();
  if (h > a.nheads || (h == a.nheads && !has_aux)) return;
  const bool aux = h == a.nheads;

  // the auxiliary wave reads head 0's tile (argmax) and folds into the shared one-hot partial
  const float* lt = hbase + (aux ? 0 : h) * per_head;
  float* xrow = aux ? hbase + a.nheads * per_head : hbase + h * per_head + ltile;
  float* gdst = !a.want_grad ? nullptr : (aux ? a.gcorr : a.gpart[h]) + (long)blockIdx.x * tile_el;
  const float kL2E = 1.4426950408889634f, kLN2 = 0.6931471805599453f;
  constexpr int CP2 = CP / 2;
  float lsum = 0.f, cnt = 0.f;
  unsigned long long corr = 0;

  auto walk = [&](auto role_c) {
    constexpr int ROLE = decltype(role_c)::value;
    // the argmax runs on head 0 (UPCE_ALL) or on the auxiliary wave
    const bool do_argmax = a.correct && (ROLE == UPCE_AUX || (ROLE == UPCE_ALL && h == 0));
    constexpr bool kSoftmax = ROLE != UPCE_AUX, kOnehot = ROLE != UPCE_HEAD;
    for (int xb = 0; xb < Wt; xb += 64) {
      const int xx = xb + lane;
      const bool xv = xx < Wt;
      const int xc = xv ? xx : Wt - 1;
      const int j0 = xj0[xc], j1 = xj1[xc];
      const float m0 = xm0[xc], m1 = xm1[xc];
      const int xend = min(xb + 63, Wt - 1);
      const bool add = xb > 0;  // later column chunks add into the rows the first one wrote
      f2 H0[CP2], H1[CP2], Rlo[CP2], Rhi[CP2];
#pragma unroll
      for (int k = 0; k < CP2; ++k) { Rlo[k] = (f2){0.f, 0.f}; Rhi[k] = (f2){0.f, 0.f}; }
      // auxiliary wave: the one-hot folds of the two low-res rows as LDS rows [64][CP] (lo, hi),
      // scattered into by one LDS atomic add per pixel and row (the lane's own row: no two lanes
      // touch one address, so the adds land in row order)
      float* clo = xrow;
      float* chi = xrow + 64 * CP;
      if constexpr (ROLE == UPCE_AUX) {
#pragma unroll
        for (int k = 0; k < CP2; ++k) {
          *(f2*)(clo + lane * CP + 2 * k) = (f2){0.f, 0.f};
          *(f2*)(chi + lane * CP + 2 * k) = (f2){0.f, 0.f};
        }
      }
      int pj[3], pc[3], plo[3], phi[3];  // this lane's x-fold pairs (low-res column, class)
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int p = min(lane + 64 * u, npair - 1);
        pj[u] = p / C;
        pc[u] = p - pj[u] * C;
        plo[u] = max(xs[pj[u]], xb);
        phi[u] = min(xe[pj[u]], xend);
      }
      auto hblend = [&](int li, f2* H) {
        const f2* L0 = (const f2*)(lt + li * rowp + j0 * CP);
        const f2* L1 = (const f2*)(lt + li * rowp + j1 * CP);
#pragma unroll
        for (int k = 0; k < CP2; ++k) H[k] = __builtin_elementwise_fma((f2){m1, m1}, L1[k], (f2){m0, m0} * L0[k]);
      };
      // x-fold of finished low-res row il (all lanes of the wave take part)
      // (the auxiliary wave's rows already sit in LDS: R == nullptr, xbuf = that row buffer)
      auto emit = [&](int il, const f2* R, const float* xbuf) {
        if (R && xv) {
#pragma unroll
          for (int k = 0; k < CP2; ++k) *(f2*)(xrow + lane * CP + 2 * k) = R[k];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS only: the row's global stores stay in flight
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < 3; ++u) {  // pairs p = lane + 64u (npair <= 3 * 64: see upce_plan)
          const int p = lane + 64 * u;
          if (p >= npair) break;
          const float* wr = wcol + pj[u] * q.wmax;
          const float* xr = xbuf + pc[u] - xb * CP;
          float s = 0.f;
          // 8 columns' LDS loads in flight per chunk (clamped, in range), then the FMAs in the
          // original ascending order: the same sum, one LDS latency per chunk instead of per column
          for (int x0 = plo[u]; x0 <= phi[u]; x0 += 8) {
            float wv[8], xv8[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const int x2 = min(x0 + k, phi[u]);
              wv[k] = wr[x2];
              xv8[k] = xr[x2 * CP];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if (x0 + k <= phi[u]) s = fmaf(wv[k], xv8[k], s);
          }
          float* o = gdst + il * npair + p;
          *o = add ? *o + s : s;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS only: the row's global stores stay in flight
        __builtin_amdgcn_wave_barrier();
      };
      // rows grouped by their top low-res row gi = r0 + li: H0 / H1 are fixed over a group, and
      // low-res row li is complete when its group ends (earlier rows fed it through Rhi)
      int li = 0;
      for (int ya = y_lo; ya < y_lo + Ht; ++li) {
        const int gi = r0 + li;
        const int yb = min(bil_first_ge(gi + 1, q.sh, q.hl, q.H), y_lo + Ht);
        const bool same = gi + 1 >= q.hl;  // bottom clamp: i1 == i0, both taps on row li
        if (kSoftmax || do_argmax) {
          hblend(li, H0);
          hblend(same ? li : li + 1, H1);
        }
        const float* L0 = lt + li * rowp;
        const float* L1 = lt + (same ? li : li + 1) * rowp;
        int tb_next = xv ? lab[(ya - y_lo) * Wt + xx] : 254;
        for (int y = ya; y < yb; ++y) {
          const int tb = tb_next;
          if (xv && y + 1 < yb) tb_next = lab[(y + 1 - y_lo) * Wt + xx];
          int i0, i1;
          float l0, l1;
          bil_src(y, q.sh, q.hl, i0, i1, l0, l1);
          if (!xv) continue;
          const bool in_range = tb < 253;
          const bool valid = tb != 254;
          f2 z[CP2];
          float mx = 0.f;
          if (kSoftmax || do_argmax) {
            // logits, packed: z = l1 * H1 + l0 * H0 (the expression of rtsds_bilinear_fwd)
#pragma unroll
            for (int k = 0; k < CP2; ++k) z[k] = __builtin_elementwise_fma((f2){l1, l1}, H1[k], (f2){l0, l0} * H0[k]);
            float mq[3] = {fmaxf(z[0].x, z[0].y), z[1].x, z[1].y};
#pragma unroll
            for (int k = 2; k < CP2; ++k) mq[k % 3] = fmaxf(mq[k % 3], fmaxf(z[k].x, z[k].y));
            mx = fmaxf(fmaxf(mq[0], mq[1]), mq[2]);
          }
          if (do_argmax) {
            int bi = 0;  // first maximum wins (torch argmax)
#pragma unroll
            for (int k = CP2 - 1; k >= 0; --k) {
              bi = z[k].y == mx ? 2 * k + 1 : bi;
              bi = z[k].x == mx ? 2 * k : bi;
            }
            // a NaN logit wins (and fmaxf skipped it): the sum of the logits is NaN then (also
            // for inf - inf, where the exact scan below is merely redundant)
            f2 zs = z[0];
#pragma unroll
            for (int k = 1; k < CP2; ++k) zs += z[k];
            const float zsum = zs.x + zs.y;
            if (__builtin_amdgcn_ballot_w64(zsum != zsum)) {  // wave-uniform: only with NaN logits
              float best = fmaf(l1, H1[0].x, l0 * H0[0].x);
              int bn = 0;
              for (int k = 1; k < CP; ++k) {
                const float zk = fmaf(l1, ((const float*)H1)[k], l0 * ((const float*)H0)[k]);
                if (zk > best || (zk != zk && best == best)) { best = zk; bn = k; }
              }
              bi = zsum != zsum ? bn : bi;
            }
            const int t = in_range ? tb : (tb == 254 ? a.ignore : -1);
            corr += (t == bi) ? 1ull : 0ull;  // t = ignore_index (or -1): never a class index < C
          }
          if constexpr (kSoftmax) {
            // z[t] from the LDS tile with the same expression as z (no register indexing)
            const int tq = in_range ? tb : 0;
            const float a00 = L0[j1 * CP + tq], a01 = L0[j0 * CP + tq], a10 = L1[j1 * CP + tq], a11 = L1[j0 * CP + tq];
            // softmax with the hardware exp2 / log2 / rcp (v_exp_f32, v_log_f32, v_rcp_f32)
            const float mxs = mx * kL2E;
            f2 sq = {0.f, 0.f};
#pragma unroll
            for (int k = 0; k < CP2; ++k) {  // z -> exp(z - max) in place
              const f2 ar = __builtin_elementwise_fma(z[k], (f2){kL2E, kL2E}, (f2){-mxs, -mxs});
              z[k] = (f2){__builtin_amdgcn_exp2f(ar.x), __builtin_amdgcn_exp2f(ar.y)};
              sq += z[k];
            }
            const float se = sq.x + sq.y;
            const float h0 = fmaf(m1, a00, m0 * a01);
            const float h1 = fmaf(m1, a10, m0 * a11);
            const float zt = in_range ? fmaf(l1, h1, l0 * h0) : NAN;
            lsum += valid ? fmaf(__builtin_amdgcn_logf(se), kLN2, mx) - zt : 0.f;
            if (h == 0) cnt += valid ? 1.f : 0.f;
            if (a.want_grad) {
              // g = softmax (- onehot(t), UPCE_ALL), folded vertically into the two low-res rows
              const float is = valid ? __builtin_amdgcn_rcpf(se) : 0.f;
              const f2 isv = {is, is}, l0v = {l0, l0}, l1v = {l1, l1};
              const int th1 = (valid && in_range) ? tb : -1;
#pragma unroll
              for (int k = 0; k < CP2; ++k) {
                f2 g;
                if constexpr (kOnehot) {
                  const f2 oh = {th1 == 2 * k ? -1.f : 0.f, th1 == 2 * k + 1 ? -1.f : 0.f};
                  g = __builtin_elementwise_fma(z[k], isv, oh);
                } else {
                  g = z[k] * isv;
                }
                Rlo[k] = __builtin_elementwise_fma(l0v, g, Rlo[k]);
                Rhi[k] = __builtin_elementwise_fma(l1v, g, Rhi[k]);
              }
            }
          } else if (a.want_grad) {
            // the auxiliary wave: -onehot(t) folded vertically into the label's class only
            if (valid && in_range) {
              atomicAdd(clo + lane * CP + tb, -l0);
              atomicAdd(chi + lane * CP + tb, -l1);
            }
          }
        }
        if (a.want_grad) {  // row li is complete
          if constexpr (ROLE == UPCE_AUX) {
            if (same) {
#pragma unroll
              for (int k = 0; k < CP2; ++k) {
                f2* lo = (f2*)(clo + lane * CP + 2 * k);
                f2* hi = (f2*)(chi + lane * CP + 2 * k);
                *lo += *hi;
                *hi = (f2){0.f, 0.f};
              }
            }
            emit(li, nullptr, clo);
#pragma unroll
            for (int k = 0; k < CP2; ++k) *(f2*)(clo + lane * CP + 2 * k) = (f2){0.f, 0.f};
            float* t2 = clo;
            clo = chi;
            chi = t2;
          } else {
            if (same) {
#pragma unroll
              for (int k = 0; k < CP2; ++k) { Rlo[k] += Rhi[k]; Rhi[k] = (f2){0.f, 0.f}; }
            }
            emit(li, Rlo, xrow);
#pragma unroll
            for (int k = 0; k < CP2; ++k) { Rlo[k] = Rhi[k]; Rhi[k] = (f2){0.f, 0.f}; }
          }
        }
        ya = yb;
      }
      const int cur = li;  // first low-res row not yet emitted (Rlo holds its contributions)
      if (a.want_grad) {  // flush row cur; rows never reached are zero
        if (cur <= TH) {
          if constexpr (ROLE == UPCE_AUX) emit(cur, nullptr, clo);
          else emit(cur, Rlo, xrow);
        }
        if (!add)
          for (int il = cur + 1; il <= TH; ++il)
            for (int p = lane; p < npair; p += 64) gdst[il * npair + p] = 0.f;
      }
    }
  };
  if constexpr (!AX) walk(std::integral_constant<int, UPCE_ALL>());
  else if (aux) walk(std::integral_constant<int, UPCE_AUX>());
  else walk(std::integral_constant<int, UPCE_HEAD>());

  if (!aux) {
    lsum = wave_sum(lsum);
    if (lane == 0) a.lpart[(long)h * q.nblocks + blockIdx.x] = lsum;
  }
  if (h == 0) {
    cnt = wave_sum(cnt);
    if (lane == 0) a.cpart[blockIdx.x] = cnt;
  }
  if (a.correct && (aux || (!has_aux && h == 0))) {
    for (int o = 32; o > 0; o >>= 1) corr += __shfl_xor(corr, o, 64);
    if (lane == 0) a.kpart[blockIdx.x] = (float)corr;
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
                                                         float* __restrict__ stat, const float* __restrict__ kpart,
                                                         unsigned long long* __restrict__ correct, int set_correct) {
  __shared__ float red[4];
  __shared__ unsigned long long kred[4];
  if (correct) {  // the argmax matches: integer sums, exact in any order
    unsigned long long k = 0;
    for (int b = threadIdx.x; b < nblocks; b += 256) k += (unsigned long long)kpart[b];
    for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o, 64);
    if ((threadIdx.x & 63) == 0) kred[threadIdx.x >> 6] = k;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long t = kred[0] + kred[1] + kred[2] + kred[3];
      *correct = set_correct ? t : *correct + t;
    }
  }
  // every array's partials of a thread loaded in one batch (8 rows in flight per array), then
  // summed in the original per-thread order b = tid, tid + 256, ...
  float acc[1 + kUpceMaxHeads];
#pragma unroll
  for (int a = 0; a <= kUpceMaxHeads; ++a) acc[a] = 0.f;
  for (int b0 = threadIdx.x; b0 < nblocks; b0 += 256 * 8) {
    float v[1 + kUpceMaxHeads][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = min(b0 + 256 * u, nblocks - 1);
      v[0][u] = cpart[b];
#pragma unroll
      for (int h = 0; h < kUpceMaxHeads; ++h) v[1 + h][u] = h < nheads ? lpart[(long)h * nblocks + b] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b0 + 256 * u < nblocks) {
#pragma unroll
        for (int a = 0; a <= kUpceMaxHeads; ++a) acc[a] += v[a][u];
      }
  }
  const float c = upce_block_sum(acc[0], red);
  if (threadIdx.x == 0) stat[0] = c;
#pragma unroll
  for (int h = 0; h < kUpceMaxHeads; ++h) {
    if (h >= nheads) break;
    const float s = upce_block_sum(acc[1 + h], red);
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
  const float* gcorr;  // the shared one-hot partials, added to every head's (or null)
  void* dx[kUpceMaxHeads];
  const float* gout;  // gout[h * gstride]
  int gstride;
  const float* count;
  UpceGeo g;
  int nheads;
};

// dx[h][img][i][j][c] = gout[h] / count * (tile partial sums covering (i, j)), fixed order:
// head h's partials, then (auxiliary wave) the shared one-hot partials.
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
    auto tsum = [&](const float* P) {
      P += (long)img * q.ntr * q.ntc * tile_el;
      auto at = [&](int rr, int cc2, int li, int lj) { return P[((long)rr * q.ntc + cc2) * tile_el + (li * TW1 + lj) * C + cc]; };
      float s = at(tr, tc, il, jl);
      if (il == 0 && tr > 0) s += at(tr - 1, tc, q.th, jl);
      if (jl == 0 && tc > 0) s += at(tr, tc - 1, il, q.tw);
      if (il == 0 && tr > 0 && jl == 0 && tc > 0) s += at(tr - 1, tc - 1, q.th, q.tw);
      return s;
    };
    float s = tsum(a.gpart[h]);
    if (a.gcorr) s += tsum(a.gcorr);
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
  // 32 full-res rows per tile: one wave per (tile, head) walks them, so shorter tiles mean more
  // waves in flight (the row loop is latency-bound at ~3 waves per SIMD)
  g.th = std::max(1, std::min(32, (int)(kUpceRows / std::ceil(fy))));
  g.wmax = (int)std::ceil((g.tw + 1) * fx) + 4;
  g.hmax = (int)std::ceil((g.th + 1) * fy) + 4;
  // kernel limits: two 64-column groups per row, <= 512 owned (column, class) pairs
  while (g.tw > 1 && (g.wmax > 128 || (g.tw + 1) * c > 192)) {
    --g.tw;
    g.wmax = (int)std::ceil((g.tw + 1) * fx) + 4;
  }
  if (g.wmax > 128 || (g.tw + 1) * c > 192) return false;  // <= 3 x-fold pairs per lane
  // tile counts from the final tile width (the loop above narrows it for small factors)
  g.ntr = (hl + g.th - 1) / g.th;
  g.ntc = (wl + g.tw - 1) / g.tw;
  g.nblocks = n * g.ntr * g.ntc;
  return (long)g.nblocks * g.ntr < (1L << 31);
}
static int upce_cp(int c) { return (c + 3) / 4 * 4; }
static size_t upce_lds_with(const UpceGeo& g, int nheads, bool aux) {
  const size_t cp = upce_cp(g.c), tile_el = (size_t)(g.th + 1) * (g.tw + 1) * cp;
  const size_t head = (((size_t)(g.tw + 1) * g.wmax + 4 * (size_t)g.wmax + 2 * (size_t)(g.tw + 1) + 3) & ~(size_t)3);
  return (head + nheads * (tile_el + 64 * cp) + (aux ? 2 * 64 * cp : 0)) * 4 + (size_t)g.hmax * g.wmax;
}
static const size_t kUpceLdsCap = 64 * 1024;
// the auxiliary wave (upce_fwd_kernel): with fewer heads than waves a workgroup can hold, and
// only when its two fold rows still fit the LDS cap -- otherwise the head waves take its roles
// (the AX = false instantiation), so the aux rows never shrink the supported geometries
static bool upce_aux(const UpceGeo& g, int nheads) {
  return nheads < kUpceMaxHeads && upce_lds_with(g, nheads, true) <= kUpceLdsCap;
}
static size_t upce_lds(const UpceGeo& g, int nheads) { return upce_lds_with(g, nheads, upce_aux(g, nheads)); }
static size_t upce_tile_el(const UpceGeo& g) { return (size_t)(g.th + 1) * (g.tw + 1) * g.c; }
// ws: stat[64] (count, per-head loss sums; offset 0, see the header) | [heads][nblocks][tile_el]
//     gradient partials | [heads][nblocks] loss partials | [nblocks] counts | (auxiliary wave)
//     [nblocks][tile_el] one-hot partials | [nblocks] argmax matches
static const size_t kUpceStat = 64;
static size_t upce_ws_floats(const UpceGeo& g, int heads) {
  return kUpceStat + (size_t)(heads + (upce_aux(g, heads) ? 1 : 0)) * g.nblocks * upce_tile_el(g) + (size_t)heads * g.nblocks +
         2 * (size_t)g.nblocks;
}
static float* upce_kpart(float* f, const UpceGeo& g, int heads) {
  return f + (size_t)(heads + (upce_aux(g, heads) ? 1 : 0)) * g.nblocks * upce_tile_el(g) + (size_t)heads * g.nblocks + g.nblocks;
}
static float* upce_gcorr(float* f, const UpceGeo& g, int heads) {
  return upce_aux(g, heads) ? f + (size_t)heads * g.nblocks * (upce_tile_el(g) + 1) + g.nblocks : nullptr;
}

extern "C" size_t rtsds_upce_workspace(int nheads, int n, int hl, int wl, int c, int H, int W, float scale_h, float scale_w) {
  UpceGeo g;
  if (nheads <= 0 || nheads > kUpceMaxHeads || !upce_plan(n, hl, wl, c, H, W, scale_h, scale_w, g)) return 0;
  if (upce_lds(g, nheads) > kUpceLdsCap) return 0;
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
  a.gcorr = upce_gcorr(f, g, nheads);
  a.kpart = upce_kpart(f, g, nheads);
  a.tgt = target;
  a.correct = correct;
  a.g = g;
  a.nheads = nheads;
  a.ignore = ignore_index;
  a.want_grad = want_grad & 1;
  hipStream_t st = (hipStream_t)stream;
  const size_t lds = upce_lds(g, nheads);
  const dim3 blk(64 * (nheads + (upce_aux(g, nheads) ? 1 : 0)));
  if (dtype != RTSDS_BF16 && dtype != RTSDS_F32) return RTSDS_ERR_UNSUPPORTED;
  switch (upce_cp(c)) {
#define UPCE_CASE(CPV)                                                                                      \
  case CPV:                                                                                                 \
    if (dtype == RTSDS_BF16 && a.gcorr) hipLaunchKernelGGL((upce_fwd_kernel<bf16, CPV, true>), dim3(g.nblocks), blk, lds, st, a); \
    else if (dtype == RTSDS_BF16) hipLaunchKernelGGL((upce_fwd_kernel<bf16, CPV, false>), dim3(g.nblocks), blk, lds, st, a);    \
    else if (a.gcorr) hipLaunchKernelGGL((upce_fwd_kernel<float, CPV, true>), dim3(g.nblocks), blk, lds, st, a);              \
    else hipLaunchKernelGGL((upce_fwd_kernel<float, CPV, false>), dim3(g.nblocks), blk, lds, st, a);                          \
    break;
    UPCE_CASE(4) UPCE_CASE(8) UPCE_CASE(12) UPCE_CASE(16) UPCE_CASE(20) UPCE_CASE(24) UPCE_CASE(28) UPCE_CASE(32)
#undef UPCE_CASE
    default: return RTSDS_ERR_UNSUPPORTED;
  }
  hipLaunchKernelGGL(upce_final_kernel, dim3(1), dim3(256), 0, st, a.lpart, a.cpart, g.nblocks, nheads, loss, loss_sum, stat,
                     a.kpart, correct, (want_grad & RTSDS_UPCE_SET_CORRECT) ? 1 : 0);
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
  a.gcorr = upce_gcorr(const_cast<float*>(f), g, nheads);
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
