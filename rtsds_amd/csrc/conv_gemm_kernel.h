#pragma once
// Implicit-GEMM convolution (forward, data-grad, weight-grad) for gfx950 / CDNA4.
//
// One kernel template serves the three GEMMs of nn.Conv2d training:
//   FWD   C[m = (n,oh,ow)][co]          = sum_{k=(r,s,ci)} X[n, oh*s-p+r*d, ...][ci] * W[co][r][s][ci]
//   DGRAD C[m = (n,ih,iw)][ci]          = sum_{k=(r,s,co)} dY[n, (ih+p-r*d)/s, ...][co] * W[co][r][s][ci]
//   WGRAD C[co][(r,s,ci)]               = sum_{pixels q} dY[q][co] * X[patch(q, r, s)][ci]
// NHWC activations make the FWD/DGRAD reduction axis (ci / co) contiguous in memory, so those
// tiles are staged "k-contiguous" (KC) and read with ds_read_b128 fragments.  WGRAD reduces
// over pixels, which are strided in NHWC: its tiles are staged pixel-major (RC, one row per
// pixel, channels contiguous -> coalesced 16-B global loads) and the MFMA fragments are
// read transposed with gfx950's ds_read_b64_tr_b16 (bf16) or plain b32 reads (f32).
//
// Tile: BM x BN x BK per 256-thread workgroup (4 waves, WM x WN), register-staged double
// buffer, one barrier per K-step.  bf16 uses v_mfma_f32_16x16x32_bf16, f32 (parity mode)
// v_mfma_f32_16x16x4_f32 (exact f32 FMA chain).
#include "conv_args.h"
#include <type_traits>
#include <utility>
#include <algorithm>
#include <cstdlib>


// (enum MODE_* and ConvArgs: conv_args.h)
template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int KS = 32;
  typedef bf16x8 frag;
  RT_DEV static f32x4 run(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int KS = 4;
  typedef float frag;
  RT_DEV static f32x4 run(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

// LDS pitches (elements).  KC: [rows][BK+pad]; bf16 pad 8 -> 80-B rows (16 consecutive rows
// hit 16 distinct 16-B slots); f32 pad 1.  RC: [BK][cols+16]: bf16 rows are 32 B mod 256 apart
// so a half-wave's 8 tr-read rows cover all 64 banks; f32 rows are 16 dwords mod 32 apart.
template <typename T, int BK> struct KCPitch { static constexpr int v = BK + (sizeof(T) == 2 ? 8 : 1); };
template <int COLS> struct RCPitch { static constexpr int v = COLS + 16; };

// ---- fragment reads --------------------------------------------------------------
// KC: lane l holds row (l&15), k-chunk (l>>4) of a 16-row block.
RT_DEV bf16x8 frag_kc(const bf16* s, int pitch, int row0, int ks, int lane) {
  return *(const bf16x8*)(s + (row0 + (lane & 15)) * pitch + ks * 32 + 8 * (lane >> 4));
}
RT_DEV float frag_kc(const float* s, int pitch, int row0, int ks, int lane) {
  return s[(row0 + (lane & 15)) * pitch + ks * 4 + (lane >> 4)];
}
// RC: tile stored [k][col].  bf16 via two ds_read_b64_tr_b16: lane 16g+4q+p addresses row
// (base + 4g + q), columns 4p..4p+3; it receives column (l&15) of those 4 rows.  Fragment
// element j <-> k row  4g+j (j<4)  /  16+4g+(j-4) (j>=4): a permutation of k shared by both
// operands, which the MFMA's k-sum does not see.
RT_DEV bf16x8 frag_rc(const bf16* s, int pitch, int col0, int ks, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const bf16* p0 = s + (ks * 32 + 4 * g + q) * pitch + col0 + 4 * p;
  const bf16* p1 = p0 + 16 * pitch;
  s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p0);
  s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p1);
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 r = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return __builtin_bit_cast(bf16x8, r);
}
RT_DEV float frag_rc(const float* s, int pitch, int col0, int ks, int lane) {
  return s[(ks * 4 + (lane >> 4)) * pitch + col0 + (lane & 15)];
}

// GL (global_load_lds) staging: the KC tile [rows][64] bf16 is written lane-linearly by the
// LDS-DMA (one wave-instruction = 8 rows of 128 B), so its bank swizzle is applied to the
// per-lane SOURCE chunk and undone on the read: row r keeps logical 16-B chunk c at physical
// slot c ^ ((r >> 1) & 7).  For the KC fragment read (lanes 0-15 rows at chunk c, 16-31 at
// c+1, ...) every ds_read_b128 lane group then covers 16 distinct 16-B bank slots.
RT_DEV int gl_swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
RT_DEV bf16x8 frag_kc_gl(const bf16* s, int row0, int ks, int lane) {
  const int row = row0 + (lane & 15);
  return *(const bf16x8*)(s + row * 64 + gl_swz(row, ks * 4 + (lane >> 4)) * 8);
}
// GL image of the RC (WGRAD) tiles: [64 pixel rows][COLS] bf16, unpadded, 16-B chunk c of row r
// at physical chunk c ^ rc_swz(r).  The transposed fragment read (ds_read_b64_tr_b16: 8 rows
// x 32 B per 32-lane group) then touches 16 distinct chunks = all 64 banks for 256-B rows.
// 64-B rows (32 columns: the 19-class weight gradients' Cout): rows r and r + 4 share banks, so
// rows 4-7 of every 8 take the other 32-B half of their row.
template <int COLS> RT_DEV int rc_swz(int row) {
  return COLS >= 128 ? (row & 7) << 1 : COLS == 32 ? ((row >> 2) & 1) << 1 : ((row >> 1) & 3) << 1;
}
// Issued as inline asm: hipcc cannot tell the transposed-read builtin apart from the LDS-DMA
// writes still in flight and would drain vmcnt(0) before every K-step's first read (losing the
// prefetch).  The caller waits lgkmcnt(0) and re-ties the registers (rc_gl_wait) before use.
RT_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p;
}
template <int COLS>
RT_DEV void frag_rc_gl_issue(const bf16* s, int col0, int ks, int lane, s16x4& t0, s16x4& t1) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = ks * 32 + 4 * g + q, r1 = r0 + 16;
  const int c = (col0 + 4 * p) >> 3, h = (p & 1) * 4;  // 16-B chunk, bf16 offset within it
  const uint32_t a0 = lds_addr(s + r0 * COLS + ((c ^ rc_swz<COLS>(r0)) << 3) + h);
  const uint32_t a1 = lds_addr(s + r1 * COLS + ((c ^ rc_swz<COLS>(r1)) << 3) + h);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(t0) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(t1) : "v"(a1));
}
RT_DEV bf16x8 rc_gl_frag(s16x4 t0, s16x4 t1) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 r = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return __builtin_bit_cast(bf16x8, r);
}
// 16 zero bytes: the DMA source of padding / out-of-range gathers.
static __device__ __attribute__((aligned(16))) bf16 g_conv_zero[8];
template <int N> RT_DEV void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int N> RT_DEV void wait_lgkmcnt() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N < 15 ? N : 15) : "memory"); }
// Fragment reads of the pipelined LDS-DMA loop as inline asm with an immediate offset from a
// per-lane base: the compiler neither waits for them (the loop counts lgkmcnt itself) nor
// re-derives their addresses.  The destination is re-tied after the wait (asm "+v") so no use
// is scheduled before the data has landed.
template <int OFF> RT_DEV void lds_rd128(bf16x8& d, uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(OFF));
}
template <int OFF> RT_DEV void lds_rdtr(s16x4& d, uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(OFF));
}
template <typename F, int... I> RT_DEV void sfor_i(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>()), ...);
}
// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1
template <int N, typename F> RT_DEV void sfor(F&& f) { sfor_i(f, std::make_integer_sequence<int, N>()); }
// Workgroup barrier of the LDS-DMA pipelines.  The s_waitcnt lgkmcnt(0) is required: without
// it the compiler may leave this wave's last ds_reads of an operand buffer outstanding across
// the barrier (their consumers, the MFMAs, are free to sink past it), and another wave's DMA
// refill of that buffer then races them -- measured as non-deterministic outputs on large
// grids (tests/test_configs_gpu.py::test_bench_conv_shapes, tools/diag/det_conv.py).
RT_DEV void gl_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename T> RT_DEV typename VecT<T>::v16 vzero() {
  typename VecT<T>::v16 z;
#pragma unroll
  for (int j = 0; j < VecT<T>::N; ++j) z[j] = (T)0.0f;
  return z;
}

// ---- main kernel -------------------------------------------------------------------
// ALA / ALB: alignment class of the A / B gathers.
//   KC A: 2 = channel count % BK == 0 (one filter tap per K-tile), 1 = % V == 0 (16-B chunks
//         never straddle a tap), 0 = scalar gather.
//   KC B: 1 = K % V == 0 (vector rows), 0 = scalar.
//   RC A/B: 1 = channel count % V == 0, 0 = scalar.
//   GL: 1 = stage A and B with global_load_lds (bf16 FWD/DGRAD, BK = 64, ALA = 2) into the
//       swizzled unpadded image above, the next K-tile's DMA in flight across the barrier
//       (counted vmcnt, raw s_barrier); 0 = register-staged double buffer.
template <typename T, int MODE, int BM, int BN, int BK, int WM, int WN, int ALA, int ALB, int GL>
__global__ void __launch_bounds__(64 * WM * WN, (GL && WM * WN == 4 && BM >= 128 && BN >= 128) ? 2 : 1)
conv_gemm_kernel(const ConvArgs P0) {
  ConvArgs P = P0;
  if (MODE == MODE_DGRAD && P0.nph > 1) {
    const ConvArgs::Phase& q = P0.phs[blockIdx.z];
    P.hp = q.hp; P.wp = q.wp; P.offh = q.offh; P.offw = q.offw; P.r0h = q.r0h; P.r0w = q.r0w;
    P.tkw = q.tkw; P.M = q.M; P.K = q.K; P.f_tkw = q.f_tkw; P.f_hw = q.f_hw; P.f_w = q.f_w;
    P.b = (const T*)P0.b + q.boff;
  }
  typedef typename VecT<T>::v16 V16;
  constexpr int V = VecT<T>::N;
  constexpr bool RC = (MODE == MODE_WGRAD);
  constexpr bool G = GL != 0;
  static_assert(!G || (sizeof(T) == 2 && BK == 64 && ALA >= 1 && ALB == 1 && BM % 32 == 0 && BN % 32 == 0 &&
                       (MODE != MODE_WGRAD || (BM >= 32 && BN >= 64))), "GL staging");
  constexpr int KCP = G ? BK : KCPitch<T, BK>::v;
  constexpr int PA = RC ? (G ? BM : RCPitch<BM>::v) : KCP;
  constexpr int PB = RC ? (G ? BN : RCPitch<BN>::v) : KCP;
  constexpr int A_EL = RC ? BK * PA : BM * PA;
  constexpr int B_EL = RC ? BK * PB : BN * PB;
  constexpr int CA = BM * BK / V, CB = BN * BK / V;      // 16-B chunks per tile
  constexpr int NW = WM * WN, NT = 64 * NW;  // waves / threads per workgroup (4 or 8 waves)
  constexpr int NA = (CA + NT - 1) / NT, NB = (CB + NT - 1) / NT;
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
  constexpr int KS = Mma<T>::KS;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(BK % KS == 0, "BK");
  static_assert(!RC || BK % (sizeof(T) == 2 ? 32 : 16) == 0, "RC BK");

  constexpr int NBUF = (GL >= 3) ? GL : 2;  // LDS operand buffers
  __shared__ __attribute__((aligned(16))) T smem[NBUF * (A_EL + B_EL)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WN) * WTM, wn0 = (wave % WN) * WTN;
  // XCD-aware remap (cdna_hip_programming.md T1, bijective form): workgroups b and b+8 run on
  // one XCD, so give each XCD a contiguous run of tiles -- M-adjacent tiles share input halo
  // rows and the same weight tile in that XCD's L2.
  // WGRAD includes the split index (the tiles of one pixel range read the same dY rows and
  // overlapping X rows: keep them on one XCD).
  int mt, nt, kz;
  {
    const int gx = gridDim.x, gxy = gx * gridDim.y;
    const int nwg = RC ? gxy * (int)gridDim.z : gxy;
    const int bid = (RC ? (int)blockIdx.z * gxy : 0) + blockIdx.y * gx + blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int t = RC ? wg % gxy : wg;
    kz = RC ? wg / gxy : (P.nph > 1 ? 0 : (int)blockIdx.z);
    // FWD / DGRAD: the N tiles of one M tile run back to back on one XCD, so each XCD's L2 keeps
    // its run of A rows across all N tiles (the weights are small and stay resident as well).
    // M-fastest order streamed A through L2 once per N tile: DeepLab's 1x1 convs with N = 1024
    // / 2048 re-read their inputs 16-32x (conv reads 53 GB per DeepLab step); 142 -> 147 img/s.
    if (!RC) {
      nt = t % (int)gridDim.y;
      mt = t / (int)gridDim.y;
    } else {
      mt = t % gx;
      nt = t / gx;
    }
  }
  const int m0 = mt * BM, n0 = nt * BN;
  if (MODE == MODE_DGRAD && P.nph > 1 && mt * BM >= P.M) return;  // phase with fewer M tiles
  const T* __restrict__ ga = (const T*)P.a;
  const T* __restrict__ gb = (const T*)P.b;

  const int nk_total = (P.K + BK - 1) / BK;
  const int kt0 = kz * P.tiles_per_split;
  const int kt1 = min(nk_total, kt0 + P.tiles_per_split);

  // ---- per-thread invariant gather state
  // KC-A rows (FWD / DGRAD): image base offset + spatial anchor of each staged row.
  long a_off[NA];
  int a_h[NA], a_w[NA];
  bool a_ok[NA];
  // RC-B column (WGRAD): fixed (tap, ci) for this thread's 16-B chunk.
  int b_r = 0, b_s = 0, b_ci = 0;
  bool b_colok = false;

  if (!RC) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int id = tid + NT * i;
      const int row = id / (BK / V);
      const int m = m0 + row;
      a_ok[i] = (id < CA) && (m < P.M);
      const int mm = a_ok[i] ? m : 0;
      if (MODE == MODE_FWD) {
        const int img = fdiv(mm, P.f_howo), rem = mm - img * P.ho * P.wo;
        const int oh = fdiv(rem, P.f_wo), ow = rem - oh * P.wo;
        a_off[i] = (long)img * P.h * P.w * P.c;
        a_h[i] = oh * P.sh - P.ph;
        a_w[i] = ow * P.sw - P.pw;
      } else {
        const int img = fdiv(mm, P.f_hw), rem = mm - img * P.hp * P.wp;
        const int th = fdiv(rem, P.f_w), tw = rem - th * P.wp;
        const int ih = th * P.psh + P.offh, iw = tw * P.psh + P.offw;
        a_off[i] = (long)img * P.ho * P.wo * P.k;
        a_h[i] = ih + P.ph;
        a_w[i] = iw + P.pw;
      }
    }
  } else {
    const int cc = tid % (BN / V);
    const int nn = n0 + cc * V;
    b_colok = nn < P.N;
    if (ALB == 1 && b_colok) {
      const int tap = fdiv(nn, P.f_c);
      b_ci = nn - tap * P.c;
      b_r = fdiv(tap, P.f_kw);
      b_s = tap - b_r * P.kw;
    }
  }

  // GL + ALA 2 (one filter tap per K-tile): LDS-DMA through buffer resources with 32-bit
  // offsets.  Each staged A row keeps its element offset at tap (0, 0) (negative in the
  // padding band is fine), the per-K-tile tap adds a wave-uniform offset, and an invalid
  // gather (padding, M edge) gets an out-of-range offset, which the DMA zero-fills (probed:
  // tools/probe/buf_lds_oob.hip).  B rows keep their byte offset; K-tiles add k0 as soffset.
  // DGRAD: stride 1, or the stride-2 parity phases (every reaching tap has matching parity, so
  // (a_h - r*dh) / 2 = (a_h >> 1) - ((r*dh) >> 1)).
  constexpr bool GB = G && !RC && ALA == 2;
  int gba_base[GB ? NA : 1], gbb_off[GB ? NB : 1];
  rsrc_t rs_a, rs_b;
  const int gsh = (MODE == MODE_DGRAD && P.sh == 2) ? 1 : 0;
  if constexpr (GB) {
    const int a_bytes = (MODE == MODE_FWD ? P.n * P.h * P.w * P.c : P.n * P.ho * P.wo * P.k) * 2;
    rs_a = make_rsrc(ga, a_bytes);
    rs_b = make_rsrc(gb, P.N * P.K * 2);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = i * (8 * NW) + wave * 8 + (lane >> 3);
      const int ch = gl_swz(row, lane & 7) * V;
      gba_base[i] = MODE == MODE_FWD ? (int)a_off[i] + (a_h[i] * P.w + a_w[i]) * P.c + ch
                                     : (int)a_off[i] + ((a_h[i] >> gsh) * P.wo + (a_w[i] >> gsh)) * P.k + ch;
      gba_base[i] *= 2;
      // opaque to the optimiser: otherwise it re-derives the offset from (hh, ww) with two
      // quarter-rate multiplies per gather inside the K loop
      asm volatile("" : "+v"(gba_base[i]));
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int row = i * (8 * NW) + wave * 8 + (lane >> 3);
      const int nrow = n0 + row;
      gbb_off[i] = nrow < P.N ? (nrow * P.K + gl_swz(row, lane & 7) * V) * 2 : (int)0x80000000;
    }
  }

  // GL WGRAD: the (tap, ci) column of each B chunk this lane stages is fixed for the whole
  // reduction (the swizzled chunk depends only on the tile row).
  int gb_r[G && RC ? NB : 1], gb_s[G && RC ? NB : 1], gb_ci[G && RC ? NB : 1];
  int gb_dh[G && RC ? NB : 1], gb_dw[G && RC ? NB : 1];  // wg_rows: row -> (d oh, d ow) in the tile
  bool gb_ok[G && RC ? NB : 1];
  if constexpr (G && RC) {
    constexpr int CPB = BN / V, RPB = 64 / CPB;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int row = (i * NW + wave) * RPB + lane / CPB;
      gb_dh[i] = P.wo >= 64 ? 0 : row / P.wo;
      gb_dw[i] = P.wo >= 64 ? row : row - gb_dh[i] * P.wo;
      const int nn = n0 + ((lane % CPB) ^ rc_swz<BN>(row)) * V;
      gb_ok[i] = nn < P.N;
      const int tap = fdiv(gb_ok[i] ? nn : 0, P.f_c);
      gb_ci[i] = (gb_ok[i] ? nn : 0) - tap * P.c;
      gb_r[i] = fdiv(tap, P.f_kw);
      gb_s[i] = tap - gb_r[i] * P.kw;
    }
  }
  // GL WGRAD on whole-row K-tiles with buffer-resource DMA: per-chunk constant parts of the
  // gather offsets; per K-tile only the tile origin (uniform) is added.  dY rows past the last
  // pixel fall past num_records and are zero-filled.
  int wga_off[G && RC ? NA : 1], wgb_ch[G && RC ? NB : 1], wgb_cw[G && RC ? NB : 1], wgb_cb[G && RC ? NB : 1];
  if constexpr (G && RC) {
    if (P.gbuf && P.wg_rows) {
      rs_a = make_rsrc(ga, P.K * P.k * 2);
      rs_b = make_rsrc(gb, P.n * P.h * P.w * P.c * 2);
      constexpr int CPA = BM / V, RPA = 64 / CPA, CPB = BN / V, RPB = 64 / CPB;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int row = (i * NW + wave) * RPA + lane / CPA;
        const int co = m0 + ((lane % CPA) ^ rc_swz<BM>(row)) * V;
        wga_off[i] = co < P.M ? (row * P.k + co) * 2 : (int)0x80000000;
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        wgb_ch[i] = gb_ok[i] ? gb_dh[i] * P.sh - P.ph + gb_r[i] * P.dh : -(1 << 30);
        wgb_cw[i] = gb_dw[i] * P.sw - P.pw + gb_s[i] * P.dw;
        wgb_cb[i] = ((wgb_ch[i] * P.w + wgb_cw[i]) * P.c + gb_ci[i]) * 2;
        asm volatile("" : "+v"(wgb_cb[i]));
      }
    }
  }

  V16 ra[NA], rb[NB];

  // ---- global -> register stage of K-tile kt
  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    if (!RC) {
      // ---- A (KC gather)
      const int Cr = (MODE == MODE_FWD) ? P.c : P.k;  // channels along the reduction
      int tap_u = 0, r_u = 0, s_u = 0, ci_u = 0;
      if (ALA == 2) {
        tap_u = k0 / Cr;
        ci_u = k0 - tap_u * Cr;
        if (MODE == MODE_FWD) {
          r_u = tap_u / P.kw;
          s_u = tap_u - r_u * P.kw;
        } else {
          const int rr = tap_u / P.tkw;
          r_u = P.r0h + rr * P.rstep;
          s_u = P.r0w + (tap_u - rr * P.tkw) * P.rstep;
        }
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int id = tid + NT * i;
        const int kc = id % (BK / V);
        V16 v = vzero<T>();
        if (ALA >= 1) {
          int r, s, ci;
          bool okk = true;
          if (ALA == 2) {
            r = r_u; s = s_u; ci = ci_u + kc * V;
          } else {
            const int kk = k0 + kc * V;
            okk = kk < P.K;
            const int tap = fdiv(kk, MODE == MODE_FWD ? P.f_c : P.f_k);
            ci = kk - tap * Cr;
            if (MODE == MODE_FWD) {
              r = fdiv(tap, P.f_kw);
              s = tap - r * P.kw;
            } else {
              const int rr = fdiv(tap, P.f_tkw);
              r = P.r0h + rr * P.rstep;
              s = P.r0w + (tap - rr * P.tkw) * P.rstep;
            }
          }
          int hh, ww;
          bool ok = a_ok[i] && okk;
          if (MODE == MODE_FWD) {
            hh = a_h[i] + r * P.dh;
            ww = a_w[i] + s * P.dw;
            ok = ok && (unsigned)hh < (unsigned)P.h && (unsigned)ww < (unsigned)P.w;
            if (ok) v = *(const V16*)(ga + a_off[i] + ((long)hh * P.w + ww) * P.c + ci);
          } else {
            int hn = a_h[i] - r * P.dh, wn = a_w[i] - s * P.dw;
            if (P.sh == 2) { ok = ok && !(hn & 1); hn >>= 1; }
            if (P.sw == 2) { ok = ok && !(wn & 1); wn >>= 1; }
            ok = ok && (unsigned)hn < (unsigned)P.ho && (unsigned)wn < (unsigned)P.wo;
            if (ok) v = *(const V16*)(ga + a_off[i] + ((long)hn * P.wo + wn) * P.k + ci);
          }
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const int kk = k0 + kc * V + j;
            if (!a_ok[i] || kk >= P.K) continue;
            const int tap = kk / Cr;
            const int ci = kk - tap * Cr;
            const int r = tap / P.kw, s = tap - r * P.kw;
            if (MODE == MODE_FWD) {
              const int hh = a_h[i] + r * P.dh, ww = a_w[i] + s * P.dw;
              if ((unsigned)hh < (unsigned)P.h && (unsigned)ww < (unsigned)P.w)
                v[j] = ga[a_off[i] + ((long)hh * P.w + ww) * P.c + ci];
            } else {
              int hn = a_h[i] - r * P.dh, wn = a_w[i] - s * P.dw;
              bool ok = true;
              if (P.sh == 2) { ok = !(hn & 1); hn >>= 1; }
              if (P.sw == 2) { ok = ok && !(wn & 1); wn >>= 1; }
              if (ok && (unsigned)hn < (unsigned)P.ho && (unsigned)wn < (unsigned)P.wo)
                v[j] = ga[a_off[i] + ((long)hn * P.wo + wn) * P.k + ci];
            }
          }
        }
        ra[i] = v;
      }
      // ---- B (KC rows of the [N][K] weight matrix)
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int id = tid + NT * i;
        const int row = id / (BK / V), kc = id % (BK / V);
        const int nrow = n0 + row, kk = k0 + kc * V;
        V16 v = vzero<T>();
        if (id < CB && nrow < P.N) {
          const T* src = gb + (long)nrow * P.K + kk;
          if (ALB == 1) {
            if (kk < P.K) v = *(const V16*)src;
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j)
              if (kk + j < P.K) v[j] = src[j];
          }
        }
        rb[i] = v;
      }
    } else {
      // ---- WGRAD A: dY rows (pixels) x Cout columns
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int id = tid + NT * i;
        const int kk = id / (BM / V), cc = id % (BM / V);
        const int q = k0 + kk, co = m0 + cc * V;
        V16 v = vzero<T>();
        if (id < CA && q < P.K) {
          const T* src = ga + (long)q * P.k + co;
          if (ALA == 1) {
            if (co < P.M) v = *(const V16*)src;
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j)
              if (co + j < P.M) v[j] = src[j];
          }
        }
        ra[i] = v;
      }
      // ---- WGRAD B: input patches, rows = output pixels, columns = (r, s, ci)
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int id = tid + NT * i;
        const int kk = id / (BN / V), cc = id % (BN / V);
        const int q = k0 + kk;
        V16 v = vzero<T>();
        if (id < CB && q < P.K) {
          const int img = fdiv(q, P.f_howo), rem = q - img * P.ho * P.wo;
          const int oh = fdiv(rem, P.f_wo), ow = rem - oh * P.wo;
          const long base = (long)img * P.h * P.w * P.c;
          const int hb = oh * P.sh - P.ph, wb = ow * P.sw - P.pw;
          if (ALB == 1) {
            const int hh = hb + b_r * P.dh, ww = wb + b_s * P.dw;
            if (b_colok && (unsigned)hh < (unsigned)P.h && (unsigned)ww < (unsigned)P.w)
              v = *(const V16*)(gb + base + ((long)hh * P.w + ww) * P.c + b_ci);
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j) {
              const int nn = n0 + cc * V + j;
              if (nn >= P.N) continue;
              const int tap = nn / P.c, ci = nn - tap * P.c;
              const int r = tap / P.kw, s = tap - r * P.kw;
              const int hh = hb + r * P.dh, ww = wb + s * P.dw;
              if ((unsigned)hh < (unsigned)P.h && (unsigned)ww < (unsigned)P.w)
                v[j] = gb[base + ((long)hh * P.w + ww) * P.c + ci];
            }
          }
        }
        rb[i] = v;
      }
    }
  };

  // GB: (channel chunk, tap row, tap column) of the next K-tile gl_issue stages.  K-tiles are
  // staged strictly in order, so the decomposition advances by one per call instead of costing
  // three scalar integer divisions (~100 SALU instructions) per K-tile.
  unsigned gw_q = 0, gw_tap = 0, gw_ntap = 1;
  int gw_rr = 0, gw_cc = 0, gw_tkw = 1;
  if constexpr (GB) {
    gw_ntap = (unsigned)(P.K / (MODE == MODE_FWD ? P.c : P.k));
    gw_tkw = MODE == MODE_FWD ? P.kw : P.tkw;
    gw_q = (unsigned)kt0 / gw_ntap;
    gw_tap = (unsigned)kt0 - gw_q * gw_ntap;
    gw_rr = (int)gw_tap / gw_tkw;
    gw_cc = (int)gw_tap - gw_rr * gw_tkw;
  }

  // ---- GL: global -> LDS DMA of K-tile kt into buffer buf (NA + NB instructions per thread)
  auto gl_issue = [&](int kt, int buf) {
    if constexpr (G && RC) {
      typedef __attribute__((address_space(3))) void* lds_t;
      typedef const __attribute__((address_space(1))) void* glb_t;
      const int k0 = kt * BK;
      T* sa = smem + buf * (A_EL + B_EL);
      T* sb = sa + A_EL;
      constexpr int CPA = BM / V, RPA = 64 / CPA;  // chunks per row, rows per wave-instruction
      constexpr int CPB = BN / V, RPB = 64 / CPB;
      if (P.gbuf && P.wg_rows) {
#pragma unroll
        for (int i = 0; i < NA; ++i) buf_lds16(rs_a, sa + (i * NW + wave) * RPA * BM, wga_off[i], k0 * P.k * 2);
        const int t_img = fdiv(k0, P.f_howo), t_rem = k0 - t_img * P.ho * P.wo;
        const int t_oh = fdiv(t_rem, P.f_wo), t_ow = t_rem - t_oh * P.wo;
        const int uh = t_oh * P.sh, uw = t_ow * P.sw;
        const int ub = (((t_img * P.h + uh) * P.w + uw) * P.c) * 2;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const bool ok = (unsigned)(uh + wgb_ch[i]) < (unsigned)P.h && (unsigned)(uw + wgb_cw[i]) < (unsigned)P.w;
          buf_lds16(rs_b, sb + (i * NW + wave) * RPB * BN, ok ? ub + wgb_cb[i] : (int)0x80000000, 0);
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {  // dY rows (pixels) x Cout columns
        const int rb = (i * NW + wave) * RPA, row = rb + lane / CPA;
        const int chunk = (lane % CPA) ^ rc_swz<BM>(row);
        const int q = k0 + row, co = m0 + chunk * V;
        const T* src = (q < P.K && co < P.M) ? ga + (long)q * P.k + co : g_conv_zero;
        __builtin_amdgcn_global_load_lds((glb_t)src, (lds_t)(sa + rb * BM), 16, 0, 0);
      }
      // tile origin (img, oh0, ow0): wave-uniform
      const int t_img = fdiv(k0, P.f_howo), t_rem = k0 - t_img * P.ho * P.wo;
      const int t_oh = fdiv(t_rem, P.f_wo), t_ow = t_rem - t_oh * P.wo;
      const T* t_base = gb + (long)t_img * P.h * P.w * P.c;
#pragma unroll
      for (int i = 0; i < NB; ++i) {  // input patches: rows = output pixels, columns = (r, s, ci)
        const int rb = (i * NW + wave) * RPB, row = rb + lane / CPB;
        const int q = k0 + row;
        const T* src = g_conv_zero;
        if (P.wg_rows) {
          const int hh = (t_oh + gb_dh[i]) * P.sh - P.ph + gb_r[i] * P.dh;
          const int ww = (t_ow + gb_dw[i]) * P.sw - P.pw + gb_s[i] * P.dw;
          if (gb_ok[i] && (unsigned)hh < (unsigned)P.h && (unsigned)ww < (unsigned)P.w)
            src = t_base + ((long)hh * P.w + ww) * P.c + gb_ci[i];
        } else if (gb_ok[i] && q < P.K) {
          const int img = fdiv(q, P.f_howo), rem = q - img * P.ho * P.wo;
          const int oh = fdiv(rem, P.f_wo), ow = rem - oh * P.wo;
          const int hh = oh * P.sh - P.ph + gb_r[i] * P.dh, ww = ow * P.sw - P.pw + gb_s[i] * P.dw;
          if ((unsigned)hh < (unsigned)P.h && (unsigned)ww < (unsigned)P.w)
            src = gb + (long)img * P.h * P.w * P.c + ((long)hh * P.w + ww) * P.c + gb_ci[i];
        }
        __builtin_amdgcn_global_load_lds((glb_t)src, (lds_t)(sb + rb * BN), 16, 0, 0);
      }
    } else if constexpr (GB) {
      T* sa = smem + buf * (A_EL + B_EL);
      T* sb = sa + A_EL;
      // K-tiles run channel-chunk-major, tap-minor: the taps of one 64-channel chunk follow
      // each other, so the tile's input rows (+ halo) for that chunk stay in L2 across the
      // taps instead of being re-fetched from MALL/HBM once per tap (the channel-major order
      // streams the whole Cin between two taps: 16 MB per XCD for the 1024-channel FFM conv).
      const int Cr = (MODE == MODE_FWD) ? P.c : P.k;
      (void)kt;  // == the walker's K-tile: q * ntap + tap
      const int tap = (int)gw_tap, ci = (int)gw_q * BK;
      const int kb = tap * Cr + ci;  // B column of this K-tile
      const int r = MODE == MODE_FWD ? gw_rr : P.r0h + gw_rr * P.rstep;
      const int sx = MODE == MODE_FWD ? gw_cc : P.r0w + gw_cc * P.rstep;
      if (++gw_cc == gw_tkw) {
        gw_cc = 0;
        ++gw_rr;
      }
      if (++gw_tap == gw_ntap) {
        gw_tap = 0;
        gw_rr = 0;
        gw_cc = 0;
        ++gw_q;
      }
      const int dhh = (r * P.dh) >> gsh, dww = (sx * P.dw) >> gsh;
      const int toff = MODE == MODE_FWD ? (dhh * P.w + dww) * P.c + ci : ci - (dhh * P.wo + dww) * P.k;
      const unsigned lim_h = MODE == MODE_FWD ? P.h : P.ho, lim_w = MODE == MODE_FWD ? P.w : P.wo;
      const int toff2 = toff * 2;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int hh = MODE == MODE_FWD ? a_h[i] + dhh : (a_h[i] >> gsh) - dhh;
        const int ww = MODE == MODE_FWD ? a_w[i] + dww : (a_w[i] >> gsh) - dww;
        const bool ok = a_ok[i] && (unsigned)hh < lim_h && (unsigned)ww < lim_w;
        const int voff = ok ? gba_base[i] + toff2 : (int)0x80000000;
        buf_lds16(rs_a, sa + (i * (8 * NW) + wave * 8) * BK, voff, 0);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i)
        buf_lds16(rs_b, sb + (i * (8 * NW) + wave * 8) * BK, gbb_off[i], kb * 2);
    } else if constexpr (G) {
      typedef __attribute__((address_space(3))) void* lds_t;
      typedef const __attribute__((address_space(1))) void* glb_t;
      const int k0 = kt * BK;
      T* sa = smem + buf * (A_EL + B_EL);
      T* sb = sa + A_EL;
      const int Cr = (MODE == MODE_FWD) ? P.c : P.k;
      // ALA 2: one filter tap per K-tile (wave-uniform); ALA 1: a tap per 16-B chunk.
      int tap_u = 0, ci_u = 0, r_u = 0, s_u = 0;
      if (ALA == 2) {
        tap_u = k0 / Cr;
        ci_u = k0 - tap_u * Cr;
        if (MODE == MODE_FWD) {
          r_u = tap_u / P.kw;
          s_u = tap_u - r_u * P.kw;
        } else {
          const int rr = tap_u / P.tkw;
          r_u = P.r0h + rr * P.rstep;
          s_u = P.r0w + (tap_u - rr * P.tkw) * P.rstep;
        }
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int row = i * (8 * NW) + wave * 8 + (lane >> 3);
        const int chunk = gl_swz(row, lane & 7);
        int ci = ci_u + chunk * V, r = r_u, sx = s_u;
        bool okk = true;
        if (ALA == 1) {
          const int kk = k0 + chunk * V;
          okk = kk < P.K;
          const int tap = fdiv(kk, MODE == MODE_FWD ? P.f_c : P.f_k);
          ci = kk - tap * Cr;
          if (MODE == MODE_FWD) {
            r = fdiv(tap, P.f_kw);
            sx = tap - r * P.kw;
          } else {
            const int rr = fdiv(tap, P.f_tkw);
            r = P.r0h + rr * P.rstep;
            sx = P.r0w + (tap - rr * P.tkw) * P.rstep;
          }
        }
        const T* src = g_conv_zero;
        if (MODE == MODE_FWD) {
          const int hh = a_h[i] + r * P.dh, ww = a_w[i] + sx * P.dw;
          if (okk && a_ok[i] && (unsigned)hh < (unsigned)P.h && (unsigned)ww < (unsigned)P.w)
            src = ga + a_off[i] + ((long)hh * P.w + ww) * P.c + ci;
        } else {
          int hn = a_h[i] - r * P.dh, wn = a_w[i] - sx * P.dw;
          bool ok = a_ok[i] && okk;
          if (P.sh == 2) { ok = ok && !(hn & 1); hn >>= 1; }
          if (P.sw == 2) { ok = ok && !(wn & 1); wn >>= 1; }
          if (ok && (unsigned)hn < (unsigned)P.ho && (unsigned)wn < (unsigned)P.wo)
            src = ga + a_off[i] + ((long)hn * P.wo + wn) * P.k + ci;
        }
        __builtin_amdgcn_global_load_lds((glb_t)src, (lds_t)(sa + (i * (8 * NW) + wave * 8) * BK), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int row = i * (8 * NW) + wave * 8 + (lane >> 3);
        const int nrow = n0 + row;
        const int kk = k0 + gl_swz(row, lane & 7) * V;
        const T* src = (nrow < P.N && kk < P.K) ? gb + (long)nrow * P.K + kk : g_conv_zero;
        __builtin_amdgcn_global_load_lds((glb_t)src, (lds_t)(sb + (i * (8 * NW) + wave * 8) * BK), 16, 0, 0);
      }
    }
  };

  // ---- register -> LDS stage
  auto store_tile = [&](int buf) {
    T* sa = smem + buf * (A_EL + B_EL);
    T* sb = sa + A_EL;
    if (!RC) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int id = tid + NT * i;
        if (id >= CA) break;
        const int row = id / (BK / V), kc = id % (BK / V);
        T* dst = sa + row * PA + kc * V;
        if (sizeof(T) == 2) *(V16*)dst = ra[i];
        else {
#pragma unroll
          for (int j = 0; j < V; ++j) dst[j] = ra[i][j];
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int id = tid + NT * i;
        if (id >= CB) break;
        const int row = id / (BK / V), kc = id % (BK / V);
        T* dst = sb + row * PB + kc * V;
        if (sizeof(T) == 2) *(V16*)dst = rb[i];
        else {
#pragma unroll
          for (int j = 0; j < V; ++j) dst[j] = rb[i][j];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int id = tid + NT * i;
        if (id >= CA) break;
        const int kk = id / (BM / V), cc = id % (BM / V);
        *(V16*)(sa + kk * PA + cc * V) = ra[i];
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int id = tid + NT * i;
        if (id >= CB) break;
        const int kk = id / (BN / V), cc = id % (BN / V);
        *(V16*)(sb + kk * PB + cc * V) = rb[i];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (GL >= 3 && kt0 < kt1) {
    // NBUF-deep ring, one barrier per K-step: tiles kt+1 .. kt+NBUF-2 stay in flight while
    // tile kt is consumed; the barrier also retires every wave's reads of tile kt-1, whose
    // buffer the DMA of tile kt+NBUF-1 then refills.
#pragma unroll
    for (int p2 = 0; p2 < NBUF - 1; ++p2)
      if (kt0 + p2 < kt1) gl_issue(kt0 + p2, p2);
    for (int kt = kt0; kt < kt1; ++kt) {
      const int it = kt - kt0, buf = it % NBUF;
      if (kt + NBUF - 2 < kt1) wait_vmcnt<(NBUF - 2) * (NA + NB)>();
      else wait_vmcnt<0>();
      gl_barrier();
      if (kt + NBUF - 1 < kt1) gl_issue(kt + NBUF - 1, (it + NBUF - 1) % NBUF);
      const T* sa = smem + buf * (A_EL + B_EL);
      const T* sb = sa + A_EL;
#pragma unroll
      for (int ks = 0; ks < BK / KS; ++ks) {
        bf16x8 fa[FM], fb[FN];
        if constexpr (RC) {
          s16x4 ta[FM][2], tb[FN][2];
#pragma unroll
          for (int i = 0; i < FM; ++i) frag_rc_gl_issue<BM>((const bf16*)sa, wm0 + i * 16, ks, lane, ta[i][0], ta[i][1]);
#pragma unroll
          for (int j = 0; j < FN; ++j) frag_rc_gl_issue<BN>((const bf16*)sb, wn0 + j * 16, ks, lane, tb[j][0], tb[j][1]);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            asm volatile("" : "+v"(ta[i][0]), "+v"(ta[i][1]));
            fa[i] = rc_gl_frag(ta[i][0], ta[i][1]);
          }
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            asm volatile("" : "+v"(tb[j][0]), "+v"(tb[j][1]));
            fb[j] = rc_gl_frag(tb[j][0], tb[j][1]);
          }
        } else {
#pragma unroll
          for (int i = 0; i < FM; ++i) fa[i] = frag_kc_gl((const bf16*)sa, wm0 + i * 16, ks, lane);
#pragma unroll
          for (int j = 0; j < FN; ++j) fb[j] = frag_kc_gl((const bf16*)sb, wn0 + j * 16, ks, lane);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  } else if (G && kt0 < kt1) {
   // LDS-DMA K loop.  The MFMA fragments are read by inline asm from per-lane bases (immediate
   // offsets) into two register sets: K-substep ks+1's reads are in flight during ks's MFMAs
   // behind a counted lgkmcnt.  (Left to the compiler, the schedule re-used one fragment pair per
   // operand and waited on each read right after issuing it: the LDS latency was exposed four
   // times per K-tile and wave.)  Two DMA schedules (profiles/r5_conv_loop_ab.txt):
   //  1 (FWD / WGRAD tiles >= 128 x 128): an NBUF-deep ring with ONE barrier per K-tile -- the
   //    barrier at the top of tile kt (after this wave's DMA of kt has landed) also retires every
   //    wave's reads of tile kt-1, so tile kt+NBUF-1's DMA goes into that buffer right after it;
   //    ResNet layer2-4 convs and weight gradients -3 to -5 %;
   //  2 (everything else, and DGRAD 128 x 128): two barriers per K-tile, the next tile's DMA
   //    issued before the wait for this one -- a barrier and a DMA issue more time to land than
   //    behind one tile's few MFMAs: the ring schedule was 5-35 % slower on these tiles, this one
   //    is 1-8 % faster than compiler-scheduled reads (layer1 weight gradients -8.5 %).
   constexpr bool PIPE = BM >= 128 && BN >= 128 && MODE != MODE_DGRAD;
   constexpr int SCHED = PIPE ? 1 : 2;
   if constexpr (G) {
    constexpr int NKS = BK / 32;
    constexpr int BUFB = (A_EL + B_EL) * (int)sizeof(T);
    constexpr int NRD = RC ? 2 * (FM + FN) : FM + FN;  // LDS read instructions per K-substep
    const uint32_t s0 = lds_addr(smem);
    // KC: one base per operand and K-substep (the chunk swizzle depends on the substep; the
    // 16-row fragment blocks are 2 KB apart).  RC: one base per fragment (the chunk swizzle of the
    // column block), substeps 32 rows apart, the second half-read 16 rows below the first.
    uint32_t ka[RC ? 1 : NKS], kb[RC ? 1 : NKS], ra[RC ? FM : 1], rb[RC ? FN : 1];
    if constexpr (!RC) {
      const int r = lane & 15;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        ka[ks] = s0 + ((wm0 + r) * 64 + gl_swz(wm0 + r, ks * 4 + (lane >> 4)) * 8) * 2;
        kb[ks] = s0 + A_EL * 2 + ((wn0 + r) * 64 + gl_swz(wn0 + r, ks * 4 + (lane >> 4)) * 8) * 2;
      }
    } else {
      const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3, r0 = 4 * g + q, h = (p & 1) * 4;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int c = (wm0 + i * 16 + 4 * p) >> 3;
        ra[i] = s0 + (r0 * BM + ((c ^ rc_swz<BM>(r0)) << 3) + h) * 2;
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int c = (wn0 + j * 16 + 4 * p) >> 3;
        rb[j] = s0 + A_EL * 2 + (r0 * BN + ((c ^ rc_swz<BN>(r0)) << 3) + h) * 2;
      }
    }
    bf16x8 fa[2][FM], fb[2][FN];
    s16x4 ta[2][FM][2], tb[2][FN][2];
    // issue the reads of K-substep K into register set S; bo: byte offset of the tile's buffer
    auto rd = [&](uint32_t bo, auto kc, auto sc) {
      constexpr int K = decltype(kc)::value, S = decltype(sc)::value;
      if constexpr (!RC) {
        const uint32_t a = ka[K] + bo, b = kb[K] + bo;
        sfor<FM>([&](auto ic) { lds_rd128<decltype(ic)::value * 2048>(fa[S][decltype(ic)::value], a); });
        sfor<FN>([&](auto jc) { lds_rd128<decltype(jc)::value * 2048>(fb[S][decltype(jc)::value], b); });
      } else {
        sfor<FM>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          lds_rdtr<K * 32 * BM * 2>(ta[S][i][0], ra[i] + bo);
          lds_rdtr<K * 32 * BM * 2 + 16 * BM * 2>(ta[S][i][1], ra[i] + bo);
        });
        sfor<FN>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          lds_rdtr<K * 32 * BN * 2>(tb[S][j][0], rb[j] + bo);
          lds_rdtr<K * 32 * BN * 2 + 16 * BN * 2>(tb[S][j][1], rb[j] + bo);
        });
      }
    };
    // the MFMAs of register set S (its reads waited for by the caller)
    auto mm = [&](auto sc) {
      constexpr int S = decltype(sc)::value;
      bf16x8 xa[FM], xb[FN];
      if constexpr (!RC) {
#pragma unroll
        for (int i = 0; i < FM; ++i) { asm volatile("" : "+v"(fa[S][i])); xa[i] = fa[S][i]; }
#pragma unroll
        for (int j = 0; j < FN; ++j) { asm volatile("" : "+v"(fb[S][j])); xb[j] = fb[S][j]; }
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          asm volatile("" : "+v"(ta[S][i][0]), "+v"(ta[S][i][1]));
          xa[i] = rc_gl_frag(ta[S][i][0], ta[S][i][1]);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          asm volatile("" : "+v"(tb[S][j][0]), "+v"(tb[S][j][1]));
          xb[j] = rc_gl_frag(tb[S][j][0], tb[S][j][1]);
        }
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[i], xb[j], acc[i][j], 0, 0, 0);
      // the next substep's lgkmcnt wait must not be hoisted above these MFMAs (asm volatile
      // orders only against other asm: the scheduler sank the MFMAs below the final wait)
      __builtin_amdgcn_sched_barrier(0);
    };
   if constexpr (SCHED == 1) {
    // NBUF-deep ring: tiles kt+1 .. kt+NBUF-2 stay in flight while tile kt is consumed
#pragma unroll
    for (int p2 = 0; p2 < NBUF - 1; ++p2)
      if (kt0 + p2 < kt1) gl_issue(kt0 + p2, p2);
    int buf = 0;  // buffer of tile kt
    for (int kt = kt0; kt < kt1; ++kt) {
      const uint32_t bo = buf * BUFB;
      // this wave's DMA of tile kt has landed (the younger tiles' stay in flight) ...
      if (kt + NBUF - 2 < kt1) wait_vmcnt<(NBUF - 2) * (NA + NB)>();
      else wait_vmcnt<0>();
      gl_barrier();  // ... every wave's; and every wave is done reading tile kt-1's buffer
      rd(bo, std::integral_constant<int, 0>(), std::integral_constant<int, 0>());
      if (kt + NBUF - 1 < kt1) gl_issue(kt + NBUF - 1, buf == 0 ? NBUF - 1 : buf - 1);
      buf = buf + 1 == NBUF ? 0 : buf + 1;
      sfor<NKS>([&](auto kc) {
        constexpr int K = decltype(kc)::value;
        if constexpr (K + 1 < NKS) {
          rd(bo, std::integral_constant<int, K + 1>(), std::integral_constant<int, (K + 1) & 1>());
          wait_lgkmcnt<NRD>();
        } else {
          wait_lgkmcnt<0>();
        }
        mm(std::integral_constant<int, K & 1>());
      });
    }
   } else if constexpr (SCHED == 2) {
    // two-barrier schedule (the next tile's DMA issued before the wait for this one) with the
    // look-ahead fragment reads of the ring schedule
    gl_issue(kt0, 0);
    for (int kt = kt0; kt < kt1; ++kt) {
      const int buf = (kt - kt0) & 1;
      if (kt + 1 < kt1) {
        gl_issue(kt + 1, buf ^ 1);
        wait_vmcnt<NA + NB>();  // tile kt landed; tile kt+1 stays in flight across the barrier
      } else {
        wait_vmcnt<0>();
      }
      gl_barrier();
      const uint32_t bo = buf * BUFB;
      rd(bo, std::integral_constant<int, 0>(), std::integral_constant<int, 0>());
      sfor<NKS>([&](auto kc) {
        constexpr int K = decltype(kc)::value;
        if constexpr (K + 1 < NKS) {
          rd(bo, std::integral_constant<int, K + 1>(), std::integral_constant<int, (K + 1) & 1>());
          wait_lgkmcnt<NRD>();
        } else {
          wait_lgkmcnt<0>();
        }
        mm(std::integral_constant<int, K & 1>());
      });
      gl_barrier();  // every wave is done reading buf before it is refilled
    }
   }
   }
  } else if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int buf = (kt - kt0) & 1;
      const bool more = kt + 1 < kt1;
      if (more) load_tile(kt + 1);
      const T* sa = smem + buf * (A_EL + B_EL);
      const T* sb = sa + A_EL;
#pragma unroll
      for (int ks = 0; ks < BK / KS; ++ks) {
        typename Mma<T>::frag fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          fa[i] = RC ? frag_rc(sa, PA, wm0 + i * 16, ks, lane) : frag_kc(sa, PA, wm0 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          fb[j] = RC ? frag_rc(sb, PB, wn0 + j * 16, ks, lane) : frag_kc(sb, PB, wn0 + j * 16, ks, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = Mma<T>::run(fa[i], fb[j], acc[i][j]);
      }
      if (more) store_tile(buf ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue: C[row][col], row = (lane>>4)*4 + e, col = lane&15 within each 16x16 block
  const int er = (lane >> 4) * 4, ec = lane & 15;
  if (MODE == MODE_WGRAD || P.slab != nullptr) {  // FWD / DGRAD split-K: fp32 partials
    float* out = (MODE == MODE_WGRAD ? (float*)P.out : P.slab) + (long)kz * P.split_stride;
    if (P.N % 4 == 0) {
      // fp32 slab rows leave as 16-B chunks: the C fragments are staged through LDS one
      // wave-row band (WTM rows) at a time, [WTM][BN + 4] fp32.
      constexpr int CP = BN + 4, CPR = BN / 4;
      static_assert(WTM * CP * 4 <= (int)sizeof(smem), "slab staging fits the operand LDS");
      float* cs = (float*)smem;
#pragma unroll
      for (int band = 0; band < WM; ++band) {
        __syncthreads();
        if (wave / WN == band) {
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) cs[(i * 16 + er + e) * CP + wn0 + j * 16 + ec] = acc[i][j][e];
        }
        __syncthreads();
        for (int c = tid; c < WTM * CPR; c += NT) {
          const int row = c / CPR, cc = c - row * CPR;
          const int gm = m0 + band * WTM + row, gn = n0 + cc * 4;
          if (gm < P.M && gn < P.N) *(f32x4*)(out + (long)gm * P.N + gn) = *(const f32x4*)(cs + row * CP + cc * 4);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int gn = n0 + wn0 + j * 16 + ec;
          if (gn >= P.N) continue;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int gm = m0 + wm0 + i * 16 + er + e;
            if (gm < P.M) out[(long)gm * P.N + gn] = acc[i][j][e];
          }
        }
    }
  } else {
   // The bf16 / fp32 output epilogue, instantiated per activation: the networks' launches
   // (none, ReLU) get it with the activation fixed at compile time, anything else reads it from
   // P.act.  A per-value runtime activation cost a chain of uniform compare-and-branches for
   // every one of a lane's 64 values (~2,000 scalar branches in a 128 x 128 tile's code).
   auto epilogue = [&](auto act_c) {
    constexpr int ACT = decltype(act_c)::value;
    T* out = (T*)P.out;
    auto act_f = [&](float v) {
      const int a = ACT >= 0 ? ACT : P.act;
      if (a == RTSDS_ACT_RELU) return fmaxf(v, 0.f);
      if (a == RTSDS_ACT_LEAKY) return v > 0.f ? v : 0.2f * v;
      if (a == RTSDS_ACT_SIGMOID) return 1.f / (1.f + expf(-v));
      return v;
    };
    auto out_row = [&](int gm) -> long {  // DGRAD phase rows scatter back to the full grid
      if (MODE == MODE_DGRAD && P.psh != 1) {
        const int img = fdiv(gm, P.f_hw), rem = gm - img * P.hp * P.wp;
        const int th = fdiv(rem, P.f_w), tw = rem - th * P.wp;
        return ((long)img * P.h + th * P.psh + P.offh) * P.w + tw * P.psh + P.offw;
      }
      return gm;
    };
    const bool has_res = MODE == MODE_FWD && P.res != nullptr;
    const bool has_mask = MODE == MODE_DGRAD && P.mask != nullptr;
    auto mask_f = [&](float g, float xv) {  // act_bwd_kernel's expression
      return xv > 0.f ? g : (P.mask_act == RTSDS_ACT_LEAKY ? 0.2f * g : 0.f);
    };
    bool stored = false;
    if constexpr (sizeof(T) == 2) {
      if (P.N % V == 0) {
        // Row-vectorised store: the 16x16 C fragments (4 rows x 1 column per lane) go through
        // LDS as bf16 [BM][BN + 8] and leave as 16-B row chunks (8 global_store_dwordx4 per
        // thread for a 128x128 tile instead of 64 scattered 2-byte stores).  Residual and
        // accumulate (y += result: ConvSum, GradJoin'd dgrad) are added on the 16-B chunks,
        // the activation after them.
        constexpr int CP = BN + 8, CPR = BN / V;
        static_assert(BM * CP <= NBUF * (A_EL + B_EL), "epilogue staging fits the operand LDS");
        T* cs = smem;
        const bool post = has_res || P.accum || has_mask;
        const bool bnb = MODE == MODE_DGRAD && P.bnb_part != nullptr;  // (host: CPR divides NT)
        float bg[V], bgx[V], bmu[V], bsc[V], bsh[V];
        if (bnb) {
          const int ch0 = n0 + (tid % CPR) * V;  // this thread's fixed channel chunk
#pragma unroll
          for (int q = 0; q < V; ++q) {
            const int ch = min(ch0 + q, P.N - 1);
            const float g = P.bnb_gamma ? P.bnb_gamma[ch] : 1.f, b = P.bnb_beta ? P.bnb_beta[ch] : 0.f;
            bmu[q] = P.bnb_mean[ch];
            bsc[q] = g * P.bnb_invstd[ch];     // bn_coef
            bsh[q] = fmaf(-bmu[q], bsc[q], b);
            bg[q] = 0.f;
            bgx[q] = 0.f;
          }
        }
        // the BatchNorm input chunks this thread folds into the statistics, loaded up front (all
        // in flight across the LDS staging): read after each chunk's store they serialised
        // behind it (the compiler cannot reorder them past the possibly-aliasing store).  The
        // 160-row tiles (10 chunks per thread) preload half of them (registers: 2 groups per
        // CU) and the other half as one batch after the first half's stores.
        constexpr int NIT = (BM * CPR + NT - 1) / NT;
        constexpr int NPL = NIT > 8 ? (NIT + 1) / 2 : NIT;
        constexpr int NXP = MODE == MODE_DGRAD ? NPL : 1;
        V16 xpre[NXP];
        const bool pmask = MODE == MODE_DGRAD && has_mask;  // (mask and accumulate exclusive)
        const bool ppre_on = pmask || P.accum;
        V16 ppre[NPL];
        auto chunk_ok = [&](int it, long& o) {
          const int c = tid + it * NT;
          const int row = c / CPR, cc = c - row * CPR;
          const int gm = m0 + row, gn = n0 + cc * V;
          const bool ok = c < BM * CPR && gm < P.M && gn < P.N;
          o = ok ? out_row(gm) * P.N + gn : 0;
          return ok;
        };
        auto load_x = [&](int it, V16& xr) {
          long o;
          if (chunk_ok(it, o)) xr = *(const V16*)((const T*)P.bnb_x + o);
        };
        auto load_p = [&](int it, V16& pr) {
          long o;
          if (chunk_ok(it, o)) pr = pmask ? *(const V16*)((const T*)P.mask + o) : *(const V16*)(out + o);
        };
        if constexpr (MODE == MODE_DGRAD) {
          if (bnb) {
#pragma unroll
            for (int it = 0; it < NPL; ++it) load_x(it, xpre[it]);
          }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = wn0 + j * 16 + ec;
          const bool ok = n0 + col < P.N;
          const float bv = (P.bias && ok) ? P.bias[n0 + col] : 0.f;
          const float sv = (MODE == MODE_FWD && P.scale && ok) ? P.scale[n0 + col] : 1.f;
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float v = fmaf(acc[i][j][e], sv, bv);
              cs[(wm0 + i * 16 + er + e) * CP + col] = from_f<T>(post ? v : act_f(v));
            }
        }
        // the mask / accumulate operand chunks, loaded before the staging barrier (all in
        // flight, the accumulators dead by now); read after each chunk's store they serialised
        if (ppre_on) {
#pragma unroll
          for (int it = 0; it < NPL; ++it) load_p(it, ppre[it]);
        }
        __syncthreads();
        auto process = [&](int it, const V16& pp, const V16& xr) {
          const int c = tid + it * NT;
          if (c >= BM * CPR) return;
          const int row = c / CPR, cc = c - row * CPR;
          const int gm = m0 + row, gn = n0 + cc * V;
          if (gm < P.M && gn < P.N) {
            const long orow = out_row(gm), o = orow * P.N + gn;
            V16 v = *(const V16*)(cs + row * CP + cc * V);
            if (post) {
              float f[V];
#pragma unroll
              for (int q = 0; q < V; ++q) f[q] = to_f(v[q]);
              if (has_res) {
                const V16 r = *(const V16*)((const T*)P.res + o);
#pragma unroll
                for (int q = 0; q < V; ++q) f[q] += to_f(r[q]);
              }
              if (has_mask) {  // (accumulate is refused together with a mask)
                const V16 r = pmask ? pp : *(const V16*)((const T*)P.mask + o);
#pragma unroll
                for (int q = 0; q < V; ++q) f[q] = mask_f(f[q], to_f(r[q]));
              }
              if (P.accum) {
                const V16 r = pmask ? *(const V16*)(out + o) : pp;
#pragma unroll
                for (int q = 0; q < V; ++q) f[q] += to_f(r[q]);
              }
#pragma unroll
              for (int q = 0; q < V; ++q) v[q] = from_f<T>(act_f(f[q]));
            }
            *(V16*)(out + (P.ldo ? orow * P.ldo + gn : o)) = v;  // (ldo: plain forward only, host-checked)
            if (MODE == MODE_DGRAD && bnb) {
#pragma unroll
              for (int q = 0; q < V; ++q) {
                const float xv = to_f(xr[q]);
                float g = to_f(v[q]);
                g *= fmaf(xv, bsc[q], bsh[q]) > 0.f ? 1.f : (P.bnb_act == RTSDS_ACT_LEAKY ? 0.2f : 0.f);
                bg[q] += g;
                bgx[q] = fmaf(g, xv - bmu[q], bgx[q]);
              }
            }
          }
        };
#pragma unroll
        for (int it = 0; it < NPL; ++it) process(it, ppre[it], xpre[MODE == MODE_DGRAD ? it : 0]);
        if constexpr (NPL < NIT) {
#pragma unroll
          for (int k = 0; k < NIT - NPL; ++k) {
            if constexpr (MODE == MODE_DGRAD) {
              if (bnb) load_x(NPL + k, xpre[k]);
            }
            if (ppre_on) load_p(NPL + k, ppre[k]);
          }
#pragma unroll
          for (int k = 0; k < NIT - NPL; ++k) process(NPL + k, ppre[k], xpre[MODE == MODE_DGRAD ? k : 0]);
        }
        if (bnb) {
          // threads tid = cc + CPR * k share chunk cc: sum their partials in a fixed order
          __syncthreads();
          float* red = (float*)smem;  // [NT][2 V]
#pragma unroll
          for (int q = 0; q < V; ++q) {
            red[tid * 2 * V + q] = bg[q];
            red[tid * 2 * V + V + q] = bgx[q];
          }
          __syncthreads();
          for (int e = tid; e < CPR * V; e += NT) {
            const int cc = e / V, q = e - cc * V, ch = n0 + cc * V + q;
            float a = 0.f, b = 0.f;
            for (int t = cc; t < NT; t += CPR) {
              a += red[t * 2 * V + q];
              b += red[t * 2 * V + V + q];
            }
            if (ch < P.N) *(float2*)(P.bnb_part + ((long)ch * gridDim.x + mt) * 2) = make_float2(a, b);
          }
        }
        stored = true;
      }
    }
    if (!stored) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int gn = n0 + wn0 + j * 16 + ec;
        if (gn >= P.N) continue;
        const float bv = P.bias ? P.bias[gn] : 0.f;
        const float sv = (MODE == MODE_FWD && P.scale) ? P.scale[gn] : 1.f;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int gm = m0 + wm0 + i * 16 + er + e;
            if (gm >= P.M) continue;
            const long orow = out_row(gm);
            float v = fmaf(acc[i][j][e], sv, bv);
            if (has_mask) v = mask_f(to_f(from_f<T>(v)), to_f(((const T*)P.mask)[orow * P.N + gn]));
            if (has_res) v += to_f(((const T*)P.res)[orow * P.N + gn]);
            if (P.accum) v += to_f(out[orow * P.N + gn]);
            out[orow * (P.ldo ? P.ldo : P.N) + gn] = from_f<T>(act_f(v));
          }
      }
    }
   };
    if (P.act == RTSDS_ACT_NONE) epilogue(std::integral_constant<int, RTSDS_ACT_NONE>());
    else if (P.act == RTSDS_ACT_RELU) epilogue(std::integral_constant<int, RTSDS_ACT_RELU>());
    else epilogue(std::integral_constant<int, -1>());
  }
  if (MODE == MODE_FWD && P.stats != nullptr) {
    // BatchNorm batch statistics fused into the producing conv: exact two-pass mean / M2 of
    // this tile's rows per output channel, from the fp32 accumulators (merged across tiles
    // with Chan's formula by bn_finalize_kernel).
    __syncthreads();
    float* red = (float*)smem;  // [WM][BN]
    const int wmi = wave / WN;
    const int nvalid = min(BM, P.M - m0);
    float mean[FN];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int gn = n0 + wn0 + j * 16 + ec;
        const float bv = (P.bias && gn < P.N) ? P.bias[gn] : 0.f;
        float sacc = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int gm = m0 + wm0 + i * 16 + er + e;
            const float v = acc[i][j][e] + bv;
            const float t = pass == 0 ? v : (v - mean[j]) * (v - mean[j]);
            if (gm < P.M) sacc += t;
          }
        sacc += __shfl_xor(sacc, 16, 64);
        sacc += __shfl_xor(sacc, 32, 64);
        if (lane < 16) red[wmi * BN + wn0 + j * 16 + ec] = sacc;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn0 + j * 16 + ec;
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) tot += red[w * BN + col];
        if (pass == 0) {
          mean[j] = tot / (float)nvalid;
        } else if (wmi == 0 && lane < 16 && n0 + col < P.N) {
          // [channel][M tile][4]: one 16-B record store
          *(f32x4*)(P.stats + ((long)(n0 + col) * gridDim.x + mt) * 4) = f32x4{(float)nvalid, mean[j], tot, 0.f};
        }
      }
      __syncthreads();
    }
  }
}

template <typename T, int MODE, int BM, int BN, int BK, int WM, int WN, int ALA, int ALB, int GL = 0>
static void launch(const ConvArgs& p, int splits, hipStream_t st) {
  dim3 grid(rt_cdiv(p.M, BM), rt_cdiv(p.N, BN), MODE == MODE_DGRAD && p.nph > 1 ? p.nph : splits);
  hipLaunchKernelGGL((conv_gemm_kernel<T, MODE, BM, BN, BK, WM, WN, ALA, ALB, GL>), grid, dim3(64 * WM * WN), 0, st, p);
}

// BK per tile: 64 where the tile is MFMA-dense (128x128, 64x64: one barrier per 64-deep
// K-step), 32 for 128x64 / narrow-N tiles whose LDS footprint would otherwise cut occupancy.
template <typename T, int MODE, int BM, int BN, int BK, int WM, int WN>
void launch_al(const ConvArgs& p, int cr, hipStream_t st, int splits) {
  if constexpr (sizeof(T) == 2 && BM % 32 == 0 && BN % 32 == 0) {
    // LDS-DMA path: every bf16 tile at BK = 64 (16-B chunks never straddle a tap: cr % 8 == 0)
    // (not for 3-channel images padded to 8: eight taps per K-tile gathered per chunk lose
    // to the register path there)
    if (cr % 32 == 0 && p.K % 8 == 0) {
      // ALA 2 (buffer-offset DMA): DGRAD only at stride 1 or in the stride-2 parity phases
      const bool gb_ok = p.gbuf && (MODE != MODE_DGRAD || (p.sh == p.sw && (p.sh == 1 || (p.sh == 2 && p.psh == 2))));
      // 8-wave tiles (one workgroup per CU): a 3-deep LDS ring (144 KB for 256 x 128)
      constexpr int GLV = WM * WN == 8 ? 3 : 2;
      if (cr % 64 == 0 && gb_ok) launch<T, MODE, BM, BN, 64, WM, WN, 2, 1, GLV>(p, splits, st);
      else launch<T, MODE, BM, BN, 64, WM, WN, 1, 1, GLV>(p, splits, st);
      return;
    }
  }
  if (cr % BK == 0) launch<T, MODE, BM, BN, BK, WM, WN, 2, 1>(p, splits, st);
  else launch<T, MODE, BM, BN, BK, WM, WN, 1, 1>(p, splits, st);
}

template <typename T, int MODE>
void dispatch_align(const ConvArgs& p, int cr, hipStream_t st, int splits) {
  int bm, bn;
  pick_tile(p.M, p.N, sizeof(T) == 2, bm, bn, MODE == MODE_FWD, p.K, MODE == MODE_DGRAD);
  if constexpr (sizeof(T) == 2) {
    if (bn == 32 && bm == 256) launch_al<T, MODE, 256, 32, 32, 4, 1>(p, cr, st, splits);
    else if (bn == 32) launch_al<T, MODE, 128, 32, 32, 4, 1>(p, cr, st, splits);
    else if (bn == 64 && bm == 128) launch_al<T, MODE, 128, 64, 32, 2, 2>(p, cr, st);
    else if (bn == 64) launch_al<T, MODE, 64, 64, 64, 2, 2>(p, cr, st);
    else if (MODE != MODE_WGRAD && bm == 160) launch_al<T, MODE, 160, 128, 64, 2, 2>(p, cr, st);
    else launch_al<T, MODE, 128, 128, 64, 2, 2>(p, cr, st);
  } else {
    if (bn == 32) launch_al<T, MODE, 128, 32, 16, 4, 1>(p, cr, st);
    else launch_al<T, MODE, 64, 64, 16, 2, 2>(p, cr, st);
  }
}

template <typename T>
void wgrad_launch(const ConvArgs& p, int bm, int bn, int splits, hipStream_t st) {
  constexpr int BK = sizeof(T) == 2 ? 64 : 16;
  if constexpr (sizeof(T) == 2) {
    // LDS-DMA staging (swizzled RC images)
    if (bm == 32) launch<T, MODE_WGRAD, 32, 128, BK, 1, 4, 1, 1, 2>(p, splits, st);
    else if (bm == 64 && bn == 64) launch<T, MODE_WGRAD, 64, 64, BK, 2, 2, 1, 1, 2>(p, splits, st);
    else if (bm == 64) launch<T, MODE_WGRAD, 64, 128, BK, 2, 2, 1, 1, 2>(p, splits, st);
    else if (bn == 64) launch<T, MODE_WGRAD, 128, 64, BK, 2, 2, 1, 1, 2>(p, splits, st);
    else launch<T, MODE_WGRAD, 128, 128, BK, 2, 2, 1, 1, 2>(p, splits, st);
  } else {
    launch<T, MODE_WGRAD, 64, 64, BK, 2, 2, 1, 1>(p, splits, st);
  }
}
