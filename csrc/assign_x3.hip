// N1 for fp32 / fp64 data on the matrix cores: bf16x3 distance + fused top-3 argmin, with an
// exact re-check of every row whose winner the error bound cannot certify.
//
// The reference computes its K-Means distances in fp64 difference form
// (Tile -> Sub -> Square -> Sum -> ArgMin, scripts/distribuitedClustering.py:221-234).  The
// exact SIMT tiles (lloyd_simt.hip assign_exact) reproduce that but run at the vector rate:
// 61 ms per headline iteration in fp32.  Here each operand is split into two bf16 terms,
// v = hi + lo + r with |r| <= 2^-18 |v| (RNE twice), and the score
//
//     s[k, i] = ||c_k||^2 - 2 x_i . c_k  ~=  cn_k + ch.xh + ch.xl + cl.xh   (ch, cl of -2c)
//
// runs as three bf16 MFMAs per product on the ring3 pipeline of assign_mfma_impl.h
// (centroid hi/lo images stream through LDS by LDS-DMA, point hi/lo fragments stay in
// registers).  The epilogue keeps each row's three smallest scores (tagged, as ring3) and
// the indices of the two smallest.  For every (row, centroid) pair |s_computed - s_exact|
// <= eps(row) (x3_eps): the split terms the three products leave out, bounded by the row's
// own ||xh||, ||xl|| and the centroid table's max ||th||, ||tl|| (Cauchy-Schwarz; RNE to
// bf16 has unit roundoff 2^-8, so each residual is <= 2^-8 |lo|); the MFMA accumulation --
// measured at <= 3.5 ulp(|C| + sum |a b|) per v_mfma_f32_16x16x32_bf16 on MI355X, neither a
// single rounding nor an fma chain (tools/probe_mfma_acc.hip, profiles/probe_mfma_acc_r05.txt)
// and taken as 8 x 2^-23 (|C| + sum |a b|) -- with the large hi.hi terms in their own chain
// (KS MFMAs from ||c||^2) and the cross terms in a second one from 0; the fp32 ||c||^2; the
// 4-bit index tag.  So
//   * gap = s2 - s1 > 2 eps: the winner is certain (the exact argmin);
//   * else, if s3 - s1 > 2 eps: the exact winner is one of the two smallest -- recomputed
//     in the data's own precision (fp32 or fp64 difference form), ties to the lower index;
//   * else (a third centroid within the bound): the row is re-assigned over all K exactly.
// The ambiguous rows go to two compacted lists (one ballot + one atomic per wave and point
// tile each): two-candidate checks, and full re-scans (lloyd_simt.hip's tiled exact kernel
// over the listed rows).  Labels therefore equal the exact argmin of the input dtype
// (fp32, or fp64 for fp64 data) up to that dtype's own rounding of the distances.
//
// Wide D (256 < D <= 1024): the point fragments no longer fit the registers, so a row chunk
// runs fcm_mfma.hip's bf16x3 distance GEMM into an [M, K] block (raw d2, no zero floor) and
// x3_rows_kernel does the top-3 / list pass over it (x3_eps_wide: one accumulator from
// ||x||^2 + ||c||^2 through all 3 DP / 16 MFMAs, worst-case split term).
#include <math.h>

#include "assign_mfma_impl.h"
#include "kernels.h"

namespace tdc {
namespace {

// ------------------------------------------------------------------------------------
// operand prep: rows of T [rows, ld] (d valid columns) -> bf16 hi/lo [rows, DP] (of -2v when
// neg2) + norm [rows] = ||v||^2 (pad centroid rows: BIG, so they never win)
// ------------------------------------------------------------------------------------
// nhl (nullable, float2 [rows]): ||hi||^2, ||lo||^2 of the row (the centroid side of the
// per-row error bound).  Norms are summed in fp64 (one rounding to fp32 at the end).
template <typename T>
__global__ __launch_bounds__(256) void x3_split_kernel(const T* __restrict__ src, int64_t rows,
                                                       int64_t valid, int d, int64_t ld, int DP,
                                                       int neg2, __bf16* __restrict__ hi,
                                                       __bf16* __restrict__ lo,
                                                       float* __restrict__ norm,
                                                       float2* __restrict__ nhl,
                                                       const T* __restrict__ shift) {
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * 4) {
    double s = 0.0, sh = 0.0, sl = 0.0;
    for (int c = lane; c < DP; c += 64) {
      // shift (nullable): the split terms and norms are of v - shift (argmin-invariant);
      // the bounds then scale with the spread of the data instead of its offset
      const T v = (row < valid && c < d) ? src[row * ld + c] - (shift ? shift[c] : (T)0) : (T)0;
      s += (double)v * (double)v;
      const T t = neg2 ? (T)-2 * v : v;
      const __bf16 th = (__bf16)(float)t;
      const __bf16 tl = (__bf16)(float)(t - (T)(float)th);
      hi[row * DP + c] = th;
      lo[row * DP + c] = tl;
      sh += (double)(float)th * (double)(float)th;
      sl += (double)(float)tl * (double)(float)tl;
    }
    s = wave_sum(s);
    if (nhl) {
      sh = wave_sum(sh);
      sl = wave_sum(sl);
    }
    if (lane == 0) {
      if (norm) norm[row] = (neg2 && row >= valid) ? BIG : (float)s;
      if (nhl) nhl[row] = row < valid ? make_float2((float)sh, (float)sl) : make_float2(0.f, 0.f);
    }
  }
}

// cstat = {max_k ||c_k||^2, max_k ||th_k||^2, max_k ||tl_k||^2} over the K valid rows (t =
// -2c split into hi + lo; nhl nullable: zeros), amb_count[0..1] = 0 (the lists of the next
// assignment).  One block.
__global__ __launch_bounds__(1024) void x3_prep_kernel(const float* __restrict__ cnorm,
                                                       const float2* __restrict__ nhl, int K,
                                                       float* __restrict__ cstat,
                                                       int* __restrict__ amb_count, int nzero) {
  __shared__ float red[3][16];
  float m = 0.f, mh = 0.f, ml = 0.f;
  for (int k = threadIdx.x; k < K; k += 1024) {
    m = fmaxf(m, cnorm[k]);
    if (nhl) {
      const float2 v = nhl[k];
      mh = fmaxf(mh, v.x);
      ml = fmaxf(ml, v.y);
    }
  }
  m = wave_max(m);
  mh = wave_max(mh);
  ml = wave_max(ml);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = m;
    red[1][threadIdx.x >> 6] = mh;
    red[2][threadIdx.x >> 6] = ml;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const bool in = threadIdx.x < 16;
    const float v0 = wave_max(in ? red[0][threadIdx.x] : 0.f);
    const float v1 = wave_max(in ? red[1][threadIdx.x] : 0.f);
    const float v2 = wave_max(in ? red[2][threadIdx.x] : 0.f);
    if (threadIdx.x == 0) {
      cstat[0] = v0;
      cstat[1] = v1;
      cstat[2] = v2;
      amb_count[0] = 0;
      amb_count[1] = 0;
      if (nzero > 2) amb_count[2] = 0;  // the prefilter's list
    }
  }
}

// Per-row bound on |score_computed - score_exact| over every centroid (see the file header).
// hx, lx: ||xh||, ||xl|| of the row; cstat: the centroid-side maxima; KS k-steps of 32.
//   split   : the products the three MFMAs leave out (xh tr, xl tl, xl tr, xr th, xr tl,
//             xr tr), by Cauchy-Schwarz on the actual hi / lo norms, |r| <= 2^-8/(1-2^-8) |lo|
//             (RNE to bf16: unit roundoff 2^-8);
//   MFMAs   : measured per instruction <= 3.5 ulp(|C| + sum |a b|) (tools/probe_mfma_acc.hip,
//             profiles/probe_mfma_acc_r05.txt), taken as 8 x 2^-23 (|C| + sum |a b|): the
//             main chain (KS MFMAs from ||c||^2), the cross chain (2 KS MFMAs from 0) and the
//             final add of the two;
//   ||c||^2 : summed in fp64, one rounding to fp32;
//   tag     : 4 index bits in the low mantissa of the score, <= 2^-19 |score|.
__device__ __forceinline__ float x3_eps(float hx, float lx, const float* cstat, int KS) {
  const float cn = cstat[0];
  const float Hc = sqrtf(cstat[1]) * 1.0001f, Lc = sqrtf(cstat[2]) * 1.0001f;
  constexpr float R8 = 0.00392157f;  // 2^-8 / (1 - 2^-8)
  const float Rc = R8 * Lc, Rx = R8 * lx;
  const float e_split = hx * Rc + lx * Lc + lx * Rc + Rx * Hc + Rx * Lc + Rx * Rc;
  const float s_main = hx * Hc, s_cross = hx * Lc + lx * Hc;
  constexpr float U8 = 8.f * 1.1920929e-7f;  // 8 x 2^-23
  const float e_acc = U8 * ((float)KS * cn + (float)(KS + 1) * s_main) +
                      U8 * (float)(2 * KS + 1) * s_cross +
                      5.9604645e-8f * (cn + s_main + s_cross);  // final add, 2^-24
  const float e_cn = 1.1920929e-7f * cn;
  const float e_tag = 1.9073486e-6f * (cn + s_main + s_cross);  // 2^-19
  return (e_split + e_acc + e_cn + e_tag) * 1.001f + 1e-30f;
}

// merge (v1, l1, v2, l2, v3) of two candidate sets (each v1 <= v2 <= v3, distinct centroids):
// the union's three smallest, ties of the first place to the lower index
__device__ __forceinline__ void top3_merge(float& v1, int& l1, float& v2, int& l2, float& v3,
                                           float ov1, int ol1, float ov2, int ol2, float ov3) {
  const bool ob = (ov1 < v1) || (ov1 == v1 && ol1 < l1);
  const float lv = ob ? v1 : ov1;  // loser of the first place
  const int ll = ob ? l1 : ol1;
  const bool o2 = (ov2 < v2) || (ov2 == v2 && ol2 < l2);
  const float sv = o2 ? ov2 : v2;
  const int sl = o2 ? ol2 : l2;
  const bool lw = (lv < sv) || (lv == sv && ll < sl);
  const float n3 = fminf(fminf(v3, ov3), fminf(fmaxf(v1, ov2), fmaxf(v2, ov1)));
  v1 = ob ? ov1 : v1;
  l1 = ob ? ol1 : l1;
  v2 = lw ? lv : sv;
  l2 = lw ? ll : sl;
  v3 = n3;
}

// the lanes with `amb` set append their row: {row, runner-up} to list2 (two-candidate check,
// count[0]) or row to listF (full exact re-scan, count[1]); per wave one ballot each and
// at most one atomic each
__device__ __forceinline__ void x3_append(bool amb, bool two, int64_t row, int l2,
                                          int2* __restrict__ list2, int* __restrict__ listF,
                                          int* __restrict__ count) {
  const unsigned long long m2 = __ballot(amb && two), mf = __ballot(amb && !two);
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  if (m2) {
    const int leader = __builtin_ctzll(m2);
    int base = 0;
    if (lane == leader) base = atomicAdd(count, __popcll(m2));
    base = __shfl(base, leader, 64);
    if (amb && two) list2[base + __popcll(m2 & below)] = make_int2((int)row, l2);
  }
  if (mf) {
    const int leader = __builtin_ctzll(mf);
    int base = 0;
    if (lane == leader) base = atomicAdd(count + 1, __popcll(mf));
    base = __shfl(base, leader, 64);
    if (amb && !two) listF[base + __popcll(mf & below)] = (int)row;
  }
}

// ------------------------------------------------------------------------------------
// DP <= 256: ring3's pipeline (64-point-wide workgroup tiles of 16x16x32 MFMAs, LDS-DMA
// centroid ring in the saddr form, early slot release) with two centroid images (hi, lo)
// per stage and two point fragment sets (hi, lo) per point tile; 3 MFMAs per k-step and
// point tile.  At D=128 a score costs 3 MFMAs (48 matrix cycles) against ~4.75 epilogue
// VALU, so the kernel is MFMA-bound where the bf16 ring3 is issue-bound.
// ------------------------------------------------------------------------------------
template <int DP, int P, int NST, int QT, int LISTED = 0>
__global__ __launch_bounds__(256, 2) void assign_x3_ring_kernel(
    const __bf16* __restrict__ Xh, const __bf16* __restrict__ Xl, int64_t N,
    const __bf16* __restrict__ Ch, const __bf16* __restrict__ Cl, const float* __restrict__ cnorm,
    int ntiles, const float* __restrict__ cstat, int32_t* __restrict__ labels,
    float* __restrict__ mind, int2* __restrict__ amb, int* __restrict__ ambF,
    int* __restrict__ amb_count, const int32_t* __restrict__ rowidx,
    const int* __restrict__ nrows, int64_t blk0) {
  constexpr int WAVES = 4;
  constexpr int BNL = 16 * QT;                 // centroids per stage
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 32;
  constexpr int TILE_B = BNL * DP * 2;         // one image (hi or lo)
  constexpr int NORM_B = BNL * 4;
  constexpr int STAGE_B = 2 * TILE_B + NORM_B;
  constexpr int PIECES = TILE_B / 1024;
  constexpr int PPW = PIECES / WAVES;
  static_assert(PIECES % WAVES == 0 && PPW >= 1, "stage split");
  constexpr int NCH = NORM_B / 16;
  constexpr int NPW = NCH / WAVES;
  static_assert(NCH % WAVES == 0 && NPW >= 1, "norm split");
  constexpr int VPS = 2 * PPW + 1;             // vmem instructions per wave per stage
  static_assert(QT * 4 <= 16, "4 tag bits");
  constexpr unsigned EMB = 15u;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE_B];

  // listed modes (after the one-product prefilter): point i is row rowidx[i], the count is
  // read on the device.  LISTED = 1: one point block per workgroup from block blk0 on, the
  // launch sized by the caller's estimate of the count (the previous step's); the
  // workgroups past the count leave before any load.  LISTED = 2: the overflow beyond such
  // a launch, a grid-stride loop on the resident workgroups (normally empty).  Sized by N
  // instead, the one-shot launch had ~35K empty workgroups at the headline shape (~0.3 ms);
  // the grid-stride loop over every block was slower (1.28 -> 1.44 ms,
  // profiles/headline_fp32_prefilter_kernel_stats_r05w.txt).
  if (LISTED) N = *nrows;
  for (int64_t blk = blk0 + blockIdx.x; blk * (WAVES * P * 16) < N; blk += gridDim.x) {
  if (LISTED == 2 && blk != blk0 + blockIdx.x) __syncthreads();  // the ring's slots are free
  // LISTED = 2: an opaque zero (asm volatile) rebuilds the lane constants per point block
  // instead of holding them through the loop (spills otherwise)
  unsigned oz = 0;
  if (LISTED == 2) asm volatile("v_mov_b32 %0, 0" : "=v"(oz));
  const int tid = (int)(threadIdx.x + oz);
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int64_t pbase = blk * (WAVES * P * 16) + (int64_t)w * (P * 16);

  bf16x8 bh[P][KS], bl[P][KS];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 16 + r;
    if (row >= N) row = N - 1;
    if (LISTED) row = rowidx[row];
    const __bf16* sh = Xh + row * DP + g * 8;
    const __bf16* sl = Xl + row * DP + g * 8;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      bh[p][kk] = *reinterpret_cast<const bf16x8*>(sh + kk * 32);
      bl[p][kk] = *reinterpret_cast<const bf16x8*>(sl + kk * 32);
    }
  }

  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int piece = w * PPW + i;
    const int L = piece * 64 + lane;
    const int row = L / CPR, cp = L % CPR;
    voff[i] = (unsigned)((row * DP + swz<DP>(row, cp) * 8) * 2);
  }
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto issue = [&](int t, int slot) __attribute__((always_inline)) {
    const __bf16* baseh = Ch + (int64_t)t * BNL * DP;
    const __bf16* basel = Cl + (int64_t)t * BNL * DP;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const unsigned dst = lds0 + slot * STAGE_B + (wu * PPW + i) * 1024;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff[i]), "s"(baseh)
                   : "memory", "m0");
    }
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const unsigned dst = lds0 + slot * STAGE_B + TILE_B + (wu * PPW + i) * 1024;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff[i]), "s"(basel)
                   : "memory", "m0");
    }
    const int nb = w * NPW;
    if (lane < NPW) {
      const float* src = cnorm + (int64_t)t * BNL + (nb + lane) * 4;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * STAGE_B + 2 * TILE_B + nb * 16),
          16, 0, 0);
    }
  };

#pragma unroll
  for (int t = 0; t < NST - 1; ++t) issue(t < ntiles ? t : ntiles - 1, t);

  asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
  __builtin_amdgcn_s_barrier();

  float B1[P], B2[P], B3[P];
  int T1[P], T2[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    B1[p] = B2[p] = B3[p] = INFINITY;
    T1[p] = T2[p] = 0;
  }

  unsigned aoff[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) aoff[kk] = lds0 + r * (DP * 2) + swz<DP>(r, kk * 4 + g) * 16;
  const unsigned noff = lds0 + 2 * TILE_B + 16 * g;

  auto stage = [&](int t, auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value;
    {
      const int tn = t + NST - 1;
      issue(tn < ntiles ? tn : ntiles - 1, (slot + NST - 1) % NST);
    }
    float m1[P], m2[P], m3[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m1[p] = m2[p] = m3[p] = INFINITY;
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      auto afrag = [&](int kk, auto img_c) __attribute__((always_inline)) {
        constexpr int img = decltype(img_c)::value;
        bf16x8 a;
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(a) : "v"(aoff[kk]), "i"(slot * STAGE_B + img * TILE_B + q * 16 * DP * 2));
        return a;
      };
      using H = std::integral_constant<int, 0>;
      using L = std::integral_constant<int, 1>;
      f32x4 n4;
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(n4) : "v"(noff), "i"(slot * STAGE_B + q * 16 * 4));
      bf16x8 ah0 = afrag(0, H{}), al0 = afrag(0, L{});
      bf16x8 ah1 = ah0, al1 = al0;
      if (KS > 1) {
        ah1 = afrag(KS > 1 ? 1 : 0, H{});
        al1 = afrag(KS > 1 ? 1 : 0, L{});
      }
      // two chains: xh.th from ||c||^2 (the large terms, KS MFMAs) and the cross terms from
      // 0 (2 KS MFMAs of ~2^-8 relative size), summed once: the large accumulator sees KS
      // roundings instead of 3 KS (the bound x3_eps)
      f32x4 acc[P], acx[P];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        bf16x8 ah2 = ah1, al2 = al1;
        if (kk + 2 < KS) {
          ah2 = afrag(kk + 2, H{});
          al2 = afrag(kk + 2, L{});
        }
        if (kk + 2 < KS) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
        else if (kk + 1 < KS) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (q == QT - 1 && kk == KS - 1) {
          // early slot release (as ring3): the stage's last fragments are in registers
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
          __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < P; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, bh[p][kk], kk == 0 ? n4 : acc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < P; ++p)
          acx[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, bl[p][kk], kk == 0 ? z4 : acx[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < P; ++p)
          acx[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al0, bh[p][kk], acx[p], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        ah0 = ah1;
        al0 = al1;
        ah1 = ah2;
        al1 = al2;
      }
      // top-3 of the phase's scores: new 3rd, new 2nd, new 1st (m1 <= m2 <= m3 kept)
#pragma unroll
      for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = __uint_as_float((__float_as_uint(acc[p][i] + acx[p][i]) & ~EMB) |
                                          (unsigned)(q * 4 + i));
          // asm: the builtins canonicalised the tagged v first (one more VALU per score);
          // v is never a signalling NaN (see assign_mfma_impl.h's top-2)
          float n1, n2, n3;
          asm("v_med3_f32 %0, %1, %2, %3" : "=v"(n3) : "v"(m2[p]), "v"(m3[p]), "v"(v));
          asm("v_med3_f32 %0, %1, %2, %3" : "=v"(n2) : "v"(m1[p]), "v"(m2[p]), "v"(v));
          asm("v_min_f32 %0, %1, %2" : "=v"(n1) : "v"(m1[p]), "v"(v));
          m3[p] = n3;
          m2[p] = n2;
          m1[p] = n1;
        }
      }
    }
    // stage triple into the running one (stage indices kept for the two smallest)
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bool up1 = m1[p] < B1[p];
      const float x = up1 ? B1[p] : m1[p];  // loser of the first place
      const int tx = up1 ? T1[p] : t;
      const bool s2 = m2[p] < B2[p];
      const float y = s2 ? m2[p] : B2[p];
      const int ty = s2 ? t : T2[p];
      B3[p] = __builtin_fminf(__builtin_fminf(B3[p], m3[p]),
                              __builtin_fminf(__builtin_fmaxf(B1[p], m2[p]), __builtin_fmaxf(B2[p], m1[p])));
      const bool xy = x < y;
      B2[p] = xy ? x : y;
      T2[p] = xy ? tx : ty;
      B1[p] = up1 ? m1[p] : B1[p];
      T1[p] = up1 ? t : T1[p];
    }
  };

  for (int t0 = 0; t0 < ntiles; t0 += NST) {
    stage(t0, std::integral_constant<int, 0>{});
    if constexpr (NST > 1) if (t0 + 1 < ntiles) stage(t0 + 1, std::integral_constant<int, 1>{});
    if constexpr (NST > 2) if (t0 + 2 < ntiles) stage(t0 + 2, std::integral_constant<int, 2 % NST>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

#pragma unroll
  for (int p = 0; p < P; ++p) {
    // ||xh||^2 and ||xl||^2 of the row (the per-row error bound), from the fragments still in
    // registers (computed here, not before the K loop: no registers held through it)
    float sh = 0.f, sl = 0.f;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float fh = (float)bh[p][kk][j], fl = (float)bl[p][kk][j];
        sh = fmaf(fh, fh, sh);
        sl = fmaf(fl, fl, sl);
      }
    sh += __shfl_xor(sh, 16, 64);
    sl += __shfl_xor(sl, 16, 64);
    sh += __shfl_xor(sh, 32, 64);
    sl += __shfl_xor(sl, 32, 64);
    const unsigned e1 = __float_as_uint(B1[p]) & EMB, e2 = __float_as_uint(B2[p]) & EMB;
    int l1 = T1[p] * BNL + (int)(e1 >> 2) * 16 + 4 * g + (int)(e1 & 3);
    int l2 = T2[p] * BNL + (int)(e2 >> 2) * 16 + 4 * g + (int)(e2 & 3);
    float v1 = __uint_as_float(__float_as_uint(B1[p]) & ~EMB);
    float v2 = __uint_as_float(__float_as_uint(B2[p]) & ~EMB);
    float v3 = __uint_as_float(__float_as_uint(B3[p]) & ~EMB);
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1)
      top3_merge(v1, l1, v2, l2, v3, __shfl_xor(v1, o, 64), __shfl_xor(l1, o, 64),
                 __shfl_xor(v2, o, 64), __shfl_xor(l2, o, 64), __shfl_xor(v3, o, 64));
    const int64_t lrow = pbase + p * 16 + r;
    const bool valid = g == 0 && lrow < N;
    const int64_t row = LISTED ? (int64_t)rowidx[lrow < N ? lrow : N - 1] : lrow;
    const float eps2 = 2.f * x3_eps(sqrtf(sh) * 1.0001f, sqrtf(sl) * 1.0001f, cstat, KS);
    if (mind) {  // + ||xh + xl||^2 turns the score into a distance (uniform branch)
      float sx = 0.f;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)bh[p][kk][j] + (float)bl[p][kk][j];
          sx = fmaf(f, f, sx);
        }
      sx += __shfl_xor(sx, 16, 64);
      sx += __shfl_xor(sx, 32, 64);
      if (valid) mind[row] = fmaxf(v1 + sx, 0.f);
    }
    if (valid) labels[row] = l1;
    x3_append(valid && !(v2 - v1 > eps2), v3 - v1 > eps2, row, l2, amb, ambF, amb_count);
  }
  if (LISTED != 2) break;  // one point block per workgroup
  }  // point blocks
}

// ------------------------------------------------------------------------------------
// wide D: top-3 / list pass over a chunk's raw d2 block G [M, K] (one wave per row)
// ------------------------------------------------------------------------------------
// The block comes from fcm_wide_dist_kernel: ONE accumulator per element from ||x||^2 +
// ||c||^2 through all 3 DP / 16 MFMAs (32x32x16), no tag.  The row's hi/lo norms are not at
// hand here, so the split term takes the worst case (||xh|| <= ||x||, ||xl|| <= 2^-8 ||x||).
__device__ __forceinline__ float x3_eps_wide(float xb, float xn, const float* cstat, int nmf) {
  const float cn = cstat[0];
  const float Hc = sqrtf(cstat[1]) * 1.0001f, Lc = sqrtf(cstat[2]) * 1.0001f;
  constexpr float R8 = 0.00392157f;
  const float hx = xb * 1.004f, lx = R8 * xb;
  const float Rc = R8 * Lc, Rx = R8 * lx;
  const float e_split = hx * Rc + lx * Lc + lx * Rc + Rx * Hc + Rx * Lc + Rx * Rc;
  const float s_all = hx * Hc + hx * Lc + lx * Hc;
  constexpr float U8 = 8.f * 1.1920929e-7f;
  const float e_acc = U8 * ((float)nmf * (xn + cn) + (float)(nmf + 1) * s_all);
  const float e_norm = 1.1920929e-7f * (xn + cn) * 2.f;
  return (e_split + e_acc + e_norm) * 1.001f + 1e-30f;
}

__global__ __launch_bounds__(256) void x3_rows_kernel(const float* __restrict__ G, int64_t M, int K,
                                                      int64_t row0, const float* __restrict__ xx,
                                                      const float* __restrict__ cstat, int nmf,
                                                      int32_t* __restrict__ labels,
                                                      int2* __restrict__ amb,
                                                      int* __restrict__ ambF,
                                                      int* __restrict__ amb_count) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t i0 = (int64_t)blockIdx.x * 4; i0 < M; i0 += nw) {
    const int64_t i = i0 + (threadIdx.x >> 6);
    const bool live = i < M;
    float v1 = INFINITY, v2 = INFINITY, v3 = INFINITY;
    int l1 = 0x7fffffff, l2 = 0x7fffffff;
    if (live) {
      const float* gr = G + i * (int64_t)K;
      for (int k = lane; k < K; k += 64) {
        const float v = gr[k];
        const bool a = v < v1, b = v < v2, c = v < v3;
        v3 = b ? v2 : (c ? v : v3);
        v2 = a ? v1 : (b ? v : v2);
        l2 = a ? l1 : (b ? k : l2);
        v1 = a ? v : v1;
        l1 = a ? k : l1;
      }
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1)
      top3_merge(v1, l1, v2, l2, v3, __shfl_xor(v1, o, 64), __shfl_xor(l1, o, 64),
                 __shfl_xor(v2, o, 64), __shfl_xor(l2, o, 64), __shfl_xor(v3, o, 64));
    const bool valid = live && lane == 0;
    float eps2 = 0.f;
    if (live) {
      const float xn = xx[i];
      eps2 = 2.f * x3_eps_wide(sqrtf(xn) * 1.0001f, xn, cstat, nmf);
    }
    if (valid) labels[row0 + i] = l1 < K ? l1 : 0;
    x3_append(valid && !(v2 - v1 > eps2), v3 - v1 > eps2, row0 + i, l2, amb, ambF, amb_count);
  }
}

// ------------------------------------------------------------------------------------
// exact re-check of the two-candidate rows (one wave per entry, grid-stride over the device
// count); the full re-scans run lloyd_simt.hip's tiled exact kernel over listF
// ------------------------------------------------------------------------------------
constexpr int X3_MAXD = 1024;

template <typename T>
__global__ __launch_bounds__(256) void x3_recheck_kernel(const T* __restrict__ X, int64_t ldx, int D,
                                                         const T* __restrict__ C,
                                                         int32_t* __restrict__ labels,
                                                         const int2* __restrict__ amb,
                                                         const int* __restrict__ amb_count) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = amb_count[0];
  for (int64_t e = (int64_t)blockIdx.x * 4 + w; e < n; e += (int64_t)gridDim.x * 4) {
    const int2 a = amb[e];
    const int64_t row = a.x;
    const T* x = X + row * ldx;
    const int l1 = labels[row], l2 = a.y;
    const T* c1 = C + (int64_t)l1 * D;
    const T* c2 = C + (int64_t)l2 * D;
    T s1 = 0, s2 = 0;
    for (int d = lane; d < D; d += 64) {
      const T xv = x[d];
      const T e1 = xv - c1[d], e2 = xv - c2[d];
      s1 = fma(e1, e1, s1);
      s2 = fma(e2, e2, s2);
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0 && (s2 < s1 || (s2 == s1 && l2 < l1))) labels[row] = l2;
  }
}

// the prefilter's flagged rows (label sign bit set) -> compact list pre (count *n): RPB rows
// per workgroup, one ballot per 64 rows and ONE atomic per workgroup (the labels of the
// listed rows are rewritten by the listed x3 pass)
constexpr int X3_COMPACT_RPB = 4096;
__global__ __launch_bounds__(256) void x3_compact_kernel(const int32_t* __restrict__ labels,
                                                         int64_t N, int32_t* __restrict__ list,
                                                         int* __restrict__ n) {
  constexpr int RPW = X3_COMPACT_RPB / 4, J = RPW / 64;
  __shared__ int s_cnt[4];
  __shared__ int s_base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * X3_COMPACT_RPB + (int64_t)w * RPW;
  unsigned long long m[J];
  int c = 0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int64_t row = r0 + j * 64 + lane;
    m[j] = __ballot(row < N && labels[row] < 0);
    c += __popcll(m[j]);
  }
  if (lane == 0) s_cnt[w] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    s_base = t ? atomicAdd(n, t) : 0;
  }
  __syncthreads();
  int base = s_base;
  for (int v = 0; v < w; ++v) base += s_cnt[v];
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if ((m[j] >> lane) & 1ull) list[base + __popcll(m[j] & below)] = (int)(r0 + j * 64 + lane);
    base += __popcll(m[j]);
  }
}

template <int DP, int P, int NST, int QT>
int launch_x3(const void* Xh, const void* Xl, int64_t N, const void* Ch, const void* Cl,
              const float* cnorm, int Kp, const float* cstat, int32_t* labels,
              float* mind, int2* amb, int* ambF, int* amb_count, const int32_t* rowidx,
              const int* nrows, int64_t est_rows, hipStream_t s) {
  constexpr int BNL = 16 * QT;
  if (Kp % BNL != 0) return (int)hipErrorInvalidValue;
  const int64_t per = 4 * P * 16;
  const int64_t blocks = (N + per - 1) / per;
  if (nrows) {
    // est_rows (> 0): the caller's estimate of the listed count; the one-shot launch covers
    // it, a small grid-stride launch covers anything beyond (normally nothing to do)
    int64_t b1 = est_rows > 0 ? (est_rows + per - 1) / per : blocks;
    if (b1 > blocks) b1 = blocks;
    hipLaunchKernelGGL((assign_x3_ring_kernel<DP, P, NST, QT, 1>), dim3((unsigned)b1),
                       dim3(256), 0, s, (const __bf16*)Xh, (const __bf16*)Xl, N, (const __bf16*)Ch,
                       (const __bf16*)Cl, cnorm, Kp / BNL, cstat, labels, mind, amb, ambF,
                       amb_count, rowidx, nrows, (int64_t)0);
    if (b1 < blocks) {
      TDC_CHECK_LAUNCH();
      static const int res = resident_blocks(assign_x3_ring_kernel<DP, P, NST, QT, 2>, 256);
      const int64_t b2 = blocks - b1 < res ? blocks - b1 : res;
      hipLaunchKernelGGL((assign_x3_ring_kernel<DP, P, NST, QT, 2>), dim3((unsigned)b2),
                         dim3(256), 0, s, (const __bf16*)Xh, (const __bf16*)Xl, N,
                         (const __bf16*)Ch, (const __bf16*)Cl, cnorm, Kp / BNL, cstat, labels,
                         mind, amb, ambF, amb_count, rowidx, nrows, b1);
    }
  } else {
    hipLaunchKernelGGL((assign_x3_ring_kernel<DP, P, NST, QT>), dim3((unsigned)blocks),
                       dim3(256), 0, s, (const __bf16*)Xh, (const __bf16*)Xl, N, (const __bf16*)Ch,
                       (const __bf16*)Cl, cnorm, Kp / BNL, cstat, labels, mind, amb, ambF,
                       amb_count, nullptr, nullptr, (int64_t)0);
  }
  TDC_CHECK_LAUNCH();
  return 0;
}

}  // namespace
}  // namespace tdc

using namespace tdc;

int tdc_x3_split(int src_dtype, const void* src, int64_t rows, int64_t valid, int d, int64_t ld,
                 int DP, int neg2, void* hi, void* lo, float* norm, float* nhl, hipStream_t s,
                 const void* shift) {
  if (rows <= 0) return 0;
  if (d > DP || DP % 32 != 0) return (int)hipErrorInvalidValue;
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  if (src_dtype == TDC_F32)
    hipLaunchKernelGGL(x3_split_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const float*)src, rows, valid, d, ld, DP, neg2, (__bf16*)hi, (__bf16*)lo, norm,
                       (float2*)nhl, (const float*)shift);
  else if (src_dtype == TDC_F64)
    hipLaunchKernelGGL(x3_split_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const double*)src, rows, valid, d, ld, DP, neg2, (__bf16*)hi, (__bf16*)lo, norm,
                       (float2*)nhl, (const double*)shift);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_x3_prep(const float* cnorm, const float* nhl, int K, float* cstat, int* amb_count,
                hipStream_t s, int nzero) {
  hipLaunchKernelGGL(x3_prep_kernel, dim3(1), dim3(1024), 0, s, cnorm, (const float2*)nhl, K,
                     cstat, amb_count, nzero);
  TDC_CHECK_LAUNCH();
  return 0;
}

// amb: int32 [3 cap] = list2 (int2 [cap]) | listF (int32 [cap]); amb_count int32 [2]
int tdc_assign_x3(const void* Xh, const void* Xl, int64_t N, int DP, const void* Ch, const void* Cl,
                  const float* cnorm, int Kp, const float* cstat, int32_t* labels,
                  float* mind, int32_t* amb, int64_t cap, int* amb_count, hipStream_t s,
                  const int32_t* rowidx, const int* nrows, int64_t est_rows) {
  if (N <= 0) return 0;
  if (N >= ((int64_t)1 << 31) || cap < N) return (int)hipErrorInvalidValue;
  if ((rowidx == nullptr) != (nrows == nullptr)) return (int)hipErrorInvalidValue;
  int2* l2 = reinterpret_cast<int2*>(amb);
  int* lf = amb + 2 * cap;
  switch (DP) {
    // LDS per stage: 2 images x 64 centroids x DP x 2 B; two workgroups (8 waves) per CU
    case 32: return launch_x3<32, 6, 3, 4>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cstat, labels, mind, l2, lf, amb_count, rowidx, nrows, est_rows, s);
    case 64: return launch_x3<64, 6, 3, 4>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cstat, labels, mind, l2, lf, amb_count, rowidx, nrows, est_rows, s);
    case 128: return launch_x3<128, 4, 2, 4>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cstat, labels, mind, l2, lf, amb_count, rowidx, nrows, est_rows, s);
    case 256: return launch_x3<256, 2, 2, 2>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cstat, labels, mind, l2, lf, amb_count, rowidx, nrows, est_rows, s);
  }
  return (int)hipErrorInvalidValue;
}

// One-product prefilter (assign_mfma_impl.h x1_eps): bf16 ring3 top-2 over (xh, th) with the
// exact labels of the certified rows, the others flagged and then listed in pre (count in
// *npre) by x3_compact_kernel for tdc_assign_x3's listed mode.  DP 64 / 128 / 256.
int tdc_x3_prefilter(const void* Xh, int64_t N, int DP, const void* Ch, const float* cnorm, int Kp,
                     const float* cstat, int32_t* labels, int32_t* pre, int* npre, hipStream_t s,
                     const float* xnhl) {
  const float2* xn2 = reinterpret_cast<const float2*>(xnhl);
  if (N <= 0) return 0;
  if (Kp % 64 != 0 || N >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  const __bf16* x = (const __bf16*)Xh;
  const __bf16* c = (const __bf16*)Ch;
  const dim3 grid((unsigned)((N + 255) / 256));
  if (DP == 64)  // P = 4 (P = 8 spills with the top-2 registers)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<64, 4, 3, 4, 4, true>), grid, dim3(256), 0,
                       s, x, N, (int64_t)DP, c, cnorm, Kp / 64, labels, nullptr, nullptr, nullptr,
                       cstat, xn2);
  else if (DP == 128)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 4, 3, 4, 4, true>), grid, dim3(256), 0,
                       s, x, N, (int64_t)DP, c, cnorm, Kp / 64, labels, nullptr, nullptr, nullptr,
                       cstat, xn2);
  else if (DP == 256)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<256, 4, 2, 4, 4, true>), grid, dim3(256), 0,
                       s, x, N, (int64_t)DP, c, cnorm, Kp / 64, labels, nullptr, nullptr, nullptr,
                       cstat, xn2);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  int64_t blocks = (N + X3_COMPACT_RPB - 1) / X3_COMPACT_RPB;
  hipLaunchKernelGGL(x3_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, s, labels, N, pre, npre);
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_x3_rows(const float* G, int64_t M, int K, int64_t row0, const float* xx, const float* cstat,
                int DP, int32_t* labels, int32_t* amb, int64_t cap, int* amb_count, hipStream_t s) {
  if (M <= 0) return 0;
  if (row0 + M >= ((int64_t)1 << 31) || cap < row0 + M) return (int)hipErrorInvalidValue;
  int64_t blocks = (M + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(x3_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, G, M, K, row0, xx,
                     cstat, 3 * DP / 16, labels, reinterpret_cast<int2*>(amb), amb + 2 * cap,
                     amb_count);
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_x3_recheck(int dtype, const void* X, int64_t ldx, int D, const void* C, int K,
                   int32_t* labels, const int32_t* amb, int64_t cap, const int* amb_count,
                   int num_cus, hipStream_t s) {
  if (D > X3_MAXD || D <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)(num_cus * 4));
  const int2* l2 = reinterpret_cast<const int2*>(amb);
  if (dtype == TDC_F32)
    hipLaunchKernelGGL(x3_recheck_kernel<float>, grid, dim3(256), 0, s, (const float*)X, ldx, D,
                       (const float*)C, labels, l2, amb_count);
  else if (dtype == TDC_F64)
    hipLaunchKernelGGL(x3_recheck_kernel<double>, grid, dim3(256), 0, s, (const double*)X, ldx, D,
                       (const double*)C, labels, l2, amb_count);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  // the rows with a third candidate inside the bound: exact re-scan over all K (tiled SIMT
  // difference form over the listed rows, their count read on the device)
  return tdc_assign_exact(dtype, X, cap, ldx, D, C, K, labels, nullptr, num_cus, s, amb + 2 * cap,
                          amb_count + 1);
}
