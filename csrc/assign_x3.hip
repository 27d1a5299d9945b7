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
// the indices of the two smallest.  For every (row, centroid) pair
//
//     |s_computed - s_exact| <= eps = tau(D) * (max_k ||c_k||^2 + 2 ||x|| max_k ||c_k||)
//
// tau(D) = (4 D + 64) 2^-23 + 2^-16 bounds, for ANY order of the fp32 additions inside and
// between the MFMAs (n terms: |error| <= (n - 1) 2^-23 sum |terms|, u taken as 2^-23 so a
// truncating adder is covered too): the dropped split terms (3 2^-18 sum |x_i c_i| per
// product, x2 for the -2c scaling), the 3 D + 1 accumulations, the fp32 ||c||^2 and the
// 4-bit index tag.  So
//   * gap = s2 - s1 > 2 eps: the winner is certain (the exact argmin);
//   * else, if s3 - s1 > 2 eps: the exact winner is one of the two smallest -- recomputed
//     in the data's own precision (fp32 or fp64 difference form), ties to the lower index;
//   * else (a third centroid within the bound): the row is re-assigned over all K exactly.
// The ambiguous rows go to a compacted list (one ballot + one atomic per wave and point
// tile); on Gaussian-blob data at the headline shape about 1 % need the two-candidate check
// and ~1e-4 the full scan.  Labels therefore equal the exact argmin of the input dtype
// (fp32, or fp64 for fp64 data) up to that dtype's own rounding of the distances.
//
// Wide D (256 < D <= 1024): the point fragments no longer fit the registers, so a row chunk
// runs fcm_mfma.hip's bf16x3 distance GEMM into an [M, K] block (raw d2, no zero floor) and
// x3_rows_kernel does the top-3 / list pass over it (bound tau * (||x|| + max ||c||)^2, the
// block includes ||x||^2).
#include <math.h>

#include "assign_mfma_impl.h"
#include "kernels.h"

namespace tdc {
namespace {

// ------------------------------------------------------------------------------------
// operand prep: rows of T [rows, ld] (d valid columns) -> bf16 hi/lo [rows, DP] (of -2v when
// neg2) + norm [rows] = ||v||^2 (pad centroid rows: BIG, so they never win)
// ------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void x3_split_kernel(const T* __restrict__ src, int64_t rows,
                                                       int64_t valid, int d, int64_t ld, int DP,
                                                       int neg2, __bf16* __restrict__ hi,
                                                       __bf16* __restrict__ lo,
                                                       float* __restrict__ norm) {
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * 4) {
    T s = 0;
    for (int c = lane; c < DP; c += 64) {
      const T v = (row < valid && c < d) ? src[row * ld + c] : (T)0;
      s += v * v;
      const T t = neg2 ? (T)-2 * v : v;
      const __bf16 th = (__bf16)(float)t;
      hi[row * DP + c] = th;
      lo[row * DP + c] = (__bf16)(float)(t - (T)(float)th);
    }
    s = wave_sum(s);
    if (lane == 0 && norm) norm[row] = (neg2 && row >= valid) ? BIG : (float)s;
  }
}

// cmax2[0] = max_k cnorm[k] over the K valid rows; amb_count[0] = 0 (the list of the next
// assignment).  One block.
__global__ __launch_bounds__(1024) void x3_prep_kernel(const float* __restrict__ cnorm, int K,
                                                       float* __restrict__ cmax2,
                                                       int* __restrict__ amb_count) {
  __shared__ float red[16];
  float m = 0.f;
  for (int k = threadIdx.x; k < K; k += 1024) m = fmaxf(m, cnorm[k]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x < 64) {
    float v = threadIdx.x < 16 ? red[threadIdx.x] : 0.f;
    v = wave_max(v);
    if (threadIdx.x == 0) {
      cmax2[0] = v;
      amb_count[0] = 0;
    }
  }
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

// one list entry per ambiguous row among the lanes with `amb` set: {row, runner-up (two-
// candidate check) or -1 (full scan)}; one ballot + at most one atomic per wave
__device__ __forceinline__ void x3_append(bool amb, bool two, int64_t row, int l2,
                                          int2* __restrict__ list, int* __restrict__ count) {
  const unsigned long long mask = __ballot(amb);
  if (mask == 0ull) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(mask);
  int base = 0;
  if (lane == leader) base = atomicAdd(count, __popcll(mask));
  base = __shfl(base, leader, 64);
  if (amb) {
    const int idx = base + __popcll(mask & ((1ull << lane) - 1ull));
    list[idx] = make_int2((int)row, two ? l2 : -1);
  }
}

// ------------------------------------------------------------------------------------
// DP <= 256: ring3's pipeline (64-point-wide workgroup tiles of 16x16x32 MFMAs, LDS-DMA
// centroid ring in the saddr form, early slot release) with two centroid images (hi, lo)
// per stage and two point fragment sets (hi, lo) per point tile; 3 MFMAs per k-step and
// point tile.  At D=128 a score costs 3 MFMAs (48 matrix cycles) against ~4.75 epilogue
// VALU, so the kernel is MFMA-bound where the bf16 ring3 is issue-bound.
// ------------------------------------------------------------------------------------
template <int DP, int P, int NST, int QT>
__global__ __launch_bounds__(256, 2) void assign_x3_ring_kernel(
    const __bf16* __restrict__ Xh, const __bf16* __restrict__ Xl, int64_t N,
    const __bf16* __restrict__ Ch, const __bf16* __restrict__ Cl, const float* __restrict__ cnorm,
    int ntiles, const float* __restrict__ cmax2p, float tau, int32_t* __restrict__ labels,
    float* __restrict__ mind, int2* __restrict__ amb, int* __restrict__ amb_count) {
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

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int64_t pbase = (int64_t)blockIdx.x * (WAVES * P * 16) + (int64_t)w * (P * 16);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  bf16x8 bh[P][KS], bl[P][KS];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 16 + r;
    if (row >= N) row = N - 1;
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

  // ||x||^2 of the split row (the bound's ||x||; +||x||^2 turns a score into a distance)
  float xs[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    float s = 0.f;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = (float)bh[p][kk][j] + (float)bl[p][kk][j];
        s = fmaf(f, f, s);
      }
    s += __shfl_xor(s, 16, 64);
    xs[p] = s + __shfl_xor(s, 32, 64);
  }

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
      f32x4 acc[P];
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
#pragma unroll
        for (int p = 0; p < P; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, bh[p][kk], kk == 0 ? n4 : acc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < P; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah0, bl[p][kk], acc[p], 0, 0, 0);
#pragma unroll
        for (int p = 0; p < P; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al0, bh[p][kk], acc[p], 0, 0, 0);
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
          const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 4 + i));
          m3[p] = __builtin_amdgcn_fmed3f(m2[p], m3[p], v);
          m2[p] = __builtin_amdgcn_fmed3f(m1[p], m2[p], v);
          m1[p] = __builtin_fminf(m1[p], v);
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

  const float cmax2 = cmax2p[0] * (1.f + 1.f / 4096.f);
  const float cmax = sqrtf(cmax2);
#pragma unroll
  for (int p = 0; p < P; ++p) {
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
    const int64_t row = pbase + p * 16 + r;
    const bool valid = g == 0 && row < N;
    const float xb = sqrtf(xs[p]) * (1.f + 1.f / 1024.f);
    const float eps2 = 2.f * tau * (cmax2 + 2.f * xb * cmax) + 1e-30f;
    if (valid) {
      labels[row] = l1;
      if (mind) mind[row] = fmaxf(v1 + xs[p], 0.f);
    }
    x3_append(valid && !(v2 - v1 > eps2), v3 - v1 > eps2, row, l2, amb, amb_count);
  }
}

// ------------------------------------------------------------------------------------
// wide D: top-3 / list pass over a chunk's raw d2 block G [M, K] (one wave per row)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void x3_rows_kernel(const float* __restrict__ G, int64_t M, int K,
                                                      int64_t row0, const float* __restrict__ xx,
                                                      const float* __restrict__ cmax2p, float tau,
                                                      int32_t* __restrict__ labels,
                                                      int2* __restrict__ amb,
                                                      int* __restrict__ amb_count) {
  const int lane = threadIdx.x & 63;
  const float cmax = sqrtf(cmax2p[0] * (1.f + 1.f / 4096.f));
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
      const float xb = sqrtf(xx[i]) * (1.f + 1.f / 1024.f);
      eps2 = 2.f * tau * (xb + cmax) * (xb + cmax) + 1e-30f;
    }
    if (valid) labels[row0 + i] = l1 < K ? l1 : 0;
    x3_append(valid && !(v2 - v1 > eps2), v3 - v1 > eps2, row0 + i, l2, amb, amb_count);
  }
}

// ------------------------------------------------------------------------------------
// exact re-check of the listed rows (one wave per entry, grid-stride over the device count)
// ------------------------------------------------------------------------------------
constexpr int X3_MAXD = 1024;

template <typename T>
__global__ __launch_bounds__(256) void x3_recheck_kernel(const T* __restrict__ X, int64_t ldx, int D,
                                                         const T* __restrict__ C, int K,
                                                         int32_t* __restrict__ labels,
                                                         const int2* __restrict__ amb,
                                                         const int* __restrict__ amb_count) {
  __shared__ T s_x[4][X3_MAXD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = amb_count[0];
  for (int64_t e = (int64_t)blockIdx.x * 4 + w; e < n; e += (int64_t)gridDim.x * 4) {
    const int2 a = amb[e];
    const int64_t row = a.x;
    const T* x = X + row * ldx;
    const int l1 = labels[row];
    if (a.y >= 0) {  // the exact winner is one of the two smallest scores
      const int l2 = a.y;
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
      continue;
    }
    // full scan: row in LDS (wave-private), lanes over centroids
    for (int d = lane; d < D; d += 64) s_x[w][d] = x[d];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    T best = (T)INFINITY;
    int bk = K;
    for (int k = lane; k < K; k += 64) {
      const T* c = C + (int64_t)k * D;
      T s = 0;
      for (int d = 0; d < D; ++d) {
        const T ev = s_x[w][d] - c[d];
        s = fma(ev, ev, s);
      }
      if (s < best) {
        best = s;
        bk = k;
      }
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const T ob = __shfl_xor(best, o, 64);
      const int ok = __shfl_xor(bk, o, 64);
      const bool take = ob < best || (ob == best && ok < bk);
      best = take ? ob : best;
      bk = take ? ok : bk;
    }
    if (lane == 0 && bk < K) labels[row] = bk;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // s_x reads done before the next entry overwrites it
  }
}

template <int DP, int P, int NST, int QT>
int launch_x3(const void* Xh, const void* Xl, int64_t N, const void* Ch, const void* Cl,
              const float* cnorm, int Kp, const float* cmax2, float tau, int32_t* labels,
              float* mind, int2* amb, int* amb_count, hipStream_t s) {
  constexpr int BNL = 16 * QT;
  if (Kp % BNL != 0) return (int)hipErrorInvalidValue;
  const int64_t per = 4 * P * 16;
  hipLaunchKernelGGL((assign_x3_ring_kernel<DP, P, NST, QT>), dim3((unsigned)((N + per - 1) / per)),
                     dim3(256), 0, s, (const __bf16*)Xh, (const __bf16*)Xl, N, (const __bf16*)Ch,
                     (const __bf16*)Cl, cnorm, Kp / BNL, cmax2, tau, labels, mind, amb, amb_count);
  TDC_CHECK_LAUNCH();
  return 0;
}

}  // namespace
}  // namespace tdc

using namespace tdc;

float tdc_x3_tau(int DP) {
  return (float)((4.0 * DP + 64.0) * ldexp(1.0, -23) + ldexp(1.0, -16));
}

int tdc_x3_split(int src_dtype, const void* src, int64_t rows, int64_t valid, int d, int64_t ld,
                 int DP, int neg2, void* hi, void* lo, float* norm, hipStream_t s) {
  if (rows <= 0) return 0;
  if (d > DP || DP % 32 != 0) return (int)hipErrorInvalidValue;
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 16384) blocks = 16384;
  if (src_dtype == TDC_F32)
    hipLaunchKernelGGL(x3_split_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const float*)src, rows, valid, d, ld, DP, neg2, (__bf16*)hi, (__bf16*)lo, norm);
  else if (src_dtype == TDC_F64)
    hipLaunchKernelGGL(x3_split_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const double*)src, rows, valid, d, ld, DP, neg2, (__bf16*)hi, (__bf16*)lo, norm);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_x3_prep(const float* cnorm, int K, float* cmax2, int* amb_count, hipStream_t s) {
  hipLaunchKernelGGL(x3_prep_kernel, dim3(1), dim3(1024), 0, s, cnorm, K, cmax2, amb_count);
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_assign_x3(const void* Xh, const void* Xl, int64_t N, int DP, const void* Ch, const void* Cl,
                  const float* cnorm, int Kp, const float* cmax2, float tau, int32_t* labels,
                  float* mind, int2* amb, int* amb_count, hipStream_t s) {
  if (N <= 0) return 0;
  if (N >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  switch (DP) {
    // LDS per stage: 2 images x 64 centroids x DP x 2 B; two workgroups (8 waves) per CU
    case 32: return launch_x3<32, 8, 3, 4>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cmax2, tau, labels, mind, amb, amb_count, s);
    case 64: return launch_x3<64, 6, 3, 4>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cmax2, tau, labels, mind, amb, amb_count, s);
    case 128: return launch_x3<128, 4, 2, 4>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cmax2, tau, labels, mind, amb, amb_count, s);
    case 256: return launch_x3<256, 2, 2, 2>(Xh, Xl, N, Ch, Cl, cnorm, Kp, cmax2, tau, labels, mind, amb, amb_count, s);
  }
  return (int)hipErrorInvalidValue;
}

int tdc_x3_rows(const float* G, int64_t M, int K, int64_t row0, const float* xx, const float* cmax2,
                float tau, int32_t* labels, int2* amb, int* amb_count, hipStream_t s) {
  if (M <= 0) return 0;
  if (row0 + M >= ((int64_t)1 << 31)) return (int)hipErrorInvalidValue;
  int64_t blocks = (M + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(x3_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, G, M, K, row0, xx,
                     cmax2, tau, labels, amb, amb_count);
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_x3_recheck(int dtype, const void* X, int64_t ldx, int D, const void* C, int K,
                   int32_t* labels, const int2* amb, const int* amb_count, int num_cus,
                   hipStream_t s) {
  if (D > X3_MAXD || D <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)(num_cus * 4));
  if (dtype == TDC_F32)
    hipLaunchKernelGGL(x3_recheck_kernel<float>, grid, dim3(256), 0, s, (const float*)X, ldx, D,
                       (const float*)C, K, labels, amb, amb_count);
  else if (dtype == TDC_F64)
    hipLaunchKernelGGL(x3_recheck_kernel<double>, grid, dim3(256), 0, s, (const double*)X, ldx, D,
                       (const double*)C, K, labels, amb, amb_count);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  return 0;
}
