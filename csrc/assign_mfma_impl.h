// Implementation of the bf16 MFMA distance + argmin kernel (see assign_mfma.hip for the
// design notes).  Shared by the library build and the ablation tool.
#pragma once
#include <type_traits>

#include "tdc_common.h"

namespace tdc {

constexpr int BN = 64;           // centroids per LDS stage = 2 MFMA row tiles of 32
constexpr float BIG = 3.0e38f;   // pad-centroid norm (finite so bit tricks stay NaN-free)

template <int DP>
__device__ __forceinline__ int swz(int r, int c) {
  constexpr int CPR = DP / 8;              // 16-byte chunks per centroid row
  constexpr int G = CPR < 16 ? CPR : 16;   // chunks per 256-byte LDS bank row
  constexpr int RPB = 16 / G;              // rows sharing a bank row
  return c ^ ((r / RPB) & (G - 1));
}

// The two superseded variants ("v1" register-staged, "ring" LDS-DMA without counted
// waits) live in tools/assign_mfma_legacy.h for the ablation harnesses.

// ------------------------------------------------------------------------------------
// Variant 3 ("ring2"): the "ring" variant (tools/assign_mfma_legacy.h) with its two stalls
// removed.
//  * the compiler cannot prove that a plain LDS read does not alias an in-flight
//    LDS-DMA, so every phase of "ring" started with s_waitcnt vmcnt(0): each stage
//    waited for the refill it had just issued (NST-1 stages ahead -> 0 ahead).  Here the
//    A fragments are read with inline-asm ds_read_b128 (explicit, counted lgkmcnt);
//  * the centroid norms ride in the ring with their tile (one extra 16-B-per-lane DMA of
//    NPW lanes per wave, so every wave issues the same count), instead of global loads
//    that also forced a vmcnt(0) at their use.
// A fragments are prefetched two k-steps ahead.
// ------------------------------------------------------------------------------------
// ABL (timing ablations only): 1 = no refill, 2 = no barrier, 4 = no epilogue,
// 8 = let the scheduler move work across the MFMA steps (valid results)
template <int DP, int P, int NST, int WAVES, int QT, int ABL = 0>
__global__ __launch_bounds__(WAVES * 64, (WAVES % 4 == 0 ? (WAVES / 4 > 1 ? WAVES / 4 : 3) : 2))
void assign_mfma_bf16_ring2_kernel(const __bf16* __restrict__ X, int64_t N, int64_t ldx,
                                   const __bf16* __restrict__ Cm2, const float* __restrict__ cnorm,
                                   int ntiles, int32_t* __restrict__ labels,
                                   float* __restrict__ mind) {
  constexpr int BNL = 32 * QT;                     // centroids per stage
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 16;
  constexpr int HALF = DP / 2;
  constexpr int TILE_B = BNL * DP * 2;
  constexpr int NORM_B = BNL * 4;
  constexpr int STAGE_B = TILE_B + NORM_B;
  constexpr int PIECES = TILE_B / 1024;
  constexpr int PPW = PIECES / WAVES;
  constexpr int NCH = NORM_B / 16;                 // 16-B norm chunks per stage
  constexpr int NPW = NCH / WAVES;                 // ... per wave
  constexpr int VPS = PPW + 1;                     // vmem instructions per wave per stage
  static_assert(PIECES % WAVES == 0 && NCH % WAVES == 0 && NPW >= 1, "stage split");
  constexpr unsigned EMB = QT * 16 <= 32 ? 31u : 63u;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE_B];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * (WAVES * P * 32) + (int64_t)w * (P * 32);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  bf16x8 bq[P][KS];
  float xn[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 32 + r;
    if (row >= N) row = N - 1;
    const bf16x8* src = reinterpret_cast<const bf16x8*>(X + row * ldx + h * HALF);
    float s = 0.f;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      bq[p][kk] = src[kk];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = (float)bq[p][kk][j];
        s = fmaf(f, f, s);
      }
    }
    xn[p] = s + __shfl_xor(s, 32, 64);
  }

  auto issue = [&](int t, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = w * PPW + i;
      const int L = piece * 64 + lane;
      const int row = L / CPR, cp = L % CPR;
      const int csrc = swz<DP>(row, cp);
      const __bf16* src = Cm2 + ((int64_t)t * BNL + row) * DP + csrc * 8;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * STAGE_B + piece * 1024), 16, 0, 0);
    }
    if (lane < NPW) {
      const float* src = cnorm + (int64_t)t * BNL + (w * NPW + lane) * 4;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * STAGE_B + TILE_B + w * NPW * 16),
          16, 0, 0);
    }
  };

#pragma unroll
  for (int t = 0; t < NST - 1; ++t) issue(t < ntiles ? t : ntiles - 1, t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
  __builtin_amdgcn_s_barrier();

  float best[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = INFINITY;
    bt[p] = 0;
  }

  // LDS read addresses: lane part precomputed once; slot / phase / norm offsets are
  // immediates (the ring loop is unrolled by NST so the slot is a compile-time constant)
  unsigned aoff[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) aoff[kk] = lds0 + r * (DP * 2) + swz<DP>(r, h * (CPR / 2) + kk) * 16;
  const unsigned noff = lds0 + TILE_B + 16 * h;

  auto stage = [&](int t, auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value;
    if constexpr (!(ABL & 1)) {
      const int tn = t + NST - 1;
      issue(tn < ntiles ? tn : ntiles - 1, (slot + NST - 1) % NST);
    }
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      auto afrag = [&](int kk) __attribute__((always_inline)) {
        bf16x8 a;
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(a) : "v"(aoff[kk]), "i"(slot * STAGE_B + q * 32 * DP * 2));
        return a;
      };
      f32x4 n4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(n4[j]) : "v"(noff), "i"(slot * STAGE_B + (q * 32 + 8 * j) * 4));
      bf16x8 a0 = afrag(0);
      bf16x8 a1 = afrag(KS > 1 ? 1 : 0);
      f32x16 acc[P];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        bf16x8 a2 = a1;
        if (kk + 2 < KS) a2 = afrag(kk + 2);
        if (kk + 2 < KS) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        else if (kk + 1 < KS) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (kk == 0) {
#pragma unroll
          for (int p = 0; p < P; ++p) {
            f32x16 init;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              init[4 * j + 0] = n4[j][0];
              init[4 * j + 1] = n4[j][1];
              init[4 * j + 2] = n4[j][2];
              init[4 * j + 3] = n4[j][3];
            }
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[p][0], init, 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int p = 0; p < P; ++p)
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[p][kk], acc[p], 0, 0, 0);
        }
        if constexpr (!(ABL & 8)) __builtin_amdgcn_sched_barrier(0);
        a0 = a1;
        a1 = a2;
      }
      if constexpr (ABL & 4) {
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
          for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(acc[p][i]));
      } else {
#pragma unroll
        for (int p = 0; p < P; ++p) {
          float m = INFINITY;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 16 + i));
            m = __builtin_fminf(m, v);
          }
          const bool up = m < best[p];
          best[p] = up ? m : best[p];
          bt[p] = up ? t : bt[p];
        }
      }
    }
    if constexpr (ABL & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");  // stage t+1 landed
    if constexpr (!(ABL & 2)) __builtin_amdgcn_s_barrier();  // ... for every wave's pieces
  };

  for (int t0 = 0; t0 < ntiles; t0 += NST) {
    stage(t0, std::integral_constant<int, 0>{});
    if constexpr (NST > 1) if (t0 + 1 < ntiles) stage(t0 + 1, std::integral_constant<int, 1>{});
    if constexpr (NST > 2) if (t0 + 2 < ntiles) stage(t0 + 2, std::integral_constant<int, 2 % NST>{});
    if constexpr (NST > 3) if (t0 + 3 < ntiles) stage(t0 + 3, std::integral_constant<int, 3 % NST>{});
    if constexpr (NST > 4) if (t0 + 4 < ntiles) stage(t0 + 4, std::integral_constant<int, 4 % NST>{});
    if constexpr (NST > 5) if (t0 + 5 < ntiles) stage(t0 + 5, std::integral_constant<int, 5 % NST>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

#pragma unroll
  for (int p = 0; p < P; ++p) {
    const float ob = __shfl_xor(best[p], 32, 64);
    const int obt = __shfl_xor(bt[p], 32, 64);
    const unsigned e0 = __float_as_uint(best[p]) & EMB, e1 = __float_as_uint(ob) & EMB;
    const int l0 = bt[p] * BNL + (int)(e0 >> 4) * 32 + (int)(e0 & 3) + 8 * (int)((e0 & 15) >> 2) + 4 * h;
    const int l1 = obt * BNL + (int)(e1 >> 4) * 32 + (int)(e1 & 3) + 8 * (int)((e1 & 15) >> 2) + 4 * (1 - h);
    const float v0 = __uint_as_float(__float_as_uint(best[p]) & ~EMB);
    const float v1 = __uint_as_float(__float_as_uint(ob) & ~EMB);
    const bool other = (v1 < v0) || (v1 == v0 && l1 < l0);
    const int64_t row = pbase + p * 32 + r;
    if (h == 0 && row < N) {
      labels[row] = other ? l1 : l0;
      if (mind) mind[row] = fmaxf((other ? v1 : v0) + xn[p], 0.f);
    }
  }
}


// ------------------------------------------------------------------------------------
// Variant 4 ("ring3"): ring2's pipeline on v_mfma_f32_16x16x32_bf16 instead of 32x32x16.
// Same FLOP per cycle and the same A-fragment LDS traffic per FLOP (each A fragment is
// shared by P=4 point tiles of 16), but MI355X holds a higher clock under the 16x16
// shape on random data (MI355X_MICROARCH.md "DVFS give-back" item 7: ~1.12-1.15x FLOP/s
// at equal cycles per FLOP).  C layout: lane l holds rows 4*(l>>4)+i (centroids) of
// column l&15 (its point); the 4 lane groups are combined once at the end.
// ------------------------------------------------------------------------------------
// TOP2: also track the second-smallest distance (mind2): one v_med3 + one v_min per
// score instead of half a v_min3 (bounds-based pruning, models/bounded.py).
//
// cstat (TOP2 only, nullable): the one-product prefilter of the fp32 / fp64 assignment
// (assign_x3.hip).  X is then the bf16 hi term xh of the data rows and Cm2 the hi term th of
// t = -2c, so a score leaves out xh.(t - th) + (x - xh).t; x1_eps bounds that per row from
// ||xh||, ||x - xh|| and the centroid maxima cstat, plus the accumulation / norm / tag terms
// of the x3 bound.  ||x - xh|| comes from the row's ||xl|| (xnhl, written once per bound
// shard by the split; x - xh = xl + xr with |xr| <= R8 |xl|), or without it from
// x - xh <= 2^-8 |xh| componentwise (RNE; +2^-16 for fp64 -> fp32 -> bf16) -- the per-row
// residual is ~0.6x that worst case and certifies ~1/6 more of the listed rows.  A row whose gap s2 - s1 exceeds 2 eps has
// the exact argmin as its label here; every other row gets its label with the sign bit set
// (x3_compact_kernel lists them for the three-product kernel: appending here took one
// same-address atomic per 16 rows and serialised the kernel's tail).
__device__ __forceinline__ float x1_eps(float hx, float lx, const float* cstat, int KS) {
  const float cn = cstat[0];
  const float Hc = sqrtf(cstat[1]) * 1.0001f, Lc = sqrtf(cstat[2]) * 1.0001f;
  constexpr float R8 = 0.00392157f;              // 2^-8 / (1 - 2^-8): |tr| <= R8 |tl|
  const float Tc = Lc * (1.f + R8);              // ||t - th||
  const float dx = lx >= 0.f ? lx * (1.f + R8)   // ||x - xh||
                             : hx * (0.00390625f + 1.5259e-5f);
  const float e_split = hx * Tc + dx * (Hc + Tc);
  const float s_main = hx * Hc;
  constexpr float U8 = 8.f * 1.1920929e-7f;      // per-MFMA accumulation (probe_mfma_acc)
  const float e_acc = U8 * ((float)KS * cn + (float)(KS + 1) * s_main);
  const float e_cn = 1.1920929e-7f * cn;
  const float e_tag = 3.8146973e-6f * (cn + s_main);  // 5 tag bits: 2^-18
  return (e_split + e_acc + e_cn + e_tag) * 1.001f + 1e-30f;
}

template <int DP, int P, int NST, int WAVES, int QT, bool TOP2 = false>
__global__ __launch_bounds__(WAVES * 64, ((DP >= 128 && (P >= 8 || (TOP2 && P >= 6))) ? 2 : WAVES == 6 ? 3 : (WAVES % 4 == 0 ? (WAVES / 4 > 1 ? WAVES / 4 : 3) : 2)))
void assign_mfma_bf16_ring3_kernel(const __bf16* __restrict__ X, int64_t N, int64_t ldx,
                                   const __bf16* __restrict__ Cm2, const float* __restrict__ cnorm,
                                   int ntiles, int32_t* __restrict__ labels,
                                   float* __restrict__ mind,
                                   const int32_t* __restrict__ rowidx = nullptr,
                                   float* __restrict__ mind2 = nullptr,
                                   const float* __restrict__ cstat = nullptr,
                                   const float2* __restrict__ xnhl = nullptr) {
  constexpr int BNL = 16 * QT;                     // centroids per stage
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 32;                      // 32-deep k-steps
  constexpr int TILE_B = BNL * DP * 2;
  constexpr int NORM_B = BNL * 4;
  constexpr int STAGE_B = TILE_B + NORM_B;
  constexpr int PIECES = TILE_B / 1024;
  // pieces / norm chunks per wave, rounded up: with a wave count that does not divide
  // them (6 waves) the last waves re-load pieces another wave also loads (identical bytes
  // to the same LDS slot), so every wave issues the same VPS DMAs per stage and the
  // stage-end vmcnt wait is exact for all of them
  constexpr int PPW = (PIECES + WAVES - 1) / WAVES;
  constexpr int NCH = NORM_B / 16;
  constexpr int NPW = (NCH + WAVES - 1) / WAVES;
  constexpr int VPS = PPW + 1;
  static_assert(NPW >= 1 && NPW <= NCH && PPW >= 1, "stage split");
  static_assert(KS >= 1, "DP >= 32");
  constexpr unsigned EMB = QT * 4 <= 16 ? 15u : 31u;  // (q, reg) id bits in the mantissa
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE_B];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;   // point column of the tile / centroid row of the A fragment
  const int g = lane >> 4;   // k-group of the operands / row group of the accumulator
  const int64_t pbase = (int64_t)blockIdx.x * (WAVES * P * 16) + (int64_t)w * (P * 16);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  bf16x8 bq[P][KS];
  float xn[P] = {};
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 16 + r;
    if (row >= N) row = N - 1;
    // indexed mode (mini-batches): point i of this launch is shard row rowidx[i], so a
    // sampled batch is never materialised
    if (rowidx) row = rowidx[row];
    const __bf16* src = X + row * ldx + g * 8;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) bq[p][kk] = *reinterpret_cast<const bf16x8*>(src + kk * 32);
  }
  // ||x||^2 only feeds the optional min-distance output: skip its ~5 VALU per element
  // when the caller does not ask for it (uniform branch)
  if (mind || mind2 || (TOP2 && cstat)) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      float s = 0.f;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = (float)bq[p][kk][j];
          s = fmaf(f, f, s);
        }
      s += __shfl_xor(s, 16, 64);
      xn[p] = s + __shfl_xor(s, 32, 64);
    }
  }

  // Per-lane byte offsets of this wave's pieces inside a stage image: loop invariant, one
  // VGPR each.  The pieces are issued by inline asm in the saddr + voffset form (stage base
  // in SGPRs, M0 = LDS destination): with the builtin, hipcc kept a 64-bit VGPR address
  // per piece and recomputed it every stage -- 256 VGPRs at P=8 against 235 this way, and
  // 1.5 % (10M rows) to 5 % (1.25M rows) more time (tools/ring3_ab.hip,
  // profiles/ring3_ab_r03.txt).  The compiler does not count these loads in its vmcnt
  // bookkeeping; the explicit stage-end waits below do (extra outstanding loads only
  // make the compiler's own vmcnt waits more conservative).  M0 is a reserved register
  // to hipcc (-Winline-asm notes the clobber): it sets M0 immediately before each of its
  // own LDS-DMA instructions (checked in the ISA: the norm DMA below), so the value this
  // asm leaves in M0 is never relied on.  The builtin with a uniform base + 32-bit offset
  // still fell back to 64-bit VGPR addresses inside the ring loop.
  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int piece = (w * PPW + i) % PIECES;
    const int L = piece * 64 + lane;
    const int row = L / CPR, cp = L % CPR;
    voff[i] = (unsigned)((row * DP + swz<DP>(row, cp) * 8) * 2);
  }
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave index in SGPRs (DMA destinations)
  auto issue = [&](int t, int slot) __attribute__((always_inline)) {
    const __bf16* base = Cm2 + (int64_t)t * BNL * DP;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = (wu * PPW + i) % PIECES;
      const unsigned dst = lds0 + slot * STAGE_B + piece * 1024;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff[i]), "s"(base)
                   : "memory", "m0");
    }
    // contiguous chunk run per wave (the DMA writes lane l at base + 16 l)
    const int nb = w * NPW < NCH - NPW ? w * NPW : NCH - NPW;
    if (lane < NPW) {
      const float* src = cnorm + (int64_t)t * BNL + (nb + lane) * 4;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * STAGE_B + TILE_B + nb * 16),
          16, 0, 0);
    }
  };

#pragma unroll
  for (int t = 0; t < NST - 1; ++t) issue(t < ntiles ? t : ntiles - 1, t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
  __builtin_amdgcn_s_barrier();

  float best[P], best2[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = INFINITY;
    best2[p] = INFINITY;
    bt[p] = 0;
  }

  // A fragment of k-step kk: row q*16 + r of the stage, 16-B chunk kk*4 + g (the XOR
  // swizzle depends on r only, so the phase is an immediate offset)
  unsigned aoff[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) aoff[kk] = lds0 + r * (DP * 2) + swz<DP>(r, kk * 4 + g) * 16;
  const unsigned noff = lds0 + TILE_B + 16 * g;  // norms of rows q*16 + 4g .. +3

  auto stage = [&](int t, auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value;
    {
      const int tn = t + NST - 1;
      issue(tn < ntiles ? tn : ntiles - 1, (slot + NST - 1) % NST);
    }
    // running key minimum of the whole stage (all QT phases): one compare/select per
    // point tile per stage instead of per phase
    float m[P], m2[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = m2[p] = INFINITY;
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      auto afrag = [&](int kk) __attribute__((always_inline)) {
        bf16x8 a;
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(a) : "v"(aoff[kk]), "i"(slot * STAGE_B + q * 16 * DP * 2));
        return a;
      };
      f32x4 n4;
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(n4) : "v"(noff), "i"(slot * STAGE_B + q * 16 * 4));
      bf16x8 a0 = afrag(0);
      bf16x8 a1 = afrag(KS > 1 ? 1 : 0);
      f32x4 acc[P];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        bf16x8 a2 = a1;
        if (kk + 2 < KS) a2 = afrag(kk + 2);
        if (kk + 2 < KS) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        else if (kk + 1 < KS) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (q == QT - 1 && kk == KS - 1) {
          // early slot release: the stage's last fragment is in registers, so the stage-end
          // wait and barrier go before its P MFMAs, which then run under the next stage's
          // refill issue and first LDS reads
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");  // stage t+1 landed
          __builtin_amdgcn_s_barrier();  // ... for every wave's pieces
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < P; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bq[p][kk], kk == 0 ? n4 : acc[p],
                                                            0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        a0 = a1;
        a1 = a2;
      }
#pragma unroll
      for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 4 + i));
          if constexpr (TOP2) {
            // m <= m2 kept.  asm: the builtins canonicalised the tagged v first (one more VALU
            // per score: 855 -> 639 per loop trip); v is never a signalling NaN (tag bits
            // only in normal values, NaN rows end with v2 - v1 = NaN and are flagged)
            float r1, r2;
            asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r2) : "v"(m[p]), "v"(m2[p]), "v"(v));
            asm("v_min_f32 %0, %1, %2" : "=v"(r1) : "v"(m[p]), "v"(v));
            m2[p] = r2;
            m[p] = r1;
          } else {
            m[p] = __builtin_fminf(m[p], v);
          }
        }
      }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if constexpr (TOP2)  // 2nd of the union of {best, best2} and {m, m2}
        best2[p] = __builtin_fminf(__builtin_fminf(best2[p], m2[p]), __builtin_fmaxf(best[p], m[p]));
      const bool up = m[p] < best[p];
      best[p] = up ? m[p] : best[p];
      bt[p] = up ? t : bt[p];
    }
  };

  for (int t0 = 0; t0 < ntiles; t0 += NST) {
    stage(t0, std::integral_constant<int, 0>{});
    if constexpr (NST > 1) if (t0 + 1 < ntiles) stage(t0 + 1, std::integral_constant<int, 1>{});
    if constexpr (NST > 2) if (t0 + 2 < ntiles) stage(t0 + 2, std::integral_constant<int, 2 % NST>{});
    if constexpr (NST > 3) if (t0 + 3 < ntiles) stage(t0 + 3, std::integral_constant<int, 3 % NST>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- combine the 4 lane groups (same point, disjoint centroid rows) ----
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const unsigned e = __float_as_uint(best[p]) & EMB;
    int lab = bt[p] * BNL + (int)(e >> 2) * 16 + 4 * g + (int)(e & 3);
    float v = __uint_as_float(__float_as_uint(best[p]) & ~EMB);
    float v2 = __uint_as_float(__float_as_uint(best2[p]) & ~EMB);
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int ol = __shfl_xor(lab, o, 64);
      if constexpr (TOP2) {
        const float ov2 = __shfl_xor(v2, o, 64);
        v2 = fminf(fminf(v2, ov2), fmaxf(v, ov));
      }
      const bool other = (ov < v) || (ov == v && ol < lab);
      v = other ? ov : v;
      lab = other ? ol : lab;
    }
    if constexpr (TOP2) {
      if (cstat) {  // uniform branch: the prefilter flags its uncertified rows
        const int64_t rr = pbase + p * 16 + r;
        const float lx = xnhl ? sqrtf(xnhl[rr < N ? rr : N - 1].y) * 1.0001f : -1.f;
        const float eps2 = 2.f * x1_eps(sqrtf(xn[p]) * 1.0001f, lx, cstat, KS);
        if (!(v2 - v > eps2)) lab |= (int)0x80000000;
      }
    }
    const int64_t row = pbase + p * 16 + r;
    if (g == 0 && row < N) {
      labels[row] = lab;
      if (mind) mind[row] = fmaxf(v + xn[p], 0.f);
      if (TOP2 && mind2) mind2[row] = fmaxf(v2 + xn[p], 0.f);
    }
  }
}

}  // namespace tdc
