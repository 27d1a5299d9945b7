// N4/N5 on MFMA: the Fuzzy C-Means tower for large K x D in fp32, on bf16 matrix cores.
//
// Reference per GPU per iteration (scripts/distribuitedClustering.py:108-137): [N,K,D]
// difference tiles -> d -> t = d^(-2/(m-1)) -> u = t / sum_k t -> NaN -> 0 -> W = u^m ->
// MatMul(W, X) (cuBLAS DGEMM) and Sum(W).  Both matrix products run here on the bf16
// matrix cores (the bf16x3 stats pass on v_mfma_f32_16x16x32_bf16, the one-product stats
// pass and the accumulate pass on v_mfma_f32_32x32x16_bf16) with fp32-grade operands from a
// hi/lo bf16 split
// (x = xh + xl, -2c = ch + cl, each lo = bf16(v - hi)):
//   x.(-2c) ~= xh.ch + xh.cl + xl.ch      (three MFMAs; the dropped xl.cl is 2^-16 relative)
//   sum_i w_ik x_i = W^T Xh + W^T Xl      (W = u^m rounded to bf16; sum_i w_ik from the same
//                                          rounded w, so each centroid is an exact convex
//                                          combination of its weights)
// Two kernels, like fcm_tower.hip:
//   fcm_mfma_stats: 8 waves x 32 points; the hi/lo point fragments stay in VGPRs,
//     64-centroid stages stream through LDS; per point sum_k t, the on-centroid rule and
//     argmin d2 -> rowinfo (see fcm_tower.hip) and the label.  From DP = 64 the stats pass
//     (fcm_mfma_stats1) runs ONE product (xh.ch) and corrects the two nearest centroids'
//     terms with the cross terms afterwards (see there).
//   fcm_mfma_accum: block = 128 centroids (32 per wave, hi/lo fragments in VGPRs) x a row
//     range.  64-point hi/lo X tiles are staged in LDS once and read twice: by rows (the
//     distance A operand) and transposed with ds_read_b64_tr_b16 (the W^T X B operand).
//     The distance accumulator (rows = points, lane = centroid) becomes the A operand of
//     W^T X without leaving registers (cdna_hip_programming.md "An accumulator tile as
//     the next MFMA's operand").  The [32 x D] W^T X tile of each wave lives in fp32
//     accumulators for the whole row range and is flushed once (fp64 atomics).
//     Blocks are mapped so that the K tiles of one row range run on the same XCD and
//     share its L2 copy of the X tile.
// Distances within 2^-16 ||x||^2 of zero count as zero (an exact hit computes 2 xl^2 ~
// 2^-17 ||x||^2): a point on a centroid keeps the reference's NaN -> 0 semantics.  Rows
// and centroids are shifted by a fixed vector (the shard mean) before the split, so the
// expansion's cancellation is relative to the data spread, not to its offset.
#include <type_traits>

#include "tdc_common.h"
#include "kernels.h"
#include "fcm_math.h"

namespace tdc {
namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr float ZERO_FLOOR = 1.52587890625e-05f;  // 2^-16 (an exact hit computes ~2^-17 |x|^2)

struct MParam {
  float expo, m;
  int pmode, mint, nz;
};

// 16-byte chunk c of row r of a [rows][DP] bf16 LDS image, XOR-swizzled so that both the
// row reads (lane = row) and the transposed reads spread over the banks (guide T10 (b)).
template <int DP>
__device__ __forceinline__ int xoff(int r, int c) {
  constexpr int CPR = DP / 8;
  const int sw = (((r & 3) << 2) | ((r >> 2) & 3)) & (CPR - 1);
  return r * DP * 2 + 16 * (c ^ sw);
}

// centroid stage image: same swizzle as the Lloyd kernels (rows of DP bf16)
template <int DP>
__device__ __forceinline__ int coff(int r, int c) {
  constexpr int CPR = DP / 8;
  constexpr int G = CPR < 16 ? CPR : 16;
  constexpr int RPB = 16 / G;
  return r * DP * 2 + 16 * (c ^ ((r / RPB) & (G - 1)));
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) {
  return __builtin_bit_cast(bf16x8, v);
}

// Membership arithmetic specialised at compile time (a runtime fuzzifier switch inside the
// unrolled epilogues quadrupled the code and thrashed the instruction cache):
//   MODE 2: m = 2  -> t = 1/d2 (v_rcp_f32), w = u*u
//   MODE 0: any m  -> t = 2^(expo log2 d2), w = 2^(m log2 u)
template <int MODE>
__device__ __forceinline__ float mt(float d2, float expo) {
  if constexpr (MODE == 2) return __builtin_amdgcn_rcpf(d2);  // rcp(0) = +inf
  else return __builtin_amdgcn_exp2f(expo * __builtin_amdgcn_logf(d2));  // log2(0) = -inf
}
template <int MODE>
__device__ __forceinline__ float mw(float u, float m) {
  if constexpr (MODE == 2) return u * u;
  else return u > 0.f ? __builtin_amdgcn_exp2f(m * __builtin_amdgcn_logf(u)) : 0.f;
}

#define TDC_GLOAD16(dst, src) \
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(src) : "memory")

// ---------------------------------------------------------------------------------------
// pass 1: per-row statistics
// ---------------------------------------------------------------------------------------
// WAVES waves x 32 points share every 64-centroid stage (8 waves: 2 per SIMD, so one wave's
// epilogue VALU runs beside the other's MFMAs); within a wave the epilogue of half q-1 is
// issued after the MFMAs of half q (software pipeline, as the Lloyd kernels).  On
// v_mfma_f32_16x16x32_bf16, the Lloyd kernels' ring3 shape: the chip holds a higher clock
// under it (MI355X_MICROARCH.md "DVFS give-back" item 7); against the 32x32x16 form of the
// same pass 0.645 vs 0.690 ms at N=1M, K=1024, D=128 (profiles/fcm_stats_shape_ab_r06am.txt).
// A wave's 32 points are two 16-point tiles and each 32-centroid half two 16-centroid tiles,
// so a lane holds 4 centroids of two points (C layout: lane l, register i = centroid
// 4 (l >> 4) + i of point l & 15); the row statistics are combined over the 4 lane groups
// at the end.
template <int DP, int MODE, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void fcm_mfma_stats_kernel(
    const __bf16* __restrict__ Xh, const __bf16* __restrict__ Xl, const float* __restrict__ xx,
    int64_t N, const __bf16* __restrict__ Ch, const __bf16* __restrict__ Cl,
    const float* __restrict__ cc, int K, int nstages, MParam prm, int32_t* __restrict__ labels,
    float* __restrict__ rowinfo) {
  constexpr int BN = 64;
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 32;                 // 32-deep k-steps
  constexpr int IMGB = BN * DP * 2;
  constexpr unsigned TB = 7u;                 // tag bits: (centroid tile, register)
  __shared__ __attribute__((aligned(16))) char s_c[2][2 * IMGB];
  __shared__ __attribute__((aligned(16))) float s_n[2][BN];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int64_t wrow = (int64_t)blockIdx.x * (WAVES * 32) + (int64_t)w * 32;

  bf16x8 bh[2][KS], bl[2][KS];
  float xn[2], zf[2];
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) {
    int64_t row = wrow + 16 * pt + r;
    if (row >= N) row = N - 1;
    const bf16x8* sh = reinterpret_cast<const bf16x8*>(Xh + row * DP + 8 * g);
    const bf16x8* sl = reinterpret_cast<const bf16x8*>(Xl + row * DP + 8 * g);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      bh[pt][kk] = sh[4 * kk];
      bl[pt][kk] = sl[4 * kk];
    }
    xn[pt] = xx[row];
    zf[pt] = ZERO_FLOOR * xn[pt];
  }

  // stage loads: as fcm_mfma_stats_kernel
  constexpr int PPI = IMGB / 1024;
  constexpr int PPW = 2 * PPI / WAVES;
  static_assert(IMGB % 1024 == 0 && (2 * PPI) % WAVES == 0 && PPI % PPW == 0, "stage pieces");
  constexpr int G = CPR < 16 ? CPR : 16;
  constexpr int RPB = 16 / G;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int hlw = (wu * PPW) / PPI;
  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int q = ((w * PPW + i) % PPI) * 64 + lane;
    const int row = q / CPR, cs = q % CPR;
    voff[i] = (unsigned)(row * DP * 2 + 16 * (cs ^ ((row / RPB) & (G - 1))));
  }
  const unsigned lds_c = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)&s_c[0][0];
  const unsigned lds_n = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)&s_n[0][0];
#define TDC_STAGE_LOAD(T_, B_)                                                            \
  {                                                                                       \
    const __bf16* base_ = (hlw ? Cl : Ch) + (int64_t)(T_) * BN * DP;                      \
    _Pragma("unroll") for (int i = 0; i < PPW; ++i) {                                     \
      const int pc_ = wu * PPW + i;                                                       \
      const unsigned dst_ = lds_c + (B_) * 2 * IMGB + (pc_ / PPI) * IMGB + (pc_ % PPI) * 1024; \
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"                  \
                   :: "s"(__builtin_amdgcn_readfirstlane(dst_)), "v"(voff[i]),             \
                      "s"(uniform_ptr(base_))                                             \
                   : "memory", "m0");                                                     \
    }                                                                                     \
    if (wu == 0 && lane < BN / 4) {                                                        \
      const float* nb_ = cc + (int64_t)(T_) * BN;                                         \
      const unsigned nd_ = lds_n + (B_) * BN * 4;                                         \
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"                  \
                   :: "s"(__builtin_amdgcn_readfirstlane(nd_)), "v"((unsigned)(lane * 16)), \
                      "s"(uniform_ptr(nb_)) : "memory", "m0");                            \
    }                                                                                     \
  }
  TDC_STAGE_LOAD(0, 0)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  float S[2] = {0.f, 0.f}, best[2] = {INFINITY, INFINITY};
  int bt[2] = {0, 0};

  // MFMAs of half Q (32 centroids = two 16-centroid tiles ct) of the stage in cb/ns
#define TDC_PHASE(ACC, Q)                                                                 \
  {                                                                                       \
    f32x4 n4[2];                                                                          \
    bf16x8 ah[2][KS], al[2][KS];                                                          \
    _Pragma("unroll") for (int ct = 0; ct < 2; ++ct) {                                    \
      n4[ct] = *reinterpret_cast<const f32x4*>(&ns[(Q) * 32 + ct * 16 + 4 * g]);          \
      const int crow = (Q) * 32 + ct * 16 + r;                                            \
      _Pragma("unroll") for (int kk = 0; kk < KS; ++kk) {                                 \
        ah[ct][kk] = as_bf16x8(*reinterpret_cast<const uint4*>(cb + coff<DP>(crow, 4 * kk + g))); \
        al[ct][kk] = as_bf16x8(*reinterpret_cast<const uint4*>(cb + IMGB + coff<DP>(crow, 4 * kk + g))); \
      }                                                                                   \
    }                                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    _Pragma("unroll") for (int kk = 0; kk < KS; ++kk)                                     \
      _Pragma("unroll") for (int ct = 0; ct < 2; ++ct)                                    \
        _Pragma("unroll") for (int pt = 0; pt < 2; ++pt) {                                \
          ACC[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ct][kk], bh[pt][kk], kk == 0 ? n4[ct] : ACC[ct][pt], 0, 0, 0); \
          ACC[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ct][kk], bl[pt][kk], ACC[ct][pt], 0, 0, 0); \
          ACC[ct][pt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[ct][kk], bh[pt][kk], ACC[ct][pt], 0, 0, 0); \
        }                                                                                 \
  }
  // epilogue of half Q of stage T_: register i of tile ct = centroid ct*16 + 4g + i of the
  // half; the tag (ct, i) orders them ascending for this lane group
#define TDC_EPI(ACC, Q, T_)                                                               \
  {                                                                                       \
    const int kvalid = K - ((T_) * BN + (Q) * 32 + 4 * g);                                \
    _Pragma("unroll") for (int pt = 0; pt < 2; ++pt) {                                    \
      float mpk = INFINITY, sp = 0.f;                                                     \
      if (kvalid >= 20) { /* every centroid of this lane group valid (all but the last stage) */ \
        _Pragma("unroll") for (int ct = 0; ct < 2; ++ct)                                  \
          _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                 \
            const float d2 = fmaxf(ACC[ct][pt][i] + xn[pt], zf[pt]);                      \
            sp += mt<MODE>(d2, prm.expo);                                                 \
            mpk = __builtin_fminf(mpk, __uint_as_float((__float_as_uint(d2) & ~TB) | (unsigned)(ct * 4 + i))); \
          }                                                                               \
      } else {                                                                            \
        _Pragma("unroll") for (int ct = 0; ct < 2; ++ct)                                  \
          _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                 \
            const bool v = ct * 16 + i < kvalid;                                          \
            const float d2 = fmaxf(ACC[ct][pt][i] + xn[pt], zf[pt]);                      \
            sp += v ? mt<MODE>(d2, prm.expo) : 0.f;                                       \
            const float pk = __uint_as_float((__float_as_uint(d2) & ~TB) | (unsigned)(ct * 4 + i)); \
            mpk = v ? __builtin_fminf(mpk, pk) : mpk;                                     \
          }                                                                               \
      }                                                                                   \
      S[pt] += sp;                                                                        \
      const bool up = mpk < best[pt];                                                     \
      best[pt] = up ? mpk : best[pt];                                                     \
      bt[pt] = up ? (2 * (T_) + (Q)) : bt[pt];                                            \
    }                                                                                     \
  }

  f32x4 acc0[2][2], acc1[2][2];
  for (int t = 0; t < nstages; ++t) {
    const int buf = t & 1;
    if (t + 1 < nstages) TDC_STAGE_LOAD(t + 1, buf ^ 1)
    const char* cb = s_c[buf];
    const float* ns = s_n[buf];
    TDC_PHASE(acc0, 0)
    if (t > 0) TDC_EPI(acc1, 1, t - 1)
    TDC_PHASE(acc1, 1)
    TDC_EPI(acc0, 0, t)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  TDC_EPI(acc1, 1, nstages - 1)
#undef TDC_PHASE
#undef TDC_EPI
#undef TDC_STAGE_LOAD

  // combine the 4 lane groups of each point: sum of t, nearest (lowest index on ties)
#pragma unroll
  for (int pt = 0; pt < 2; ++pt) {
    float s = S[pt];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const unsigned e = __float_as_uint(best[pt]) & TB;
    float v = __uint_as_float(__float_as_uint(best[pt]) & ~TB);
    int l = bt[pt] * 32 + (int)(e >> 2) * 16 + 4 * g + (int)(e & 3);
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int ol = __shfl_xor(l, o, 64);
      const bool other = (ov < v) || (ov == v && ol < l);
      v = other ? ov : v;
      l = other ? ol : l;
    }
    const int64_t row = wrow + 16 * pt + r;
    if (g == 0 && row < N) {
      const bool on = v <= __uint_as_float(__float_as_uint(zf[pt]) & ~TB);
      labels[row] = (on && prm.nz) ? 0 : l;
      rowinfo[row] = on ? (prm.nz ? 0.f : -1.f) : __builtin_amdgcn_rcpf(s);
    }
  }
}

// ---------------------------------------------------------------------------------------
// pass 1, one product (DP >= 64): the row statistics need fp32-faithful distances only where
// they dominate.  sum_k t_k is ruled by the nearest centroids, whose d2 is small against
// ||x||^2 + ||c||^2 (the expansion's cancellation), while the far terms carry the bf16
// product's ~2^-9 / sqrt(D) relative error harmlessly.  So the MFMAs compute xh.ch only
// (a third of the bf16x3 work, hi centroid images only), the epilogue keeps each row's
// two nearest centroids (tag-in-mantissa min + v_med3 runner-up), and at the end the two
// get the cross terms xh.cl + xl.ch on the VALU (the lo point fragments stay in registers,
// the centroid rows come from L2): their d2 then equals the accumulate pass's bf16x3 value
// up to fp32 rounding, and sum_k t_k swaps their one-product terms for the corrected ones.
// The label (nearest of the two) and the on-centroid rule use the corrected d2.
// ---------------------------------------------------------------------------------------
template <int DP, int MODE, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void fcm_mfma_stats1_kernel(
    const __bf16* __restrict__ Xh, const __bf16* __restrict__ Xl, const float* __restrict__ xx,
    int64_t N, const __bf16* __restrict__ Ch, const __bf16* __restrict__ Cl,
    const float* __restrict__ cc, int K, int nstages, MParam prm, int32_t* __restrict__ labels,
    float* __restrict__ rowinfo, float4* __restrict__ fix) {
  constexpr int BN = 64;
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 16;
  constexpr int HALF = DP / 2;
  constexpr int IMGB = BN * DP * 2;           // bytes of one hi stage image
  // stage ring: a stage's compute (~1K cycles per SIMD) is shorter than its DMA's latency
  // from L2 under load, so stage t + NSTS - 1 is issued while stage t computes (with two
  // slots the pass waited out every stage: ~4.8K cycles per 64-centroid stage, SQ_WAIT_ANY
  // 26 % + SQ_WAIT_INST_ANY 39 % of wave cycles, profiles/pmc_fcm10m_one_vs_x3_r05h.txt)
  constexpr int NSTS = 4;
  __shared__ __attribute__((aligned(16))) char s_c[NSTS][IMGB];
  __shared__ __attribute__((aligned(16))) float s_n[NSTS][BN];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * (WAVES * 32) + (int64_t)w * 32 + r;
  const int64_t row = row0 < N ? row0 : N - 1;

  // hi point fragments for the MFMAs; the lo ones are loaded for the fix-up at the end (the
  // same bytes, 32 VGPRs fewer through the loop: they hold the next half's A fragments)
  bf16x8 bh[KS], bl[KS];
  {
    const bf16x8* sh = reinterpret_cast<const bf16x8*>(Xh + row * DP + h * HALF);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) bh[kk] = sh[kk];
  }
  const float xn = xx[row];
  const float zf = ZERO_FLOOR * xn;

  // hi stage images by LDS-DMA, as the bf16x3 kernel (source-side swizzle, saddr form)
  constexpr int PPI = IMGB / 1024;
  constexpr int PPW = PPI / WAVES;
  static_assert(IMGB % 1024 == 0 && PPI % WAVES == 0 && PPW >= 1, "stage pieces");
  constexpr int G = CPR < 16 ? CPR : 16;
  constexpr int RPB = 16 / G;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int q = (w * PPW + i) * 64 + lane;
    const int rr = q / CPR, cs = q % CPR;
    voff[i] = (unsigned)(rr * DP * 2 + 16 * (cs ^ ((rr / RPB) & (G - 1))));
  }
  const unsigned lds_c = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)&s_c[0][0];
  const unsigned lds_n = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)&s_n[0][0];
  auto stage_load = [&](int T, int B) __attribute__((always_inline)) {
    const __bf16* base = Ch + (int64_t)T * BN * DP;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const unsigned dst = lds_c + B * IMGB + (wu * PPW + i) * 1024;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff[i]),
                      "s"(uniform_ptr(base))
                   : "memory", "m0");
    }
    // every wave loads the stage's norms (identical bytes to the same slot), so every wave
    // issues PPW + 1 DMAs per stage and the ring's vmcnt waits are exact for all of them
    if (lane < BN / 4) {
      const float* nb = cc + (int64_t)T * BN;
      const unsigned nd = lds_n + B * BN * 4;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(nd)), "v"((unsigned)(lane * 16)),
                      "s"(uniform_ptr(nb)) : "memory", "m0");
    }
  };
  constexpr int VPS = PPW + 1;
  // (stages past the end reload the last one into a free slot: uniform DMA counts)
#pragma unroll
  for (int t = 0; t < NSTS - 1; ++t) stage_load(t < nstages ? t : nstages - 1, t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NSTS - 2) * VPS) : "memory");  // stage 0 landed
  __syncthreads();

  // keys: the tagged d2 bits compared as int32 (no canonicalising v_max per v_min_f32; all
  // negative keys order below the positive ones, reversed among themselves -- a negative
  // one-product d2 lies within the product error of 0 and the fix-up re-sorts the two)
  constexpr int KINF = 0x7f800000;
  float S = 0.f;
  int best = KINF, best2 = KINF;
  int bt = 0, bt2 = 0;
  // top-2 fold of one tile's (m, m2) into (best, bt), (best2, bt2)
  auto fold = [&](int m, int m2, int tt) __attribute__((always_inline)) {
    const bool up = m < best;
    const int c = up ? best : m;
    const int ct = up ? bt : tt;
    const bool s2 = m2 < c;
    const int cand = s2 ? m2 : c;
    const int candt = s2 ? tt : ct;
    const bool up2 = cand < best2;
    best2 = up2 ? cand : best2;
    bt2 = up2 ? candt : bt2;
    best = up ? m : best;
    bt = up ? tt : bt;
  };
  // register i = centroid (i&3)+8(i>>2)+4h of the half; the key is the UNclamped one-product
  // d2 with the register index in its low mantissa bits, and t is taken of the key itself
  // (2^-19 relative off d2), so the fix-up can take out exactly the term it added
  // (the floor as an int32 max of the bits: zf >= 0, so every negative key maps to zf and
  // the positive ones order as their bits -- fmaxf of the bit-cast key cost a canonicalising
  // v_max_f32 per element on top of the max itself)
  const int zfi = __float_as_int(zf);
  auto elem = [&](float a, int i, int& m, int& m2, float& sp) __attribute__((always_inline)) {
    const int pk = (int)((__float_as_uint(a + xn) & ~15u) | (unsigned)i);
    sp += mt<MODE>(__int_as_float(max(pk, zfi)), prm.expo);
    // median of (m, m2, pk) with m <= m2 kept: one v_med3_i32 (the max(m, min(m2, pk))
    // spelling compiled to a v_min + v_max pair)
    int md;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(md) : "v"(m), "v"(m2), "v"(pk));
    m2 = md;
    m = min(m, pk);
  };
  // two top-2 sets (m <= m2 each) -> one
  auto merge2 = [](int& m, int& m2, int mo, int m2o) __attribute__((always_inline)) {
    m2 = min(max(m, mo), min(m2, m2o));
    m = min(m, mo);
  };
  // the MFMAs of half Q into acc; with EPI, the previous tile's epilogue (accp: all 32
  // centroids real) issues between them, 16/KS elements per MFMA: at one product the
  // epilogue VALU is as long as the MFMA chain, and in program order after it the wave
  // would leave the matrix pipe idle for its whole length
  // A fragments of half Q of a stage (both halves are read at the stage start, so the
  // second half's reads are in flight under the first half's MFMAs)
  auto frags = [&](bf16x8 (&ah)[KS], int Q, const char* cb) __attribute__((always_inline)) {
    const int crow = Q * 32 + r;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
      ah[kk] = as_bf16x8(*reinterpret_cast<const uint4*>(cb + coff<DP>(crow, h * (CPR / 2) + kk)));
  };
  auto phase = [&](f32x16& acc, int Q, const bf16x8 (&ah)[KS], const float* ns,
                   const f32x16& accp, int ttp, auto epi_c) __attribute__((always_inline)) {
    constexpr bool EPI = decltype(epi_c)::value;
    f32x16 init;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 n4 = *reinterpret_cast<const f32x4*>(&ns[Q * 32 + 8 * g4 + 4 * h]);
#pragma unroll
      for (int e = 0; e < 4; ++e) init[4 * g4 + e] = n4[e];
    }
    // even and odd elements in two independent chains (running sum, top-2), merged once
    // per phase: one chain serialised every v_add / v_min on its predecessor
    int m = KINF, m2 = KINF, mo = KINF, m2o = KINF;
    float sp = 0.f, spo = 0.f;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[kk], bh[kk], kk == 0 ? init : acc, 0, 0, 0);
      if constexpr (EPI) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (i * KS / 16 == kk) {
            if (i & 1) elem(accp[i], i, mo, m2o, spo);
            else elem(accp[i], i, m, m2, sp);
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (EPI) {
      S += sp + spo;
      merge2(m, m2, mo, m2o);
      fold(m, m2, ttp);
    }
  };
  // stand-alone epilogue with the pad-centroid mask (the last stage)
  auto epi = [&](const f32x16& acc, int Q, int T) __attribute__((always_inline)) {
    const int kvalid = K - (T * BN + Q * 32 + 4 * h);
    int m = KINF, m2 = KINF;
    float sp = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const bool v = (i & 3) + 8 * (i >> 2) < kvalid;
      int m_ = m, m2_ = m2;
      float sp_ = sp;
      elem(acc[i], i, m_, m2_, sp_);
      m = v ? m_ : m;
      m2 = v ? m2_ : m2;
      sp = v ? sp_ : sp;
    }
    S += sp;
    fold(m, m2, 2 * T + Q);
  };
  using WITH = std::integral_constant<bool, true>;
  using WITHOUT = std::integral_constant<bool, false>;

  f32x16 acc0, acc1;
  for (int t = 0; t < nstages; ++t) {
    const int buf = t % NSTS;
    {
      // slot (t + NSTS - 1) % NSTS was last read in stage t - 1, before its barrier
      const int tn = t + NSTS - 1;
      stage_load(tn < nstages ? tn : nstages - 1, tn % NSTS);
    }
    const char* cb = s_c[buf];
    const float* ns = s_n[buf];
    bf16x8 ah0[KS], ah1[KS];
    frags(ah0, 0, cb);
    frags(ah1, 1, cb);
    // wave-uniform: are all 32 centroids of half (t-1, 1) / (t, 0) real?
    if (t > 0 && K - ((t - 1) * BN + 32) >= 32) {
      phase(acc0, 0, ah0, ns, acc1, 2 * t - 1, WITH{});
    } else {
      phase(acc0, 0, ah0, ns, acc1, 0, WITHOUT{});
      if (t > 0) epi(acc1, 1, t - 1);
    }
    if (K - t * BN >= 32) {
      phase(acc1, 1, ah1, ns, acc0, 2 * t, WITH{});
    } else {
      phase(acc1, 1, ah1, ns, acc0, 0, WITHOUT{});
      epi(acc0, 0, t);
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NSTS - 2) * VPS) : "memory");  // stage t + 1 landed
    __syncthreads();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  {
    const bf16x8* sl = reinterpret_cast<const bf16x8*>(Xl + row * DP + h * HALF);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) bl[kk] = sl[kk];
  }
  epi(acc1, 1, nstages - 1);

  // ---- the row's two nearest over both lane halves, by (d2, label): same in both lanes ----
  S += __shfl_xor(S, 32, 64);
  auto lab_of = [&](float v, int t) {
    const unsigned e = __float_as_uint(v) & 15u;
    return t * 32 + (int)(e & 3) + 8 * (int)(e >> 2) + 4 * h;
  };
  auto lt = [](float a, int la, float b, int lb) { return a < b || (a == b && la < lb); };
  // the keys as floats (tag bits kept: the t the loop added was taken of exactly these)
  const float v0 = __int_as_float(best), w0 = __int_as_float(best2);
  const int l0 = lab_of(v0, bt), k0 = lab_of(w0, bt2);
  const float v1 = __shfl_xor(v0, 32, 64), w1 = __shfl_xor(w0, 32, 64);
  const int l1 = __shfl_xor(l0, 32, 64), k1 = __shfl_xor(k0, 32, 64);
  float va = v0, vb = v1;
  int la = l0, lb = l1;
  if (lt(v1, l1, v0, l0)) { va = v1; la = l1; vb = v0; lb = l0; }
  if (lt(w0, k0, vb, lb)) { vb = w0; lb = k0; }
  if (lt(w1, k1, vb, lb)) { vb = w1; lb = k1; }
  const bool has_b = vb < INFINITY && lb < K;
  // m = 2: the runner-up's correction matters only while its term is within 1/32 of the
  // nearest's (the one-product error of d2 relative to d2 falls as 1/d2, so the term
  // error falls as 1/d2^2); flatter t = d2^(-1/(m-1)) of other m: always
  const bool fix_b = has_b && (MODE != 2 || fmaxf(vb, zf) < 32.f * fmaxf(va, zf));

  // ---- cross terms xh.cl + xl.ch of the two over this lane's half, summed over halves ----
  // (both rows at once, two 16-B chunk pairs per scheduling region: the loads of a region
  // are in flight together without every chunk of both rows held in registers at once)
  auto cross = [&](int k) __attribute__((always_inline)) {
    const bf16x8* ph = reinterpret_cast<const bf16x8*>(Ch + (int64_t)k * DP + h * HALF);
    const bf16x8* pl = reinterpret_cast<const bf16x8*>(Cl + (int64_t)k * DP + h * HALF);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int k4 = 0; k4 < KS; k4 += 4) {
      bf16x8 chv[4], clv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        chv[u] = ph[k4 + u];
        clv[u] = pl[k4 + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s0 = fmaf((float)bh[k4 + u][j], (float)clv[u][j], s0);
          s1 = fmaf((float)bl[k4 + u][j], (float)chv[u][j], s1);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    return s0 + s1;
  };
  // (lanes r and r+32 hold the same row's two halves and take the same branches)
  float xa = cross(la), xb = 0.f;
  if (fix_b) xb = cross(lb);
  xa += __shfl_xor(xa, 32, 64);
  xb += __shfl_xor(xb, 32, 64);
  const float da = fmaxf(va + xa, zf);
  const float db = has_b ? fmaxf(vb + xb, zf) : INFINITY;
  float Sf = S - mt<MODE>(fmaxf(va, zf), prm.expo) + mt<MODE>(da, prm.expo);
  if (fix_b) Sf += mt<MODE>(db, prm.expo) - mt<MODE>(fmaxf(vb, zf), prm.expo);
  const bool bwin = lt(db, lb, da, la);
  const float dmin = bwin ? db : da;
  const int lab = bwin ? lb : la;
  if (h == 0 && row0 < N) {
    const bool on = dmin <= zf;
    labels[row0] = (on && prm.nz) ? 0 : lab;
    rowinfo[row0] = on ? (prm.nz ? 0.f : -1.f) : __builtin_amdgcn_rcpf(Sf);
    // the two corrected d2 the sum used, for the one-product accumulate pass
    if (fix)
      fix[row0] = make_float4(da, fix_b ? db : 0.f, __int_as_float(la),
                              __int_as_float(fix_b ? lb : -1));
  }
}

// ---------------------------------------------------------------------------------------
// pass 2: W^T X and the column sums of a 128-centroid tile over a row range; the block's
// [128 x D] fp32 partial goes to its own slab (no atomics), reduced by fcm_reduce_kernel
// ---------------------------------------------------------------------------------------
// WAVES = 4: one wave per SIMD, each wave owns 32 centroids over both 32-point halves of a
// tile, memberships of one half software-pipelined between the MFMAs of the other.
// WAVES = 8: two waves per SIMD, wave w owns centroid group w & 3 and point half w >> 2
// (no intra-wave pipeline: the other wave on the SIMD issues its MFMAs under this wave's
// membership VALU); the two halves' W^T X partials meet in LDS at the end.
//
// STAG (8 waves): the two waves of a SIMD (w and w + 4, same centroid group, point halves 0
// and 1) run the same program and with one barrier per tile they ran in lockstep -- both
// in their distance MFMAs, then both in their membership VALU, then both in W^T X, so the
// VALU segment stood beside an idle matrix pipe.  Staggered, waves 4-7 defer each tile's
// memberships and W^T X by one tile (distances carried across the barrier in registers,
// MI355X_MICROARCH.md item 9): in one barrier interval wave w runs dist(t) | memb(t) |
// W^T X(t) while wave w + 4 runs memb(t-1) | W^T X(t-1) | dist(t), so each one's
// membership VALU issues beside the other's MFMAs.  Tile t is then read in two intervals:
// three LDS tile buffers.
//
// ONE (DP >= 64, with the stats pass's fix-up rows): the distances are ONE product, xh.ch,
// like the stats pass's (fcm_mfma_stats1), and each row's two nearest centroids take the
// stats pass's corrected d2 (fix = {d2a, d2b, la, lb} per row; lb = -1 when the stats pass
// kept the runner-up's one-product term).  The memberships then use the same d2 as the
// denominator sum_k t_k of the stats pass (up to the fp32 rounding of the two MFMA orders),
// and the distance MFMAs drop from 3 x DP/16 to DP/16 per 32 x 32 tile.
//
// RAW: the shard's own bf16 rows (unshifted, Xr) are W^T X's one operand -- ONE product
// per tile, exact in its products (bf16 w times bf16 x into fp32) -- and the reduction adds
// no shift back.  For bf16 data only (the rows ARE those bf16 numbers; fp32 rows keep
// W^T Xh + W^T Xl).  With ONE the tile holds [xh | xr]; with the bf16x3 distances
// [xh | xl | xr] (NIMG = 3).
template <int DP, int MODE, bool NZ, int WAVES, bool STAG, bool ONE, bool RAW>
__global__ __launch_bounds__(WAVES * 64, 1) void fcm_mfma_accum_kernel(
    const __bf16* __restrict__ Xh, const __bf16* __restrict__ Xl, const float* __restrict__ xx,
    const float* __restrict__ rowinfo, const float* __restrict__ fix, int64_t N,
    const __bf16* __restrict__ Xr, const __bf16* __restrict__ Ch,
    const __bf16* __restrict__ Cl, const float* __restrict__ cc, int K, int nkt,
    int64_t rows_per_split, int xcd_map, MParam prm, float* __restrict__ part,
    float* __restrict__ part_ws, int KP) {
  constexpr int TP = 64;                  // points per LDS tile (two 32-point sub-tiles)
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 16;
  constexpr int HALF = DP / 2;
  constexpr int NDT = DP / 32;            // 32-feature output tiles
  constexpr int IMG = TP * DP * 2;        // bytes of one hi (or lo) image
  constexpr int NT = WAVES * 64;
  static_assert(WAVES == 4 || WAVES == 8, "4 or 8 waves");
  static_assert(!STAG || WAVES == 8, "the stagger pairs the two waves of a SIMD");
  static_assert(!ONE || WAVES == 8, "one-product form: 8 waves");
  // tile images: xh, then xl (bf16x3 distances, or W^T X's lo operand), then xr (RAW)
  constexpr int NIMG = (RAW && !ONE) ? 3 : 2;
  // STAG: a 4-slot tile ring with two tiles in flight (tile it + 2 loads while tile it
  // computes and tile it - 1 finishes its lagging W^T X): one interval's work (~1.8K cycles
  // per SIMD) is shorter than a 32-KB tile's DMA latency under load.  The row statistics
  // then arrive by LDS-DMA too (no register staging to wait on), the zero floor is taken
  // of xx in the membership step, and a partial last tile's padded rows are patched in LDS
  // after their DMA lands.
  // (the bf16x3 8-wave form measured the same with a 3-slot ring of this kind -- 16.6 vs
  // 16.2-16.8 ms, profiles/bench_fcm10m_x3_r05r.json.log -- and spilled 7 VGPRs: it keeps
  // its double buffer with register-staged statistics)
  constexpr bool RING = STAG;
  constexpr int NBUF = STAG ? 4 : 2;
  constexpr int SXB = NBUF * NIMG * IMG;
  // row statistics per tile row: xx, 1/S, (non-STAG: the zero floor 2^-16 xx,) + (ONE)
  // d2a, d2b, la, lb
  constexpr int RSF = RING ? 2 : 3;       // index of d2a
  constexpr int NRS = ONE ? RSF + 4 : (RING ? 2 : 3);
  __shared__ __attribute__((aligned(16))) char s_xf[SXB];
#define s_x(B_) (s_xf + (B_) * NIMG * IMG)
  __shared__ __attribute__((aligned(16))) float s_rs[NBUF][NRS][TP];
  __shared__ __attribute__((aligned(16))) float s_rsdummy[RING ? TP : 1];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  // XCD-aware order: the K tiles of one row range are consecutive on one XCD
  int64_t L = blockIdx.x;
  if (xcd_map) {
    const int64_t per = (int64_t)gridDim.x / 8;
    L = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const int kt = (int)(L % nkt);
  const int64_t split = L / nkt;
  const int64_t a = split * rows_per_split;
  const int64_t b = min(N, a + rows_per_split);
  const int cg = w & 3;                   // centroid group
  const int kw = kt * 128 + cg * 32;      // this wave's 32 centroids
  const int kc = kw + r;                  // this lane's centroid (column of the distances)

  bf16x8 ch[KS], cl[KS];
  float ccl;
  {
    const bf16x8* sh = reinterpret_cast<const bf16x8*>(Ch + (int64_t)kc * DP + h * HALF);
    const bf16x8* sl = reinterpret_cast<const bf16x8*>(Cl + (int64_t)kc * DP + h * HALF);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      ch[kk] = sh[kk];
      if constexpr (!ONE) cl[kk] = sl[kk];
    }
    ccl = cc[kc];
  }

  const bf16x2 ONES2 = {(__bf16)1.0f, (__bf16)1.0f};
  f32x16 out[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) out[dt][i] = 0.f;
  float wsum = 0.f;

  // X tiles arrive by LDS-DMA (as the stats pass's centroid stages): source-side XOR
  // swizzle (xoff is an involution in the chunk index), rows past the range clamped to its
  // last row through the per-lane offset, inline asm in the saddr + voffset form.  Only
  // the 2 x 64 row statistics still go through registers (padded rows get special
  // values).
  constexpr int PPI = IMG / 1024;               // 1-KiB pieces per (hi or lo) image
  constexpr int PPW = NIMG * PPI / WAVES;       // pieces per wave per tile
  static_assert(IMG % 1024 == 0 && (NIMG * PPI) % WAVES == 0, "tile pieces");
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave index in SGPRs (DMA destinations)
  int prow[PPW];
  unsigned pcol[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int q = ((w * PPW + i) % PPI) * 64 + lane;  // destination chunk in the image
    prow[i] = q / CPR;
    pcol[i] = (unsigned)(xoff<DP>(prow[i], q % CPR) - prow[i] * DP * 2);  // = source chunk
  }
  const unsigned lds_x = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)&s_xf[0];
  const unsigned lds_rs = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)&s_rs[0][0][0];
  const unsigned lds_dummy = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)&s_rsdummy[0];
  float pv = 0.f;
#define TDC_TILE_LOAD(R0_, B_)                                                            \
  {                                                                                       \
    const int last_ = (int)(b - 1 - (R0_));                                               \
    _Pragma("unroll") for (int i = 0; i < PPW; ++i) {                                     \
      const int pc_ = wu * PPW + i;                                                       \
      const int im_ = pc_ / PPI;                                                          \
      const __bf16* base_ = (im_ == 0 ? Xh : (im_ == 1 ? Xl : Xr)) + (R0_) * DP;          \
      const int rr_ = prow[i] < last_ ? prow[i] : last_;                                  \
      const unsigned dst_ = lds_x + (B_) * NIMG * IMG + im_ * IMG + (pc_ % PPI) * 1024;   \
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"                  \
                   :: "s"(__builtin_amdgcn_readfirstlane(dst_)),                          \
                      "v"((unsigned)(rr_ * DP * 2) + pcol[i]), "s"(uniform_ptr(base_))    \
                   : "memory", "m0");                                                     \
    }                                                                                     \
    if (tid < NRS * TP) {                                                                 \
      /* wave w loads statistic w of the tile's rows; padded rows: a huge norm keeps t   \
         finite (rcp(0) * info 0 would be NaN), no fix-up centroid */                    \
      const int64_t gr = (R0_) + lane;                                                    \
      if (w == 0 || w == 2) {                                                             \
        pv = gr < b ? xx[gr] : 1.0e30f;                                                   \
        if (w == 2) pv *= ZERO_FLOOR;                                                     \
      } else if (w == 1) pv = gr < b ? rowinfo[gr] : 0.f;                                 \
      else pv = gr < b ? fix[gr * 4 + (w - 3)] : (w >= 5 ? __int_as_float(-1) : 0.f);     \
    }                                                                                     \
  }
  // STAG: images and statistics of one tile by LDS-DMA, VPS = PPW + 1 per wave: wave w < NRS
  // brings statistic w of the 64 rows (rows past the range clamped, patched later); the
  // others a dummy copy into scratch, so every wave's vmcnt count is the same
  constexpr int VPS = PPW + 1;
#define TDC_TILE_DMA(R0_, B_)                                                             \
  {                                                                                       \
    const int last_ = (int)(b - 1 - (R0_));                                               \
    _Pragma("unroll") for (int i = 0; i < PPW; ++i) {                                     \
      const int pc_ = wu * PPW + i;                                                       \
      const int im_ = pc_ / PPI;                                                          \
      const __bf16* base_ = (im_ == 0 ? Xh : (im_ == 1 ? Xl : Xr)) + (R0_) * DP;          \
      const int rr_ = prow[i] < last_ ? prow[i] : last_;                                  \
      const unsigned dst_ = lds_x + (B_) * NIMG * IMG + im_ * IMG + (pc_ % PPI) * 1024;   \
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"                  \
                   :: "s"(__builtin_amdgcn_readfirstlane(dst_)),                          \
                      "v"((unsigned)(rr_ * DP * 2) + pcol[i]), "s"(uniform_ptr(base_))    \
                   : "memory", "m0");                                                     \
    }                                                                                     \
    {                                                                                     \
      /* (the dummy copies re-read xx: fix is null without the one-product form) */       \
      const int st_ = wu < NRS ? wu : 0;                                                  \
      const int lr_ = lane < last_ ? lane : last_;                                        \
      const float* sb_ = st_ == 0 ? xx + (R0_) : st_ == 1 ? rowinfo + (R0_)               \
                                                          : fix + (R0_) * 4 + (st_ - RSF); \
      const unsigned so_ = st_ < RSF ? (unsigned)lr_ * 4u : (unsigned)lr_ * 16u;           \
      const unsigned sd_ = wu < NRS ? lds_rs + ((B_) * NRS + wu) * TP * 4 : lds_dummy;    \
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, %2"                    \
                   :: "s"(__builtin_amdgcn_readfirstlane(sd_)), "v"(so_),                 \
                      "s"(uniform_ptr(sb_)) : "memory", "m0");                            \
    }                                                                                     \
  }
  // rows of a partial tile past the range: a huge norm keeps t finite (rcp(0) * info 0
  // would be NaN), no fix-up centroid (after this wave's own statistics DMA landed)
#define TDC_TILE_PATCH(R0_, B_)                                                           \
  if ((R0_) + TP > b && w < NRS) {                                                        \
    const int valid_ = (int)(b - (R0_));                                                  \
    if (lane >= valid_)                                                                   \
      s_rs[B_][w][lane] = w == 0 ? 1.0e30f : (w >= RSF + 2 ? __int_as_float(-1) : 0.f);   \
  }
#define TDC_TILE_STORE(B_)                                                                \
  {                                                                                       \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                      \
    if (tid < NRS * TP) s_rs[B_][w][lane] = pv;                                          \
  }
  if constexpr (RING) {
    // tiles 0 and 1 in flight, wait for tile 0 (every block has >= 1 tile: a < b)
    TDC_TILE_DMA(a, 0)
    TDC_TILE_DMA(a + TP < b ? a + TP : a, 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VPS) : "memory");
    TDC_TILE_PATCH(a, 0)
  } else if (a < b) {
    TDC_TILE_LOAD(a, 0)
    TDC_TILE_STORE(0)
  }
  __syncthreads();

  // transposed-read lane geometry (T10): group g, row q4, column quad p4
  const int g = lane >> 4, gi = lane & 15, q4 = gi >> 2, p4 = gi & 3;
  constexpr int EPK = 16 / KS;          // membership elements per distance k-step
  constexpr int EPW = 16 / (2 * NDT);   // membership elements per W^T X (s, dt) step
#define TDC_DIST(ACC, SUB, INTERLEAVE)                                                    \
  if constexpr (ONE) {                                                                    \
    /* one product: the A fragments read two k-steps ahead (an LDS read outlives one    \
       32-cycle MFMA; the registers of the lo fragments pay for the deeper ring) */     \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) ACC[i] = ccl;                         \
    const int prow = (SUB) * 32 + r;                                                      \
    bf16x8 af[KS];                                                                        \
    _Pragma("unroll") for (int kk = 0; kk < 2 && kk < KS; ++kk)                           \
      af[kk] = as_bf16x8(*reinterpret_cast<const uint4*>(xh + xoff<DP>(prow, h * (CPR / 2) + kk))); \
    _Pragma("unroll") for (int kk = 0; kk < KS; ++kk) {                                   \
      if (kk + 2 < KS)                                                                    \
        af[kk + 2] = as_bf16x8(*reinterpret_cast<const uint4*>(xh + xoff<DP>(prow, h * (CPR / 2) + kk + 2))); \
      ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk], ch[kk], ACC, 0, 0, 0);        \
      INTERLEAVE(kk * EPK, EPK)                                                           \
    }                                                                                     \
  } else {                                                                                \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) ACC[i] = ccl;                         \
    const int prow = (SUB) * 32 + r;                                                      \
    bf16x8 ah = as_bf16x8(*reinterpret_cast<const uint4*>(xh + xoff<DP>(prow, h * (CPR / 2)))); \
    bf16x8 al;                                                                            \
    if constexpr (!ONE) al = as_bf16x8(*reinterpret_cast<const uint4*>(xl + xoff<DP>(prow, h * (CPR / 2)))); \
    _Pragma("unroll") for (int kk = 0; kk < KS; ++kk) {                                   \
      const int kn = kk + 1 < KS ? kk + 1 : kk;                                           \
      const bf16x8 ahn = as_bf16x8(*reinterpret_cast<const uint4*>(xh + xoff<DP>(prow, h * (CPR / 2) + kn))); \
      bf16x8 aln;                                                                         \
      if constexpr (!ONE) aln = as_bf16x8(*reinterpret_cast<const uint4*>(xl + xoff<DP>(prow, h * (CPR / 2) + kn))); \
      ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, ch[kk], ACC, 0, 0, 0);            \
      if constexpr (!ONE) {                                                               \
        ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, cl[kk], ACC, 0, 0, 0);          \
        ACC = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, ch[kk], ACC, 0, 0, 0);          \
      }                                                                                   \
      INTERLEAVE(kk * EPK, EPK)                                                           \
      ah = ahn;                                                                           \
      if constexpr (!ONE) al = aln;                                                       \
    }                                                                                     \
  }
  // memberships of elements [I0, I0 + CNT) of half SUB (distances in ACC) -> WH
#define TDC_MEMB(ACC, WH, I0, CNT)                                                    \
  _Pragma("unroll") for (int q = 0; q < (CNT); ++q) {                                     \
    const int i = (I0) + q, g4 = i >> 2, e = i & 3;                                       \
    const float zf = ZERO_FLOOR * xq[g4][e];                                              \
    const float d2 = fmaxf(ACC[i] + xq[g4][e], zf);                                       \
    float u = mt<MODE>(d2, prm.expo) * iq[g4][e];                                         \
    if constexpr (!NZ) u = iq[g4][e] < 0.f ? (d2 <= zf ? 1.f : 0.f) : u;                  \
    const float wv = mw<MODE>(u, prm.m);                                                  \
    const __bf16 bhv = (__bf16)wv;                                                        \
    WH[i >> 3][i & 7] = bhv;                                                              \
    wsum += (float)bhv;  /* the rounded weight: each centroid an exact convex combination */ \
  }
#define TDC_LOADQ(SUB)                                                                    \
  _Pragma("unroll") for (int g4 = 0; g4 < 4; ++g4) {                                      \
    const int pt = (SUB) * 32 + 8 * g4 + 4 * h;                                           \
    xq[g4] = *reinterpret_cast<const f32x4*>(&s_rs[buf][0][pt]);                          \
    iq[g4] = *reinterpret_cast<const f32x4*>(&s_rs[buf][1][pt]);                          \
  }
  // W^T X of half SUB (weights WH): A = W (row = centroid, k = points), B = X^T via
  // transposed reads (T10); INTERLEAVE runs between the (s, dt) steps
#define TDC_TRLD(SUB, T_, H0, H1, L0, L1)                                                \
  {                                                                                       \
    const int s_ = (T_) / NDT, dt_ = (T_) % NDT;                                          \
    const int c0 = (dt_ * 32 + 16 * (g & 1)) >> 3;                                        \
    const int rA = (SUB) * 32 + 16 * s_ + 4 * (g >> 1) + q4;                              \
    const int oA = xoff<DP>(rA, c0 + (p4 >> 1)) + 8 * (p4 & 1);                           \
    const int oB = xoff<DP>(rA + 8, c0 + (p4 >> 1)) + 8 * (p4 & 1);                       \
    if constexpr (!RAW) {                                                                 \
      H0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xh + oA));                \
      H1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xh + oB));                \
    }                                                                                     \
    L0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xw + oA));                  \
    L1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xw + oB));                  \
  }
  // W^T X of half SUB (weights WH, bf16): A = W (row = centroid, k = points), B = X^T hi and
  // lo via transposed reads (T10), prefetched one (s, dt) step ahead; INTERLEAVE runs between
#define TDC_WTX(SUB, WH, INTERLEAVE, LAST)                                            \
  if constexpr (RAW) {                                                                    \
    /* one product per (s, dt) step: the transposed reads run three steps ahead */       \
    constexpr int NSTEP = 2 * NDT, PFW = 3;                                               \
    s16x4 lr0[NSTEP], lr1[NSTEP], hdum0, hdum1;                                           \
    _Pragma("unroll") for (int t = 0; t < PFW && t < NSTEP; ++t)                          \
      TDC_TRLD(SUB, t, hdum0, hdum1, lr0[t], lr1[t])                                      \
    _Pragma("unroll") for (int t = 0; t < NSTEP; ++t) {                                   \
      if (t + PFW < NSTEP) TDC_TRLD(SUB, t + PFW, hdum0, hdum1, lr0[t + PFW], lr1[t + PFW]) \
      const int s = t / NDT, dt = t % NDT;                                                \
      const bf16x8 xb = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lr0[t], lr1[t], 0, 1, 2, 3, 4, 5, 6, 7)); \
      if (t + 1 == NSTEP) { LAST }                                                        \
      out[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(WH[s], xb, out[dt], 0, 0, 0);     \
      INTERLEAVE(t * EPW, EPW)                                                            \
    }                                                                                     \
  } else {                                                                                \
    s16x4 h0, h1, l0, l1;                                                                 \
    TDC_TRLD(SUB, 0, h0, h1, l0, l1)                                                      \
    _Pragma("unroll") for (int t = 0; t < 2 * NDT; ++t) {                                 \
      s16x4 nh0, nh1, nl0, nl1;                                                           \
      if (t + 1 < 2 * NDT) TDC_TRLD(SUB, t + 1, nh0, nh1, nl0, nl1)                       \
      const int s = t / NDT, dt = t % NDT;                                                \
      bf16x8 xbh;                                                                         \
      if constexpr (!RAW) xbh = __builtin_bit_cast(bf16x8, __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7)); \
      const bf16x8 xbl = __builtin_bit_cast(bf16x8, __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7)); \
      if (t + 1 == 2 * NDT) { LAST }                                                      \
      if constexpr (!RAW)                                                                 \
        out[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(WH[s], xbh, out[dt], 0, 0, 0);  \
      out[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(WH[s], xbl, out[dt], 0, 0, 0);    \
      INTERLEAVE(t * EPW, EPW)                                                            \
      if (t + 1 < 2 * NDT) { h0 = nh0; h1 = nh1; l0 = nl0; l1 = nl1; }                   \
    }                                                                                     \
  }
#define TDC_NONE(I0, CNT)
#define TDC_MEMB0(I0, CNT) TDC_MEMB(acc0, wh0, I0, CNT)
#define TDC_MEMB1(I0, CNT) TDC_MEMB(acc1, wh1, I0, CNT)
  // the 8-wave membership step of half SUB: row statistics read from LDS buffer B_ per group
  // of 4 elements (no xq/iq arrays live across the distance MFMAs: the 2-wave register
  // budget is 256)
#define TDC_MEMB8(ACC, WH, SUB, B_)                                                       \
  _Pragma("unroll") for (int g4 = 0; g4 < 4; ++g4) {                                      \
    const int pt = (SUB) * 32 + 8 * g4 + 4 * h;                                           \
    const f32x4 xq4 = *reinterpret_cast<const f32x4*>(&s_rs[B_][0][pt]);                  \
    const f32x4 iq4 = *reinterpret_cast<const f32x4*>(&s_rs[B_][1][pt]);                  \
    f32x4 zf4;                                                                            \
    if constexpr (RING) zf4 = xq4 * ZERO_FLOOR;                                           \
    else zf4 = *reinterpret_cast<const f32x4*>(&s_rs[B_][2][pt]);                         \
    f32x4 da4, db4;                                                                       \
    i32x4 la4, lb4;                                                                       \
    if constexpr (ONE) {                                                                  \
      da4 = *reinterpret_cast<const f32x4*>(&s_rs[B_][RSF][pt]);                          \
      db4 = *reinterpret_cast<const f32x4*>(&s_rs[B_][RSF + 1][pt]);                      \
      la4 = *reinterpret_cast<const i32x4*>(&s_rs[B_][RSF + 2][pt]);                      \
      lb4 = *reinterpret_cast<const i32x4*>(&s_rs[B_][RSF + 3][pt]);                      \
    }                                                                                     \
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                       \
      const int i = 4 * g4 + e;                                                           \
      const float zf = zf4[e];                                                            \
      /* the floor as an int32 max (zf >= 0; fmaxf canonicalised the LDS operand) */     \
      float d2 = __int_as_float(max(__float_as_int(ACC[i] + xq4[e]), __float_as_int(zf))); \
      if constexpr (ONE) {                                                                \
        d2 = kc == la4[e] ? da4[e] : d2;                                                  \
        d2 = kc == lb4[e] ? db4[e] : d2;                                                  \
      }                                                                                   \
      float u = mt<MODE>(d2, prm.expo) * iq4[e];                                          \
      if constexpr (!NZ) u = iq4[e] < 0.f ? (d2 <= zf ? 1.f : 0.f) : u;                   \
      const float wv = mw<MODE>(u, prm.m);                                                \
      const __bf16 bhv = (__bf16)wv;                                                      \
      WH[i >> 3][i & 7] = bhv;                                                            \
      /* the rounded weights summed a pair at a time (v_dot2c with (1, 1)) */            \
      if (e & 1) {                                                                        \
        const bf16x2 pr_ = {WH[i >> 3][(i & 7) - 1], bhv};                                \
        /* (inline asm: the builtin with a constant (1, 1) is folded back into two      \
           converts and two adds) */                                                      \
        asm("v_dot2c_f32_bf16 %0, %1, %2" : "+v"(wsum) : "v"(pr_), "v"(ONES2));          \
      }                                                                                   \
    }                                                                                     \
  }
  if constexpr (STAG) {
    // interval it: tile it in slot it % 4 (landed at the end of interval it - 1), tile
    // it - 1 (the lagging waves' memberships and W^T X) in slot (it + 3) % 4, tile it + 1
    // landing, tile it + 2 loading into the slot tile it - 2 left
    const int sub = w >> 2;
    const int64_t ntile = (b - a + TP - 1) / TP;
    f32x16 acc0;
    bf16x8 wh0[2];
    for (int64_t it = 0; it <= ntile; ++it) {
      const bool cur = it < ntile;
      const int bc = (int)(it & 3), bp = (int)((it + 3) & 3), bl2 = (int)((it + 2) & 3);
      {
        // (past the end: the last tile again into the free slot -- uniform DMA counts)
        const int64_t t2 = it + 2 < ntile ? it + 2 : ntile - 1;
        TDC_TILE_DMA(a + t2 * TP, bl2)
      }
      const char* xh_c = s_x(bc);
      const char* xl_c = s_x(bc) + IMG;
      const char* xw_c = s_x(bc) + (NIMG - 1) * IMG;
      const char* xw_p = s_x(bp) + (NIMG - 1) * IMG;
      if (sub == 0) {
        if (cur) {
          const char* xh = xh_c;
          const char* xl = xl_c;
          const char* xw = xw_c;
          TDC_DIST(acc0, 0, TDC_NONE)
          TDC_MEMB8(acc0, wh0, 0, bc)
          TDC_WTX(0, wh0, TDC_NONE, )
        }
      } else {
        if (it > 0) {
          // (W^T X reads xh only without RAW, when the tile is [xh | xl])
          const char* xh = s_x(bp);
          const char* xl = xw_p;
          const char* xw = xw_p;
          TDC_MEMB8(acc0, wh0, 1, bp)
          TDC_WTX(1, wh0, TDC_NONE, )
        }
        if (cur) {
          const char* xh = xh_c;
          const char* xl = xl_c;
          const char* xw = xw_c;
          TDC_DIST(acc0, 1, TDC_NONE)
        }
      }
      // tile it + 1 landed (only tile it + 2's DMAs may still be in flight)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VPS) : "memory");
      if (it + 1 < ntile) TDC_TILE_PATCH(a + (it + 1) * TP, (int)((it + 1) & 3))
      __syncthreads();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the reloads past the end
    __syncthreads();
  } else {
  {
  int buf = 0;
  for (int64_t r0 = a; r0 < b; r0 += TP) {
    const bool more = r0 + TP < b;
    // buffer buf ^ 1 was last read in the previous tile, before its barrier
    if (more) TDC_TILE_LOAD(r0 + TP, buf ^ 1)
    const char* xh = s_x(buf);
    const char* xl = s_x(buf) + IMG;
    const char* xw = s_x(buf) + (NIMG - 1) * IMG;
    // Software pipeline over the two 32-point halves, written out explicitly so that the
    // membership VALU of one half issues between the MFMAs of the other (one wave per
    // SIMD: nothing else hides it):
    //   dist(0) | dist(1) + memberships(0) | W^T X(0) + memberships(1) | W^T X(1)
    f32x16 acc0, acc1;
    bf16x8 wh0[2], wh1[2];
    f32x4 xq[4], iq[4];
    if constexpr (WAVES == 4) {
      TDC_DIST(acc0, 0, TDC_NONE)
      TDC_LOADQ(0)
      TDC_DIST(acc1, 1, TDC_MEMB0)
      TDC_LOADQ(1)
      TDC_WTX(0, wh0, TDC_MEMB1, )
      TDC_WTX(1, wh1, TDC_NONE, )
    } else {
      const int sub = w >> 2;
      TDC_DIST(acc0, sub, TDC_NONE)
      TDC_MEMB8(acc0, wh0, sub, buf)
      // early tile release: the tile's last transposed X reads are in registers, so the
      // next tile's row statistics and the barrier go before the last three W^T X MFMAs,
      // which then run under the next tile's first LDS reads (fcm10m -0.5 %)
      TDC_WTX(sub, wh0, TDC_NONE, { if (more) TDC_TILE_STORE(buf ^ 1) __syncthreads(); })
    }
    if (WAVES == 4) {
      if (more) TDC_TILE_STORE(buf ^ 1)
      __syncthreads();
    }
    buf ^= 1;
  }
  }
  }
#undef TDC_NONE
#undef TDC_MEMB0
#undef TDC_MEMB1
#undef TDC_DIST
#undef TDC_MEMB
#undef TDC_LOADQ
#undef TDC_WTX
#undef TDC_TRLD
#undef TDC_MEMB8
#undef TDC_TILE_LOAD
#undef TDC_TILE_STORE

  if constexpr (WAVES == 8) {
    // the point-half-1 waves hand their W^T X partials (and column sums) to the half-0
    // waves of the same centroid group through the (now idle) tile buffers
    static_assert(4 * 32 * DP * 4 <= SXB, "exchange fits the tile buffers");
    float* xo = reinterpret_cast<float*>(&s_xf[0]) + cg * 32 * DP;
    float* xw = &s_rs[0][0][0] + cg * 32;
    __syncthreads();
    const float wpair = wsum + __shfl_xor(wsum, 32, 64);  // all lanes take part in the swap
    if (w >= 4) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) xo[(i * NDT + dt) * 64 + lane] = out[dt][i];
      if (h == 0) xw[r] = wpair;
    }
    __syncthreads();
    if (w >= 4) return;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) out[dt][i] += xo[(i * NDT + dt) * 64 + lane];
    wsum += (h == 0) ? xw[r] : 0.f;
  }
  // ---- slab: out rows (registers) = centroids kw + (i&3)+8(i>>2)+4h, lane = feature ----
  float* slab = part + split * (int64_t)KP * DP;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = kw + (i & 3) + 8 * (i >> 2) + 4 * h;
      slab[(int64_t)k * DP + dt * 32 + r] = out[dt][i];
    }
  }
  wsum += __shfl_xor(wsum, 32, 64);
  if (h == 0) part_ws[split * (int64_t)KP + kc] = wsum;
}

// wx[k, d] += sum_s part[s, k, d] + mu[d] sum_s part_ws[s, k] (fp64: the slabs hold
// sum w (x - mu) of the shifted rows), ws[k] += sum_s part_ws[s, k]
__global__ __launch_bounds__(256) void fcm_reduce_kernel(const float* __restrict__ part,
                                                         const float* __restrict__ part_ws,
                                                         int64_t splits, int K, int KP, int DP,
                                                         int D, const float* __restrict__ mu,
                                                         double* __restrict__ wx,
                                                         double* __restrict__ ws) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t tot = (int64_t)K * DP;
  if (e < tot) {
    const int k = (int)(e / DP), d = (int)(e % DP);
    if (d < D) {
      double s = 0.0, w = 0.0;
      for (int64_t sp = 0; sp < splits; ++sp) {
        s += (double)part[(sp * KP + k) * (int64_t)DP + d];
        w += (double)part_ws[sp * KP + k];
      }
      wx[(int64_t)k * D + d] += s + (mu ? (double)mu[d] * w : 0.0);
    }
  } else if (e < tot + K) {
    const int k = (int)(e - tot);
    double s = 0.0;
    for (int64_t sp = 0; sp < splits; ++sp) s += (double)part_ws[sp * KP + k];
    ws[k] += s;
  }
}

// ---------------------------------------------------------------------------------------
// operand prep: rows of fp32 [rows, ld] (d valid columns) -> hi/lo bf16 [rows, DP] (+ norm)
// neg2: centroids (hi/lo of -2c, norm of c); pad rows (>= valid) are zero, norm 0
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ src, int64_t rows,
                                                         int64_t valid, int d, int64_t ld, int DP,
                                                         int neg2, const float* __restrict__ shift,
                                                         __bf16* __restrict__ hi,
                                                         __bf16* __restrict__ lo,
                                                         float* __restrict__ norm) {
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * 4) {
    float s = 0.f;
    for (int c = lane; c < DP; c += 64) {
      const float v = (row < valid && c < d) ? src[row * ld + c] - (shift ? shift[c] : 0.f) : 0.f;
      s = fmaf(v, v, s);
      const float t = neg2 ? -2.f * v : v;
      const __bf16 vh = (__bf16)t;
      const __bf16 vl = (__bf16)(t - (float)vh);
      hi[row * DP + c] = vh;
      lo[row * DP + c] = vl;
    }
    s = wave_sum(s);
    // centroid pad rows: a huge norm keeps their distances (and memberships) negligible
    if (lane == 0 && norm) norm[row] = (neg2 && row >= valid) ? 1.0e30f : s;
  }
}

MParam make_mparam(double m, int nz) {
  MParam p;
  p.expo = (float)(-1.0 / (m - 1.0));
  p.m = (float)m;
  p.pmode = fcm_pmode(m);
  p.mint = fcm_mint(m);
  p.nz = nz;
  return p;
}

template <int DP>
int launch_mstats(const void* Xh, const void* Xl, const float* xx, int64_t N, const void* Ch,
                  const void* Cl, const float* cc, int K, int Kp, double m, int nz,
                  int32_t* labels, float* rowinfo, float* fix, hipStream_t s) {
  constexpr int WAVES = 8;
  const int64_t blocks = (N + WAVES * 32 - 1) / (WAVES * 32);
  const MParam p = make_mparam(m, nz);
#define TDC_LS(MODE)                                                                          \
  hipLaunchKernelGGL((fcm_mfma_stats_kernel<DP, MODE, WAVES>), dim3((unsigned)blocks), dim3(WAVES * 64), 0, s, \
                     (const __bf16*)Xh, (const __bf16*)Xl, xx, N, (const __bf16*)Ch,          \
                     (const __bf16*)Cl, cc, K, Kp / 64, p, labels, rowinfo)
#define TDC_LS1(MODE)                                                                         \
  hipLaunchKernelGGL((fcm_mfma_stats1_kernel<DP, MODE, WAVES>), dim3((unsigned)blocks), dim3(WAVES * 64), 0, s, \
                     (const __bf16*)Xh, (const __bf16*)Xl, xx, N, (const __bf16*)Ch,          \
                     (const __bf16*)Cl, cc, K, Kp / 64, p, labels, rowinfo, (float4*)fix)
  // one product + fix-up from DP = 64 (fcm10m 19.05 -> 18.60 ms, profiles/fcm_stats1_ab_r04m.txt)
  // only for the one-product form (fix rows requested): its row normaliser is wrong where a
  // third centroid sits within the one-product error of the nearest two (duplicate
  // centroids of a tight blob: sum w +55 % on clustered data, profiles/
  // fcm_bf16_witness_diag_it10_r06g.txt), so the bf16x3 form keeps bf16x3 in both passes;
  // at DP = 32 the bf16x3 kernel's 6 MFMAs per tile are not what bounds it
  bool done = false;
  if constexpr (DP >= 64) {
    if (fix) {
      if (m == 2.0) TDC_LS1(2); else TDC_LS1(0);
      done = true;
    }
  }
  if (!done) {
    if (m == 2.0) TDC_LS(2); else TDC_LS(0);
  }
#undef TDC_LS
#undef TDC_LS1
  TDC_CHECK_LAUNCH();
  return 0;
}

// row ranges of the accumulate pass: ~2 blocks per CU in total, whole 64-point tiles
inline void accum_geometry(int64_t N, int K, int num_cus, int* nkt, int64_t* splits, int64_t* rps) {
  *nkt = (K + 127) / 128;
  const int64_t tiles = (N + 63) / 64;
  int64_t sp = ((int64_t)num_cus * 2 + *nkt - 1) / *nkt;
  if (sp > tiles) sp = tiles;
  if (sp < 1) sp = 1;
  *rps = ((tiles + sp - 1) / sp) * 64;
  *splits = (N + *rps - 1) / *rps;
}

template <int DP>
int launch_maccum(const void* Xh, const void* Xl, const void* Xr, const float* xx,
                  const float* rowinfo, const float* fix, int64_t N, const void* Ch, const void* Cl, const float* cc, int K, int Kp,
                  int D, double m, int nz, float* part, const float* mu, double* wx, double* ws,
                  int num_cus, hipStream_t s) {
  int nkt;
  int64_t splits, rps;
  accum_geometry(N, K, num_cus, &nkt, &splits, &rps);
  const int64_t nb = splits * nkt;
  const int xcd = (nb % 8 == 0) ? 1 : 0;
  float* part_ws = part + splits * (int64_t)Kp * DP;
  const MParam p = make_mparam(m, nz);
  // 8 waves (2 per SIMD): one wave's epilogue VALU runs beside the other's MFMAs; the
  // one-wave software-pipelined WAVES=4 form measured slower (docs/PERF_NOTES.md)
  // The one-product form runs when the stats pass left its fix-up rows (DP >= 64), always
  // staggered (fcm10m 16.65 -> 16.02 ms, profiles/fcm10m_*_r05e.txt), with the raw bf16 rows
  // as the W^T X operand when the caller has them (Xr); the bf16x3 form keeps the lockstep
  // loop (staggered, its extra live registers spill: 17.7 -> 19.7 ms)
  // (one product + raw rows: the tile is [xh | xr], so xr rides in the second image slot)
  const bool one = DP >= 64 && fix;
  const void* X2 = (one && Xr) ? Xr : Xl;
#define TDC_LA(MODE, NZV, ST, ONEV, RAWV)                                                     \
  hipLaunchKernelGGL((fcm_mfma_accum_kernel<DP, MODE, NZV, 8, ST, ONEV, RAWV>),               \
                     dim3((unsigned)nb), dim3(512), 0, s, (const __bf16*)Xh,                   \
                     (const __bf16*)X2, xx, rowinfo, fix, N, (const __bf16*)Xr,                \
                     (const __bf16*)Ch, (const __bf16*)Cl, cc, K, nkt, rps, xcd, p, part,      \
                     part_ws, Kp)
#define TDC_LA2(MODE, NZV)                                                                    \
  if (one) {                                                                                  \
    if (Xr) TDC_LA(MODE, NZV, DP >= 64, DP >= 64, DP >= 64);                                  \
    else TDC_LA(MODE, NZV, DP >= 64, DP >= 64, false);                                        \
  } else if (Xr && DP >= 64) {                                                                \
    TDC_LA(MODE, NZV, false, false, DP >= 64);                                                \
  } else {                                                                                    \
    TDC_LA(MODE, NZV, false, false, false);                                                   \
  }
  if (m == 2.0) {
    if (nz) { TDC_LA2(2, true) } else { TDC_LA2(2, false) }
  } else {
    if (nz) { TDC_LA2(0, true) } else { TDC_LA2(0, false) }
  }
#undef TDC_LA2
#undef TDC_LA
  TDC_CHECK_LAUNCH();
  const int64_t tot = (int64_t)K * DP + K;
  // (raw rows: the slabs hold sum w x of the unshifted rows, nothing to add back)
  hipLaunchKernelGGL(fcm_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, part,
                     part_ws, splits, K, Kp, DP, D, (Xr && DP >= 64) ? nullptr : mu, wx, ws);
  TDC_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------------------
// Wide D (DP = 256 ... 1024, multiples of 128): the tower's operands no longer fit a wave's
// registers (a 32-point hi/lo fragment set is DP/2 VGPRs, the [32 x DP] W^T X tile DP/2
// accumulators), so the wide path runs over row chunks with the [rows, K] block in HBM,
// like fcm_wide.hip, but both products on the matrix cores (the same hi/lo bf16 split):
//   wide_dist : G[r, k] = ||x||^2 + ||c||^2 + x.(-2c)  (3 MFMAs per product), a point within
//               2^-16 ||x||^2 of a centroid stored as exactly 0 (fcm_wide_rows' on-centroid
//               rule), 128-point x 128-centroid tiles, 32-feature hi/lo stages by LDS-DMA
//   (fcm_wide_rows turns d2 into w = u^m in place, csrc/fcm_wide.hip)
//   wide_wtx  : W^T X of 128-centroid x 128-feature output tiles over a row range: the W
//               stage (fp32 w -> bf16, column sums of the rounded w) goes through registers into row-major LDS
//               images, X hi/lo by LDS-DMA; both MFMA operands come from transposed reads
//               (ds_read_b64_tr_b16), so neither needs a transposed copy in HBM
// ---------------------------------------------------------------------------------------
constexpr int WT = 128;  // tile edge (points / centroids / features)

// 64-byte rows (32 bf16 features) of a stage image: chunk c of row r at 16 (c ^ ((r>>2)&3))
// -- every ds_read_b128 lane group of the 32x32x16 operand read is conflict-free
__device__ __forceinline__ int w64off(int r, int c) { return r * 64 + 16 * (c ^ ((r >> 2) & 3)); }
// 256-byte rows (128 bf16): the row/transpose dual-use image (b) of the guide (T10)
__device__ __forceinline__ int w256off(int r, int c) {
  return r * 256 + 16 * (c ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

// G [M, K] fp32 for the M rows of the chunk (grid: M/128 x Kp/128 tiles, XCD-grouped so the
// centroid tiles of one row tile share an L2).  4 waves, wave (wr, wc) owns points
// wr*64 + [0, 64) x centroids wc*64 + [0, 64): 2 x 2 MFMA tiles of 32x32.
__global__ __launch_bounds__(256, 2) void fcm_wide_dist_kernel(
    const __bf16* __restrict__ Xh, const __bf16* __restrict__ Xl, const float* __restrict__ xx,
    int64_t M, int DP, const __bf16* __restrict__ Ch, const __bf16* __restrict__ Cl,
    const float* __restrict__ cc, int K, int nct, float* __restrict__ G, int zfloor) {
  constexpr int IMG = WT * 64;          // one (hi or lo, X or C) 32-feature stage image
  constexpr int STAGE = 4 * IMG;        // Xh | Xl | Ch | Cl
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  __shared__ float s_xn[WT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int wr = w >> 1, wc = w & 1;
  int64_t L = blockIdx.x;
  {  // XCD-aware order: consecutive work items (the centroid tiles of a row tile) on one XCD
    const int64_t per = (int64_t)gridDim.x / 8;
    if (per * 8 == (int64_t)gridDim.x) L = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const int ct = (int)(L % nct);
  const int64_t r0 = (L / nct) * WT;
  const int k0 = ct * WT;
  const int64_t ldb = (int64_t)DP * 2;  // row pitch in bytes (X and C alike)

  // LDS-DMA pieces: wave w loads image w (Xh, Xl, Ch, Cl) of every stage, 8 x 1 KiB pieces
  // of 16 rows; the swizzle is applied on the source side (w64off is an involution in c)
  unsigned voff[8];
  const int last = (int)min((int64_t)WT - 1, M - 1 - r0);  // X rows past the chunk: clamped
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int row = p * 16 + (lane >> 2), cs = lane & 3;
    const int rr = (w < 2 && row > last) ? last : row;
    voff[p] = (unsigned)(rr * ldb + 16 * (cs ^ ((row >> 2) & 3)));
  }
  const __bf16* src0 = w == 0 ? Xh + r0 * DP : w == 1 ? Xl + r0 * DP
                     : w == 2 ? Ch + (int64_t)k0 * DP : Cl + (int64_t)k0 * DP;
  const char* srcb = reinterpret_cast<const char*>(uniform_ptr(src0));
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    const char* base = srcb + (int64_t)st * 64;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const unsigned dst = lds0 + buf * STAGE + wu * IMG + p * 1024;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff[p]), "s"(base)
                   : "memory", "m0");
    }
  };
  const int nst = DP / 32;
  issue(0, 0);
  if (tid < WT) s_xn[tid] = (r0 + tid < M) ? xx[r0 + tid] : 0.f;

  // accumulators start at ||x||^2 + ||c||^2 (registers: points, lanes: centroids)
  f32x16 acc[2][2];
  __syncthreads();  // s_xn
#pragma unroll
  for (int tj = 0; tj < 2; ++tj) {
    const float cn = cc[k0 + wc * 64 + tj * 32 + r];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 xn4 = *reinterpret_cast<const f32x4*>(&s_xn[wr * 64 + ti * 32 + 8 * g4 + 4 * h]);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[ti][tj][4 * g4 + e] = xn4[e] + cn;
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // fragment addresses: row R (point or centroid), k16 step s, half h -> chunk 2s + h
  const int xr = (r >> 2) & 3;
  unsigned ao[2][2], bo[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      ao[t][st] = lds0 + 0 * IMG + (wr * 64 + t * 32 + r) * 64 + 16 * ((2 * st + h) ^ xr);
      bo[t][st] = lds0 + 2 * IMG + (wc * 64 + t * 32 + r) * 64 + 16 * ((2 * st + h) ^ xr);
    }
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) issue(st + 1, buf ^ 1);
    const unsigned bo_ = buf * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(ah[t]) : "v"(ao[t][ks] + bo_));
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(al[t]) : "v"(ao[t][ks] + bo_), "i"(IMG));
        asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(bh[t]) : "v"(bo[t][ks] + bo_));
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bl[t]) : "v"(bo[t][ks] + bo_), "i"(IMG));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ti], bh[tj], acc[ti][tj], 0, 0, 0);
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[ti], bl[tj], acc[ti][tj], 0, 0, 0);
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[ti], bh[tj], acc[ti][tj], 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage st + 1 landed (this wave's part)
    __syncthreads();
  }
  // epilogue: lanes = centroids (coalesced 128-B row segments), registers = points
#pragma unroll
  for (int tj = 0; tj < 2; ++tj) {
    const int k = k0 + wc * 64 + tj * 32 + r;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int pr = wr * 64 + ti * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        const int64_t row = r0 + pr;
        if (row < M && k < K) {
          const float d2 = acc[ti][tj][i];
          G[row * (int64_t)K + k] = (zfloor && d2 <= ZERO_FLOOR * s_xn[pr]) ? 0.f : d2;
        }
      }
  }
}

// part[split, k, d] (+ part_ws[split, k] from the feature-tile-0 blocks) of
// sum_{rows of the split} w[r, k] x[r, d]; reduced by fcm_reduce_kernel
__global__ __launch_bounds__(256, 2) void fcm_wide_wtx_kernel(
    const float* __restrict__ W, const __bf16* __restrict__ Xh, const __bf16* __restrict__ Xl,
    int64_t M, int DP, int K, int Kp, int nkt, int ndt, int64_t rows_per_split,
    float* __restrict__ part, float* __restrict__ part_ws) {
  constexpr int RS = 32;                 // data rows per stage (two k16 steps)
  constexpr int IMG = RS * 256;          // one [32 rows x 128] bf16 image
  constexpr int STAGE = 3 * IMG;         // W (bf16) | Xh | Xl
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  int64_t L = blockIdx.x;
  {
    const int64_t per = (int64_t)gridDim.x / 8;
    if (per * 8 == (int64_t)gridDim.x) L = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const int kt = (int)(L % nkt);
  const int dt = (int)((L / nkt) % ndt);
  const int64_t split = L / ((int64_t)nkt * ndt);
  const int k0 = kt * WT, d0 = dt * WT;
  const int64_t a = split * rows_per_split;
  const int64_t b = min(M, a + rows_per_split);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- W stage through registers: thread -> data row tid/8, centroids 16 (tid%8) + [0,16)
  const int wrow = tid >> 3, wcol = (tid & 7) * 16;
  const bool kin = k0 + wcol < K;        // K % 16 == 0 is not required: per-element below
  float4 wv[4];
  float wsum[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) wsum[e] = 0.f;
  auto wload = [&](int64_t rb) __attribute__((always_inline)) {
    const int64_t row = rb + wrow;
    const bool ok = row < b;
    const float* src = W + (ok ? row : a) * (int64_t)K + k0 + wcol;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok && kin) {
        if ((K & 3) == 0 && k0 + wcol + 16 <= K) v = *reinterpret_cast<const float4*>(src + 4 * q);
        else {
          float t[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = (k0 + wcol + 4 * q + e < K) ? src[4 * q + e] : 0.f;
          v = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
      wv[q] = v;
    }
  };
  // W rounded to bf16 (RNE), the column sums taken of the same rounded weights: each
  // centroid is an exact convex combination (as the register tower, fcm_mfma_accum_kernel)
  auto wstore = [&](int buf) __attribute__((always_inline)) {
    bf16x8 hv[2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float f[4] = {wv[q].x, wv[q].y, wv[q].z, wv[q].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = 4 * q + e;
        const __bf16 hb = (__bf16)f[e];
        hv[j >> 3][j & 7] = hb;
        wsum[j] += (float)hb;
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int off = w256off(wrow, (wcol >> 3) + c);
      *reinterpret_cast<bf16x8*>(smem + buf * STAGE + off) = hv[c];
    }
  };
  // ---- X stage by LDS-DMA: waves 0-1 load Xh pieces, 2-3 Xl; 4 pieces of 4 rows each
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int ximg = wu >> 1;              // 0: Xh, 1: Xl
  unsigned xoffv[4];
  int xrow[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int row = ((w & 1) * 4 + p) * 4 + (lane >> 4), cs = lane & 15;
    xrow[p] = row;
    xoffv[p] = (unsigned)(16 * (cs ^ (((row & 3) << 2) | ((row >> 2) & 3))));
  }
  const char* xsrc = reinterpret_cast<const char*>(uniform_ptr(ximg ? Xl : Xh));
  auto xissue = [&](int64_t rb, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int pc = (wu & 1) * 4 + p;
      const unsigned dst = lds0 + buf * STAGE + (1 + ximg) * IMG + pc * 1024;
      int64_t row = rb + xrow[p];
      if (row >= b) row = b - 1;  // rows past the range: any valid row (their w is 0)
      const unsigned vo = (unsigned)((row - a) * (int64_t)DP * 2 + d0 * 2) + xoffv[p];
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(vo),
                      "s"(xsrc + a * (int64_t)DP * 2)
                   : "memory", "m0");
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[ti][tj][i] = 0.f;

  // transposed-read lane geometry (T10): group g, row q4, column quad p4
  const int g = lane >> 4, gi = lane & 15, q4 = gi >> 2, p4 = gi & 3;
  // per (operand tile t, k16 step s): byte offsets of the two 4-row blocks
  unsigned wo[2][2][2], xo[2][2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int rA = 16 * s + 4 * (g >> 1) + q4;
      const int cw = (wr * 64 + t * 32 + 16 * (g & 1)) >> 3;
      const int cx = (wc * 64 + t * 32 + 16 * (g & 1)) >> 3;
      wo[t][s][0] = lds0 + w256off(rA, cw + (p4 >> 1)) + 8 * (p4 & 1);
      wo[t][s][1] = lds0 + w256off(rA + 8, cw + (p4 >> 1)) + 8 * (p4 & 1);
      xo[t][s][0] = lds0 + IMG + w256off(rA, cx + (p4 >> 1)) + 8 * (p4 & 1);
      xo[t][s][1] = lds0 + IMG + w256off(rA + 8, cx + (p4 >> 1)) + 8 * (p4 & 1);
    }

  if (a < b) {
    wload(a);
    xissue(a, 0);
    wstore(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int buf = 0;
  for (int64_t rb = a; rb < b; rb += RS) {
    const bool more = rb + RS < b;
    if (more) {
      wload(rb + RS);
      xissue(rb + RS, buf ^ 1);
    }
    const unsigned bo_ = buf * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      s16x4 wh[2][2], xh[2][2], xl[2][2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          wh[t][q] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(wo[t][s][q] + bo_));
          xh[t][q] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(xo[t][s][q] + bo_));
          xl[t][q] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(xo[t][s][q] + bo_ + IMG));
        }
#pragma unroll
      for (int ti = 0; ti < 2; ++ti) {
        const bf16x8 ah = __builtin_bit_cast(bf16x8, __builtin_shufflevector(wh[ti][0], wh[ti][1], 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int tj = 0; tj < 2; ++tj) {
          const bf16x8 bh = __builtin_bit_cast(bf16x8, __builtin_shufflevector(xh[tj][0], xh[tj][1], 0, 1, 2, 3, 4, 5, 6, 7));
          const bf16x8 bl = __builtin_bit_cast(bf16x8, __builtin_shufflevector(xl[tj][0], xl[tj][1], 0, 1, 2, 3, 4, 5, 6, 7));
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc[ti][tj], 0, 0, 0);
          acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc[ti][tj], 0, 0, 0);
        }
      }
    }
    if (more) wstore(buf ^ 1);  // its previous contents were read before the last barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    buf ^= 1;
  }
  // ---- output: registers = centroids (i&3)+8(i>>2)+4h, lanes = features
  const int r = lane & 31, h = lane >> 5;
  float* slab = part + split * (int64_t)Kp * DP;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = k0 + wr * 64 + ti * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
        const int d = d0 + wc * 64 + tj * 32 + r;
        slab[(int64_t)k * DP + d] = acc[ti][tj][i];
      }
  if (dt == 0) {  // column sums of W: the 32 threads of one centroid group meet in LDS
    float* red = reinterpret_cast<float*>(smem);  // idle after the last barrier
#pragma unroll
    for (int e = 0; e < 16; ++e) red[wrow * WT + wcol + e] = wsum[e];
    __syncthreads();
    if (tid < WT) {
      float sacc = 0.f;
      for (int q = 0; q < RS; ++q) sacc += red[q * WT + tid];
      part_ws[split * (int64_t)Kp + k0 + tid] = sacc;
    }
  }
}

}  // namespace
}  // namespace tdc

using namespace tdc;

int tdc_fcm_split_rows(const float* src, int64_t rows, int64_t valid, int d, int64_t ld, int DP,
                       int neg2, const float* shift, void* hi, void* lo, float* norm,
                       hipStream_t s) {
  if (rows <= 0) return 0;
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(split_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, rows, valid,
                     d, ld, DP, neg2, shift, (__bf16*)hi, (__bf16*)lo, norm);
  TDC_CHECK_LAUNCH();
  return 0;
}

// wide-D row-chunk passes (see fcm_wide_dist_kernel): geometry of the W^T X partial slabs
static void wide_wtx_geometry(int64_t M, int Kp, int DP, int num_cus, int* nkt, int* ndt,
                              int64_t* splits, int64_t* rps) {
  *nkt = Kp / WT;
  *ndt = DP / WT;
  const int64_t tiles = (M + 31) / 32;
  const int64_t items = (int64_t)(*nkt) * (*ndt);
  int64_t sp = ((int64_t)num_cus * 2 + items - 1) / items;
  if (sp > tiles) sp = tiles;
  if (sp < 1) sp = 1;
  *rps = ((tiles + sp - 1) / sp) * 32;
  *splits = (M + *rps - 1) / *rps;
}

int64_t tdc_fcm_mfma_wide_workspace(int64_t M, int Kp, int DP, int num_cus) {
  int nkt, ndt;
  int64_t splits, rps;
  wide_wtx_geometry(M, Kp, DP, num_cus, &nkt, &ndt, &splits, &rps);
  return splits * (int64_t)Kp * (DP + 1);
}

int tdc_fcm_mfma_wide(int pass, const void* Xh, const void* Xl, const float* xx, int64_t M,
                      int DP, int D, const void* Ch, const void* Cl, const float* cc, int K,
                      int Kp, float* G, float* work, const float* shift, double* wx, double* ws,
                      int num_cus, hipStream_t s) {
  if (M <= 0 || K <= 0) return 0;
  if (DP % WT != 0 || DP < WT || DP > 1024 || Kp % WT != 0 || Kp < K || D > DP)
    return (int)hipErrorInvalidValue;
  if (pass == 0 || pass == 1) {
    // pass 1: raw d2 (no on-centroid floor) for the K-Means wide path (assign_x3.hip)
    const int nct = Kp / WT;
    const int64_t nb = ((M + WT - 1) / WT) * nct;
    hipLaunchKernelGGL(fcm_wide_dist_kernel, dim3((unsigned)nb), dim3(256), 0, s,
                       (const __bf16*)Xh, (const __bf16*)Xl, xx, M, DP, (const __bf16*)Ch,
                       (const __bf16*)Cl, cc, K, nct, G, pass == 0 ? 1 : 0);
    TDC_CHECK_LAUNCH();
    return 0;
  }
  if (pass != 2) return (int)hipErrorInvalidValue;
  int nkt, ndt;
  int64_t splits, rps;
  wide_wtx_geometry(M, Kp, DP, num_cus, &nkt, &ndt, &splits, &rps);
  float* part_ws = work + splits * (int64_t)Kp * DP;
  const int64_t nb = splits * nkt * ndt;
  hipLaunchKernelGGL(fcm_wide_wtx_kernel, dim3((unsigned)nb), dim3(256), 0, s, (const float*)G,
                     (const __bf16*)Xh, (const __bf16*)Xl, M, DP, K, Kp, nkt, ndt, rps, work,
                     part_ws);
  TDC_CHECK_LAUNCH();
  const int64_t tot = (int64_t)K * DP + K;
  hipLaunchKernelGGL(fcm_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, work,
                     part_ws, splits, K, Kp, DP, D, shift, wx, ws);
  TDC_CHECK_LAUNCH();
  return 0;
}

int64_t tdc_fcm_mfma_workspace(int64_t N, int K, int Kp, int DP, int num_cus) {
  int nkt;
  int64_t splits, rps;
  accum_geometry(N, K, num_cus, &nkt, &splits, &rps);
  return splits * (int64_t)Kp * (DP + 1);
}

int64_t tdc_fcm_mfma_rowinfo_len(int64_t N, int DP) {
  return DP >= 64 ? ((N + 3) / 4) * 4 + 4 * N : N;
}
int tdc_fcm_mfma(int pass, const void* Xh, const void* Xl, const void* Xr, const float* xx,
                 int64_t N, int DP, int D, const void* Ch, const void* Cl, const float* cc, int K,
                 int Kp, double m, int nan_to_zero, int32_t* labels, float* rowinfo,
                 int64_t rowinfo_len, double* wx, double* ws, float* work, const float* shift,
                 int num_cus, hipStream_t s) {
  if (N <= 0 || K <= 0) return 0;
  if (Kp % 128 != 0 || Kp < K) return (int)hipErrorInvalidValue;
  if (rowinfo_len < N) return (int)hipErrorInvalidValue;
  // the fix-up rows follow the [N] statistics (16-byte aligned) when the caller sized
  // rowinfo for them (tdc_fcm_mfma_rowinfo_len); without them the accumulate pass runs the
  // bf16x3 distances
  float* fix = (DP >= 64 && rowinfo_len >= tdc_fcm_mfma_rowinfo_len(N, DP))
                   ? rowinfo + ((N + 3) / 4) * 4 : nullptr;
#define TDC_FM(DPV)                                                                           \
  if (DP == DPV) {                                                                            \
    if (pass == 0)                                                                            \
      return launch_mstats<DPV>(Xh, Xl, xx, N, Ch, Cl, cc, K, Kp, m, nan_to_zero, labels,     \
                                rowinfo, fix, s);                                             \
    return launch_maccum<DPV>(Xh, Xl, Xr, xx, rowinfo, fix, N, Ch, Cl, cc, K, Kp, D, m,       \
                              nan_to_zero, work, shift, wx, ws, num_cus, s);                  \
  }
  TDC_FM(32)
  TDC_FM(64)
  TDC_FM(128)
#undef TDC_FM
  return (int)hipErrorInvalidValue;
}
