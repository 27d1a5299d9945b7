// Superseded bf16 MFMA assign variants, kept for the ablation harnesses in tools/
// (ablate_assign.hip): "v1" (register-staged centroid tiles, 32x32x16 MFMA) and "ring"
// (LDS-DMA ring without counted waits).  The library kernels are in
// csrc/assign_mfma_impl.h (ring2 for D=32, ring3 otherwise).  Build with -I csrc.
#pragma once
#include "assign_mfma_impl.h"

namespace tdc {

// ABL: ablation switches for tools/ablate_assign.hip (0 in the library):
//   1 = skip epilogue (accumulators kept live), 2 = skip next-stage staging,
//   4 = skip the per-stage barrier (timing only; results invalid), 8 = non-temporal X loads
template <int DP, int P, int ABL = 0>
__global__ __launch_bounds__(256, 2) void assign_mfma_bf16_kernel(
    const __bf16* __restrict__ X, int64_t N, int64_t ldx, const __bf16* __restrict__ Cm2,
    const float* __restrict__ cnorm, int ntiles, int32_t* __restrict__ labels,
    float* __restrict__ mind) {
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 16;
  constexpr int HALF = DP / 2;
  constexpr int STAGE = BN * DP;
  constexpr int CHUNKS = BN * CPR;
  constexpr int CPT = (CHUNKS + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 s_c[2 * STAGE];
  __shared__ __attribute__((aligned(16))) float s_n[2 * BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * (4 * P * 32) + (int64_t)w * (P * 32);

  // ---- point fragments: resident in VGPRs for the whole centroid loop ----
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
      // plain loads: non-temporal X loads measured 15-20 % slower (ablate_assign)
      if constexpr (ABL & 8) bq[p][kk] = __builtin_nontemporal_load(src + kk);
      else bq[p][kk] = src[kk];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = (float)bq[p][kk][j];
        s = fmaf(f, f, s);
      }
    }
    xn[p] = s + __shfl_xor(s, 32, 64);
  }

  // ---- centroid stage staging (global -> regs -> swizzled LDS) ----
  uint4 pre[CPT];
  float npre = 0.f;
  // stage 0 straight into buffer 0
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int q = tid + i * 256;
    if (CHUNKS % 256 == 0 || q < CHUNKS) {
      const int row = q / CPR, c = q % CPR;
      *reinterpret_cast<uint4*>(s_c + row * DP + swz<DP>(row, c) * 8) =
          *reinterpret_cast<const uint4*>(Cm2 + (int64_t)row * DP + c * 8);
    }
  }
  if (tid < BN) s_n[tid] = cnorm[tid];
  __syncthreads();

  float best[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = INFINITY;
    bt[p] = 0;
  }
  // Software pipeline over the two 32-centroid halves (q) of each 64-centroid stage:
  //   phase 1 of stage t: MFMAs of q=0 into acc0  ||  epilogue of acc1 (stage t-1, q=1)
  //   phase 2 of stage t: MFMAs of q=1 into acc1  ||  epilogue of acc0 (stage t,   q=0)
  // so the and_or/min VALU work fills the MFMA issue gaps of the same wave.  Epilogues
  // run in increasing centroid order, so the strict '<' keeps first-index ties.
  f32x16 acc0[P], acc1[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc1[p][i] = 3.0e38f;  // stage -1 dummy: never selected
  }

#define TDC_EPILOGUE(ACC, Q, T_)                                                           \
  _Pragma("unroll") for (int p = 0; p < P; ++p) {                                          \
    float m = INFINITY;                                                                    \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                       \
      const float v = __uint_as_float((__float_as_uint(ACC[p][i]) & ~31u) |                \
                                      (unsigned)((Q) * 16 + i));                           \
      m = __builtin_fminf(m, v);                                                           \
    }                                                                                      \
    const bool up = m < best[p];                                                           \
    best[p] = up ? m : best[p];                                                            \
    bt[p] = up ? (T_) : bt[p];                                                             \
  }

#define TDC_PHASE(ACC, Q)                                                                  \
  {                                                                                        \
    const int row = (Q) * 32 + r;                                                          \
    const f32x4 n0 = *reinterpret_cast<const f32x4*>(ns + (Q) * 32 + 4 * h);               \
    const f32x4 n1 = *reinterpret_cast<const f32x4*>(ns + (Q) * 32 + 8 + 4 * h);           \
    const f32x4 n2 = *reinterpret_cast<const f32x4*>(ns + (Q) * 32 + 16 + 4 * h);          \
    const f32x4 n3 = *reinterpret_cast<const f32x4*>(ns + (Q) * 32 + 24 + 4 * h);          \
    f32x16 init;                                                                           \
    init[0] = n0[0]; init[1] = n0[1]; init[2] = n0[2]; init[3] = n0[3];                    \
    init[4] = n1[0]; init[5] = n1[1]; init[6] = n1[2]; init[7] = n1[3];                    \
    init[8] = n2[0]; init[9] = n2[1]; init[10] = n2[2]; init[11] = n2[3];                  \
    init[12] = n3[0]; init[13] = n3[1]; init[14] = n3[2]; init[15] = n3[3];                \
    bf16x8 a_cur = *reinterpret_cast<const bf16x8*>(cs + row * DP + swz<DP>(row, h * (CPR / 2)) * 8); \
    _Pragma("unroll") for (int kk = 0; kk < KS; ++kk) {                                    \
      const int kn = kk + 1 < KS ? kk + 1 : kk;                                            \
      const bf16x8 a_nxt = *reinterpret_cast<const bf16x8*>(                               \
          cs + row * DP + swz<DP>(row, h * (CPR / 2) + kn) * 8);                           \
      _Pragma("unroll") for (int p = 0; p < P; ++p) ACC[p] =                               \
          __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_cur, bq[p][kk], kk == 0 ? init : ACC[p], 0, 0, 0); \
      a_cur = a_nxt;                                                                       \
    }                                                                                      \
  }

#define TDC_KEEP(ACC)                                     \
  _Pragma("unroll") for (int p = 0; p < P; ++p)           \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(ACC[p][i]));
  for (int t = 0; t < ntiles; ++t) {
    const int buf = (ABL & 2) ? 0 : (t & 1);
    // issue the next stage's loads first; they land under this stage's MFMAs
    // (the last iteration re-loads the final stage: no branch, no reader)
    const int tn = (t + 1 < ntiles) ? t + 1 : t;
    // Issued by inline asm so hipcc cannot sink them next to their ds_write (it treats
    // const __restrict__ loads as invariant and moves them past any barrier): their
    // latency then hides under this stage's MFMAs.  hipcc does not count asm loads, so
    // the explicit vmcnt(0) below (naming every destination) is the only wait.
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int q = tid + i * 256;
      if ((ABL & 2) == 0 && (CHUNKS % 256 == 0 || q < CHUNKS)) {
        const int row = q / CPR, c = q % CPR;
        const __bf16* src = Cm2 + ((int64_t)tn * BN + row) * DP + c * 8;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(pre[i]) : "v"(src) : "memory");
      }
    }
    if constexpr ((ABL & 2) == 0) {
      const float* src = cnorm + tn * BN + (tid & (BN - 1));
      asm volatile("global_load_dword %0, %1, off" : "=v"(npre) : "v"(src) : "memory");
    }

    const __bf16* cs = s_c + buf * STAGE;
    const float* ns = s_n + buf * BN;
    TDC_PHASE(acc0, 0)
    if constexpr (ABL & 1) { TDC_KEEP(acc1) } else { TDC_EPILOGUE(acc1, 1, t - 1) }
    TDC_PHASE(acc1, 1)
    if constexpr (ABL & 1) { TDC_KEEP(acc0) } else { TDC_EPILOGUE(acc0, 0, t) }

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr ((ABL & 2) == 0) {
      __bf16* dst = s_c + (buf ^ 1) * STAGE;
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int q = tid + i * 256;
        if (CHUNKS % 256 == 0 || q < CHUNKS) {
          const int row = q / CPR, c = q % CPR;
          *reinterpret_cast<uint4*>(dst + row * DP + swz<DP>(row, c) * 8) = pre[i];
        }
      }
      if (tid < BN) s_n[(buf ^ 1) * BN + tid] = npre;
    }
    if constexpr ((ABL & 4) == 0) __syncthreads();
  }
  TDC_EPILOGUE(acc1, 1, ntiles - 1)
#undef TDC_KEEP
#undef TDC_PHASE
#undef TDC_EPILOGUE

  // ---- combine the two lane halves (same point, disjoint centroid rows) ----
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const float ob = __shfl_xor(best[p], 32, 64);
    const int obt = __shfl_xor(bt[p], 32, 64);
    const unsigned e0 = __float_as_uint(best[p]) & 31u, e1 = __float_as_uint(ob) & 31u;
    const int l0 = bt[p] * BN + (int)(e0 >> 4) * 32 + (int)(e0 & 3) + 8 * (int)((e0 & 15) >> 2) + 4 * h;
    const int l1 = obt * BN + (int)(e1 >> 4) * 32 + (int)(e1 & 3) + 8 * (int)((e1 & 15) >> 2) + 4 * (1 - h);
    const float v0 = __uint_as_float(__float_as_uint(best[p]) & ~31u);
    const float v1 = __uint_as_float(__float_as_uint(ob) & ~31u);
    const bool other = (v1 < v0) || (v1 == v0 && l1 < l0);
    const int64_t row = pbase + p * 32 + r;
    if (h == 0 && row < N) {
      labels[row] = other ? l1 : l0;
      if (mind) mind[row] = fmaxf((other ? v1 : v0) + xn[p], 0.f);
    }
  }
}

// ------------------------------------------------------------------------------------
// Variant 2 ("ring"): centroid stages arrive by LDS-DMA (global_load_lds_dwordx4) into an
// NST-deep ring, no staging VGPRs and no ds_write pass; loads run NST-1 stages ahead
// behind a counted vmcnt and a raw s_barrier (cdna_hip_programming.md §5 "glds vs
// register staging", "Pipelining across barriers").  The DMA destination is
// lane-linear, so the XOR swizzle moves to the per-lane SOURCE address (rule 21).
// A workgroup of WAVES waves shares each stage: per-point centroid traffic through
// L2/LDS-DMA is 1/(WAVES*P*32) of C per point, the lever that decides this kernel
// (ablate_assign: no-staging build 1.89 ms vs 2.30 ms with 4-wave groups).
// The centroid norms (the accumulator init) are read straight from global (L1-resident).
// ------------------------------------------------------------------------------------
template <int DP, int P, int NST, int WAVES, int QT, int ABL = 0>
__global__ __launch_bounds__(WAVES * 64, (WAVES % 4 == 0 ? (WAVES / 4 > 1 ? WAVES / 4 : 3) : 2))
void assign_mfma_bf16_ring_kernel(const __bf16* __restrict__ X, int64_t N, int64_t ldx,
                                  const __bf16* __restrict__ Cm2, const float* __restrict__ cnorm,
                                  int ntiles, int32_t* __restrict__ labels,
                                  float* __restrict__ mind) {
  constexpr int BNL = 32 * QT;                     // centroids per stage
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 16;
  constexpr int HALF = DP / 2;
  constexpr int TILE_B = BNL * DP * 2;
  constexpr int PIECES = TILE_B / 1024;            // 1 KiB per wave-instruction
  constexpr int PPW = PIECES / WAVES;
  static_assert(PIECES % WAVES == 0, "stage must split evenly over the waves");
  constexpr int G = CPR < 16 ? CPR : 16;
  constexpr int RPB = 16 / G;
  constexpr unsigned EMB = QT * 16 <= 32 ? 31u : 63u;  // (q, reg) id bits in the mantissa
  __shared__ __attribute__((aligned(16))) char smem[NST * TILE_B];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * (WAVES * P * 32) + (int64_t)w * (P * 32);

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
      const int L = piece * 64 + lane;            // linear 16-B chunk index in the stage
      const int row = L / CPR, cp = L % CPR;
      const int csrc = cp ^ ((row / RPB) & (G - 1));
      const __bf16* src = Cm2 + ((int64_t)t * BNL + row) * DP + csrc * 8;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * TILE_B + piece * 1024), 16, 0, 0);
    }
  };

#pragma unroll
  for (int t = 0; t < NST - 1; ++t) issue(t < ntiles ? t : ntiles - 1, t);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * PPW) : "memory");
  __builtin_amdgcn_s_barrier();

  float best[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = INFINITY;
    bt[p] = 0;
  }
  f32x16 acc[P];

#define TDC_EPILOGUE(Q, T_)                                                                \
  _Pragma("unroll") for (int p = 0; p < P; ++p) {                                          \
    float m = INFINITY;                                                                    \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) {                                       \
      const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) |                \
                                      (unsigned)((Q) * 16 + i));                           \
      m = __builtin_fminf(m, v);                                                           \
    }                                                                                      \
    const bool up = m < best[p];                                                           \
    best[p] = up ? m : best[p];                                                            \
    bt[p] = up ? (T_) : bt[p];                                                             \
  }
#define TDC_KEEP()                                                                         \
  _Pragma("unroll") for (int p = 0; p < P; ++p)                                            \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(acc[p][i]));
#define TDC_PHASE(Q)                                                                       \
  {                                                                                        \
    const int row = (Q) * 32 + r;                                                          \
    const float* nsrc = cnorm + (int64_t)t * BNL + (Q) * 32 + 4 * h;                       \
    const f32x4 n0 = *reinterpret_cast<const f32x4*>(nsrc);                                \
    const f32x4 n1 = *reinterpret_cast<const f32x4*>(nsrc + 8);                            \
    const f32x4 n2 = *reinterpret_cast<const f32x4*>(nsrc + 16);                           \
    const f32x4 n3 = *reinterpret_cast<const f32x4*>(nsrc + 24);                           \
    f32x16 init;                                                                           \
    init[0] = n0[0]; init[1] = n0[1]; init[2] = n0[2]; init[3] = n0[3];                    \
    init[4] = n1[0]; init[5] = n1[1]; init[6] = n1[2]; init[7] = n1[3];                    \
    init[8] = n2[0]; init[9] = n2[1]; init[10] = n2[2]; init[11] = n2[3];                  \
    init[12] = n3[0]; init[13] = n3[1]; init[14] = n3[2]; init[15] = n3[3];                \
    bf16x8 a_cur = *reinterpret_cast<const bf16x8*>(cs + row * DP + swz<DP>(row, h * (CPR / 2)) * 8); \
    _Pragma("unroll") for (int kk = 0; kk < KS; ++kk) {                                    \
      const int kn = kk + 1 < KS ? kk + 1 : kk;                                            \
      const bf16x8 a_nxt = *reinterpret_cast<const bf16x8*>(                               \
          cs + row * DP + swz<DP>(row, h * (CPR / 2) + kn) * 8);                           \
      _Pragma("unroll") for (int p = 0; p < P; ++p) acc[p] =                               \
          __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_cur, bq[p][kk], kk == 0 ? init : acc[p], 0, 0, 0); \
      a_cur = a_nxt;                                                                       \
    }                                                                                      \
  }

  for (int t = 0; t < ntiles; ++t) {
    const int slot = t % NST;
    {  // refill the slot read in stage t-1 (every wave passed the barrier after it)
      const int tn = t + NST - 1;
      issue(tn < ntiles ? tn : ntiles - 1, (t + NST - 1) % NST);
    }
    const __bf16* cs = reinterpret_cast<const __bf16*>(smem + slot * TILE_B);
#pragma unroll
    for (int q = 0; q < QT; ++q) {
      TDC_PHASE(q)
      if constexpr (ABL & 1) { TDC_KEEP() } else { TDC_EPILOGUE(q, t) }
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * PPW) : "memory");  // stage t+1 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... for every wave's pieces
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the dummy tail DMAs
#undef TDC_KEEP
#undef TDC_PHASE
#undef TDC_EPILOGUE

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

}  // namespace tdc
