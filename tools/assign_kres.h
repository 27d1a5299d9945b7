// N1 variant "kres": K-resident bf16 MFMA distance + argmin.
//
// The ring kernels (assign_mfma_impl.h) stream every centroid stage through LDS once per
// point block: a 64-row refill (16 one-KiB LDS-DMA pieces) and a workgroup barrier per
// stage.  Their ablations put the refill alone at 12 % of the headline kernel and the
// MFMA pipe at 64-71 % busy (profiles/assign_ring3_ablation_r02.txt,
// pmc_assign_ring3_p8_vs_p4_r02.txt).  Here the centroid table never moves inside the
// main loop:
//
//   * the table is cut into `ksplit` row slices of at most R rows (R*DP*2 bytes ~ 128 KiB,
//     e.g. K=1024 x D=128 -> 2 slices of 512); one workgroup per CU loads ONE slice into
//     LDS once, at launch (plus its ||c||^2 row norms), and keeps it for its lifetime;
//   * after that single barrier every wave runs on its own: it takes 64-point units
//     (P=4 tiles of 16 points, bf16 B fragments in VGPRs) round-robin, sweeps the whole
//     slice with v_mfma_f32_16x16x32_bf16 (A fragments = centroid rows, ds_read_b128 with
//     the ring kernels' XOR swizzle: conflict-free) and the and_or + min epilogue of the
//     ring3 kernel, and prefetches the next unit's points into a second register set while
//     it computes -- no barriers, no refill, and a wave-granular tail (a 1.25M-row shard
//     is 19.5K units for 2048 waves);
//   * workgroups come in ksplit-tuples that sweep the same units with different slices;
//     blocks b and b+8 share an XCD under round-robin placement, so a tuple is
//     {g, g+8, ...} and its X rows meet in one L2 (speed only, never correctness);
//   * ksplit == 1 writes labels directly; otherwise each slice writes a (score, label)
//     key per point and kres_merge_kernel picks the minimum (lower slice = lower label on
//     ties, the same first-index rule as the ring kernels).
//
// Scores are ||c||^2 - 2 x.c (accumulator initialised with the norm); with `mind` the
// point norm is added before the key is written, so the merged key is the distance.
#pragma once
#include "assign_mfma_impl.h"  // csrc/ (build with -I csrc)

namespace tdc {

template <int DP>
struct KresGeom {
  static constexpr int ROWB = DP * 2;
  // rows per slice: ~128 KiB of bf16 rows (+ 4 B norm per row), a multiple of 64
  static constexpr int R = (128 * 1024) / ROWB;
  static constexpr int LDS = R * ROWB + R * 4;
};

// One wave's unit: P tiles of 16 points.  Lane (r, g) holds point tile_base + r, features
// [kk*32 + g*8, +8) for k-step kk (the same permutation for A and B).
template <int DP, int P>
__device__ __forceinline__ void kres_load_points(const __bf16* __restrict__ X, int64_t N,
                                                 int64_t ldx, int64_t pbase, int r, int g,
                                                 bf16x8 (&bq)[P][DP / 32]) {
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 16 + r;
    if (row >= N) row = N - 1;
    const __bf16* src = X + row * ldx + g * 8;
#pragma unroll
    for (int kk = 0; kk < DP / 32; ++kk) bq[p][kk] = *reinterpret_cast<const bf16x8*>(src + kk * 32);
  }
}

// Tile pipeline of one unit: for tile t the A fragments of tile t+1 are read first, then
// the MFMAs of tile t run interleaved (sched_group_barrier) with the epilogue of tile t-1,
// whose accumulators are long complete -- so neither the LDS read latency nor the MFMA
// result latency is exposed, and the epilogue VALU fills the MFMA issue gaps of the SAME
// wave (the co-resident waves are independent: no barrier ever aligns them).
template <int DP, int P>
__device__ __forceinline__ void kres_unit(const char* __restrict__ smem, int nst, int row0,
                                          int r, int g, int64_t pbase, int64_t N,
                                          const bf16x8 (&bq)[P][DP / 32], int ksplit,
                                          int slice, int32_t* __restrict__ labels,
                                          float* __restrict__ mind, float2* __restrict__ keys) {
  constexpr int KS = DP / 32;
  constexpr int ROWB = DP * 2;
  constexpr int R = KresGeom<DP>::R;
  constexpr unsigned EMB = 15u;  // (tile q, reg i) id of a 64-row stage: 4 mantissa bits
  const float* snorm = reinterpret_cast<const float*>(smem + R * ROWB);
  unsigned aoff[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) aoff[kk] = r * ROWB + swz<DP>(r, kk * 4 + g) * 16;
  auto read_tile = [&](int t, bf16x8 (&a)[KS], f32x4& n4) __attribute__((always_inline)) {
    const int base = t * 16;
    n4 = *reinterpret_cast<const f32x4*>(snorm + base + 4 * g);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
      a[kk] = *reinterpret_cast<const bf16x8*>(smem + base * ROWB + aoff[kk]);
  };
  float best[P], m[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = INFINITY;
    m[p] = INFINITY;
    bt[p] = 0;
  }
  // epilogue of tile q (0..3) of stage st: tagged running min; the stage's min meets the
  // best after its 4th tile
  auto epilogue = [&](const f32x4 (&acc)[P], int q, int st) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 4 + i));
        m[p] = __builtin_fminf(m[p], v);
      }
    if (q == 3) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const bool up = m[p] < best[p];
        best[p] = up ? m[p] : best[p];
        bt[p] = up ? st : bt[p];
        m[p] = INFINITY;
      }
    }
  };
  auto mfmas = [&](const bf16x8 (&a)[KS], const f32x4& n4, f32x4 (&acc)[P]) __attribute__((always_inline)) {
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
      for (int p = 0; p < P; ++p)
        acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk], bq[p][kk], kk == 0 ? n4 : acc[p],
                                                          0, 0, 0);
  };
  // interleave: P*KS MFMAs, each followed by up to 2 VALU of the previous epilogue
  auto interleave = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_group_barrier(0x100, KS + 1, 0);  // next tile's LDS reads first
#pragma unroll
    for (int j = 0; j < P * KS; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // two VALU
    }
    __builtin_amdgcn_sched_barrier(0);  // the tile's code stays in its own region
  };
  bf16x8 a0[KS], a1[KS];
  f32x4 n0, n1;
  f32x4 acc0[P], acc1[P];
  const int ntl = nst * 4;
  auto clampt = [&](int t) __attribute__((always_inline)) { return t < ntl ? t : ntl - 1; };
  // prologue: tile 0 (set 0)
  read_tile(0, a0, n0);
  read_tile(1, a1, n1);
  mfmas(a0, n0, acc0);
  // one stage (4 tiles) per iteration; tile q uses register set q & 1, the epilogue of
  // tile q-1 runs beside the MFMAs of tile q (q = 0 closes the previous stage)
  for (int st = 0; st < nst; ++st) {
    const int t0 = st * 4;
    read_tile(clampt(t0 + 2), a0, n0);  // tile q=1: MFMAs on set 1, epilogue of q=0
    mfmas(a1, n1, acc1);
    epilogue(acc0, 0, st);
    interleave();
    read_tile(clampt(t0 + 3), a1, n1);  // q=2: set 0, epilogue of q=1
    mfmas(a0, n0, acc0);
    epilogue(acc1, 1, st);
    interleave();
    read_tile(clampt(t0 + 4), a0, n0);  // q=3: set 1, epilogue of q=2
    mfmas(a1, n1, acc1);
    epilogue(acc0, 2, st);
    interleave();
    if (st + 1 < nst) {                  // next stage's q=0: set 0, epilogue of q=3
      read_tile(clampt(t0 + 5), a1, n1);
      mfmas(a0, n0, acc0);
      epilogue(acc1, 3, st);
      interleave();
    } else {
      epilogue(acc1, 3, st);
    }
  }
  // combine the 4 lane groups (same point, disjoint centroid rows)
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const unsigned e = __float_as_uint(best[p]) & EMB;
    int lab = row0 + bt[p] * 64 + (int)(e >> 2) * 16 + 4 * g + (int)(e & 3);
    float v = __uint_as_float(__float_as_uint(best[p]) & ~EMB);
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int ol = __shfl_xor(lab, o, 64);
      const bool other = (ov < v) || (ov == v && ol < lab);
      v = other ? ov : v;
      lab = other ? ol : lab;
    }
    const int64_t row = pbase + p * 16 + r;
    if (g == 0 && row < N) {
      if (ksplit == 1) {
        labels[row] = lab;
        // ||x||^2 is added by a follow-up pass (kres_mind_kernel): the points' norms stay
        // off the register budget
        if (mind) mind[row] = v;
      } else {
        keys[(int64_t)slice * N + row] = make_float2(v, __int_as_float(lab));
      }
    }
  }
}

// ring3's phase code (assign_mfma_impl.h: inline-asm ds_read_b128 with explicit lgkmcnt,
// A fragments two k-steps ahead, P MFMAs per k-step between sched barriers) on the
// resident slice: no refill, no barrier.
template <int DP, int P>
__device__ __forceinline__ void kres_unit_r3(const char* __restrict__ smem, int nst, int row0,
                                             int r, int g, int64_t pbase, int64_t N,
                                             const bf16x8 (&bq)[P][DP / 32], int ksplit,
                                             int slice, int32_t* __restrict__ labels,
                                             float* __restrict__ mind, float2* __restrict__ keys) {
  constexpr int KS = DP / 32;
  constexpr int ROWB = DP * 2;
  constexpr int R = KresGeom<DP>::R;
  constexpr unsigned EMB = 15u;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)smem;
  unsigned aoff0[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) aoff0[kk] = lds0 + r * ROWB + swz<DP>(r, kk * 4 + g) * 16;
  const unsigned noff0 = lds0 + R * ROWB + 16 * g;
  float best[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = INFINITY;
    bt[p] = 0;
  }
  for (int st = 0; st < nst; ++st) {
    unsigned aoff[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) aoff[kk] = aoff0[kk] + st * 64 * ROWB;
    const unsigned noff = noff0 + st * 64 * 4;
    float m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = INFINITY;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      auto afrag = [&](int kk) __attribute__((always_inline)) {
        bf16x8 a;
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(a) : "v"(aoff[kk]), "i"(q * 16 * ROWB));
        return a;
      };
      f32x4 n4;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(n4) : "v"(noff), "i"(q * 16 * 4));
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
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 4 + i));
          m[p] = __builtin_fminf(m[p], v);
        }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bool up = m[p] < best[p];
      best[p] = up ? m[p] : best[p];
      bt[p] = up ? st : bt[p];
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const unsigned e = __float_as_uint(best[p]) & EMB;
    int lab = row0 + bt[p] * 64 + (int)(e >> 2) * 16 + 4 * g + (int)(e & 3);
    float v = __uint_as_float(__float_as_uint(best[p]) & ~EMB);
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int ol = __shfl_xor(lab, o, 64);
      const bool other = (ov < v) || (ov == v && ol < lab);
      v = other ? ov : v;
      lab = other ? ol : lab;
    }
    const int64_t row = pbase + p * 16 + r;
    if (g == 0 && row < N) {
      if (ksplit == 1) {
        labels[row] = lab;
        if (mind) mind[row] = v;
      } else {
        keys[(int64_t)slice * N + row] = make_float2(v, __int_as_float(lab));
      }
    }
  }
}

// grid: a multiple of 8 * ksplit workgroups of 64 * WAVES threads, one per CU
template <int DP, int P, int WAVES, bool PREFETCH, bool R3 = false>
__global__ __launch_bounds__(WAVES * 64, WAVES / 4)
void assign_kres_kernel(const __bf16* __restrict__ X, int64_t N, int64_t ldx,
                        const __bf16* __restrict__ Cm2, const float* __restrict__ cnorm, int Kp,
                        int ksplit, int32_t* __restrict__ labels, float* __restrict__ mind,
                        float2* __restrict__ keys) {
  constexpr int KS = DP / 32;
  constexpr int ROWB = DP * 2;
  constexpr int CPR = DP / 8;
  constexpr int R = KresGeom<DP>::R;
  __shared__ __attribute__((aligned(16))) char smem[KresGeom<DP>::LDS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int slice = (blockIdx.x >> 3) % ksplit;
  const int grp = (blockIdx.x / (8 * ksplit)) * 8 + (blockIdx.x & 7);
  const int ngrp = gridDim.x / ksplit;
  const int row0 = slice * R;
  const int rows = min(R, Kp - row0);  // a multiple of 64

  // ---- the slice, once: rows x 16-B chunks, XOR-swizzled as the ring kernels' stages ----
  for (int q = tid; q < rows * CPR; q += WAVES * 64) {
    const int rr = q / CPR, c = q % CPR;
    const uint4 v = *reinterpret_cast<const uint4*>(Cm2 + (int64_t)(row0 + rr) * DP + c * 8);
    *reinterpret_cast<uint4*>(smem + rr * ROWB + swz<DP>(rr, c) * 16) = v;
  }
  for (int q = tid; q < rows; q += WAVES * 64)
    reinterpret_cast<float*>(smem + R * ROWB)[q] = cnorm[row0 + q];
  __syncthreads();

  const int nst = rows / 64;
  const int64_t nunits = (N + 16 * P - 1) / (16 * P);
  const int64_t stride = (int64_t)ngrp * WAVES;
  int64_t u = (int64_t)grp * WAVES + w;
  if (u >= nunits) return;
  if constexpr (!PREFETCH) {
    for (; u < nunits; u += stride) {
      bf16x8 bq[P][KS];
      kres_load_points<DP, P>(X, N, ldx, u * 16 * P, r, g, bq);
      if constexpr (R3)
        kres_unit_r3<DP, P>(smem, nst, row0, r, g, u * 16 * P, N, bq, ksplit, slice, labels, mind, keys);
      else
        kres_unit<DP, P>(smem, nst, row0, r, g, u * 16 * P, N, bq, ksplit, slice, labels, mind, keys);
    }
  } else {
    // two register sets: the next unit's rows load while this one computes (the loads are
    // unconditional -- clamped to the last unit -- so the vmcnt bookkeeping is static)
    bf16x8 bqa[P][KS], bqb[P][KS];
    kres_load_points<DP, P>(X, N, ldx, u * 16 * P, r, g, bqa);
    for (;;) {
      const int64_t u1 = u + stride;
      kres_load_points<DP, P>(X, N, ldx, (u1 < nunits ? u1 : nunits - 1) * 16 * P, r, g, bqb);
      kres_unit<DP, P>(smem, nst, row0, r, g, u * 16 * P, N, bqa, ksplit, slice, labels, mind, keys);
      if (u1 >= nunits) break;
      const int64_t u2 = u1 + stride;
      kres_load_points<DP, P>(X, N, ldx, (u2 < nunits ? u2 : nunits - 1) * 16 * P, r, g, bqa);
      kres_unit<DP, P>(smem, nst, row0, r, g, u1 * 16 * P, N, bqb, ksplit, slice, labels, mind, keys);
      if (u2 >= nunits) break;
      u = u2;
    }
  }
}

// ksplit > 1: labels[i] = label of the smallest key over the slices (ties: lower slice);
// mind (optional) = max(0, score + ||x_i||^2)
__global__ __launch_bounds__(256) void kres_merge_kernel(const float2* __restrict__ keys,
                                                         int ksplit, int64_t N,
                                                         int32_t* __restrict__ labels,
                                                         float* __restrict__ mind,
                                                         const float* __restrict__ xnorm) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * 256) {
    float2 b = keys[i];
    for (int s = 1; s < ksplit; ++s) {
      const float2 k = keys[(int64_t)s * N + i];
      if (k.x < b.x) b = k;
    }
    labels[i] = __float_as_int(b.y);
    if (mind) mind[i] = fmaxf(b.x + xnorm[i], 0.f);
  }
}

// ksplit == 1 with mind: mind[i] = max(0, score_i + ||x_i||^2) in place
__global__ __launch_bounds__(256) void kres_mind_kernel(float* __restrict__ mind, int64_t N,
                                                        const float* __restrict__ xnorm) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < N;
       i += (int64_t)gridDim.x * 256)
    mind[i] = fmaxf(mind[i] + xnorm[i], 0.f);
}

// ||x_i||^2 of bf16 rows (only when a min distance is asked for)
template <int DP>
__global__ __launch_bounds__(256) void kres_xnorm_kernel(const __bf16* __restrict__ X, int64_t N,
                                                         int64_t ldx, float* __restrict__ xnorm) {
  // 16 lanes per row, DP/16 features per lane
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int sub = threadIdx.x & 15;
  for (int64_t row = t >> 4; row < N; row += ((int64_t)gridDim.x * 256) >> 4) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < DP / 16; ++j) {
      const float f = (float)X[row * ldx + sub * (DP / 16) + j];
      s = fmaf(f, f, s);
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
    if (sub == 0) xnorm[row] = s;
  }
}

}  // namespace tdc
