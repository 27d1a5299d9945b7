// A/B harness (round 6): does the headline assign lose its idle third to point-fragment
// prologues that run in lockstep?  Variants of the production ring3 kernel
// (csrc/assign_mfma_impl.h, assign_mfma_bf16_ring3_kernel<128, 8, 2, 4, 4>) on the headline
// shape, timed interleaved in one process, labels compared with production.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/ring3_persist_ab.hip -o gpubin/ring3_persist_ab
//   ./gpubin/ring3_persist_ab [N] [K] [reps]
//
// Every block of the production launch (19531 x 512 points) begins by loading its 128 KB of
// point fragments from HBM; all first-round blocks start together and run equal work, so the
// loads of the whole chip arrive as one burst per round (the HBM-bound prologue row of
// MI355X_MICROARCH.md, ~11 B/cycle/CU), while the K loop itself reads almost nothing.
// Variants (template flags of ring3p_kernel):
//   PERSIST  grid = resident slots (2 per CU); each workgroup loops over point blocks
//            b, b + grid, ...  (static stride; the ring and lane constants are reused)
//   RELOAD   (PERSIST only) the next block's point fragments are loaded right after the
//            current block's last MFMA (before its lane-group merge and label stores), and
//            the last stage issues no dead refill, so the loads overlap the block's tail and
//            the next ring prologue (a reload inside the last stage made hipcc spill 300+
//            VGPRs, peeled or behind a uniform branch)
//   stagger  (runtime) a first-round workgroup sleeps hash(blockIdx) % S x ~1k cycles
//            before it starts: the chip's prologue bursts spread over a block time
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <vector>

#include "assign_mfma_impl.h"

using namespace tdc;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

// PF > 0 (non-persistent): in each of the block's last PF stages every wave touches a share of
// the rows of block blockIdx.x + pf_stride (the block the dispatcher most likely starts next
// on this XCD: blocks go round-robin over the 8 XCDs) with 4-byte LDS-DMA loads into a sink,
// one 128-B line per lane, so that block's point prologue hits the XCD's L2 instead of HBM
template <int DP, int P, int NST, int WAVES, int QT, bool PERSIST, bool RELOAD, int PF = 0>
__global__ __launch_bounds__(WAVES * 64, 2)
void ring3p_kernel(const __bf16* __restrict__ X, int64_t N, int64_t ldx,
                   const __bf16* __restrict__ Cm2, const float* __restrict__ cnorm, int ntiles,
                   int32_t* __restrict__ labels, int64_t nblk, int stagger, int stag_blocks,
                   unsigned long long* __restrict__ stamps = nullptr, int pf_stride = 0) {
  static_assert(!RELOAD || (PERSIST && NST == 2), "reload: persistent, two-slot ring");
  static_assert(PF == 0 || !PERSIST, "prefetch: one block per workgroup");
  static_assert(PF == 0 || NST == 2, "prefetch: the stage-end wait must be vmcnt(0)");
  // stamps (diagnostic build only, non-persistent): per block, from wave 0 lane 0 --
  // s_memtime at entry, after the prologue barrier (points + first ring stage landed), after
  // the K loop, and the CU id (HW_ID bits 8-15 | XCC_ID << 8)
  unsigned long long st0 = 0, st1 = 0;
  if (stamps) st0 = __builtin_amdgcn_s_memtime();
  constexpr int BNL = 16 * QT;
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 32;
  constexpr int TILE_B = BNL * DP * 2;
  constexpr int NORM_B = BNL * 4;
  constexpr int STAGE_B = TILE_B + NORM_B;
  constexpr int PIECES = TILE_B / 1024;
  constexpr int PPW = (PIECES + WAVES - 1) / WAVES;
  constexpr int NCH = NORM_B / 16;
  constexpr int NPW = (NCH + WAVES - 1) / WAVES;
  constexpr int VPS = PPW + 1;
  constexpr unsigned EMB = QT * 4 <= 16 ? 15u : 31u;
  constexpr int PER = WAVES * P * 16;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE_B + (PF ? WAVES * 256 : 0)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // prefetch lines: PER rows x DP x 2 B of the next block = PER * DP / 64 lines of 128 B,
  // split over the waves and the PF stages (lane = one line)
  constexpr int LINES = PER * DP * 2 / 128;
  constexpr int LPS = PF ? (LINES + WAVES * PF * 64 - 1) / (WAVES * PF * 64) : 0;  // instrs/stage
  const int64_t pfb = (int64_t)blockIdx.x + pf_stride;
  const bool pf_on = PF && pf_stride > 0 && pfb < nblk;
  const __bf16* pf_base = X + (pf_on ? pfb * PER * ldx : 0);
  const int64_t pf_lines = pf_on ? min((int64_t)LINES, ((N - pfb * PER) * ldx * 2 + 127) / 128) : 0;
  auto prefetch = [&](int j) __attribute__((always_inline)) {  // j: 0 .. PF-1
#pragma unroll
    for (int i = 0; i < LPS; ++i) {
      int64_t line = ((int64_t)(j * LPS + i) * WAVES + w) * 64 + lane;
      if (line >= pf_lines) line = pf_lines - 1;
      const unsigned voffp = (unsigned)(line * 128);
      const unsigned dst = lds0 + NST * STAGE_B + w * 256;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voffp), "s"(pf_base)
                   : "memory", "m0");
    }
  };

  if (stagger > 0 && (int)blockIdx.x < stag_blocks) {
    unsigned h = (unsigned)blockIdx.x * 2654435761u;
    h ^= h >> 15;
    const int n = (int)(h % (unsigned)stagger);
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(16);
  }

  bf16x8 bq[P][KS];
  // point fragments by buffer loads: a wave-uniform descriptor per (block, wave) over the
  // wave's P x 16 rows (rows past N read as 0 by the descriptor's bounds check), one VGPR
  // of per-lane offset, the tile offset p x 16 rows in soffset, kk in the immediate
  const unsigned vrow = (unsigned)(r * ldx * 2 + g * 16);
  const int wu0 = __builtin_amdgcn_readfirstlane(w);
  auto rsrc_of = [&](int64_t blk) __attribute__((always_inline)) {
    const int64_t row0 = blk * PER + (int64_t)wu0 * (P * 16);
    const int64_t left = N - row0;
    const int64_t bytes = left <= 0 ? 0 : (left * ldx * 2 < (1 << 30) ? left * ldx * 2 : (1 << 30));
    const void* base = uniform_ptr(X + (left <= 0 ? 0 : row0 * ldx));
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                             __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
  };
  auto load_points = [&](__amdgpu_buffer_rsrc_t rs, int kk) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)vrow + kk * 64,
                                                     (int)(p * 16 * ldx * 2), 0);
      bq[p][kk] = __builtin_bit_cast(bf16x8, v);
    }
  };

  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int piece = (w * PPW + i) % PIECES;
    const int L = piece * 64 + lane;
    const int row = L / CPR, cp = L % CPR;
    voff[i] = (unsigned)((row * DP + swz<DP>(row, cp) * 8) * 2);
  }
  const int wu = __builtin_amdgcn_readfirstlane(w);
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
    const int nb = w * NPW < NCH - NPW ? w * NPW : NCH - NPW;
    if (lane < NPW) {
      const float* src = cnorm + (int64_t)t * BNL + (nb + lane) * 4;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * STAGE_B + TILE_B + nb * 16),
          16, 0, 0);
    }
  };
  unsigned aoff[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) aoff[kk] = lds0 + r * (DP * 2) + swz<DP>(r, kk * 4 + g) * 16;
  const unsigned noff = lds0 + TILE_B + 16 * g;

  const int64_t step = PERSIST ? (int64_t)gridDim.x : nblk;
  int64_t blk = blockIdx.x;
  if (blk >= nblk) return;
  {
    const auto rs0 = rsrc_of(blk);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) load_points(rs0, kk);
  }

  for (; blk < nblk; blk += step) {
    const int64_t nxt = blk + step;
    if (!RELOAD && blk != (int64_t)blockIdx.x) {
      const auto rsb = rsrc_of(blk);
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) load_points(rsb, kk);
    }
    const auto rsn = rsrc_of(nxt);
#pragma unroll
    for (int t = 0; t < NST - 1; ++t) issue(t < ntiles ? t : ntiles - 1, t);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
    __builtin_amdgcn_s_barrier();
    if (stamps) st1 = __builtin_amdgcn_s_memtime();

    float best[P];
    int bt[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      best[p] = INFINITY;
      bt[p] = 0;
    }

    auto stage = [&](int t, auto slot_c) __attribute__((always_inline)) {
      constexpr int slot = decltype(slot_c)::value;
      // RELOAD: the block's last stage issues no refill (uniform branch)
      const bool last = RELOAD && t == ntiles - 1;
      if constexpr (PF > 0) {
        // the oldest load of the stage, so the stage-end vmcnt wait finds it landed first
        if (pf_on && t >= ntiles - PF) prefetch(t - (ntiles - PF));
      }
      if (!last) {
        const int tn = t + NST - 1;
        issue(tn < ntiles ? tn : ntiles - 1, (slot + NST - 1) % NST);
      }
      float m[P];
#pragma unroll
      for (int p = 0; p < P; ++p) m[p] = INFINITY;
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
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
            __builtin_amdgcn_s_barrier();
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
            m[p] = __builtin_fminf(m[p], v);
          }
        }
      }
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const bool up = m[p] < best[p];
        best[p] = up ? m[p] : best[p];
        bt[p] = up ? t : bt[p];
      }
    };

    for (int t0 = 0; t0 < ntiles; t0 += NST) {
      stage(t0, std::integral_constant<int, 0>{});
      if constexpr (NST > 1) if (t0 + 1 < ntiles) stage(t0 + 1, std::integral_constant<int, 1>{});
      if constexpr (NST > 2) if (t0 + 2 < ntiles) stage(t0 + 2, std::integral_constant<int, 2 % NST>{});
    }
    if constexpr (RELOAD) {
      // the next block's point fragments, issued before this block's merge / label stores
      // (in-place asm "+v": the destination is unprotected until the prologue's vmcnt(0),
      // which precedes every use)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int p = 0; p < P; ++p)
          asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
                       : "+v"(bq[p][kk])
                       : "v"(vrow), "s"(rsn), "s"((int)(p * 16 * ldx * 2)), "i"(kk * 64)
                       : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }

    if (stamps) {
      const unsigned long long st2 = __builtin_amdgcn_s_memtime();
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      if (tid == 0) {
        stamps[blk * 4 + 0] = st0;
        stamps[blk * 4 + 1] = st1;
        stamps[blk * 4 + 2] = st2;
        stamps[blk * 4 + 3] = (unsigned long long)(((hw >> 8) & 0xffu) | ((xcc & 0xfu) << 8));
      }
    }
    const int64_t pbase = blk * PER + (int64_t)w * (P * 16);
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const unsigned e = __float_as_uint(best[p]) & EMB;
      int lab = bt[p] * BNL + (int)(e >> 2) * 16 + 4 * g + (int)(e & 3);
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
      if (g == 0 && row < N) labels[row] = lab;
    }
    if constexpr (PERSIST) __builtin_amdgcn_s_barrier();  // every wave past its last LDS read
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ring2x: the 32x32x16 shape with ring3's refinements (saddr-form LDS-DMA, stage-level
// running minimum, early slot release, two waves per SIMD).  A 32x32x16 MFMA holds the
// SIMD's issue for 8 of its 32 cycles (16x16x32: 8 of 16), so the tag + min epilogue
// (16 scores per lane per tile) leaves slack where ring3 is issue-bound.
template <int DP, int P, int NST, int WAVES, int QT>
__global__ __launch_bounds__(WAVES * 64, 2)
void ring2x_kernel(const __bf16* __restrict__ X, int64_t N, int64_t ldx,
                   const __bf16* __restrict__ Cm2, const float* __restrict__ cnorm, int ntiles,
                   int32_t* __restrict__ labels) {
  constexpr int BNL = 32 * QT;
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 16;
  constexpr int HALF = DP / 2;
  constexpr int TILE_B = BNL * DP * 2;
  constexpr int NORM_B = BNL * 4;
  constexpr int STAGE_B = TILE_B + NORM_B;
  constexpr int PIECES = TILE_B / 1024;
  constexpr int PPW = (PIECES + WAVES - 1) / WAVES;
  constexpr int NCH = NORM_B / 16;
  constexpr int NPW = (NCH + WAVES - 1) / WAVES;
  constexpr int VPS = PPW + 1;
  constexpr unsigned EMB = QT * 16 <= 32 ? 31u : 63u;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE_B];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * (WAVES * P * 32) + (int64_t)w * (P * 32);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  bf16x8 bq[P][KS];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 32 + r;
    if (row >= N) row = N - 1;
    const bf16x8* src = reinterpret_cast<const bf16x8*>(X + row * ldx + h * HALF);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) bq[p][kk] = src[kk];
  }
  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int piece = (w * PPW + i) % PIECES;
    const int L = piece * 64 + lane;
    const int row = L / CPR, cp = L % CPR;
    voff[i] = (unsigned)((row * DP + swz<DP>(row, cp) * 8) * 2);
  }
  const int wu = __builtin_amdgcn_readfirstlane(w);
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
  float best[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = INFINITY;
    bt[p] = 0;
  }
  unsigned aoff[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) aoff[kk] = lds0 + r * (DP * 2) + swz<DP>(r, h * (CPR / 2) + kk) * 16;
  const unsigned noff = lds0 + TILE_B + 16 * h;
  auto stage = [&](int t, auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value;
    {
      const int tn = t + NST - 1;
      issue(tn < ntiles ? tn : ntiles - 1, (slot + NST - 1) % NST);
    }
    float m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = INFINITY;
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
      bf16x8 a1 = afrag(1);
      f32x16 acc[P];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        bf16x8 a2 = a1;
        if (kk + 2 < KS) a2 = afrag(kk + 2);
        if (kk + 2 < KS) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        else if (kk + 1 < KS) asm volatile("s_waitcnt lgkmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (q == QT - 1 && kk == KS - 1) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
          __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < P; ++p) {
          if (kk == 0) {
            f32x16 init;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              init[4 * j + 0] = n4[j][0];
              init[4 * j + 1] = n4[j][1];
              init[4 * j + 2] = n4[j][2];
              init[4 * j + 3] = n4[j][3];
            }
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[p][0], init, 0, 0, 0);
          } else {
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[p][kk], acc[p], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        a0 = a1;
        a1 = a2;
      }
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 16 + i));
          m[p] = __builtin_fminf(m[p], v);
        }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const bool up = m[p] < best[p];
      best[p] = up ? m[p] : best[p];
      bt[p] = up ? t : bt[p];
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
    const float ob = __shfl_xor(best[p], 32, 64);
    const int obt = __shfl_xor(bt[p], 32, 64);
    const unsigned e0 = __float_as_uint(best[p]) & EMB, e1 = __float_as_uint(ob) & EMB;
    const int l0 = bt[p] * BNL + (int)(e0 >> 4) * 32 + (int)(e0 & 3) + 8 * (int)((e0 & 15) >> 2) + 4 * h;
    const int l1 = obt * BNL + (int)(e1 >> 4) * 32 + (int)(e1 & 3) + 8 * (int)((e1 & 15) >> 2) + 4 * (1 - h);
    const float v0 = __uint_as_float(__float_as_uint(best[p]) & ~EMB);
    const float v1 = __uint_as_float(__float_as_uint(ob) & ~EMB);
    const bool other = (v1 < v0) || (v1 == v0 && l1 < l0);
    const int64_t row = pbase + p * 32 + r;
    if (h == 0 && row < N) labels[row] = other ? l1 : l0;
  }
}

static uint64_t sm64(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static double unif(uint64_t& s) { return (sm64(s) >> 11) * (1.0 / 9007199254740992.0); }
static uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

constexpr int DP = 128;
static int g_cus = 256;

struct Bufs {
  const __bf16* x;
  int64_t n;
  const __bf16* c;
  const float* cn;
  int kp;
  int* lab;
};

static void prod(const Bufs& b, hipStream_t s) {
  const int64_t per = 4 * 8 * 16;
  hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 8, 2, 4, 4>),
                     dim3((unsigned)((b.n + per - 1) / per)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / 64, b.lab, nullptr);
}

static unsigned long long* g_stamps = nullptr;

template <int PF>
static void pfv(const Bufs& b, hipStream_t s, int stride) {
  const int64_t per = 4 * 8 * 16;
  const int64_t nblk = (b.n + per - 1) / per;
  hipLaunchKernelGGL((ring3p_kernel<128, 8, 2, 4, 4, false, false, PF>), dim3((unsigned)nblk),
                     dim3(256), 0, s, b.x, b.n, (int64_t)DP, b.c, b.cn, b.kp / 64, b.lab, nblk, 0,
                     0, nullptr, stride);
}

template <bool PERSIST, bool RELOAD>
static void var(const Bufs& b, hipStream_t s, int stagger, int slots = 2, bool stamp = false) {
  const int64_t per = 4 * 8 * 16;
  const int64_t nblk = (b.n + per - 1) / per;
  const int64_t grid = PERSIST ? std::min<int64_t>(nblk, (int64_t)g_cus * slots) : nblk;
  hipLaunchKernelGGL((ring3p_kernel<128, 8, 2, 4, 4, PERSIST, RELOAD>), dim3((unsigned)grid),
                     dim3(256), 0, s, b.x, b.n, (int64_t)DP, b.c, b.cn, b.kp / 64, b.lab, nblk,
                     stagger, g_cus * 2, stamp ? g_stamps : nullptr);
}

// per-block stamps -> where the prologue cycles go and whether co-resident blocks' prologues
// overlap (printed summary)
static void analyse_stamps(int64_t nblk) {
  std::vector<unsigned long long> h((size_t)nblk * 4);
  CK(hipMemcpy(h.data(), g_stamps, h.size() * 8, hipMemcpyDeviceToHost));
  struct B { unsigned long long s0, s1, s2; unsigned cu; };
  std::vector<B> v;
  v.reserve(nblk);
  unsigned long long tmin = ~0ull, tmax = 0;
  for (int64_t i = 0; i < nblk; ++i) {
    B b{h[4 * i], h[4 * i + 1], h[4 * i + 2], (unsigned)h[4 * i + 3]};
    if (b.s1 < b.s0 || b.s2 < b.s1) continue;
    v.push_back(b);
    tmin = std::min(tmin, b.s0);
    tmax = std::max(tmax, b.s2);
  }
  double pro = 0, loop = 0;
  std::vector<double> pr;
  for (auto& b : v) {
    pro += (double)(b.s1 - b.s0);
    loop += (double)(b.s2 - b.s1);
    pr.push_back((double)(b.s1 - b.s0));
  }
  std::sort(pr.begin(), pr.end());
  const double n = (double)v.size();
  printf("  stamps: %zu blocks, span %.3g cycles; prologue (entry -> first barrier) mean %.0f "
         "p10 %.0f p50 %.0f p90 %.0f cycles; K loop mean %.0f cycles; prologue share of block "
         "time %.1f %%\n",
         v.size(), (double)(tmax - tmin), pro / n, pr[(size_t)(0.1 * n)], pr[(size_t)(0.5 * n)],
         pr[(size_t)(0.9 * n)], loop / n, 100.0 * pro / (pro + loop));
  // per CU: how much of each block's prologue overlaps another block's K loop on that CU
  std::map<unsigned, std::vector<B>> cu;
  for (auto& b : v) cu[b.cu].push_back(b);
  double ov = 0, ov2 = 0, tot = 0;
  size_t ncu = cu.size();
  for (auto& kv : cu) {
    auto& bl = kv.second;
    std::sort(bl.begin(), bl.end(), [](const B& a, const B& c) { return a.s0 < c.s0; });
    for (size_t i = 0; i < bl.size(); ++i) {
      const double a0 = (double)bl[i].s0, a1 = (double)bl[i].s1;
      double covered = 0, both = 0;  // other block in its loop / in its own prologue
      for (size_t j = (i > 8 ? i - 8 : 0); j < std::min(bl.size(), i + 8); ++j) {
        if (j == i) continue;
        const double l0 = std::max(a0, (double)bl[j].s1), l1 = std::min(a1, (double)bl[j].s2);
        if (l1 > l0) covered += l1 - l0;
        const double p0 = std::max(a0, (double)bl[j].s0), p1 = std::min(a1, (double)bl[j].s1);
        if (p1 > p0) both += p1 - p0;
      }
      ov += covered;
      ov2 += both;
      tot += a1 - a0;
    }
  }
  printf("  per CU (%zu CUs): %.1f %% of prologue cycles run beside another block's K loop, "
         "%.1f %% beside another block's prologue\n", ncu, 100.0 * ov / tot, 100.0 * ov2 / tot);
}

template <int P, int NST, int QT>
static void r2x(const Bufs& b, hipStream_t s) {
  const int64_t per = 4 * P * 32;
  hipLaunchKernelGGL((ring2x_kernel<128, P, NST, 4, QT>), dim3((unsigned)((b.n + per - 1) / per)),
                     dim3(256), 0, s, b.x, b.n, (int64_t)DP, b.c, b.cn, b.kp / (32 * QT), b.lab);
}

template <typename F>
static float timeit(F f, int reps) {
  f();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) f();
  CK(hipDeviceSynchronize());
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<float, std::milli>(t1 - t0).count() / reps;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 10000000;
  const int K = argc > 2 ? atoi(argv[2]) : 1024;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const int Kp = (K + 127) / 128 * 128;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  g_cus = prop.multiProcessorCount;
  printf("N=%lld K=%d D=%d CUs=%d\n", (long long)N, K, DP, g_cus);
  if ((Kp / 64) % 2) {
    printf("K/64 must be even\n");
    return 1;
  }
  uint64_t seed = 12345;
  std::vector<float> cen((size_t)K * DP);
  for (auto& v : cen) v = (float)(unif(seed) * 20.0 - 10.0);
  std::vector<uint16_t> xh((size_t)N * DP);
  for (int64_t i = 0; i < N; ++i) {
    const int k = (int)(sm64(seed) % (uint64_t)K);
    for (int d = 0; d < DP; d += 2) {
      const double u1 = unif(seed) + 1e-300, u2 = unif(seed);
      const double rr = sqrt(-2.0 * log(u1));
      xh[(size_t)i * DP + d] = f2bf((float)(cen[(size_t)k * DP + d] + rr * cos(6.283185307179586 * u2)));
      xh[(size_t)i * DP + d + 1] =
          f2bf((float)(cen[(size_t)k * DP + d + 1] + rr * sin(6.283185307179586 * u2)));
    }
  }
  std::vector<uint16_t> cm2((size_t)Kp * DP, 0);
  std::vector<float> cn(Kp, 3.0e38f);
  for (int k = 0; k < K; ++k) {
    const int64_t i = (int64_t)(sm64(seed) % (uint64_t)N);
    double s = 0;
    for (int d = 0; d < DP; ++d) {
      const float c = bf2f(xh[(size_t)i * DP + d]);
      cm2[(size_t)k * DP + d] = f2bf(-2.f * c);
      s += (double)c * c;
    }
    cn[k] = (float)s;
  }
  __bf16 *dx, *dc;
  float* dcn;
  int *l0, *l1;
  CK(hipMalloc(&dx, xh.size() * 2));
  CK(hipMalloc(&dc, cm2.size() * 2));
  CK(hipMalloc(&dcn, cn.size() * 4));
  CK(hipMalloc(&l0, N * 4));
  CK(hipMalloc(&l1, N * 4));
  CK(hipMemcpy(dx, xh.data(), xh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, cm2.data(), cm2.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcn, cn.data(), cn.size() * 4, hipMemcpyHostToDevice));
  Bufs b0{dx, N, dc, dcn, Kp, l0}, b1{dx, N, dc, dcn, Kp, l1};
  std::vector<int> h0(N), h1(N);
  auto check = [&](const char* name) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h0.data(), l0, N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), l1, N * 4, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < N; ++i) bad += h0[i] != h1[i];
    printf("  %-28s mismatches vs production: %lld\n", name, (long long)bad);
    fflush(stdout);
  };
  prod(b0, 0);
#define TRY(NAME, ...)                     \
  CK(hipMemset(l1, 0xff, N * 4));          \
  __VA_ARGS__;                             \
  check(NAME);
  {
    const int64_t nblk = (N + 511) / 512;
    CK(hipMalloc(&g_stamps, (size_t)nblk * 4 * 8));
    CK(hipMemset(g_stamps, 0, (size_t)nblk * 4 * 8));
    for (int i = 0; i < 3; ++i) var<false, false>(b1, 0, 0);
    TRY("copy + stamps", (var<false, false>(b1, 0, 0, 2, true)))
    analyse_stamps(nblk);
    for (int i = 0; i < 3; ++i) var<false, false>(b1, 0, 0);
    TRY("copy + stamps (again)", (var<false, false>(b1, 0, 0, 2, true)))
    analyse_stamps(nblk);
    TRY("stagger 100 + stamps", (var<false, false>(b1, 0, 100, 2, true)))
    analyse_stamps(nblk);
  }
  // tail: the launch is 38.15 rounds of 512 resident blocks at 10M; time the same kernel over
  // whole rounds (multiples of 512 blocks) and per row
  const int64_t rows_round = (int64_t)g_cus * 2 * 512;
  const int64_t n_whole = N / rows_round * rows_round;
  Bufs bw{dx, n_whole, dc, dcn, Kp, l1};
  for (int round = 0; round < 3; ++round) {
    const float t0 = timeit([&] { prod(b0, 0); }, reps);
    const float t1 = timeit([&] { prod(bw, 0); }, reps);
    printf("round %d: prod N=%lld %.4f ms (%.3f ns/row) | N=%lld (whole rounds) %.4f ms (%.3f ns/row) "
           "-> tail cost %.1f us\n",
           round, (long long)N, t0, t0 * 1e6 / N, (long long)n_whole, t1, t1 * 1e6 / n_whole,
           (t0 - t1 * (double)N / n_whole) * 1e3);
    fflush(stdout);
  }
  return 0;
}
