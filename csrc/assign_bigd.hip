// N1/N8 for wide embeddings: fused distance + argmin for D in (256, 1024] (bf16) and for
// block-scaled fp8 (OCP e4m3 + E8M0 scales, D a multiple of 256 up to 1024), plus the
// fp8 row quantiser.  BASELINE config 5: N=50M, D=768, K=65536.
//
// Reference: the same K-Means tower (`scripts/distribuitedClustering.py:221-234`); the
// reference had no reduced-precision path at all (float64 everywhere).
//
// Why a second kernel (vs assign_mfma.hip, D <= 256):
//   * a 32-point B fragment set is D/8 VGPRs per lane in the fp8 MX layout (96 at D=768)
//     and D/4 in bf16 (128 at D=512): one point tile per wave, 8 waves per workgroup, so
//     one centroid stage in LDS is reused by 256 points;
//   * the centroid table no longer fits an XCD's 4 MiB L2 (65536 x 768 fp8 = 48 MiB), so
//     the K loop is split into GROUPS of ~3 MiB and the grid is ordered XCD-major:
//     block b runs on XCD b % 8, and the work items of one XCD are a contiguous
//     (group-major) range, so every XCD keeps exactly one centroid group L2-resident
//     while it sweeps the points.  Per-group winners are merged with a 64-bit atomicMin
//     on (order-preserving score bits << 32 | centroid id): min score, lowest id on ties;
//   * fp8 uses v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate on CDNA4; the
//     unscaled fp8 MFMA only runs at the bf16 rate).  Each lane feeds 32 bytes
//     features of one row as two 16-feature halves of two consecutive scale blocks
//     (layout probed on the hardware, see fp8_off), so the per-lane E8M0 scale operand
//     is one of the row's block exponents.  The -2 of the expansion is folded
//     into the centroid operand (sign bit + 1 in the exponent), the accumulator is
//     initialised with ||c~||^2, so the epilogue is pure min.
//
// Schedule per workgroup (WAVES waves x 32 points): centroid tiles of 32 rows stream
// through an NST-deep LDS ring filled by global_load_lds (LDS-DMA, 16 B per lane,
// XOR-swizzled on the source side so ds_read_b128 lane groups are conflict-free);
// per-tile norms / scales for tile t+1 are loaded one stage early, BEFORE the ring
// refill, so the only vmcnt wait per stage is the counted one on the ring.
#include <stdlib.h>

#include <type_traits>

#include "kernels.h"
#include "tdc_common.h"

namespace tdc {
namespace bigd {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
constexpr float BIGN = 3.0e38f;

struct OpBf16 {
  static constexpr int ES = 2;   // storage bytes per feature
  static constexpr int FB = 16;  // operand bytes per lane per MFMA
  static constexpr bool SCALED = false;
  typedef bf16x8 frag;
};
struct OpFp8 {
  static constexpr int ES = 1;
  static constexpr int FB = 32;
  static constexpr bool SCALED = true;
  typedef i32x8 frag;
};

template <int RB>
__device__ __forceinline__ int swz(int r, int c) {
  constexpr int CPR = RB / 16;
  constexpr int G = CPR < 16 ? CPR : 16;
  constexpr int RPB = 16 / G;
  return c ^ ((r / RPB) & (G - 1));
}

__device__ __forceinline__ unsigned ord_bits(float v) {
  const unsigned u = __float_as_uint(v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_bits(unsigned o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// Operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 (probed with tools/probe_mfma_scale.hip):
// byte j of lane (r, h) is k = 32*(j/16) + 16*h + (j%16), and the E8M0 scale of K-block b
// (k in [32b, 32b+32)) comes from lane r + 32*b.  So one 32-feature quantisation block
// is split over both lane halves (16 features each), and MFMA step kk covers blocks
// 2kk and 2kk+1: lane half h reads features 64kk + 16h + [0,16) and 64kk + 32 + 16h +
// [0,16), and supplies the scale of block 2kk + h.
__device__ __forceinline__ int fp8_off(int kk, int h, int u) { return 64 * kk + 32 * u + 16 * h; }

// SEL: the byte of the scale registers the MFMA applies (its op_sel; probed with
// tools/probe_mfma_scale_opsel.hip: SEL = byte index 0..3 of the 32-bit scale operand)
template <class OP, int SEL = 0>
__device__ __forceinline__ f32x16 mma(const typename OP::frag& a, const typename OP::frag& b,
                                      const f32x16& c, int sa, int sb) {
  if constexpr (OP::SCALED) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, SEL, sa, SEL, sb);
  } else {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
}

// D: padded feature count.  X rows: ldx BYTES apart.  Xs/Cs: E8M0 scales [rows, D/32].
// ABL (timing ablations, 0 in production; results are invalid otherwise):
//   1 = no ring refill after the prologue, 2 = no per-stage barrier, 4 = no epilogue
// QH: 32-centroid row tiles per ring stage (QH=2 halves the per-stage barrier / refill /
// norm-load overhead per MFMA; the stage index t then counts QH-tile stages).
// TOP2: also the runner-up centroid (labels2) and both distances (mind/mind2), for the
// exact re-check of near ties (recheck_top2_kernel); single K-group only.
template <class OP, int D, int WAVES, int NST, int ABL = 0, int QH = 1, bool TOP2 = false>
__global__ __launch_bounds__(WAVES * 64, 1) void assign_bigd_kernel(
    const uint8_t* __restrict__ X, const uint8_t* __restrict__ Xs, int64_t N, int64_t ldx,
    const uint8_t* __restrict__ Cm2, const uint8_t* Cs,
    const float* cnorm, int ntiles, int kg_tiles, int64_t npb, int64_t n_items,
    int64_t items_per_xcd, const float* __restrict__ xnorm, int32_t* __restrict__ labels,
    float* __restrict__ mind, unsigned long long* __restrict__ keys,
    int32_t* __restrict__ labels2 = nullptr, float* __restrict__ mind2 = nullptr) {
  constexpr int RB = D * OP::ES;        // bytes per row
  constexpr int HALFB = RB / 2;         // lane half h covers bytes [h*HALFB, (h+1)*HALFB)
  constexpr int NK = HALFB / OP::FB;    // MFMAs per 32x32 tile
  constexpr int CPR = RB / 16;
  constexpr int UPF = OP::FB / 16;      // 16-B LDS reads per fragment
  constexpr int TILE_B = QH * 32 * RB;
  constexpr int PIECES = TILE_B / 1024;
  constexpr int PPW = PIECES / WAVES;
  constexpr int SB = D / 32;            // scale bytes per row
  constexpr int NSW = OP::SCALED ? NK / 2 : 1;  // scale dwords per lane (= the row's)
  // per-stage side region, DMA'd with the tile: ||c||^2 of the QH*32 rows, then (fp8)
  // their E8M0 scale rows; every wave issues exactly ONE extra LDS-DMA for it (LPW lanes)
  constexpr int NRM_B = QH * 32 * 4;
  constexpr int EXB = NRM_B + (OP::SCALED ? QH * 32 * SB : 0);
  constexpr int EXC = EXB / 16;
  constexpr int LPW = (EXC + WAVES - 1) / WAVES;
  constexpr int STAGE_B = TILE_B + WAVES * LPW * 16;
  constexpr int VPS = PPW + 1;          // vector-memory ops per wave per stage
  static_assert(EXB % 16 == 0 && LPW <= 64, "side region");
  static_assert(RB % 256 == 0, "row bytes must be a multiple of 256");
  static_assert(PIECES % WAVES == 0, "stage must split evenly over the waves");
  static_assert(!OP::SCALED || NK % 2 == 0, "fp8: D must be a multiple of 128");
  constexpr unsigned EMB = 15u;
  // MFMAs of a stage issued after its barrier (their fragments already in registers):
  // fp8 D=768 69.4 -> 67.7 ms, D=512 26.5 -> 24.7 ms per pass (profiles/early_release_ab_r04s.txt)
  constexpr int ER = 2;
  static_assert(ER >= 1 && ER <= 2 && NK >= 2, "early release after the last fragment reads");
  // deferred epilogue (below) where its extra accumulator registers fit: one wave per SIMD
  // (512 VGPR+AGPR) below D = 1024 bf16 (where hipcc then re-loads the point fragments
  // instead), or two with at most 96 point-fragment VGPRs (fp8 up to D = 768)
  constexpr bool DEFER = (WAVES <= 4 && HALFB / 4 <= 224) || (OP::SCALED && HALFB / 4 <= 96);
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // ---- XCD-major work item: (centroid group g, point block pb) ----
  const int64_t b = blockIdx.x;
  const int64_t item = (b & 7) * items_per_xcd + (b >> 3);
  if (item >= n_items) return;  // whole block, before any barrier
  const int g = (int)(item / npb);
  const int64_t pb = item - (int64_t)g * npb;
  const int t0 = g * kg_tiles;
  const int t1 = min(ntiles, t0 + kg_tiles);
  const int nt = t1 - t0;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t prow = pb * (WAVES * 32) + w * 32 + r;
  const int64_t xrow = prow < N ? prow : N - 1;

  // ---- point fragments (B operand), resident for the whole group ----
  typename OP::frag bq[NK];
  if constexpr (OP::SCALED) {
    const uint8_t* src = X + xrow * ldx;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const i32x4 lo = *reinterpret_cast<const i32x4*>(src + fp8_off(kk, h, 0));
      const i32x4 hi = *reinterpret_cast<const i32x4*>(src + fp8_off(kk, h, 1));
      bq[kk] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  } else {
    const uint8_t* src = X + xrow * ldx + h * HALFB;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
      bq[kk] = *reinterpret_cast<const typename OP::frag*>(src + kk * OP::FB);
  }
  // E8M0 scales: lane half h applies the scale of block 2kk + h, byte 2(kk & 1) + h of
  // scale dword kk >> 1.  The dwords are shifted right by 8h once, so the byte is
  // 2(kk & 1) for both halves and the MFMA's byte select (op_sel) picks it: no per-MFMA
  // shift / mask (it was ~2 VALU per MFMA).
  const int hsh = 8 * h;
  int xs[NSW];
  if constexpr (OP::SCALED) {
    const int* s = reinterpret_cast<const int*>(Xs + xrow * SB);
#pragma unroll
    for (int i = 0; i < NSW; ++i) xs[i] = (int)((unsigned)s[i] >> hsh);
  }
  // fp8 A fragments: per-lane LDS byte offsets inside a 32-row tile, one VGPR per
  // distinct (chunk & 15): chunk 4kk + 2u + h of row r sits at swizzled chunk
  // 16 (kk >> 2) + ((4 (kk & 3) + 2u + h) ^ (r & 15)) (swz with 16 chunk groups), so the
  // kk >> 2 part is a ds_read immediate offset.  The per-read address arithmetic of the
  // generic form was ~3 VALU per MFMA.
  unsigned aoff8[8];
  if constexpr (OP::SCALED) {
    static_assert(RB >= 256 && NK % 4 == 0 || NK < 4, "fp8 swizzle: 16-chunk groups");
#pragma unroll
    for (int m = 0; m < 8; ++m)
      aoff8[m] = (unsigned)(r * RB + 16 * ((2 * m + h) ^ (r & 15)));
  }
  const unsigned lds_base =
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ring refill: per-lane byte offsets of this wave's pieces inside a stage (loop
  // invariant), issued by inline asm in the saddr + voffset form with M0 = the LDS
  // destination (the builtin made hipcc rebuild a 64-bit VGPR address per piece every
  // stage; the same change measured 1-5 % on the D <= 256 kernel, assign_mfma_impl.h).
  // The compiler does not count these loads; the explicit stage-end vmcnt waits do.
  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int L = (w * PPW + i) * 64 + lane;  // 16-B chunk index inside the stage
    const int row = L / CPR, cp = L % CPR;
    voff[i] = (unsigned)(row * RB + swz<RB>(row, cp) * 16);
  }
  const int wu = __builtin_amdgcn_readfirstlane(w);  // wave index in SGPRs (DMA destinations)
  auto issue = [&](int t, int slot) __attribute__((always_inline)) {
    const uint8_t* base = Cm2 + (int64_t)t * (32 * QH) * RB;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = wu * PPW + i;
      const unsigned dst = lds_base + slot * STAGE_B + piece * 1024;
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                   :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff[i]), "s"(base)
                   : "memory", "m0");
    }
    if (lane < LPW) {
      const int c = w * LPW + lane;  // 16-B chunk of the side region
      const uint8_t* src = reinterpret_cast<const uint8_t*>(cnorm);  // (pad chunks: dummy)
      if (c < NRM_B / 16)
        src = reinterpret_cast<const uint8_t*>(cnorm + (int64_t)t * (QH * 32)) + c * 16;
      else if (OP::SCALED && c < EXC)
        src = Cs + (int64_t)t * (QH * 32) * SB + (c - NRM_B / 16) * 16;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * STAGE_B + TILE_B + w * LPW * 16),
          16, 0, 0);
    }
  };
  float best = INFINITY, best2 = INFINITY;
  int bt = 0, bt2 = 0;
  // Deferred epilogue (DEFER): the min-reduction of tile i runs between the MFMAs of tile
  // i+1 (accp, independent of the chain in flight), so the VALU issues under the matrix
  // pipe instead of after every chain, where both waves of a SIMD sat in it at the same
  // time (fp8 D=768: 72.0 -> 69.8 ms per 2M x 65536 pass, profiles/fp8_defer_epi_ab_r04f.txt).
  f32x16 accp;
#pragma unroll
  for (int j = 0; j < 16; ++j) accp[j] = INFINITY;  // no pending tile: min stays +inf
  int ttp = 0;
  float pm = INFINITY, pm2 = INFINITY;
  auto epi_elem = [&](int j) __attribute__((always_inline)) {
    const float v = __uint_as_float((__float_as_uint(accp[j]) & ~EMB) | (unsigned)j);
    if constexpr (TOP2) {
      // pm <= pm2 kept.  asm as in ring3's top-2 epilogue (assign_mfma_impl.h): the builtins
      // canonicalise the tagged v first (one more VALU per score); v is never a signalling
      // NaN (tag bits only in normal values)
      float r1, r2;
      asm("v_med3_f32 %0, %1, %2, %3" : "=v"(r2) : "v"(pm), "v"(pm2), "v"(v));
      asm("v_min_f32 %0, %1, %2" : "=v"(r1) : "v"(pm), "v"(v));
      pm2 = r2;
      pm = r1;
    } else {
      pm = __builtin_fminf(pm, v);
    }
  };
  auto epi_fold = [&]() __attribute__((always_inline)) {
    const bool up = pm < best;
    if constexpr (TOP2) {  // runner-up of {best, best2} U {pm, pm2}, with its tile
      const float c = up ? best : pm;
      const int ct = up ? bt : ttp;
      const bool s2 = pm2 < c;
      const float cand = s2 ? pm2 : c;
      const int candt = s2 ? ttp : ct;
      const bool up2 = cand < best2;
      best2 = up2 ? cand : best2;
      bt2 = up2 ? candt : bt2;
    }
    best = up ? pm : best;
    bt = up ? ttp : bt;
    pm = pm2 = INFINITY;
  };
  // one ring stage: the tile, its norms and its scales all arrived by LDS-DMA NST-1
  // stages ago, so the only vmcnt wait per stage is the counted one on the ring.  The ring
  // slot is a compile-time constant (the stage loop below is unrolled by NST): the LDS
  // addresses of the slot and of the refill destinations fold into immediates instead of a
  // runtime i % NST and its address arithmetic every stage (~2.7 SALU per MFMA before).
  auto stage = [&](int i, auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value;
    const int t = t0 + i;
    if constexpr (!(ABL & 1)) {
      const int in = i + NST - 1;
      issue(t0 + (in < nt ? in : nt - 1), (slot + NST - 1) % NST);
    }
#pragma unroll
    for (int qh = 0; qh < QH; ++qh) {
    // LDS byte address of this lane's row in the slot
    const unsigned rbase = lds_base + slot * STAGE_B + (qh * 32 + r) * RB;
    const unsigned xbase = lds_base + slot * STAGE_B + TILE_B;
    // accumulator init = ||c||^2 of rows qh*32 + 8j + 4h + [0,4) (32x32 C layout) and the
    // scale row of centroid row qh*32 + r; issued before the fragments, so the first
    // counted lgkmcnt wait below also covers them
    f32x16 acc;
    const unsigned nbase = xbase + (qh * 32 + 4 * h) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 v;
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(nbase), "i"(32 * j));
      acc[4 * j + 0] = v[0];
      acc[4 * j + 1] = v[1];
      acc[4 * j + 2] = v[2];
      acc[4 * j + 3] = v[3];
    }
    int sa_row[NSW];
    if constexpr (OP::SCALED) {
      // the row's E8M0 scales as 8-byte reads (rows are SB = D/32 bytes apart: 8-B aligned).
      // At D=768 the 24-B row pitch made every ds_read_b32 2-way bank-conflicted (lanes r and
      // r+16); ds_read_b64 over 64 banks is conflict-free there, and half the instructions.
      static_assert(NSW % 2 == 0, "scale dwords in pairs");
      const unsigned sbase = xbase + NRM_B + (qh * 32 + r) * SB;
#pragma unroll
      for (int j = 0; j < NSW / 2; ++j) {
        i32x2 v;
        asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(sbase), "i"(8 * j));
        sa_row[2 * j] = v[0];
        sa_row[2 * j + 1] = v[1];
      }
    }
    const unsigned qbase = lds_base + slot * STAGE_B + qh * 32 * RB;
    // A fragments via inline-asm ds_read_b128: the compiler cannot prove they do not
    // alias the in-flight LDS-DMA ring refill, so compiler-visible LDS reads get a
    // vmcnt(0) in front of them (= waiting for the refill just issued, every stage).
    // Issued two MFMAs ahead; the lgkmcnt waits are explicit.
    auto lds_frag = [&](int kk) __attribute__((always_inline)) {
      typename OP::frag a;
      i32x4 lo, hi;
      if constexpr (UPF == 1) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(lo) : "v"(rbase + swz<RB>(r, h * (CPR / 2) + kk) * 16));
        a = __builtin_bit_cast(typename OP::frag, lo);
      } else {
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(lo) : "v"(qbase + aoff8[2 * (kk & 3)]), "i"(256 * (kk >> 2)));
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(hi) : "v"(qbase + aoff8[2 * (kk & 3) + 1]), "i"(256 * (kk >> 2)));
        a = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      return a;
    };
    typename OP::frag a0 = lds_frag(0);
    typename OP::frag a1 = lds_frag(NK > 1 ? 1 : 0);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      typename OP::frag a2 = a1;
      if (kk + 2 < NK) a2 = lds_frag(kk + 2);
      // reads still allowed in flight when a0 is consumed: those of a1 and a2
      constexpr int PER = UPF;  // ds_read instructions per fragment
      if (qh == QH - 1 && kk == NK - ER) {
        // early slot release: the stage's last ER fragments are in registers, so the
        // stage-end wait and barrier go here and those ER MFMAs run after it, under the
        // next stage's refill issue and first LDS reads (instead of the matrix pipe idling
        // through the barrier and the next stage's read latency)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (ABL & 1) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");  // stage i+1 landed
        }
        if constexpr (!(ABL & 2)) __builtin_amdgcn_s_barrier();  // ... for every wave's pieces
      } else if (kk + 2 < NK) {
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(2 * PER) : "memory");
      } else if (kk + 1 < NK) {
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(PER) : "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (OP::SCALED) {
        // the scale row was read before the fragments, so it has landed by the first wait
        if (kk == 0) {
#pragma unroll
          for (int j = 0; j < NSW; ++j) sa_row[j] = (int)((unsigned)sa_row[j] >> hsh);
        }
      }
      if constexpr (OP::SCALED) {  // block 2kk+h: dword kk>>1, byte 2(kk&1) after >> 8h
        if ((kk & 1) == 0) acc = mma<OP, 0>(a0, bq[kk], acc, sa_row[kk >> 1], xs[kk >> 1]);
        else acc = mma<OP, 2>(a0, bq[kk], acc, sa_row[kk >> 1], xs[kk >> 1]);
      } else {
        acc = mma<OP>(a0, bq[kk], acc, 0, 0);
      }
      // the previous tile's epilogue, spread over the chain (folds to constants unrolled)
      if constexpr (DEFER && !(ABL & 4)) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (j * NK / 16 == kk) epi_elem(j);
      }
      __builtin_amdgcn_sched_barrier(0);
      a0 = a1;
      a1 = a2;
    }
    if constexpr (ABL & 4) {
#pragma unroll
      for (int j = 0; j < 16; ++j) asm volatile("" ::"v"(acc[j]));
    } else if constexpr (DEFER) {
      epi_fold();
      accp = acc;
      ttp = t * QH + qh;  // 32-row tile index
    } else {
      accp = acc;
      ttp = t * QH + qh;
#pragma unroll
      for (int j = 0; j < 16; ++j) epi_elem(j);
      epi_fold();
    }
    }  // qh
  };

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(t0 + (s < nt ? s : nt - 1), s);
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
  __builtin_amdgcn_s_barrier();

  for (int i = 0; i < nt; i += NST) {
    stage(i, std::integral_constant<int, 0>{});
    if constexpr (NST > 1) if (i + 1 < nt) stage(i + 1, std::integral_constant<int, 1 % NST>{});
    if constexpr (NST > 2) if (i + 2 < nt) stage(i + 2, std::integral_constant<int, 2 % NST>{});
    if constexpr (NST > 3) if (i + 3 < nt) stage(i + 3, std::integral_constant<int, 3 % NST>{});
  }
  static_assert(NST <= 4, "stage loop unrolled up to 4 slots");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DEFER && !(ABL & 4)) {  // the last tile's epilogue
#pragma unroll
    for (int j = 0; j < 16; ++j) epi_elem(j);
    epi_fold();
  }

  const float ob = __shfl_xor(best, 32, 64);
  const int obt = __shfl_xor(bt, 32, 64);
  const unsigned e0 = __float_as_uint(best) & EMB, e1 = __float_as_uint(ob) & EMB;
  const int l0 = bt * 32 + (int)(e0 & 3) + 8 * (int)(e0 >> 2) + 4 * h;
  const int l1 = obt * 32 + (int)(e1 & 3) + 8 * (int)(e1 >> 2) + 4 * (1 - h);
  const float v0 = __uint_as_float(__float_as_uint(best) & ~EMB);
  const float v1 = __uint_as_float(__float_as_uint(ob) & ~EMB);
  const bool other = (v1 < v0) || (v1 == v0 && l1 < l0);
  if constexpr (TOP2) {  // merge the two lane halves' runner-ups
    const float ob2 = __shfl_xor(best2, 32, 64);
    const int obt2 = __shfl_xor(bt2, 32, 64);
    const unsigned f0 = __float_as_uint(best2) & EMB, f1 = __float_as_uint(ob2) & EMB;
    const int k0 = bt2 * 32 + (int)(f0 & 3) + 8 * (int)(f0 >> 2) + 4 * h;
    const int k1 = obt2 * 32 + (int)(f1 & 3) + 8 * (int)(f1 >> 2) + 4 * (1 - h);
    const float w0 = __uint_as_float(__float_as_uint(best2) & ~EMB);
    const float w1 = __uint_as_float(__float_as_uint(ob2) & ~EMB);
    // candidates: the loser of the two bests, and both runner-ups
    float cv = other ? v0 : v1;
    int cl = other ? l0 : l1;
    if (w0 < cv) { cv = w0; cl = k0; }
    if (w1 < cv) { cv = w1; cl = k1; }
    if (h == 0 && prow < N && labels2) {
      labels2[prow] = cl;
      if (mind2) mind2[prow] = fmaxf(cv + xnorm[prow], 0.f);
    }
  }
  if (h == 0 && prow < N) {
    const int lab = other ? l1 : l0;
    const float v = other ? v1 : v0;
    if (keys) {
      const unsigned long long key = ((unsigned long long)ord_bits(v) << 32) | (unsigned)lab;
      atomicMin(keys + prow, key);
    } else {
      labels[prow] = lab;
      if (mind) mind[prow] = fmaxf(v + xnorm[prow], 0.f);
    }
  }
}

// keys -> labels / mind, and reset keys for the next pass
__global__ __launch_bounds__(256) void keys_finalize_kernel(unsigned long long* __restrict__ keys,
                                                            int64_t N, const float* __restrict__ xnorm,
                                                            int32_t* __restrict__ labels,
                                                            float* __restrict__ mind) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const unsigned long long k = keys[i];
  labels[i] = (int32_t)(unsigned)(k & 0xffffffffull);
  if (mind) mind[i] = fmaxf(unord_bits((unsigned)(k >> 32)) + xnorm[i], 0.f);
  keys[i] = ~0ull;
}

// ------------------------------------------------------------------ fp8 quantiser (N8)
template <typename T>
__device__ __forceinline__ float ldf(const T* p) { return (float)*p; }

// One wave per row.  Lane l owns features [base + 8l, base + 8l + 8) of each 512-wide span;
// a 32-feature scale block = 4 consecutive lanes.  E8M0 exponent e = ilogb(amax) - 7 puts
// the block max in [128, 256) (no saturation, 13 binades of headroom below it).
// neg2: centroid operand (-2*c): sign flipped, exponent + 1, and norm = ||c~||^2 of the
// UN-negated dequantised row.  Rows >= valid: zero bytes, scale 1.0, norm = BIGN.
template <typename T>
__global__ __launch_bounds__(256) void quant_fp8_kernel(const T* __restrict__ X, int64_t rows,
                                                        int64_t valid, int d, int64_t ldx, int DP,
                                                        int neg2, uint8_t* __restrict__ Q,
                                                        uint8_t* __restrict__ S,
                                                        float* __restrict__ norm) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bool pad = row >= valid;
  float nsum = 0.f;
  for (int base = 0; base < DP; base += 512) {
    const int c0 = base + 8 * lane;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      v[j] = (!pad && c < d) ? ldf(X + row * ldx + c) : 0.f;
    }
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) am = fmaxf(am, fabsf(v[j]));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    if (c0 >= DP) continue;  // after the shuffles (all lanes took part)
    int e = am > 0.f ? ilogbf(am) - 7 : -127;
    e = e < -127 ? -127 : (e > 126 ? 126 : e);
    const float inv = ldexpf(1.f, -e);
    const float sc = ldexpf(1.f, e);
    int p0 = 0, p1 = 0;
    p0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, p0, false);
    p0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, p0, true);
    p1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, p1, false);
    p1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, p1, true);
    float f[8];
    f[0] = __builtin_amdgcn_cvt_f32_fp8(p0, 0); f[1] = __builtin_amdgcn_cvt_f32_fp8(p0, 1);
    f[2] = __builtin_amdgcn_cvt_f32_fp8(p0, 2); f[3] = __builtin_amdgcn_cvt_f32_fp8(p0, 3);
    f[4] = __builtin_amdgcn_cvt_f32_fp8(p1, 0); f[5] = __builtin_amdgcn_cvt_f32_fp8(p1, 1);
    f[6] = __builtin_amdgcn_cvt_f32_fp8(p1, 2); f[7] = __builtin_amdgcn_cvt_f32_fp8(p1, 3);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = f[j] * sc;
      nsum = fmaf(x, x, nsum);
    }
    if (neg2 && !pad) {
      p0 ^= 0x80808080;
      p1 ^= 0x80808080;
    }
    int2 pk;
    pk.x = p0;
    pk.y = p1;
    *reinterpret_cast<int2*>(Q + row * DP + c0) = pk;
    if ((lane & 3) == 0) S[row * (DP / 32) + c0 / 32] = (uint8_t)(e + 127 + (neg2 ? 1 : 0));
  }
  nsum = wave_sum(nsum);
  if (lane == 0 && norm) norm[row] = pad ? BIGN : nsum;
}

}  // namespace bigd
}  // namespace tdc

using namespace tdc::bigd;

namespace {
template <class OP, int D, int WAVES, int NST, int ABL = 0, int QH = 1, bool TOP2 = false>
int launch_bigd(const void* X, const void* Xs, int64_t N, int64_t ldx_bytes, const void* Cm2,
                const void* Cs, const float* cnorm, int Kp, int kg_tiles, const float* xnorm,
                int32_t* labels, float* mind, unsigned long long* keys, hipStream_t stream,
                int32_t* labels2 = nullptr, float* mind2 = nullptr) {
  // = the kernel's STAGE_B: tile + one 16-B side chunk per lane of LPW lanes per wave
  constexpr int TILE_B = QH * 32 * D * OP::ES;
  constexpr int EXB = QH * 32 * 4 + (OP::SCALED ? QH * 32 * (D / 32) : 0);
  constexpr int LPW = (EXB / 16 + WAVES - 1) / WAVES;
  const size_t lds = (size_t)NST * (TILE_B + WAVES * LPW * 16);
  auto kern = assign_bigd_kernel<OP, D, WAVES, NST, ABL, QH, TOP2>;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  // stages of QH 32-row tiles (the caller checked Kp % (32*QH) == 0); a K-group is a
  // whole number of stages (the group size is an L2-residency tunable, labels do not
  // depend on it)
  const int ntiles = Kp / (32 * QH);
  if (kg_tiles > 0) kg_tiles = kg_tiles / QH > 0 ? kg_tiles / QH : 1;
  if (kg_tiles <= 0 || kg_tiles > ntiles) kg_tiles = ntiles;
  const int ngroups = (ntiles + kg_tiles - 1) / kg_tiles;
  if (ngroups > 1 && keys == nullptr) return (int)hipErrorInvalidValue;
  if (TOP2 && ngroups > 1) return (int)hipErrorInvalidValue;  // runner-up: one K-group only
  const int64_t per = (int64_t)WAVES * 32;
  const int64_t npb = (N + per - 1) / per;
  const int64_t n_items = npb * ngroups;
  const int64_t ipx = (n_items + 7) / 8;
  dim3 grid((unsigned)(ipx * 8));
  hipLaunchKernelGGL(kern, grid, dim3(WAVES * 64), lds, stream, (const uint8_t*)X,
                     (const uint8_t*)Xs, N, ldx_bytes, (const uint8_t*)Cm2, (const uint8_t*)Cs,
                     cnorm, ntiles, kg_tiles, npb, n_items, ipx, xnorm, labels, mind,
                     ngroups > 1 ? keys : nullptr, labels2, mind2);
  TDC_CHECK_LAUNCH();
  if (ngroups > 1) {
    hipLaunchKernelGGL(keys_finalize_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0,
                       stream, keys, N, xnorm, labels, mind);
    TDC_CHECK_LAUNCH();
  }
  return 0;
}
}  // namespace

int tdc_assign_bigd_supported(int dtype, int DP) {
  // (bf16 D > 512: one wave per SIMD, the point fragments spill into AGPRs; 56-64 KiB
  // stages 2 deep above D=768; D > 1024 would not fit the register file)
  if (dtype == TDC_FP8) return DP == 256 || DP == 512 || DP == 768 || DP == 1024;
  if (dtype == TDC_BF16)
    return DP == 384 || DP == 512 || DP == 640 || DP == 768 || DP == 896 || DP == 1024;
  return 0;
}

int tdc_assign_bigd(int dtype, const void* X, const void* Xs, int64_t N, int64_t ldx, int DP,
                    const void* Cm2, const void* Cs, const float* cnorm, int Kp, int kg_tiles,
                    const float* xnorm, int32_t* labels, float* mind, unsigned long long* keys,
                    hipStream_t stream, int32_t* labels2, float* mind2) {
  if (N <= 0) return 0;
  if (Kp % 32 != 0) return (int)hipErrorInvalidValue;
  if (labels2 != nullptr) {  // fp8 with runner-up (near-tie re-check)
    if (dtype != TDC_FP8) return (int)hipErrorInvalidValue;
    switch (DP) {
      case 256: return launch_bigd<OpFp8, 256, 8, 4, 0, 1, true>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream, labels2, mind2);
      case 512: return launch_bigd<OpFp8, 512, 8, 4, 0, 1, true>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream, labels2, mind2);
      case 768:
        if (Kp % 64 == 0)
          return launch_bigd<OpFp8, 768, 8, 3, 0, 2, true>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream, labels2, mind2);
        return launch_bigd<OpFp8, 768, 8, 4, 0, 1, true>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream, labels2, mind2);
      case 1024: return launch_bigd<OpFp8, 1024, 8, 4, 0, 1, true>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream, labels2, mind2);
    }
    return (int)hipErrorInvalidValue;
  }
  if (dtype == TDC_FP8) {
    switch (DP) {
      case 256: return launch_bigd<OpFp8, 256, 8, 4>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      case 512: return launch_bigd<OpFp8, 512, 8, 4>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      case 768: {
        // 64-row stages (QH=2): 206.5 vs 211.8 ms (grouped), 197.3 vs 200.8 ms (one group)
        // at N=5M.  The ablations (ABL) are instantiated by tools harnesses only.
        if (Kp % 64 == 0)
          return launch_bigd<OpFp8, 768, 8, 3, 0, 2>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
        return launch_bigd<OpFp8, 768, 8, 4>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      }
      case 1024: return launch_bigd<OpFp8, 1024, 8, 4>(X, Xs, N, ldx, Cm2, Cs, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
    }
  } else if (dtype == TDC_BF16) {
    const int64_t ldb = ldx * 2;
    switch (DP) {
      case 384: return launch_bigd<OpBf16, 384, 8, 4>(X, nullptr, N, ldb, Cm2, nullptr, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      // D >= 512: the point fragments (D/4 VGPRs) need one wave per SIMD (4-wave groups,
      // accumulators in AGPRs; 8 waves spilled 45 VGPRs at D=512); 32-48 KiB stages, 3 deep
      case 512: return launch_bigd<OpBf16, 512, 4, 3>(X, nullptr, N, ldb, Cm2, nullptr, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      case 640: return launch_bigd<OpBf16, 640, 4, 3>(X, nullptr, N, ldb, Cm2, nullptr, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      case 768: return launch_bigd<OpBf16, 768, 4, 3>(X, nullptr, N, ldb, Cm2, nullptr, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      case 896: return launch_bigd<OpBf16, 896, 4, 2>(X, nullptr, N, ldb, Cm2, nullptr, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
      case 1024: return launch_bigd<OpBf16, 1024, 4, 2>(X, nullptr, N, ldb, Cm2, nullptr, cnorm, Kp, kg_tiles, xnorm, labels, mind, keys, stream);
    }
  }
  return (int)hipErrorInvalidValue;
}

namespace {
// Exact re-check of the fp8 winner against the runner-up: one wave per point whose fp8
// margin d2 - d1 is within tau * d2 (the quantisation noise of both operands), distances
// in fp32 difference form from the full-precision row and centroids.  Points with a
// clear margin exit after reading two floats.
template <typename XT>
__global__ __launch_bounds__(256) void recheck_top2_kernel(const XT* __restrict__ X, int64_t ldx,
                                                           int D, const float* __restrict__ C,
                                                           int32_t* __restrict__ labels,
                                                           const int32_t* __restrict__ labels2,
                                                           const float* __restrict__ d1,
                                                           const float* __restrict__ d2, float tau,
                                                           int64_t N, int* __restrict__ flips) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= N) return;
  const float a = d1[i], b = d2[i];
  if (!(b - a <= tau * b)) return;  // clear margin (NaN-safe: NaN re-checks)
  const int l1 = labels[i], l2 = labels2[i];
  if (l1 == l2) return;
  const XT* x = X + i * ldx;
  const float* c1 = C + (int64_t)l1 * D;
  const float* c2 = C + (int64_t)l2 * D;
  float s1 = 0.f, s2 = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float xv = (float)x[d];
    const float e1 = xv - c1[d], e2 = xv - c2[d];
    s1 = fmaf(e1, e1, s1);
    s2 = fmaf(e2, e2, s2);
  }
  s1 = tdc::wave_sum(s1);
  s2 = tdc::wave_sum(s2);
  if (lane == 0 && (s2 < s1 || (s2 == s1 && l2 < l1))) {
    labels[i] = l2;
    if (flips) atomicAdd(flips, 1);
  }
}
}  // namespace

int tdc_recheck_top2(int x_dtype, const void* X, int64_t N, int64_t ldx, int D, const float* C,
                     int32_t* labels, const int32_t* labels2, const float* d1, const float* d2,
                     float tau, int* flips, hipStream_t stream) {
  if (N <= 0) return 0;
  const dim3 grid((unsigned)((N + 3) / 4));
  if (x_dtype == TDC_BF16)
    hipLaunchKernelGGL(recheck_top2_kernel<__bf16>, grid, dim3(256), 0, stream, (const __bf16*)X,
                       ldx, D, C, labels, labels2, d1, d2, tau, N, flips);
  else if (x_dtype == TDC_F32)
    hipLaunchKernelGGL(recheck_top2_kernel<float>, grid, dim3(256), 0, stream, (const float*)X,
                       ldx, D, C, labels, labels2, d1, d2, tau, N, flips);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_quant_fp8(int src_dtype, const void* X, int64_t rows, int64_t valid, int d, int64_t ldx,
                  int DP, int neg2, void* Q, void* S, float* norm, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (DP % 32 != 0 || d > DP) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)((rows + 3) / 4));
  switch (src_dtype) {
    case TDC_F32:
      hipLaunchKernelGGL(quant_fp8_kernel<float>, grid, dim3(256), 0, stream, (const float*)X, rows,
                         valid, d, ldx, DP, neg2, (uint8_t*)Q, (uint8_t*)S, norm);
      break;
    case TDC_F64:
      hipLaunchKernelGGL(quant_fp8_kernel<double>, grid, dim3(256), 0, stream, (const double*)X,
                         rows, valid, d, ldx, DP, neg2, (uint8_t*)Q, (uint8_t*)S, norm);
      break;
    case TDC_BF16:
      hipLaunchKernelGGL(quant_fp8_kernel<__bf16>, grid, dim3(256), 0, stream, (const __bf16*)X,
                         rows, valid, d, ldx, DP, neg2, (uint8_t*)Q, (uint8_t*)S, norm);
      break;
    default:
      return (int)hipErrorInvalidValue;
  }
  TDC_CHECK_LAUNCH();
  return 0;
}
