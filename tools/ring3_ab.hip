// A/B harness: schedule variants of the production ring3 assign kernel
// (csrc/assign_mfma_impl.h, assign_mfma_bf16_ring3_kernel) on the headline shape, timed
// interleaved in one process (cdna_hip_programming.md §5.4 rule 24), labels compared.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/ring3_ab.hip -o build/ring3_ab
//   ./build/ring3_ab [N] [K] [reps]
//
// Variants (VAR bits of ring3x_kernel, a copy of the production kernel):
//   1: the next stage's LDS-DMA pieces are issued one per phase (at the phase start)
//      instead of all at the start of the stage (the guide's issue-cost row:
//      ~60 cycles per piece among bare MFMAs, 100-185 inside a phase already carrying
//      pieces and fragment reads)
//   2: s_setprio(1) around every MFMA cluster (guide T5)
//   4: index tags carry the stage within a super-stage of 16 (8 tag bits)
//   8: half-P software pipeline inside each phase: the MFMAs of point tiles 0..P/2-1 run
//      with the tag + min epilogue of tiles P/2..P-1 of the previous phase between them,
//      then the MFMAs of tiles P/2.. with the epilogue of tiles 0..P/2-1 of this phase
//      (no extra accumulators: each half's registers are read before they are rewritten),
//      instead of 32 MFMAs and then a 48-VALU epilogue burst
// Data: Gaussian blobs around K uniform(-10,10) centres (splitmix64 + Box-Muller).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <int DP, int P, int NST, int WAVES, int QT, int VAR>
__global__ __launch_bounds__(WAVES * 64, ((DP >= 128 && P >= 8) ? 2 : 3))
void ring3x_kernel(const __bf16* __restrict__ X, int64_t N, int64_t ldx,
                   const __bf16* __restrict__ Cm2, const float* __restrict__ cnorm, int ntiles,
                   int32_t* __restrict__ labels) {
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
  constexpr bool SPREAD = (VAR & 1) != 0;
  constexpr bool PRIO = (VAR & 2) != 0;
  static_assert(!SPREAD || PPW <= QT, "one piece per phase");
  // VAR 4: the tag also carries the stage within a super-stage of 16 stages (8 tag bits for
  // QT=4), so the per-stage compare / select of the running best becomes one v_min_f32
  // per point tile, and the compare / select runs once per super-stage
  constexpr bool STAGETAG = (VAR & 4) != 0;
  constexpr bool HALFP = (VAR & 8) != 0;
  static_assert(!HALFP || (P % 2 == 0 && !STAGETAG && !SPREAD && KS == 4), "half-P form");
  static_assert(!STAGETAG || QT == 4, "stage tags: 4 (q, reg) bits + 4 stage bits");
  if (STAGETAG && ntiles > 16) return;  // experiment covers K <= 1024
  constexpr unsigned EMB = STAGETAG ? 255u : (QT * 4 <= 16 ? 15u : 31u);
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE_B];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 15;
  const int g = lane >> 4;
  const int64_t pbase = (int64_t)blockIdx.x * (WAVES * P * 16) + (int64_t)w * (P * 16);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  bf16x8 bq[P][KS];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 16 + r;
    if (row >= N) row = N - 1;
    const __bf16* src = X + row * ldx + g * 8;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) bq[p][kk] = *reinterpret_cast<const bf16x8*>(src + kk * 32);
  }

  // per-lane byte offsets of this wave's pieces inside a stage (loop invariant: one VGPR
  // each; the stage base is wave-uniform, so the DMA takes the saddr + voffset form)
  unsigned voff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int pc = (w * PPW + i) % PIECES;
    const int L = pc * 64 + lane;
    const int row = L / CPR, cp = L % CPR;
    voff[i] = (unsigned)((row * DP + swz<DP>(row, cp) * 8) * 2);
  }
  // inline asm (saddr + voffset, M0 = LDS destination): with the builtin, hipcc hoists a
  // 64-bit VGPR address per piece and stage out of the unrolled ring loop and spills them
  auto piece = [&](int t, int slot, int i) __attribute__((always_inline)) {
    const int pc = (w * PPW + i) % PIECES;
    const __bf16* base = Cm2 + (int64_t)t * BNL * DP;
    const unsigned dst = lds0 + slot * STAGE_B + pc * 1024;
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2"
                 :: "s"(__builtin_amdgcn_readfirstlane(dst)), "v"(voff[i]), "s"(base) : "memory", "m0");
  };
  auto norms = [&](int t, int slot) __attribute__((always_inline)) {
    const int nb = w * NPW < NCH - NPW ? w * NPW : NCH - NPW;
    if (lane < NPW) {
      const float* src = cnorm + (int64_t)t * BNL + (nb + lane) * 4;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(smem + slot * STAGE_B + TILE_B + nb * 16),
          16, 0, 0);
    }
  };
  auto issue = [&](int t, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) piece(t, slot, i);
    norms(t, slot);
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
  for (int kk = 0; kk < KS; ++kk) aoff[kk] = lds0 + r * (DP * 2) + swz<DP>(r, kk * 4 + g) * 16;
  const unsigned noff = lds0 + TILE_B + 16 * g;
  unsigned vmask = ~EMB;
  asm volatile("" : "+v"(vmask));  // keep the non-inline mask in one VGPR

  auto stage = [&](int t, auto slot_c) __attribute__((always_inline)) {
    constexpr int slot = decltype(slot_c)::value;
    constexpr int nslot = (slot + NST - 1) % NST;
    const int tn0 = t + NST - 1;
    const int tn = tn0 < ntiles ? tn0 : ntiles - 1;
    if constexpr (!SPREAD) issue(tn, nslot);
    float m[P];
#pragma unroll
    for (int p = 0; p < P; ++p) m[p] = STAGETAG ? best[p] : INFINITY;
    const unsigned stag = STAGETAG ? (unsigned)((t & 15) << 4) : 0u;
    if constexpr (HALFP) {
      constexpr int H = P / 2;
      f32x4 acc[P];
      auto epi1 = [&](int p, int q) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 4 + i));
          m[p] = __builtin_fminf(m[p], v);
        }
      };
      bf16x8 a[KS];
#pragma unroll
      for (int q = 0; q < QT; ++q) {
        f32x4 n4;
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(n4) : "v"(noff), "i"(slot * STAGE_B + q * 16 * 4));
#pragma unroll
        for (int kk = 0; kk < KS; ++kk)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(a[kk]) : "v"(aoff[kk]), "i"(slot * STAGE_B + q * 16 * DP * 2));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        // tiles 0..H-1 of phase q, with the epilogue of tiles H.. of phase q-1
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
          for (int p = 0; p < H; ++p)
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk], bq[p][kk], kk == 0 ? n4 : acc[p], 0, 0, 0);
          if (q > 0) {
#pragma unroll
            for (int p = H + kk * H / KS; p < H + (kk + 1) * H / KS; ++p) epi1(p, q - 1);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        // tiles H.. of phase q, with the epilogue of tiles 0..H-1 of phase q
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
#pragma unroll
          for (int p = H; p < P; ++p)
            acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kk], bq[p][kk], kk == 0 ? n4 : acc[p], 0, 0, 0);
#pragma unroll
          for (int p = kk * H / KS; p < (kk + 1) * H / KS; ++p) epi1(p, q);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int p = H; p < P; ++p) epi1(p, QT - 1);
    }
#pragma unroll
    for (int q = 0; q < (HALFP ? 0 : QT); ++q) {
      auto afrag = [&](int kk) __attribute__((always_inline)) {
        bf16x8 a;
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(a) : "v"(aoff[kk]), "i"(slot * STAGE_B + q * 16 * DP * 2));
        return a;
      };
      if constexpr (SPREAD) {  // one piece per phase, before the phase's fragment reads
        if (q < PPW) piece(tn, nslot, q);
        if (q == QT - 1) norms(tn, nslot);
      }
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
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int p = 0; p < P; ++p)
          acc[p] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bq[p][kk], kk == 0 ? n4 : acc[p],
                                                            0, 0, 0);
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        a0 = a1;
        a1 = a2;
      }
#pragma unroll
      for (int p = 0; p < P; ++p) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v;
          if constexpr (STAGETAG) {  // one v_and_or_b32: mask in a VGPR, tag in an SGPR
            const unsigned tg = __builtin_amdgcn_readfirstlane(stag | (unsigned)(q * 4 + i));
            v = __uint_as_float((__float_as_uint(acc[p][i]) & vmask) | tg);
          } else {
            v = __uint_as_float((__float_as_uint(acc[p][i]) & ~EMB) | (unsigned)(q * 4 + i));
          }
          m[p] = __builtin_fminf(m[p], v);
        }
      }
    }
    if constexpr (STAGETAG) {
#pragma unroll
      for (int p = 0; p < P; ++p) best[p] = m[p];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      if constexpr (STAGETAG) {
        // experiment: one super-stage (ntiles <= 16, K <= 1024): best is a plain minimum
      } else {
        const bool up = m[p] < best[p];
        best[p] = up ? m[p] : best[p];
        bt[p] = up ? t : bt[p];
      }
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"((NST - 2) * VPS) : "memory");
    __builtin_amdgcn_s_barrier();
  };

  for (int t0 = 0; t0 < ntiles; t0 += NST) {
    stage(t0, std::integral_constant<int, 0>{});
    if constexpr (NST > 1) if (t0 + 1 < ntiles) stage(t0 + 1, std::integral_constant<int, 1>{});
    if constexpr (NST > 2) if (t0 + 2 < ntiles) stage(t0 + 2, std::integral_constant<int, 2 % NST>{});
    if constexpr (NST > 3) if (t0 + 3 < ntiles) stage(t0 + 3, std::integral_constant<int, 3 % NST>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

#pragma unroll
  for (int p = 0; p < P; ++p) {
    const unsigned e = __float_as_uint(best[p]) & EMB;
    int lab = STAGETAG ? (bt[p] * 16 + (int)(e >> 4)) * BNL + (int)((e & 15) >> 2) * 16 + 4 * g + (int)(e & 3)
                       : bt[p] * BNL + (int)(e >> 2) * 16 + 4 * g + (int)(e & 3);
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

static void prod4(const Bufs& b, hipStream_t s) {  // the short-launch (< 4M rows) schedule
  const int64_t per = 4 * 4 * 16;
  hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 4, 3, 4, 4>),
                     dim3((unsigned)((b.n + per - 1) / per)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / 64, b.lab, nullptr);
}

template <int P, int NST, int QT, int VAR>
static void var(const Bufs& b, hipStream_t s) {
  const int64_t per = 4 * P * 16;
  hipLaunchKernelGGL((ring3x_kernel<128, P, NST, 4, QT, VAR>),
                     dim3((unsigned)((b.n + per - 1) / per)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / (16 * QT), b.lab);
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
  printf("N=%lld K=%d D=%d\n", (long long)N, K, DP);
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
    printf("  %-24s mismatches vs production: %lld\n", name, (long long)bad);
    fflush(stdout);
  };
  prod(b0, 0);
#define TRY(NAME, ...)                     \
  CK(hipMemset(l1, 0xff, N * 4));          \
  __VA_ARGS__(b1, 0);                      \
  check(NAME);
  TRY("copy (VAR 0)", var<8, 2, 4, 0>)
  TRY("spread", var<8, 2, 4, 1>)
  TRY("setprio", var<8, 2, 4, 2>)
  TRY("spread+setprio", var<8, 2, 4, 3>)
  TRY("P4 NST3 spread", var<4, 3, 4, 1>)
  TRY("prod P4 NST3", prod4)
  TRY("stage tags P8", var<8, 2, 4, 4>)
  TRY("stage tags P4 NST3", var<4, 3, 4, 4>)
  TRY("half-P pipeline P8", var<8, 2, 4, 8>)
  TRY("copy P8 NST3", var<8, 3, 4, 0>)
  const double flop = 2.0 * (double)N * Kp * DP;
  for (int round = 0; round < 3; ++round) {
    const float t0 = timeit([&] { prod(b0, 0); }, reps);
    const float t1 = timeit([&] { var<8, 2, 4, 0>(b1, 0); }, reps);
    const float t3 = timeit([&] { var<8, 2, 4, 4>(b1, 0); }, reps);
    const float t5 = timeit([&] { prod4(b1, 0); }, reps);
    const float t6 = timeit([&] { var<4, 3, 4, 4>(b1, 0); }, reps);
    const float t7 = timeit([&] { var<8, 2, 4, 8>(b1, 0); }, reps);
    const float t8 = timeit([&] { var<8, 3, 4, 0>(b1, 0); }, reps);
    printf("round %d: prod P8 %.3f ms (%.0f TF/s) | copy P8 %.3f | stagetag P8 %.3f | "
           "prod P4N3 %.3f | stagetag P4N3 %.3f | half-P P8 %.3f | copy P8 NST3 %.3f\n",
           round, t0, flop / t0 / 1e9, t1, t3, t5, t6, t7, t8);
    fflush(stdout);
  }
  return 0;
}
