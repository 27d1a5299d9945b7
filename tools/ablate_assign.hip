// Ablation / A-B harness for the bf16 MFMA assign kernels (cdna_hip_programming.md §7:
// ablate before optimising; §5.4 rule 24: compare variants in ONE process, interleaved).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/ablate_assign.hip -o build/ablate_assign
//   ./build/ablate_assign [N] [K]          (stand-alone, HIP runtime from /opt/rocm)
//   tools/ablate_in_torch.py               (same code as a .so inside a PyTorch process)
//
// Data: Gaussian blobs around K uniform(-10,10) centers (splitmix64 + Box-Muller) -- the
// kernel's clock under load is data dependent, so never time on constant/trivial fills.
// Correctness: labels are poisoned (-1) before every checked run and compared against the
// register-staged kernel.  ABL != 0 variants remove work and give invalid labels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "assign_mfma_impl.h"
#include "assign_mfma_legacy.h"  // tools/

using namespace tdc;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

// NST == 0: register-staged kernel; else LDS-DMA ring kernel with WAVES x QT geometry
template <int DP, int P, int ABL, int NST = 0, int WAVES = 4, int QT = 2>
void launch(const __bf16* X, int64_t N, const __bf16* C, const float* cn, int Kp, int* lab,
            float* md, hipStream_t s) {
  const int64_t per = (NST ? WAVES : 4) * P * 32;
  const dim3 grid((unsigned)((N + per - 1) / per));
  const int ntiles = Kp / (NST ? 32 * QT : 64);
  if constexpr (NST == 0)
    hipLaunchKernelGGL((assign_mfma_bf16_kernel<DP, P, ABL>), grid, dim3(256), 0, s, X, N,
                       (int64_t)DP, C, cn, ntiles, lab, md);
  else
    hipLaunchKernelGGL((assign_mfma_bf16_ring_kernel<DP, P, NST, WAVES, QT, ABL>), grid,
                       dim3(WAVES * 64), 0, s, X, N, (int64_t)DP, C, cn, ntiles, lab, md);
}

// wall-clock ms per launch over `reps` launches, device-synchronised around the batch
template <int DP, int P, int ABL, int NST = 0, int WAVES = 4, int QT = 2>
float timed(const __bf16* X, int64_t N, const __bf16* C, const float* cn, int Kp, int* lab,
            float* md, int reps = 10) {
  launch<DP, P, ABL, NST, WAVES, QT>(X, N, C, cn, Kp, lab, md, 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) launch<DP, P, ABL, NST, WAVES, QT>(X, N, C, cn, Kp, lab, md, 0);
  CK(hipDeviceSynchronize());
  const auto t1 = std::chrono::steady_clock::now();
  return std::chrono::duration<float, std::milli>(t1 - t0).count() / reps;
}

struct Problem {
  int64_t N;
  int K;
  __bf16 *X, *C;
  float *cn, *md;
  int* lab;
};

static Problem make_problem(int64_t N, int K) {
  constexpr int DP = 128;
  uint64_t st = 0x9E3779B97F4A7C15ull;
  auto u01 = [&]() {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return ((z >> 11) + 0.5) * (1.0 / 9007199254740992.0);
  };
  auto gauss = [&]() {
    return (float)(std::sqrt(-2.0 * std::log(u01())) * std::cos(6.283185307179586 * u01()));
  };
  std::vector<float> cf((size_t)K * DP);
  for (auto& v : cf) v = (float)(__bf16)(10.f * (float)(2.0 * u01() - 1.0));
  std::vector<__bf16> hc(cf.size()), hx((size_t)N * DP);
  std::vector<float> hn(K);
  for (int k = 0; k < K; ++k) {
    float s2 = 0.f;
    for (int d = 0; d < DP; ++d) {
      const float v = cf[(size_t)k * DP + d];
      hc[(size_t)k * DP + d] = (__bf16)(-2.f * v);
      s2 += v * v;
    }
    hn[k] = s2;
  }
  for (int64_t i = 0; i < N; ++i) {
    const int b = (int)(u01() * K);
    for (int d = 0; d < DP; ++d) hx[i * DP + d] = (__bf16)(cf[(size_t)b * DP + d] + gauss());
  }
  Problem p{N, K, nullptr, nullptr, nullptr, nullptr, nullptr};
  CK(hipMalloc(&p.X, hx.size() * 2));
  CK(hipMalloc(&p.C, hc.size() * 2));
  CK(hipMalloc(&p.cn, K * 4));
  CK(hipMalloc(&p.lab, N * 4));
  CK(hipMalloc(&p.md, N * 4));
  CK(hipMemcpy(p.X, hx.data(), hx.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(p.C, hc.data(), hc.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(p.cn, hn.data(), K * 4, hipMemcpyHostToDevice));
  return p;
}

// poisoned-output comparison of the ring kernel against the register-staged kernel
static void check(const Problem& p) {
  std::vector<int> a(p.N), b(p.N);
  CK(hipMemset(p.lab, 0xff, p.N * 4));
  launch<128, 2, 0>(p.X, p.N, p.C, p.cn, p.K, p.lab, p.md, 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(a.data(), p.lab, p.N * 4, hipMemcpyDeviceToHost));
  CK(hipMemset(p.lab, 0xff, p.N * 4));
  launch<128, 2, 0, 3, 4, 2>(p.X, p.N, p.C, p.cn, p.K, p.lab, p.md, 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(b.data(), p.lab, p.N * 4, hipMemcpyDeviceToHost));
  std::vector<int> c(p.N);
  CK(hipMemset(p.lab, 0xff, p.N * 4));
  launch<128, 2, 0, 3, 12, 3>(p.X, p.N, p.C, p.cn, p.K, p.lab, p.md, 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(c.data(), p.lab, p.N * 4, hipMemcpyDeviceToHost));
  size_t diff12 = 0, unset_c = 0;
  for (int64_t i = 0; i < p.N; ++i) { diff12 += a[i] != c[i]; unset_c += c[i] < 0; }
  printf("check: w12q3 unset %zu, mismatches %zu\n", unset_c, diff12);
  size_t unset_a = 0, unset_b = 0, diff = 0;
  for (int64_t i = 0; i < p.N; ++i) {
    unset_a += a[i] < 0;
    unset_b += b[i] < 0;
    diff += a[i] != b[i];
  }
  printf("check: regstage unset %zu, ring unset %zu, mismatches %zu of %lld\n", unset_a,
         unset_b, diff, (long long)p.N);
}

extern "C" int ablate_main(long long n_arg, int k_arg) {
  const int64_t N = n_arg > 0 ? n_arg : 10000000;
  const int K = ((k_arg > 0 ? k_arg : 1152) + 191) / 192 * 192;  // divisible by 64 and 96
  Problem p = make_problem(N, K);
  check(p);
  const double flop = 2.0 * N * K * 128;
  const char* names[] = {"regstage", "regstage no_epilogue", "regstage no_staging",
                         "ring w4 q2 n3 (library)", "ring w12 q3 n3", "ring w12 q3 n2",
                         "ring w8 q2 n3", "ring w12 q3 n3 no_epi"};
  constexpr int NV = 8;
  float best[NV];
  for (float& b : best) b = 1e30f;
  for (int round = 0; round < 3; ++round) {
    best[0] = std::min(best[0], timed<128, 2, 0>(p.X, N, p.C, p.cn, K, p.lab, p.md));
    best[1] = std::min(best[1], timed<128, 2, 1>(p.X, N, p.C, p.cn, K, p.lab, p.md));
    best[2] = std::min(best[2], timed<128, 2, 2>(p.X, N, p.C, p.cn, K, p.lab, p.md));
    best[3] = std::min(best[3], timed<128, 2, 0, 3, 4, 2>(p.X, N, p.C, p.cn, K, p.lab, p.md));
    best[4] = std::min(best[4], timed<128, 2, 0, 3, 12, 3>(p.X, N, p.C, p.cn, K, p.lab, p.md));
    best[5] = std::min(best[5], timed<128, 2, 0, 2, 12, 3>(p.X, N, p.C, p.cn, K, p.lab, p.md));
    best[6] = std::min(best[6], timed<128, 2, 0, 3, 8, 2>(p.X, N, p.C, p.cn, K, p.lab, p.md));
    best[7] = std::min(best[7], timed<128, 2, 1, 3, 12, 3>(p.X, N, p.C, p.cn, K, p.lab, p.md));
  }
  for (int v = 0; v < NV; ++v)
    printf("%-26s %8.3f ms  %7.1f TFLOP/s\n", names[v], best[v], flop / best[v] / 1e9);
  check(p);
  return 0;
}

// time the library-configuration ring kernel on caller-provided buffers (torch tensors)
extern "C" float ablate_ring_on(const void* X, long long N, const void* C, const float* cn,
                                int Kp, int* lab, float* md) {
  return timed<128, 2, 0, 3, 4, 2>((const __bf16*)X, N, (const __bf16*)C, cn, Kp, lab, md);
}

#ifndef ABLATE_NO_MAIN
int main(int argc, char** argv) {
  return ablate_main(argc > 1 ? atoll(argv[1]) : 0, argc > 2 ? atoi(argv[2]) : 0);
}
#endif
