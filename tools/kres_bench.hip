// A/B harness: the K-resident assign (csrc/assign_kres.h) against the production ring3
// kernel (csrc/assign_mfma_impl.h) on the same data, in one process, interleaved
// (cdna_hip_programming.md §5.4 rule 24).  Labels are compared point by point.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc -I tools tools/kres_bench.hip -o build/kres_bench
//   ./build/kres_bench [N] [K]
//
// Data: Gaussian blobs around K uniform(-10,10) centres (splitmix64 + Box-Muller); the
// clock under load is data dependent, so never time on constant fills.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "assign_kres.h"

using namespace tdc;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

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
  float2* keys;
};

static void ring3(const Bufs& b, hipStream_t s) {
  const int64_t per8 = 4 * 8 * 16;
  hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 8, 2, 4, 4>),
                     dim3((unsigned)((b.n + per8 - 1) / per8)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / 64, b.lab, nullptr);
}

static void ring3p4(const Bufs& b, hipStream_t s) {  // the short-launch schedule
  const int64_t per = 4 * 4 * 16;
  hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 4, 3, 4, 4>),
                     dim3((unsigned)((b.n + per - 1) / per)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / 64, b.lab, nullptr);
}

template <int P, int WAVES, bool PF, bool R3 = false>
static void kres(const Bufs& b, hipStream_t s, int cus) {
  constexpr int R = KresGeom<DP>::R;
  const int ksplit = (b.kp + R - 1) / R;
  int grid = cus / (8 * ksplit) * (8 * ksplit);
  hipLaunchKernelGGL((assign_kres_kernel<DP, P, WAVES, PF, R3>), dim3((unsigned)grid),
                     dim3(WAVES * 64), 0, s, b.x, b.n, (int64_t)DP, b.c, b.cn, b.kp, ksplit, b.lab,
                     nullptr, b.keys);
  if (ksplit > 1)
    hipLaunchKernelGGL(kres_merge_kernel, dim3(cus * 8), dim3(256), 0, s, b.keys, ksplit, b.n,
                       b.lab, nullptr, nullptr);
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
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const int Kp = (K + 63) / 64 * 64;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  printf("N=%lld K=%d D=%d CUs=%d\n", (long long)N, K, DP, cus);

  // blobs
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
  // centroids: K random data rows, -2c in bf16, ||c||^2 (pad rows: BIG)
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
  float2* keys;
  CK(hipMalloc(&dx, xh.size() * 2));
  CK(hipMalloc(&dc, cm2.size() * 2));
  CK(hipMalloc(&dcn, cn.size() * 4));
  CK(hipMalloc(&l0, N * 4));
  CK(hipMalloc(&l1, N * 4));
  CK(hipMalloc(&keys, (size_t)N * 8 * ((Kp + KresGeom<DP>::R - 1) / KresGeom<DP>::R)));
  CK(hipMemcpy(dx, xh.data(), xh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, cm2.data(), cm2.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcn, cn.data(), cn.size() * 4, hipMemcpyHostToDevice));

  Bufs b0{dx, N, dc, dcn, Kp, l0, keys}, b1{dx, N, dc, dcn, Kp, l1, keys};
  std::vector<int> h0(N), h1(N);
  auto check = [&](const char* name) {
    CK(hipMemcpy(h0.data(), l0, N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), l1, N * 4, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < N; ++i) bad += h0[i] != h1[i];
    printf("  %-28s mismatches vs ring3: %lld\n", name, (long long)bad);
  };
  const double flop = 2.0 * (double)N * Kp * DP;
  ring3(b0, 0);
  CK(hipMemset(l1, 0xff, N * 4));
  kres<8, 8, false, true>(b1, 0, cus);
  CK(hipDeviceSynchronize());
  check("kres r3 P8 W8");
  CK(hipMemset(l1, 0xff, N * 4));
  kres<4, 12, false, true>(b1, 0, cus);
  CK(hipDeviceSynchronize());
  check("kres r3 P4 W12");
  CK(hipMemset(l1, 0xff, N * 4));
  kres<4, 8, false>(b1, 0, cus);
  CK(hipDeviceSynchronize());
  check("kres P4 W8");
  CK(hipMemset(l1, 0xff, N * 4));
  kres<4, 8, false, true>(b1, 0, cus);
  CK(hipDeviceSynchronize());
  check("kres r3 P4 W8");
  CK(hipMemset(l1, 0xff, N * 4));
  ring3p4(b1, 0);
  CK(hipDeviceSynchronize());
  check("ring3 P4 (short-launch)");
  for (int round = 0; round < 3; ++round) {
    const float tp4 = timeit([&] { ring3p4(b1, 0); }, reps);
    printf("round %d: ring3 P4 NST3 %.3f ms\n", round, tp4);
    const float t0 = timeit([&] { ring3(b0, 0); }, reps);
    const float t1 = timeit([&] { kres<8, 8, false, true>(b1, 0, cus); }, reps);
    const float t2 = timeit([&] { kres<4, 12, false, true>(b1, 0, cus); }, reps);
    const float t3 = timeit([&] { kres<4, 8, false>(b1, 0, cus); }, reps);
    const float t4 = timeit([&] { kres<4, 8, false, true>(b1, 0, cus); }, reps);
    printf("round %d: ring3 %.3f ms (%.0f TF/s) | r3P8W8 %.3f | r3P4W12 %.3f | P4W8pipe %.3f | r3P4W8 %.3f ms\n",
           round, t0, flop / t0 / 1e9, t1, t2, t3, t4);
  }
  return 0;
}
