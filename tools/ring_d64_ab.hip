// A/B harness at D=64 (the mini-batch config's dimension, K=4096): the production ring3
// schedule (v_mfma_f32_16x16x32_bf16) against the ring2 schedule (32x32x16) in one
// process, interleaved, labels compared.  At D=64 the 16x16x32 shape carries 2 MFMAs per
// 16x16 output tile, so the argmin epilogue (1.5 VALU per score) plus the MFMA issue hold
// (8 of 16 cycles) exceed the MFMA time; 32x32x16 holds 8 of 32 cycles.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/ring_d64_ab.hip -o gpubin/ring_d64_ab
//   ./gpubin/ring_d64_ab [N] [K] [reps]
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

constexpr int DP = 64;

struct Bufs {
  const __bf16* x;
  int64_t n;
  const __bf16* c;
  const float* cn;
  int kp;
  int* lab;
};

template <int P, int NST, int QT>
static void r3(const Bufs& b, hipStream_t s) {
  const int64_t per = 4 * P * 16;
  hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<DP, P, NST, 4, QT>),
                     dim3((unsigned)((b.n + per - 1) / per)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / (16 * QT), b.lab, nullptr);
}
template <int P, int NST, int QT>
static void r2(const Bufs& b, hipStream_t s) {
  const int64_t per = 4 * P * 32;
  hipLaunchKernelGGL((assign_mfma_bf16_ring2_kernel<DP, P, NST, 4, QT>),
                     dim3((unsigned)((b.n + per - 1) / per)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / (32 * QT), b.lab, nullptr);
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
  const int64_t N = argc > 1 ? atoll(argv[1]) : 4000000;
  const int K = argc > 2 ? atoi(argv[2]) : 4096;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const int Kp = (K + 255) / 256 * 256;
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
    printf("  %-28s mismatches vs production ring3: %lld\n", name, (long long)bad);
    fflush(stdout);
  };
  r3<8, 3, 8>(b0, 0);
#define TRY(NAME, ...)                     \
  CK(hipMemset(l1, 0xff, N * 4));          \
  __VA_ARGS__(b1, 0);                      \
  check(NAME);
  TRY("ring3 P8 NST3 QT4", r3<8, 3, 4>)
  TRY("ring2 P4 NST3 QT2", r2<4, 3, 2>)
  TRY("ring2 P4 NST3 QT4", r2<4, 3, 4>)
  TRY("ring2 P2 NST3 QT4", r2<2, 3, 4>)
  TRY("ring2 P4 NST2 QT4", r2<4, 2, 4>)
  const double flop = 2.0 * (double)N * Kp * DP;
  for (int round = 0; round < 3; ++round) {
    const float t0 = timeit([&] { r3<8, 3, 8>(b0, 0); }, reps);
    const float t1 = timeit([&] { r3<8, 3, 4>(b1, 0); }, reps);
    const float t2 = timeit([&] { r2<4, 3, 2>(b1, 0); }, reps);
    const float t3 = timeit([&] { r2<4, 3, 4>(b1, 0); }, reps);
    const float t4 = timeit([&] { r2<2, 3, 4>(b1, 0); }, reps);
    const float t5 = timeit([&] { r2<4, 2, 4>(b1, 0); }, reps);
    printf("round %d: ring3 P8 QT8 (prod) %.3f ms (%.0f TF/s) | r3 QT4 %.3f | r2 P4 QT2 %.3f | "
           "r2 P4 QT4 %.3f | r2 P2 QT4 %.3f | r2 P4 NST2 QT4 %.3f\n",
           round, t0, flop / t0 / 1e9, t1, t2, t3, t4, t5);
    fflush(stdout);
  }
  return 0;
}
