// A/B harness (round 6): point tiles per wave of the one-product prefilter of the fp32 / fp64
// K-Means path (assign_mfma_bf16_ring3_kernel<..., TOP2 = true> with the x1_eps bound,
// csrc/assign_x3.hip tdc_x3_prefilter), D = 128, K = 1024, timed interleaved; labels (with
// the uncertified rows' sign bit) compared with the production P = 4 launch.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/top2_ab.hip -o gpubin/top2_ab
//   ./gpubin/top2_ab [N] [reps]
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

constexpr int DP = 128;

struct Bufs {
  const __bf16* x;
  int64_t n;
  const __bf16* c;
  const float* cn;
  int kp;
  int* lab;
  const float* cstat;
  const float2* xnhl;
};

template <int P, int NST>
static void top2(const Bufs& b, hipStream_t s) {
  const int64_t per = 4 * P * 16;
  hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, P, NST, 4, 4, true>),
                     dim3((unsigned)((b.n + per - 1) / per)), dim3(256), 0, s, b.x, b.n,
                     (int64_t)DP, b.c, b.cn, b.kp / 64, b.lab, nullptr, nullptr, nullptr, b.cstat,
                     b.xnhl);
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
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int K = 1024, Kp = 1024;
  printf("N=%lld K=%d D=%d (top-2 prefilter)\n", (long long)N, K, DP);
  uint64_t seed = 99;
  std::vector<float> cen((size_t)K * DP);
  for (auto& v : cen) v = (float)(unif(seed) * 20.0 - 10.0);
  std::vector<uint16_t> xh((size_t)N * DP);
  std::vector<float> xnhl((size_t)N * 2);
  for (int64_t i = 0; i < N; ++i) {
    const int k = (int)(sm64(seed) % (uint64_t)K);
    double sh = 0, sl = 0;
    for (int d = 0; d < DP; ++d) {
      const double u1 = unif(seed) + 1e-300, u2 = unif(seed);
      const float v = (float)(cen[(size_t)k * DP + d] + sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
      const uint16_t h = f2bf(v);
      xh[(size_t)i * DP + d] = h;
      const float l = v - bf2f(h);
      sh += (double)bf2f(h) * bf2f(h);
      sl += (double)l * l;
    }
    xnhl[2 * i] = (float)sh;
    xnhl[2 * i + 1] = (float)sl;
  }
  std::vector<uint16_t> cm2((size_t)Kp * DP, 0);
  std::vector<float> cn(Kp, 3.0e38f);
  float cmax = 0, hmax = 0, lmax = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t i = (int64_t)(sm64(seed) % (uint64_t)N);
    double s = 0, h2 = 0, l2 = 0;
    for (int d = 0; d < DP; ++d) {
      const float c = bf2f(xh[(size_t)i * DP + d]);
      const float t = -2.f * c;
      const uint16_t th = f2bf(t);
      cm2[(size_t)k * DP + d] = th;
      s += (double)c * c;
      h2 += (double)bf2f(th) * bf2f(th);
      l2 += (double)(t - bf2f(th)) * (t - bf2f(th));
    }
    cn[k] = (float)s;
    cmax = std::max(cmax, (float)s);
    hmax = std::max(hmax, (float)h2);
    lmax = std::max(lmax, (float)l2);
  }
  float cstat[3] = {cmax, hmax, lmax};
  __bf16 *dx, *dc;
  float *dcn, *dcs, *dxn;
  int *l0, *l1;
  CK(hipMalloc(&dx, xh.size() * 2));
  CK(hipMalloc(&dc, cm2.size() * 2));
  CK(hipMalloc(&dcn, cn.size() * 4));
  CK(hipMalloc(&dcs, 12));
  CK(hipMalloc(&dxn, xnhl.size() * 4));
  CK(hipMalloc(&l0, N * 4));
  CK(hipMalloc(&l1, N * 4));
  CK(hipMemcpy(dx, xh.data(), xh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, cm2.data(), cm2.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcn, cn.data(), cn.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dcs, cstat, 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(dxn, xnhl.data(), xnhl.size() * 4, hipMemcpyHostToDevice));
  Bufs b0{dx, N, dc, dcn, Kp, l0, dcs, (const float2*)dxn};
  Bufs b1{dx, N, dc, dcn, Kp, l1, dcs, (const float2*)dxn};
  std::vector<int> h0(N), h1(N);
  top2<4, 3>(b0, 0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h0.data(), l0, N * 4, hipMemcpyDeviceToHost));
  int64_t flagged = 0;
  for (int64_t i = 0; i < N; ++i) flagged += h0[i] < 0;
  printf("  production P=4: %.2f %% of the rows flagged for the three-product pass\n",
         100.0 * flagged / N);
  auto check = [&](const char* name) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h1.data(), l1, N * 4, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < N; ++i) bad += h0[i] != h1[i];
    printf("  %-24s mismatches vs P=4: %lld\n", name, (long long)bad);
    fflush(stdout);
  };
#define TRY(NAME, ...)            \
  CK(hipMemset(l1, 0xff, N * 4)); \
  __VA_ARGS__;                    \
  check(NAME);
  TRY("P=6 NST=2", (top2<6, 2>(b1, 0)))
  TRY("P=6 NST=3", (top2<6, 3>(b1, 0)))
  TRY("P=8 NST=2 (20 spills)", (top2<8, 2>(b1, 0)))
  for (int round = 0; round < 3; ++round) {
    const float t0 = timeit([&] { top2<4, 3>(b0, 0); }, reps);
    const float t1 = timeit([&] { top2<6, 2>(b1, 0); }, reps);
    const float t2 = timeit([&] { top2<6, 3>(b1, 0); }, reps);
    const float t3 = timeit([&] { top2<8, 2>(b1, 0); }, reps);
    printf("round %d: P=4 NST=3 (production) %.3f ms | P=6 NST=2 %.3f | P=6 NST=3 %.3f | "
           "P=8 NST=2 %.3f\n", round, t0, t1, t2, t3);
    fflush(stdout);
  }
  return 0;
}
