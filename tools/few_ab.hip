// A/B harness (round 6): the few-rows exact re-scan of the fp32 / fp64 MFMA path
// (csrc/lloyd_simt.hip assign_exact_few_kernel + exact_few_merge_kernel), fp64, K=1024,
// D=128: rows per workgroup RB and grid size, at listed counts around the ~60 rows the
// fp64 N=2M step re-scans.  Labels compared with RB=8 (the earlier fixed choice).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc tools/few_ab.hip -o gpubin/few_ab
//   ./gpubin/few_ab [reps]
#include "../csrc/lloyd_simt.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

static uint64_t sm64(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct Prob {
  const double* X;
  int64_t ldx;
  int D;
  const double* C;
  int K;
  int32_t* labels;
  double* mind;
  const int32_t* rowidx;
  const int* nptr;
  double* part_d;
  int* part_k;
};

// rb = 0: production (RB by the listed count), else forced
static void few(const Prob& p, int rb, int grid, hipStream_t s) {
  const int dpad = (p.D + 31) / 32 * 32;
  const size_t lds = (size_t)dpad * EXACT_FEW_RB * sizeof(double);
  hipLaunchKernelGGL((assign_exact_few_kernel<double>), dim3(grid), dim3(256), lds, s, p.X,
                     p.ldx, p.D, p.C, p.K, p.labels, p.mind, p.rowidx, p.nptr, p.part_d, p.part_k,
                     rb);
  hipLaunchKernelGGL((exact_few_merge_kernel<double>), dim3((EXACT_FEW_PARTS + 255) / 256),
                     dim3(256), 0, s, p.K, grid, p.labels, p.mind, p.rowidx, p.nptr, p.part_d,
                     p.part_k, rb);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const int64_t N = 200000;
  const int D = 128, K = 1024;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint64_t seed = 7;
  std::vector<double> x((size_t)N * D), c((size_t)K * D);
  for (auto& v : c) v = (double)(sm64(seed) % 20000) / 1000.0 - 10.0;
  for (int64_t i = 0; i < N; ++i) {
    const int k = (int)(sm64(seed) % K);
    for (int d = 0; d < D; ++d)
      x[(size_t)i * D + d] = c[(size_t)k * D + d] + ((double)(sm64(seed) % 2000) / 1000.0 - 1.0);
  }
  std::vector<int32_t> ridx(N);
  for (int64_t i = 0; i < N; ++i) ridx[i] = (int32_t)((i * 7919) % N);
  double *dx, *dc, *dm, *pd;
  int32_t *dl, *dr;
  int *dn, *pk;
  CK(hipMalloc(&dx, x.size() * 8));
  CK(hipMalloc(&dc, c.size() * 8));
  CK(hipMalloc(&dm, N * 8));
  CK(hipMalloc(&dl, N * 4));
  CK(hipMalloc(&dr, N * 4));
  CK(hipMalloc(&dn, 4));
  CK(hipMalloc(&pd, (size_t)EXACT_FEW_PARTS * 8));
  CK(hipMalloc(&pk, (size_t)EXACT_FEW_PARTS * 4));
  CK(hipMemcpy(dx, x.data(), x.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, c.data(), c.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dr, ridx.data(), N * 4, hipMemcpyHostToDevice));
  Prob p{dx, D, D, dc, K, dl, dm, dr, dn, pd, pk};
  std::vector<int32_t> h0(N), h1(N);
  printf("few-rows re-scan, fp64 D=%d K=%d, %d CUs, %d reps\n", D, K, cus, reps);
  for (int n : {0, 60, 240, 1000, 4000}) {
    CK(hipMemcpy(dn, &n, 4, hipMemcpyHostToDevice));
    CK(hipMemset(dl, 0xff, N * 4));
    few(p, 8, 2 * cus, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h0.data(), dl, N * 4, hipMemcpyDeviceToHost));
    auto run = [&](const char* name, auto f) {
      CK(hipMemset(dl, 0xff, N * 4));
      f();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h1.data(), dl, N * 4, hipMemcpyDeviceToHost));
      int64_t bad = 0;
      for (int i = 0; i < n; ++i) bad += h0[ridx[i]] != h1[ridx[i]];
      for (int i = 0; i < 3; ++i) f();
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < reps; ++i) f();
      CK(hipDeviceSynchronize());
      const auto t1 = std::chrono::steady_clock::now();
      printf("  n=%5d %-22s %8.2f us per call (few + merge)  mismatches %lld\n", n, name,
             std::chrono::duration<double, std::micro>(t1 - t0).count() / reps, (long long)bad);
      fflush(stdout);
    };
    run("RB=8 (round-6 a)", [&] { few(p, 8, 2 * cus, 0); });
    run("RB=4", [&] { few(p, 4, 2 * cus, 0); });
    run("RB=2", [&] { few(p, 2, 2 * cus, 0); });
    run("RB=1", [&] { few(p, 1, 2 * cus, 0); });
    run("RB by count (prod)", [&] { few(p, 0, 2 * cus, 0); });
  }
  return 0;
}
