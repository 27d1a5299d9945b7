// Probe: sustained v_mfma_f64_16x16x4f64 throughput on the whole chip (register operands,
// 8 independent accumulators per wave, 1 or 2 waves per SIMD), against which the fp64 FCM
// GEMM kernels (csrc/fcm_wide.hip) are priced.
//   hipcc --offload-arch=gfx950 -O3 tools/probe_f64_mfma.hip -o gpubin/probe_f64_mfma
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void probe(double* out, int iters, double a0, double b0) {
  f64x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f64x4{0.0, 0.0, 0.0, 0.0};
  double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[0] = s;  // keep the chain live
}

template <int NACC>
void run(double* out, int cus, int wps, int iters) {
  const int blocks = cus * wps;  // 4 waves per block: one per SIMD per block
  hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
  (void)hipDeviceSynchronize();
  for (int rep = 0; rep < 2; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(probe<NACC>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    (void)hipDeviceSynchronize();
    auto t1 = std::chrono::steady_clock::now();
    const double s = std::chrono::duration<double>(t1 - t0).count();
    const double flop = (double)blocks * 4 * iters * NACC * 16 * 16 * 4 * 2;
    printf("accumulators %2d, waves/SIMD %d: %.3f ms, %.1f TF/s fp64 MFMA\n", NACC, wps, s * 1e3,
           flop / s / 1e12);
  }
}

int main() {
  double* out;
  (void)hipMalloc(&out, 8);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int wps = 1; wps <= 4; ++wps) run<8>(out, cus, wps, 4096);
  for (int wps = 1; wps <= 2; ++wps) run<16>(out, cus, wps, 2048);
  run<4>(out, cus, 4, 8192);
  return 0;
}
