// Probe (round 6): FLOP/s of the two block-scaled fp8 MFMA shapes on random operands,
// v_mfma_scale_f32_32x32x64_f8f6f4 against v_mfma_scale_f32_16x16x128_f8f6f4 (the same
// cycles per FLOP on paper).  MI355X_MICROARCH.md "DVFS give-back" item 7 measured the bf16
// 16x16 shape at ~1.12-1.15x the FLOP/s of the 32x32 one on random data (a higher held
// clock); this checks whether the fp8 shapes differ the same way before any kernel work.
// Operands in registers (random e4m3 bytes, NaN patterns cleared, random E8M0 scales near
// 1), independent accumulators, every SIMD busy, each arm run for ~1.5 s, alternated.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_fp8_shape.hip -o gpubin/probe_fp8_shape
//   ./gpubin/probe_fp8_shape [iters]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// 4 accumulators of 32x32 (64 VGPRs) vs 8 of 16x16 (32 VGPRs): the same 4096 outputs per
// wave and the same FLOP per loop trip (4 x 131072 = 8 x 65536)
__global__ __launch_bounds__(256) void loop32(const int* __restrict__ src, float* __restrict__ out,
                                              int iters) {
  const int l = threadIdx.x & 63;
  i32x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = src[(blockIdx.x * 64 + l) * 16 + i];
    b[i] = src[(blockIdx.x * 64 + l) * 16 + 8 + i];
  }
  const int sa = 127 + (src[l] & 3) - 1, sb = 127 + ((src[l] >> 2) & 3) - 1;
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 0, 0, 0, sa, 0, sb);
    c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, c1, 0, 0, 0, sb, 0, sa);
    c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c2, 0, 0, 0, sa, 0, sa);
    c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, b, c3, 0, 0, 0, sb, 0, sb);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void loop16(const int* __restrict__ src, float* __restrict__ out,
                                              int iters) {
  const int l = threadIdx.x & 63;
  i32x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = src[(blockIdx.x * 64 + l) * 16 + i];
    b[i] = src[(blockIdx.x * 64 + l) * 16 + 8 + i];
  }
  const int sa = 127 + (src[l] & 3) - 1, sb = 127 + ((src[l] >> 2) & 3) - 1;
  f32x4 c[8] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      c[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4((j & 1) ? b : a, (j & 2) ? b : a,
                                                             c[j], 0, 0, 0, sa, 0, sb);
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int blocks = prop.multiProcessorCount * 2;  // 2 waves per SIMD
  std::vector<int> h((size_t)blocks * 64 * 16);
  uint64_t s = 12345;
  for (auto& v : h) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    // random e4m3 bytes with the NaN codes (S.1111.111) cleared: bit 0 of each byte off
    v = (int)((uint32_t)(s >> 32) & 0xFEFEFEFEu);
  }
  int* d;
  float* o;
  CK(hipMalloc(&d, h.size() * 4));
  CK(hipMalloc(&o, (size_t)blocks * 256 * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const double flop = (double)blocks * 4 * iters * 4 * 131072.0;  // 4 waves per block
  auto run = [&](bool big) {
    const auto t0 = std::chrono::steady_clock::now();
    int n = 0;
    double el = 0;
    do {
      if (big) hipLaunchKernelGGL(loop32, dim3(blocks), dim3(256), 0, 0, d, o, iters);
      else hipLaunchKernelGGL(loop16, dim3(blocks), dim3(256), 0, 0, d, o, iters);
      CK(hipDeviceSynchronize());
      ++n;
      el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (el < 1.5);
    return flop * n / el / 1e12;
  };
  printf("blocks %d x 256 threads, %d iters, %.3g FLOP per launch\n", blocks, iters, flop);
  for (int r = 0; r < 3; ++r) {
    const double t32 = run(true), t16 = run(false);
    printf("round %d: 32x32x64 %.0f TF/s | 16x16x128 %.0f TF/s | ratio %.3f\n", r, t32, t16, t16 / t32);
    fflush(stdout);
  }
  return 0;
}
