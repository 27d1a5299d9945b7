// Probe of the scale-byte select (opsel) of v_mfma_scale_f32_32x32x64_f8f6f4 on gfx950:
// A = B = e4m3 1.0 everywhere, the A (or B) scale register holds four different E8M0
// exponents (bytes 127..130 = 1, 2, 4, 8), the other scale is 1.0.  Every output is then
// 64 x the selected scale, so output / 64 names the byte that opsel picked.
//   hipcc --offload-arch=gfx950 -O3 tools/probe_mfma_scale_opsel.hip -o gpubin/probe_opsel
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int OPSEL, int WHICH>
__global__ void probe(float* out) {
  const int l = threadIdx.x;
  i32x8 one8;
  for (int i = 0; i < 8; ++i) one8[i] = 0x38383838;  // e4m3 1.0 in every byte
  const int s4 = 127 | (128 << 8) | (129 << 16) | (130 << 24), s1 = 127;
  f32x16 c = {};
  if (WHICH == 0) c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(one8, one8, c, 0, 0, OPSEL, s4, 0, s1);
  else c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(one8, one8, c, 0, 0, 0, s1, OPSEL, s4);
  out[l] = c[0];
  out[64 + l] = c[15];
}

template <int OPSEL, int WHICH>
void run(float* d) {
  float h[128];
  hipLaunchKernelGGL((probe<OPSEL, WHICH>), dim3(1), dim3(64), 0, 0, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  float mn = h[0], mx = h[0];
  for (int i = 0; i < 128; ++i) { mn = h[i] < mn ? h[i] : mn; mx = h[i] > mx ? h[i] : mx; }
  printf("operand %c opsel %d: out/64 min %g max %g\n", WHICH ? 'B' : 'A', OPSEL, mn / 64, mx / 64);
}

int main() {
  float* d;
  hipMalloc(&d, 128 * 4);
  run<0, 0>(d); run<1, 0>(d); run<2, 0>(d); run<3, 0>(d);
  run<0, 1>(d); run<1, 1>(d); run<2, 1>(d); run<3, 1>(d);
  return 0;
}
