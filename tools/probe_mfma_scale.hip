// Probe of v_mfma_scale_f32_32x32x64_f8f6f4 operand/scale semantics on gfx950.
// For each (lane L, byte j) of the A operand: A = one e4m3 "1.0" at (L, j), B = all 1.0,
// per-lane A scale = 2^(lane-32) (E8M0 127 + lane - 32), B scale = 1.  The output row that
// lights up gives the A row of (L, j); its value 2^(s-32) names the lane whose scale
// was applied.  Prints "L j row scale_lane".
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(float* out, int L, int j, int which) {
  const int l = threadIdx.x;
  i32x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, b;
  const int one = 0x38;  // e4m3 1.0
  for (int i = 0; i < 8; ++i) b[i] = one | (one << 8) | (one << 16) | (one << 24);
  i32x8 x = {0, 0, 0, 0, 0, 0, 0, 0};
  if (l == L) x[j >> 2] = one << (8 * (j & 3));
  int sx = 127 + l - 32, so = 127;
  f32x16 c = {};
  if (which == 0) c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(x, b, c, 0, 0, 0, sx, 0, so);
  else c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, x, c, 0, 0, 0, so, 0, sx);
  for (int i = 0; i < 16; ++i) out[l * 16 + i] = c[i];
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 16 * 4);
  float h[64 * 16];
  for (int which = 0; which < 2; ++which) {
    printf("# operand %s\n", which == 0 ? "A" : "B");
    for (int L : {0, 1, 31, 32, 33, 63}) {
      for (int j = 0; j < 32; ++j) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, L, j, which);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        // C/D: col = lane & 31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
        int nz = 0, row = -1, col = -1;
        float v = 0;
        for (int l = 0; l < 64; ++l)
          for (int i = 0; i < 16; ++i)
            if (h[l * 16 + i] != 0.f) {
              ++nz;
              row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
              col = l & 31;
              v = h[l * 16 + i];
            }
        int e = 0;
        frexpf(v, &e);
        printf("L=%2d j=%2d nonzeros=%4d last(row=%2d col=%2d) value=%g scale_lane=%d\n", L, j, nz, row,
               col, v, e - 1 + 32);
      }
    }
  }
  return 0;
}
