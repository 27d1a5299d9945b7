// Probe: how does v_mfma_f32_16x16x32_bf16 round?  For random bf16 A/B and fp32 C, compare
// every output bit-for-bit with
//   (a) C + sum_k a_k b_k computed exactly (fp64: 32 bf16 products are exact in fp64 and
//       their sum with C is exact to 2^-53 relative here) and rounded ONCE to fp32 (RNE);
//   (b) a k-ordered fp32 fmaf chain starting from C;
// and record the largest |MFMA - exact| in units of ulp(max(|C|, sum|a b|)).
// Used to set the accumulation term of the assign_x3 error bound (csrc/assign_x3.hip).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_mfma_acc tools/probe_mfma_acc.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// A [16][32], B [32][16] row-major bf16 (as uint16 bits), C/D [16][16] fp32, T tiles
__global__ void probe(const uint16_t* A, const uint16_t* B, const float* C, float* D, int T) {
  const int t = blockIdx.x;
  if (t >= T) return;
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  const uint16_t* a = A + (size_t)t * 512;
  const uint16_t* b = B + (size_t)t * 512;
  bf16x8 av, bv;
  for (int j = 0; j < 8; ++j) {
    uint16_t ab = a[r * 32 + 8 * g + j], bb = b[(8 * g + j) * 16 + r];
    av[j] = __builtin_bit_cast(__bf16, ab);
    bv[j] = __builtin_bit_cast(__bf16, bb);
  }
  f32x4 c;
  for (int i = 0; i < 4; ++i) c[i] = C[(size_t)t * 256 + (4 * g + i) * 16 + r];
  f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) D[(size_t)t * 256 + (4 * g + i) * 16 + r] = d[i];
}

static float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static uint64_t rng = 88172645463325252ull;
static double urand() {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return (rng >> 11) * (1.0 / 9007199254740992.0);
}

int main() {
  const int T = 20000;
  uint16_t* A = (uint16_t*)malloc(T * 512 * 2);
  uint16_t* B = (uint16_t*)malloc(T * 512 * 2);
  float* C = (float*)malloc(T * 256 * 4);
  float* D = (float*)malloc(T * 256 * 4);
  for (int t = 0; t < T; ++t) {
    const int mode = t % 4;  // 0 random, 1 large C + small products, 2 cancelling, 3 mixed exponents
    for (int i = 0; i < 512; ++i) {
      double x = urand() * 2 - 1, y = urand() * 2 - 1;
      if (mode == 3) { x *= ldexp(1.0, (int)(urand() * 20) - 10); y *= ldexp(1.0, (int)(urand() * 20) - 10); }
      A[t * 512 + i] = f2bf((float)x);
      B[t * 512 + i] = f2bf((float)y);
    }
    for (int i = 0; i < 256; ++i) {
      double c = urand() * 2 - 1;
      if (mode == 1) c *= 1e4;
      C[t * 256 + i] = (float)c;
    }
    if (mode == 2) {  // rows of A: second half negates the first (sums cancel to ~C)
      for (int r = 0; r < 16; ++r)
        for (int k = 0; k < 16; ++k) A[t * 512 + r * 32 + 16 + k] = A[t * 512 + r * 32 + k] ^ 0x8000;
      for (int k = 0; k < 16; ++k)
        for (int c = 0; c < 16; ++c) B[t * 512 + (16 + k) * 16 + c] = B[t * 512 + k * 16 + c];
    }
  }
  uint16_t *dA, *dB;
  float *dC, *dD;
  hipMalloc(&dA, T * 1024); hipMalloc(&dB, T * 1024); hipMalloc(&dC, T * 1024); hipMalloc(&dD, T * 1024);
  hipMemcpy(dA, A, T * 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, B, T * 1024, hipMemcpyHostToDevice);
  hipMemcpy(dC, C, T * 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD, T);
  hipMemcpy(D, dD, T * 1024, hipMemcpyDeviceToHost);
  long match_once[4] = {0}, match_chain[4] = {0}, total[4] = {0};
  double worst[4] = {0};
  for (int t = 0; t < T; ++t) {
    const int mode = t % 4;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        const float c = C[t * 256 + i * 16 + j];
        double ex = c, mag = fabs(c);
        float ch = c;
        for (int k = 0; k < 32; ++k) {
          const double p = (double)bf2f(A[t * 512 + i * 32 + k]) * bf2f(B[t * 512 + k * 16 + j]);
          ex += p;
          mag += fabs(p);
          ch = fmaf(bf2f(A[t * 512 + i * 32 + k]), bf2f(B[t * 512 + k * 16 + j]), ch);
        }
        const float d = D[t * 256 + i * 16 + j];
        total[mode]++;
        if (d == (float)ex) match_once[mode]++;
        if (d == ch) match_chain[mode]++;
        const double ulp = ldexp(1.0, ilogb(mag) - 23);
        const double e = fabs((double)d - ex) / ulp;
        if (e > worst[mode]) worst[mode] = e;
      }
  }
  const char* names[4] = {"random", "large C", "cancelling", "mixed exponents"};
  for (int m = 0; m < 4; ++m)
    printf("%-16s outputs %ld  == exact-sum rounded once: %.6f  == k-ordered fmaf chain: %.6f  "
           "max |err| / ulp(sum|terms|): %.3f\n", names[m], total[m],
           (double)match_once[m] / total[m], (double)match_chain[m] / total[m], worst[m]);
  return 0;
}
