// Shared device helpers for the tdc (tensorflow-distributed-clustering, MI355X-native)
// HIP kernels.  gfx950 / CDNA4 only: 64-lane waves, MFMA, 160 KiB LDS per CU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TDC_WAVE 64

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define TDC_CHECK_LAUNCH()                                                         \
  do {                                                                             \
    hipError_t _e = hipGetLastError();                                             \
    if (_e != hipSuccess) return (int)_e;                                          \
  } while (0)

namespace tdc {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Typed element load/convert helpers (X may be bf16 / fp32 / fp64).
template <typename T> __device__ __forceinline__ float to_f(T v) { return (float)v; }
template <typename T, typename A> __device__ __forceinline__ A to_acc(T v) { return (A)v; }

// Atomic add on global memory for float / double (gfx950 has native
// global_atomic_add_f32 / _f64; agent scope is the default).
__device__ __forceinline__ void atomic_add(float* p, float v) { atomicAdd(p, v); }
__device__ __forceinline__ void atomic_add(double* p, double v) { atomicAdd(p, v); }
// fixed-point partials (deterministic update): two's-complement wrap-around add
__device__ __forceinline__ void atomic_add(long long* p, long long v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v);
}

// A wave-uniform pointer in SGPRs (readfirstlane of both halves): the saddr operand of
// an inline-asm global / LDS-DMA load, when the compiler cannot prove the value uniform.
__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (const void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// Stage rows [r0, r0 + 256) of a CONTIGUOUS row-major X (ldx == D, 16-B aligned base)
// into LDS with 16-byte loads.  Returns the number of valid rows; the caller syncs before
// reading s_x[row * D + d].
template <typename T>
__device__ __forceinline__ int stage_rows_lds(const T* __restrict__ X, int64_t N, int D,
                                              int64_t r0, T* s_x) {
  const int rows = (int)((N - r0) < 256 ? (N - r0) : 256);
  const T* src = X + r0 * D;
  if (rows == 256) {
    const int nch = 256 * D * (int)sizeof(T) / 16;
    for (int c = threadIdx.x; c < nch; c += 256)
      reinterpret_cast<uint4*>(s_x)[c] = reinterpret_cast<const uint4*>(src)[c];
  } else {
    for (int e = threadIdx.x; e < rows * D; e += 256) s_x[e] = src[e];
  }
  return rows;
}

// Row `row` of a row-major X into registers, branch-free: the row is clamped to N - 1 and
// features d >= D re-read feature D - 1 (always in bounds), so the loads need no exec-mask
// branches and the compiler's vmcnt tracking stays exact across a ping-pong prefetch loop.
// row_mask zeroes the d >= D copies once the data is used.
template <typename T, int DMAX>
__device__ __forceinline__ void row_load(const T* __restrict__ X, int64_t row, int64_t N,
                                         int64_t ldx, int D, T (&v)[DMAX]) {
  const T* p = X + (row < N ? row : N - 1) * ldx;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) v[d] = p[d < D ? d : D - 1];
}
template <typename T, int DMAX>
__device__ __forceinline__ void row_mask(int D, T (&v)[DMAX]) {
#pragma unroll
  for (int d = 0; d < DMAX; ++d) v[d] = d < D ? v[d] : (T)0;
}

// Blocks of `kernel` (block threads, static LDS only) the whole GPU holds at once: the
// grid of a grid-stride kernel.  A larger grid leaves a second, partial round of blocks
// that runs at a fraction of the occupancy (every block has the same row count).
template <typename F>
inline int resident_blocks(F kernel, int block) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess)
    per = 1;
  return (per > 0 ? per : 1) * (cus > 0 ? cus : 1);
}

}  // namespace tdc
