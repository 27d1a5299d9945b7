// Bounds-based pruning for exact Lloyd iterations (models/bounded.py; Hamerly 2010's
// single lower bound).  Per row i: ub = upper bound on the distance to its centroid,
// lb = lower bound on the distance to every other centroid (Euclidean, not squared).
// After the centroids move by drift[k]:  ub += drift[a(i)],  lb -= max_k drift[k].
// While ub < lb the row's label cannot change, so only the rows that fail the test are
// re-assigned (indexed top-2 MFMA kernel) and only the rows whose label changed move
// their contribution between clusters.
//
// Both kernels append to a compact list with one global atomic per block (block_reserve).
#include "tdc_common.h"
#include "kernels.h"

namespace tdc {

// Appends are reserved ONCE PER BLOCK and in ONE pass: each thread keeps its tile's hit
// flags in a register bitmask, the block scans the per-thread hit counts, reserves its
// slice of the output with one global atomic and every thread writes its hits at its
// exclusive prefix.  (A per-wave atomic on the single counter serialised ~156K
// same-address atomics at N=10M; the earlier two-pass form re-read the bounds and took
// 74 us per 10M-row filter.)
constexpr int BF_ROWS = 16;                 // rows per thread (4 x 16-B vectors)
constexpr int BF_TILE = 256 * BF_ROWS;      // rows per block
constexpr int BS_ROWS = 4;                  // active entries per thread in the scatter

// exclusive block prefix of `hits` (256 threads) + the block's base in the output
__device__ __forceinline__ int block_reserve(int hits, int* count, int* s_wave, int* s_base) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = hits;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) s_wave[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    *s_base = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  int off = *s_base + incl - hits;
  for (int v = 0; v < w; ++v) off += s_wave[v];
  return off;
}

__device__ __forceinline__ bool move_bounds(float& u, float& l, int lab, const float* drift,
                                            float md, float slack) {
  u += drift[lab];
  l -= md;
  return !(u * (1.f + slack) < l);  // NaN bounds re-assign
}

template <bool VEC>
__global__ __launch_bounds__(256) void bounds_filter_kernel(const int32_t* __restrict__ labels,
                                                            int64_t N, float* __restrict__ ub,
                                                            float* __restrict__ lb,
                                                            const float* __restrict__ drift,
                                                            const float* __restrict__ maxdrift,
                                                            float slack, int32_t* __restrict__ active,
                                                            int* __restrict__ count) {
  __shared__ int s_wave[4], s_base;
  const float md = *maxdrift;
  const int64_t tile0 = (int64_t)blockIdx.x * BF_TILE;
  unsigned flags = 0u;  // bit 4v+e: row tile0 + v*1024 + 4*tid + e
#pragma unroll
  for (int v = 0; v < BF_ROWS / 4; ++v) {
    const int64_t i = tile0 + v * 1024 + 4 * threadIdx.x;
    if (VEC && i + 3 < N) {
      const int4 lab = *reinterpret_cast<const int4*>(labels + i);
      float4 u = *reinterpret_cast<const float4*>(ub + i);
      float4 l = *reinterpret_cast<const float4*>(lb + i);
      unsigned f = 0u;
      f |= (unsigned)move_bounds(u.x, l.x, lab.x, drift, md, slack);
      f |= (unsigned)move_bounds(u.y, l.y, lab.y, drift, md, slack) << 1;
      f |= (unsigned)move_bounds(u.z, l.z, lab.z, drift, md, slack) << 2;
      f |= (unsigned)move_bounds(u.w, l.w, lab.w, drift, md, slack) << 3;
      *reinterpret_cast<float4*>(ub + i) = u;
      *reinterpret_cast<float4*>(lb + i) = l;
      flags |= f << (4 * v);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (i + e < N) {
          float u = ub[i + e], l = lb[i + e];
          if (move_bounds(u, l, labels[i + e], drift, md, slack)) flags |= 1u << (4 * v + e);
          ub[i + e] = u;
          lb[i + e] = l;
        }
      }
    }
  }
  int k = block_reserve(__popc(flags), count, s_wave, &s_base);
  while (flags) {
    const int b = __ffs(flags) - 1;
    flags &= flags - 1u;
    active[k++] = (int32_t)(tile0 + (b >> 2) * 1024 + 4 * threadIdx.x + (b & 3));
  }
}

__global__ __launch_bounds__(256) void bounds_scatter_kernel(
    const int32_t* __restrict__ active, const int* __restrict__ count, int64_t cap,
    const int32_t* __restrict__ blab, const float* __restrict__ d1, const float* __restrict__ d2,
    int32_t* __restrict__ labels, float* __restrict__ ub, float* __restrict__ lb,
    int32_t* __restrict__ moved_idx, int32_t* __restrict__ moved_old,
    int32_t* __restrict__ moved_new, int* __restrict__ mcount) {
  __shared__ int s_wave[4], s_base;
  const int64_t M = min((int64_t)*count, cap);
  const int64_t j0 = (int64_t)blockIdx.x * (256 * BS_ROWS) + threadIdx.x;
  int32_t idx[BS_ROWS], old[BS_ROWS], nw[BS_ROWS];
  unsigned flags = 0u;
#pragma unroll
  for (int e = 0; e < BS_ROWS; ++e) {  // active rows are distinct: no write conflicts
    const int64_t j = j0 + e * 256;
    idx[e] = old[e] = nw[e] = 0;
    if (j < M) {
      idx[e] = active[j];
      nw[e] = blab[j];
      old[e] = labels[idx[e]];
      labels[idx[e]] = nw[e];
      ub[idx[e]] = sqrtf(d1[j]);
      lb[idx[e]] = sqrtf(d2[j]);
      if (old[e] != nw[e]) flags |= 1u << e;
    }
  }
  int k = block_reserve(__popc(flags), mcount, s_wave, &s_base);
#pragma unroll
  for (int e = 0; e < BS_ROWS; ++e) {
    if (flags & (1u << e)) {
      moved_idx[k] = idx[e];
      moved_old[k] = old[e];
      moved_new[k] = nw[e];
      ++k;
    }
  }
}

}  // namespace tdc

using namespace tdc;

int tdc_bounds_filter(const int32_t* labels, int64_t N, float* ub, float* lb, const float* drift,
                      const float* maxdrift, float slack, int32_t* active, int* count,
                      hipStream_t s) {
  if (N <= 0) return 0;
  const dim3 grid((unsigned)((N + BF_TILE - 1) / BF_TILE));
  const bool vec = ((reinterpret_cast<uintptr_t>(labels) | reinterpret_cast<uintptr_t>(ub) |
                     reinterpret_cast<uintptr_t>(lb)) & 15u) == 0;
  if (vec)
    hipLaunchKernelGGL(bounds_filter_kernel<true>, grid, dim3(256), 0, s, labels, N, ub, lb,
                       drift, maxdrift, slack, active, count);
  else
    hipLaunchKernelGGL(bounds_filter_kernel<false>, grid, dim3(256), 0, s, labels, N, ub, lb,
                       drift, maxdrift, slack, active, count);
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_bounds_scatter(const int32_t* active, const int* count, int64_t cap, const int32_t* blab,
                       const float* d1, const float* d2, int32_t* labels, float* ub, float* lb,
                       int32_t* moved_idx, int32_t* moved_old, int32_t* moved_new, int* mcount,
                       hipStream_t s) {
  if (cap <= 0) return 0;
  const dim3 grid((unsigned)((cap + 256 * BS_ROWS - 1) / (256 * BS_ROWS)));
  hipLaunchKernelGGL(bounds_scatter_kernel, grid, dim3(256), 0, s, active, count, cap,
                     blab, d1, d2, labels, ub, lb, moved_idx, moved_old, moved_new, mcount);
  TDC_CHECK_LAUNCH();
  return 0;
}
