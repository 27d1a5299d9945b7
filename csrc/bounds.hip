// Bounds-based pruning for exact Lloyd iterations (models/bounded.py; Hamerly 2010's
// single lower bound).  Per row i: ub = upper bound on the distance to its centroid,
// lb = lower bound on the distance to every other centroid (Euclidean, not squared).
// After the centroids move by drift[k]:  ub += drift[a(i)],  lb -= max_k drift[k].
// While ub < lb the row's label cannot change, so only the rows that fail the test are
// re-assigned (indexed top-2 MFMA kernel) and only the rows whose label changed move
// their contribution between clusters.
//
// Both kernels append to a compact list with one global atomic per block (see BlockAppend).
#include "tdc_common.h"
#include "kernels.h"

namespace tdc {

// index of this lane among the set lanes of mask below it
__device__ __forceinline__ int lane_rank(unsigned long long mask, int lane) {
  return __popcll(mask & ((1ull << lane) - 1ull));
}

// Appends are reserved ONCE PER BLOCK: each block owns a contiguous range of rows, counts
// its hits in a first pass, reserves its slice of the output with one global atomic and
// writes in a second pass (LDS cursor).  A per-wave atomic on the single counter
// serialised ~156K same-address atomics at N=10M (1.8 ms for a 40 MB pass).
constexpr int BOUNDS_BLOCKS = 1024;

struct BlockAppend {
  int* s_wave;    // [4] per-wave hit counts
  int* s_base;    // [1] block base in the output
  int* s_cursor;  // [1] running offset inside the block's slice
  __device__ __forceinline__ void reserve(int wave_hits, int* count) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) s_wave[w] = wave_hits;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int tot = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
      *s_base = tot ? atomicAdd(count, tot) : 0;
      *s_cursor = 0;
    }
    __syncthreads();
  }
  // slot of this lane's hit (call with the wave's ballot; lanes without a hit ignore it)
  __device__ __forceinline__ int slot(unsigned long long mask) {
    const int lane = threadIdx.x & 63;
    int off = 0;
    if (lane == 0) off = atomicAdd(s_cursor, __popcll(mask));
    off = __shfl(off, 0, 64);
    return *s_base + off + lane_rank(mask, lane);
  }
};

__device__ __forceinline__ void block_range(int64_t n, int64_t& r0, int64_t& r1) {
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  r0 = (int64_t)blockIdx.x * per;
  r1 = min(n, r0 + per);
}

__global__ __launch_bounds__(256) void bounds_filter_kernel(const int32_t* __restrict__ labels,
                                                            int64_t N, float* __restrict__ ub,
                                                            float* __restrict__ lb,
                                                            const float* __restrict__ drift,
                                                            const float* __restrict__ maxdrift,
                                                            float slack, int32_t* __restrict__ active,
                                                            int* __restrict__ count) {
  __shared__ int s_wave[4], s_base, s_cursor;
  BlockAppend app{s_wave, &s_base, &s_cursor};
  const float md = *maxdrift;
  int64_t r0, r1;
  block_range(N, r0, r1);
  // pass 1: move the bounds, count the rows that may change label
  int hits = 0;
  for (int64_t i0 = r0; i0 < r1; i0 += 256) {  // block-uniform trip count
    const int64_t i = i0 + threadIdx.x;
    bool act = false;
    if (i < r1) {
      const float u = ub[i] + drift[labels[i]];
      const float l = lb[i] - md;
      ub[i] = u;
      lb[i] = l;
      act = !(u * (1.f + slack) < l);  // NaN bounds re-assign
    }
    hits += __popcll(__ballot(act));
  }
  app.reserve(hits, count);
  if (hits == 0 && s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3] == 0) return;
  // pass 2: same rows, same thread -> the bounds it wrote; append the hits
  for (int64_t i0 = r0; i0 < r1; i0 += 256) {
    const int64_t i = i0 + threadIdx.x;
    bool act = false;
    if (i < r1) act = !(ub[i] * (1.f + slack) < lb[i]);
    const unsigned long long mask = __ballot(act);
    if (mask == 0ull) continue;  // wave-uniform
    const int k = app.slot(mask);
    if (act) active[k] = (int32_t)i;
  }
}

__global__ __launch_bounds__(256) void bounds_scatter_kernel(
    const int32_t* __restrict__ active, const int* __restrict__ count, int64_t cap,
    const int32_t* __restrict__ blab, const float* __restrict__ d1, const float* __restrict__ d2,
    int32_t* __restrict__ labels, float* __restrict__ ub, float* __restrict__ lb,
    int32_t* __restrict__ moved_idx, int32_t* __restrict__ moved_old,
    int32_t* __restrict__ moved_new, int* __restrict__ mcount) {
  __shared__ int s_wave[4], s_base, s_cursor;
  BlockAppend app{s_wave, &s_base, &s_cursor};
  const int64_t M = min((int64_t)*count, cap);
  int64_t r0, r1;
  block_range(M, r0, r1);
  // pass 1: count label changes (labels untouched yet; active rows are distinct)
  int hits = 0;
  for (int64_t j0 = r0; j0 < r1; j0 += 256) {
    const int64_t j = j0 + threadIdx.x;
    const bool mv = j < r1 && labels[active[j]] != blab[j];
    hits += __popcll(__ballot(mv));
  }
  app.reserve(hits, mcount);
  // pass 2: append the changes, then install the new labels and bounds
  for (int64_t j0 = r0; j0 < r1; j0 += 256) {
    const int64_t j = j0 + threadIdx.x;
    bool mv = false;
    int32_t i = 0, old = 0, nw = 0;
    if (j < r1) {
      i = active[j];
      nw = blab[j];
      old = labels[i];
      mv = old != nw;
    }
    const unsigned long long mask = __ballot(mv);
    if (mask != 0ull) {
      const int k = app.slot(mask);
      if (mv) {
        moved_idx[k] = i;
        moved_old[k] = old;
        moved_new[k] = nw;
      }
    }
    if (j < r1) {
      labels[i] = nw;
      ub[i] = sqrtf(d1[j]);
      lb[i] = sqrtf(d2[j]);
    }
  }
}

}  // namespace tdc

using namespace tdc;

int tdc_bounds_filter(const int32_t* labels, int64_t N, float* ub, float* lb, const float* drift,
                      const float* maxdrift, float slack, int32_t* active, int* count,
                      hipStream_t s) {
  if (N <= 0) return 0;
  int64_t g = (N + 255) / 256;
  if (g > BOUNDS_BLOCKS) g = BOUNDS_BLOCKS;
  hipLaunchKernelGGL(bounds_filter_kernel, dim3((unsigned)g), dim3(256), 0, s, labels, N, ub, lb,
                     drift, maxdrift, slack, active, count);
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_bounds_scatter(const int32_t* active, const int* count, int64_t cap, const int32_t* blab,
                       const float* d1, const float* d2, int32_t* labels, float* ub, float* lb,
                       int32_t* moved_idx, int32_t* moved_old, int32_t* moved_new, int* mcount,
                       hipStream_t s) {
  if (cap <= 0) return 0;
  int64_t g = (cap + 255) / 256;
  if (g > BOUNDS_BLOCKS) g = BOUNDS_BLOCKS;
  hipLaunchKernelGGL(bounds_scatter_kernel, dim3((unsigned)g), dim3(256), 0, s, active, count, cap,
                     blab, d1, d2, labels, ub, lb, moved_idx, moved_old, moved_new, mcount);
  TDC_CHECK_LAUNCH();
  return 0;
}
