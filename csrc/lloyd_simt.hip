// Exact-arithmetic (fp32 / fp64) K-Means kernels for low-dimensional data, and the
// LDS-privatised centroid update (N2) used by every dtype.
//
// * lloyd_small: ONE pass over the shard computes labels AND per-cluster sums/counts.
//   This is the whole reference K-Means tower (scripts/distribuitedClustering.py:217-248:
//   Tile/Sub/Square/Sum/ArgMin + K x (Where, Gather, Mean) + CPU Bincount) for the
//   reference's own configs (D=5, K<=15, fp64).  Distances use the difference form
//   sum((x-c)^2) like the reference; the per-cluster partials live in VGPRs
//   (predicated FMA, static indices) so there is no atomic contention even at K=3,
//   and are reduced wave -> LDS -> one global atomic per (cluster, dim) per block.
// * assign_simt: difference-form argmin for larger K (centroids staged through LDS).
// * update_lds: per-block LDS histogram of sum(x) and count, sliced over D so that
//   K x D_slice fits LDS; one flush of global atomics per block.
#include <type_traits>

#include "tdc_common.h"
#include "kernels.h"

namespace tdc {

// ------------------------------------------------------------------------------------
// fused small-K Lloyd step
// ------------------------------------------------------------------------------------
// labels may be null: the fit's final label pass writes them, the steps need only the sums.
// LPR lanes share a row: lane part p = lane % LPR owns clusters p*KL .. p*KL+KL-1, so the
// K x D fp64 accumulators per lane shrink LPR-fold (K = 15, D = 5: 245 VGPRs / 2 waves per
// SIMD at LPR = 1, ~140 / 3 waves at LPR = 2); the partial argmins meet by lane swaps.
template <typename T, typename ACC, int KL, int DMAX, int LPR>
__global__ __launch_bounds__(256) void lloyd_small_kernel(
    const T* __restrict__ X, int64_t N, int64_t ldx, int D, const T* __restrict__ C, int K,
    int32_t* __restrict__ labels, T* __restrict__ mind, ACC* __restrict__ sums,
    ACC* __restrict__ counts) {
  constexpr int KMAX = KL * LPR;
  __shared__ T s_c[KMAX * DMAX];
  __shared__ T s_red[4][KMAX * (DMAX + 1)];
  const int tid = threadIdx.x;
  for (int i = tid; i < KMAX * DMAX; i += 256) {
    const int k = i / DMAX, d = i % DMAX;
    s_c[i] = (k < K && d < D) ? C[k * D + d] : (T)0;
  }
  __syncthreads();
  const int part = LPR == 1 ? 0 : (tid % LPR);
  const T* sc = s_c + part * KL * DMAX;

  T acc[KL][DMAX];
  T cnt[KL];  // counted with the one-hot selector itself: one add instead of cmp + select + add
#pragma unroll
  for (int k = 0; k < KL; ++k) {
    cnt[k] = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) acc[k][d] = 0;
  }

  // One row per LPR lanes, grid-stride, ping-pong prefetch: the loads of the next row are
  // issued before the current row's distances and one-hot accumulation, into the other
  // register set (no copy, so the compiler's vmcnt waits stay partial); with two waves per
  // SIMD and no prefetch the HBM latency was exposed.  (Wave-private LDS staging of 64-row
  // tiles with 16-B loads measured no better than these 8-B row loads:
  // docs/PERF_NOTES.md "Reference configs".)
  auto row = [&](T (&x)[DMAX], int64_t r) {
    row_mask(D, x);
    // larger tiles: re-read the centroids from LDS (broadcast) every row instead of
    // letting the compiler hoist K x D of them into VGPRs next to the K x D accumulators
    if constexpr (KL >= 8 || LPR > 1) asm volatile("" ::: "memory");
    const bool valid = r < N;
    T bd = (T)INFINITY;  // NaN distances (poisoned centroid, empty_cluster='nan') never win
    int best = 0;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      const int k = part * KL + j;
      if (LPR > 1 || k < K) {  // LPR == 1: wave-uniform skip
        T dd = 0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          const T df = x[d] - sc[j * DMAX + d];
          dd = fma(df, df, dd);
        }
        if (k < K && dd < bd) {  // strict: first minimum wins (TF ArgMin)
          bd = dd;
          best = k;
        }
      }
    }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) {  // partial argmins of the row's lanes
      const T od = __shfl_xor(bd, o, 64);
      const int ob = __shfl_xor(best, o, 64);
      if (od < bd || (od == bd && ob < best)) {
        bd = od;
        best = ob;
      }
    }
    if (valid && part == 0) {
      if (labels) labels[r] = best;
      if (mind) mind[r] = bd;
    }
    if (!valid) best = -1;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      const int k = part * KL + j;
      if (LPR > 1 || k < K) {
        const T sel = (k == best) ? (T)1 : (T)0;
        cnt[j] += sel;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) acc[j][d] = fma(sel, x[d], acc[j][d]);
      }
    }
  };
  const int64_t stride = (int64_t)gridDim.x * (256 / LPR);
  int64_t r = ((int64_t)blockIdx.x * 256 + tid) / LPR;
  T xa[DMAX], xb[DMAX];
  if (r < N) row_load(X, r, N, ldx, D, xa);
  for (; r < N; r += 2 * stride) {
    row_load(X, r + stride, N, ldx, D, xb);
    row(xa, r);
    row_load(X, r + 2 * stride, N, ldx, D, xa);
    row(xb, r + stride);
  }

  // wave reduce over the lanes of one part -> LDS -> block total -> one global atomic
  // per (k, d)
  const int lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int j = 0; j < KL; ++j) {
#pragma unroll
    for (int d = 0; d <= DMAX; ++d) {
      T v = (d < DMAX) ? acc[j][d] : cnt[j];
#pragma unroll
      for (int o = 32; o >= LPR; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane < LPR) s_red[w][(lane * KL + j) * (DMAX + 1) + d] = v;
    }
  }
  __syncthreads();
  for (int i = tid; i < K * (DMAX + 1); i += 256) {
    const int k = i / (DMAX + 1), d = i % (DMAX + 1);
    if (d >= D && d != DMAX) continue;
    const T v = s_red[0][i] + s_red[1][i] + s_red[2][i] + s_red[3][i];
    if (d == DMAX) {
      if (v != (T)0) atomic_add(&counts[k], (ACC)v);
    } else if (v != (T)0) {
      atomic_add(&sums[k * D + d], (ACC)v);
    }
  }
}

// ------------------------------------------------------------------------------------
// exact assignment, any K (centroid tiles through LDS), D <= DMAX
// ------------------------------------------------------------------------------------
template <typename T, int DMAX>
__global__ __launch_bounds__(256) void assign_simt_kernel(const T* __restrict__ X, int64_t N,
                                                          int64_t ldx, int D,
                                                          const T* __restrict__ C, int K,
                                                          int32_t* __restrict__ labels,
                                                          T* __restrict__ mind) {
  constexpr int KT = 256;  // centroids per LDS tile
  __shared__ T s_c[KT * DMAX];
  const int tid = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * 256 + tid;
  T x[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) x[d] = (i < N && d < D) ? X[i * ldx + d] : (T)0;
  T bd = (T)INFINITY;
  int best = 0;
  for (int k0 = 0; k0 < K; k0 += KT) {
    const int kt = min(KT, K - k0);
    __syncthreads();
    for (int j = tid; j < kt * DMAX; j += 256) {
      const int k = j / DMAX, d = j % DMAX;
      s_c[j] = (d < D) ? C[(int64_t)(k0 + k) * D + d] : (T)0;
    }
    __syncthreads();
    for (int k = 0; k < kt; ++k) {
      T dd = 0;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const T df = x[d] - s_c[k * DMAX + d];
        dd = fma(df, df, dd);
      }
      if (dd < bd) {
        bd = dd;
        best = k0 + k;
      }
    }
  }
  if (i < N) {
    labels[i] = best;
    if (mind) mind[i] = bd;
  }
}

// ------------------------------------------------------------------------------------
// LDS-privatised, D-sliced centroid update
// ------------------------------------------------------------------------------------
template <typename XT, int VEC> struct VecLoad;
template <> struct VecLoad<float, 4> {
  __device__ static void load(const float* p, float (&v)[4]) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
};
template <> struct VecLoad<double, 2> {
  __device__ static void load(const double* p, double (&v)[2]) {
    const double2 t = *reinterpret_cast<const double2*>(p);
    v[0] = t.x; v[1] = t.y;
  }
};
template <> struct VecLoad<__bf16, 4> {
  __device__ static void load(const __bf16* p, float (&v)[4]) {
    const uint2 t = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
  }
};
template <typename XT> struct VecLoad1 {
  template <typename LT> __device__ static void load(const XT* p, LT (&v)[1]) { v[0] = (LT)p[0]; }
};
// LDS accumulation type: fp64 data keeps fp64 partials (compat mode), else fp32
template <typename XT> struct LdsT { typedef float type; };
template <> struct LdsT<double> { typedef double type; };

template <typename XT, typename ACC, int VEC>
__global__ __launch_bounds__(256) void update_lds_kernel(const XT* __restrict__ X, int64_t N,
                                                         int64_t ldx, int D, int DS,
                                                         const int32_t* __restrict__ labels,
                                                         int K, ACC* __restrict__ sums,
                                                         ACC* __restrict__ counts,
                                                         int nslices, int64_t rows_per_block) {
  typedef typename LdsT<XT>::type LT;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  const int stride = DS + 1;  // pad: breaks the power-of-2 bank aliasing across clusters
  LT* s_sum = reinterpret_cast<LT*>(smem_raw);
  int* s_cnt = reinterpret_cast<int*>(s_sum + (size_t)K * stride);
  const int tid = threadIdx.x;
  const int slice = blockIdx.x % nslices;
  const int64_t chunk = blockIdx.x / nslices;
  const int d0 = slice * DS;
  const int ds = min(DS, D - d0);
  for (int i = tid; i < K * stride; i += 256) s_sum[i] = (LT)0;
  for (int i = tid; i < K; i += 256) s_cnt[i] = 0;
  __syncthreads();

  const int tpr = DS / VEC;   // threads per row
  const int rpi = 256 / tpr;  // rows per block iteration
  const int j = tid % tpr, rsub = tid / tpr;
  const int dd = j * VEC;
  const int64_t r0 = chunk * rows_per_block;
  const int64_t r1 = min(N, r0 + rows_per_block);
  constexpr int R = 8;  // rows per thread in flight: hides the label -> row load chain
  for (int64_t row0 = r0 + rsub; row0 < r1; row0 += (int64_t)rpi * R) {
    int lab[R];
    LT v[R][VEC];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int64_t row = row0 + (int64_t)u * rpi;
      lab[u] = row < r1 ? labels[row] : -1;
      if ((unsigned)lab[u] >= (unsigned)K) lab[u] = -1;  // never index LDS out of range
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int64_t row = row0 + (int64_t)u * rpi;
      if (lab[u] >= 0 && dd < ds) {
        if constexpr (VEC == 1) VecLoad1<XT>::load(X + row * ldx + d0 + dd, v[u]);
        else VecLoad<XT, VEC>::load(X + row * ldx + d0 + dd, v[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (lab[u] < 0) continue;
      if (dd < ds) {
        LT* dst = s_sum + lab[u] * stride + dd;
#pragma unroll
        for (int e = 0; e < VEC; ++e) atomicAdd(dst + e, v[u][e]);
      }
      if (j == 0) atomicAdd(s_cnt + lab[u], 1);
    }
  }
  __syncthreads();
  for (int i = tid; i < K * ds; i += 256) {
    const int k = i / ds, d = i % ds;
    if (s_cnt[k]) atomic_add(&sums[(int64_t)k * D + d0 + d], (ACC)s_sum[k * stride + d]);
  }
  if (slice == 0)
    for (int k = tid; k < K; k += 256)
      if (s_cnt[k]) atomic_add(&counts[k], (ACC)s_cnt[k]);
}

}  // namespace tdc

using namespace tdc;

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
namespace {

int grid_for(int64_t N, int per_block, int cap) {
  int64_t g = (N + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

template <typename T, typename ACC, int KL, int DMAX, int LPR>
int launch_small(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K,
                 int32_t* labels, void* mind, void* sums, void* counts, hipStream_t s) {
  // grid-stride over the rows with exactly the blocks the GPU holds at once: a larger grid
  // leaves a second, partial round of blocks running at a fraction of the occupancy
  static const int resident = resident_blocks(lloyd_small_kernel<T, ACC, KL, DMAX, LPR>, 256);
  const int g = grid_for(N * LPR, 256, resident);
  hipLaunchKernelGGL((lloyd_small_kernel<T, ACC, KL, DMAX, LPR>), dim3(g), dim3(256), 0, s,
                     (const T*)X, N, ldx, D, (const T*)C, K, labels, (T*)mind, (ACC*)sums,
                     (ACC*)counts);
  TDC_CHECK_LAUNCH();
  return 0;
}

// (clusters per lane, DMAX, lanes per row) register tiles compiled for the fused kernel
template <typename T, typename ACC>
int dispatch_small(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K,
                   int32_t* labels, void* mind, void* sums, void* counts, hipStream_t s) {
#define TDC_SMALL(KL, DM, LPR)                                                            \
  if (K <= (KL) * (LPR) && D <= DM)                                                       \
    return launch_small<T, ACC, KL, DM, LPR>(X, N, ldx, D, C, K, labels, mind, sums, counts, s);
  TDC_SMALL(4, 4, 1)
  if (D == 5) {  // the reference's own configs (D = 5, K in {3, 6, 9, 12, 15}): exact tiles
    TDC_SMALL(4, 5, 1)
    TDC_SMALL(4, 5, 2)
    TDC_SMALL(6, 5, 2)
    TDC_SMALL(8, 5, 2)
  }
  TDC_SMALL(4, 8, 1)
  TDC_SMALL(8, 4, 1)
  TDC_SMALL(8, 8, 1)
  TDC_SMALL(16, 4, 1)
  if constexpr (sizeof(T) == 4) {
    TDC_SMALL(16, 8, 1)
    TDC_SMALL(8, 16, 1)
  }
  TDC_SMALL(4, 16, 1)
  if constexpr (sizeof(T) == 4) {
    TDC_SMALL(32, 4, 1)
  } else {
    TDC_SMALL(16, 6, 1)
    // fp64 K <= 16 x D <= 8 and K <= 32 x D <= 4: two lanes per row (a one-lane tile
    // would hold 128 fp64 accumulators = 256 VGPRs)
    TDC_SMALL(8, 8, 2)
    TDC_SMALL(16, 4, 2)
  }
#undef TDC_SMALL
  return (int)hipErrorInvalidValue;
}

}  // namespace

int tdc_lloyd_small_supported(int dtype, int K, int D) {
  if (dtype == TDC_F32) return (K <= 16 && D <= 8) || (K <= 8 && D <= 16) || (K <= 32 && D <= 4);
  if (dtype == TDC_F64)
    return (K <= 16 && D <= 8) || (K <= 4 && D <= 16) || (K <= 32 && D <= 4);
  return 0;
}

int tdc_lloyd_small(int dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                    const void* C, int K, int32_t* labels, void* mind, void* sums, void* counts,
                    hipStream_t s) {
  if (N <= 0) return 0;
  if (dtype == TDC_F32) {
    if (acc_dtype == TDC_F64)
      return dispatch_small<float, double>(X, N, ldx, D, C, K, labels, mind, sums, counts, s);
    return dispatch_small<float, float>(X, N, ldx, D, C, K, labels, mind, sums, counts, s);
  }
  if (dtype == TDC_F64)
    return dispatch_small<double, double>(X, N, ldx, D, C, K, labels, mind, sums, counts, s);
  return (int)hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------
// exact assignment for ANY D (fp32 / fp64, difference form like the reference's
// Sub/Square/Sum, `scripts/distribuitedClustering.py:228-230`): (16 MR)-row x 128-centroid
// block tiles, 16 x 16 threads with an MR-row x 8-centroid register micro-tile, rows and centroids
// staged through LDS feature-major in 32-feature chunks (LDS use independent of D), so a
// thread's MR rows / 8 centroids of one feature are ds_read_b128 pieces; fp32 runs
// on packed math (v_pk_add_f32 / v_pk_fma_f32: two centroids per instruction).  The argmin
// is kept per row and merged over the 16 centroid lanes at the end.  Replaces the
// library-GEMM fallback for fp32 D > 64 / fp64 D > 32 (the GEMM expansion loses the
// exact-difference precision).
// ------------------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));

// x - c for a centroid pair c with x broadcast from one half of a row pair (VOP3P op_sel:
// no register copy to build the (x, x) pair, which cost more moves than the math)
__device__ __forceinline__ f32x2 pk_sub_lo(f32x2 xp, f32x2 c) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]"
      : "=v"(r) : "v"(xp), "v"(c));
  return r;
}
__device__ __forceinline__ f32x2 pk_sub_hi(f32x2 xp, f32x2 c) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]"
      : "=v"(r) : "v"(xp), "v"(c));
  return r;
}

// MR rows x 8 centroids per thread: fp32 MR = 8 (packed pairs, 64 accumulators), fp64 MR = 4
template <typename T> struct ExactCfg { static constexpr int MR = 8; };
template <> struct ExactCfg<double> { static constexpr int MR = 4; };

// A listed re-scan (rowidx / nptr below) of at most this many rows runs on
// assign_exact_few_kernel instead: the 128-row tiles would leave all but a handful of CUs idle.
constexpr int EXACT_FEW_MAX = 32768, EXACT_FEW_MAXD = 1024;

constexpr int EXACT_FEW_RB = 8, EXACT_FEW_PARTS = 8192;
// rows per workgroup by the listed count (read on the device): few rows want short
// per-thread chains over more workgroups, many rows the centroid slice reused over 8 rows
// (fp64 D=128 K=1024, few + merge: 60 rows 36.1 us at 8 -> 18.0 at 2; 240 rows 37.0 -> 21.4
// at 2 or 4; 1000 rows 43.4 / 41.2 at 8 / 4; 4000 rows 126 at 8, 140 at 4;
// profiles/few_rows_rb_ab_r06aa.txt).  force (A/B harness): 0 = by count, else that RB.
__device__ __forceinline__ int exact_few_rb(int n, int force) {
  return force ? force : (n <= 160 ? 2 : n <= 1536 ? 4 : EXACT_FEW_RB);
}
__device__ __forceinline__ int exact_few_splits(int n, int nkc, int grid, int rb) {
  const int rg = (n + rb - 1) / rb;
  int sp = rg > 0 ? grid / rg : 1;
  if (sp > nkc) sp = nkc;
  if (sp < 1) sp = 1;
  if ((int64_t)sp * rg * rb > EXACT_FEW_PARTS) sp = 1;
  return sp;
}


// the per-row minimum over the K splits of assign_exact_few_kernel (nothing to do at S = 1),
// grid-stride over the listed rows: exact_few_merge_kernel, or the empty launch of
// assign_exact_kernel when the listed rows were few (one launch fewer per step)
template <typename T>
__device__ __forceinline__ void exact_few_merge_rows(int K, int few_grid, int n, int force_rb,
                                                     int32_t* __restrict__ labels,
                                                     T* __restrict__ mind,
                                                     const int32_t* __restrict__ rowidx,
                                                     const T* __restrict__ part_d,
                                                     const int* __restrict__ part_k) {
  const int S = exact_few_splits(n, (K + 255) / 256, few_grid, exact_few_rb(n, force_rb));
  if (S <= 1) return;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (int64_t)gridDim.x * blockDim.x) {
    T b = part_d[r * S];
    int k = part_k[r * S];
    for (int sp = 1; sp < S; ++sp) {  // ascending k: strict < keeps the lower index
      const T v = part_d[r * S + sp];
      if (v < b) {
        b = v;
        k = part_k[r * S + sp];
      }
    }
    const int64_t orow = rowidx[r];
    labels[orow] = k;
    if (mind) mind[orow] = b;
  }
}

// rowidx (nullable): row i of the launch is row rowidx[i] of X (and of labels / mind), with
// the row count read from the device (nptr) -- the full re-scan of the rows the fp32/fp64
// MFMA assignment could not certify (assign_x3.hip), sized on the device
template <typename T>
__global__ __launch_bounds__(256) void assign_exact_kernel(const T* __restrict__ X, int64_t N,
                                                           int64_t ldx, int D,
                                                           const T* __restrict__ C, int K,
                                                           int32_t* __restrict__ labels,
                                                           T* __restrict__ mind,
                                                           const int32_t* __restrict__ rowidx,
                                                           const int* __restrict__ nptr,
                                                           int few_max, int few_grid = 0,
                                                           const T* __restrict__ part_d = nullptr,
                                                           const int* __restrict__ part_k = nullptr) {
  constexpr int MR = ExactCfg<T>::MR;
  constexpr int R = 16 * MR, KT = 128, DC = 32;
  constexpr int PX = R + 4, PC = KT + 4;  // row pitch (16-B aligned, spreads the store banks)
  __shared__ __attribute__((aligned(16))) T s_x[DC][PX];
  __shared__ __attribute__((aligned(16))) T s_c[DC][PC];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  constexpr bool F32 = sizeof(T) == 4;
  if (nptr) {
    N = *nptr;
    if (N <= few_max) {  // assign_exact_few_kernel has them; merge its K splits here
      if (part_d) exact_few_merge_rows<T>(K, few_grid, (int)N, 0, labels, mind, rowidx, part_d, part_k);
      return;
    }
  }
  for (int64_t r0 = (int64_t)blockIdx.x * R; r0 < N; r0 += (int64_t)gridDim.x * R) {
    T best[MR];
    int bk[MR];
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      best[i] = (T)INFINITY;
      bk[i] = 0;
    }
    for (int k0 = 0; k0 < K; k0 += KT) {
      // fp32: MR x 4 packed centroid pairs; fp64: MR x 8 scalars
      typename std::conditional<F32, f32x2[MR][4], double[MR][8]>::type acc;
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < (F32 ? 4 : 8); ++j) {
          if constexpr (F32) acc[i][j] = f32x2{0.f, 0.f};
          else acc[i][j] = 0.0;
        }
      for (int dc = 0; dc < D; dc += DC) {
        __syncthreads();
        // coalesced along the features, stored feature-major (transposed)
        for (int e = tid; e < R * DC; e += 256) {
          const int r = e / DC, d = e % DC;
          const int64_t xr = rowidx ? (int64_t)rowidx[r0 + r < N ? r0 + r : N - 1] : r0 + r;
          s_x[d][r] = (r0 + r < N && dc + d < D) ? X[xr * ldx + dc + d] : (T)0;
        }
        for (int e = tid; e < KT * DC; e += 256) {
          const int r = e / DC, d = e % DC;
          s_c[d][r] = (k0 + r < K && dc + d < D) ? C[(int64_t)(k0 + r) * D + dc + d] : (T)0;
        }
        __syncthreads();
#pragma unroll 2
        for (int d = 0; d < DC; ++d) {
          if constexpr (F32) {
            const f32x2* xs = reinterpret_cast<const f32x2*>(&s_x[d][ty * MR]);
            const f32x2* cs = reinterpret_cast<const f32x2*>(&s_c[d][tx * 8]);
            f32x2 xp[MR / 2], c2[4];
#pragma unroll
            for (int m = 0; m < MR / 2; ++m) xp[m] = xs[m];
#pragma unroll
            for (int j = 0; j < 4; ++j) c2[j] = cs[j];
#pragma unroll
            for (int m = 0; m < MR / 2; ++m)
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const f32x2 d0 = pk_sub_lo(xp[m], c2[j]);
                const f32x2 d1 = pk_sub_hi(xp[m], c2[j]);
                acc[2 * m][j] = __builtin_elementwise_fma(d0, d0, acc[2 * m][j]);
                acc[2 * m + 1][j] = __builtin_elementwise_fma(d1, d1, acc[2 * m + 1][j]);
              }
          } else {
            T xv[MR], cv[8];
#pragma unroll
            for (int i = 0; i < MR; ++i) xv[i] = s_x[d][ty * MR + i];
#pragma unroll
            for (int j = 0; j < 8; ++j) cv[j] = s_c[d][tx * 8 + j];
#pragma unroll
            for (int i = 0; i < MR; ++i)
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const T df = xv[i] - cv[j];
                acc[i][j] = fma(df, df, acc[i][j]);
              }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = k0 + tx * 8 + j;  // ascending per thread: strict < keeps the first
        if (k < K) {
#pragma unroll
          for (int i = 0; i < MR; ++i) {
            T v;
            if constexpr (F32) v = acc[i][j >> 1][j & 1];
            else v = acc[i][j];
            if (v < best[i]) {
              best[i] = v;
              bk[i] = k;
            }
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < MR; ++i) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const T ob = __shfl_xor(best[i], o, 64);
        const int ok = __shfl_xor(bk[i], o, 64);
        if (ob < best[i] || (ob == best[i] && ok < bk[i])) {
          best[i] = ob;
          bk[i] = ok;
        }
      }
      const int64_t row = r0 + ty * MR + i;
      if (tx == 0 && row < N) {
        const int64_t orow = rowidx ? (int64_t)rowidx[row] : row;
        labels[orow] = bk[i];
        if (mind) mind[orow] = best[i];
      }
    }
  }
}

// The listed re-scan when it is short (<= EXACT_FEW_MAX rows; the x3 path lists ~0.02% of N):
// RB rows per workgroup with one centroid of each 256-centroid chunk per thread, so a few
// thousand rows still spread over every CU (on the 128-row tiles 1.7k rows kept 14 CUs busy
// for 0.5 ms).  Same fma chain in ascending d from 0 as assign_exact_kernel (zero padding adds
// fma(0, 0, acc) = acc), so the distances are bit-identical; ties go to the lower index.
// K split (round 6): with few listed rows the row groups alone leave most of the grid idle
// (~60 fp64 rows: 8 workgroups streaming all K, ~120 us), so each row group's 256-centroid
// chunks are split over S workgroups, S = the idle share of the grid (the same on every
// workgroup: it depends only on the device-side count), each writing its (min, index) to
// part_d / part_k; exact_few_merge_kernel then takes the per-row minimum over the splits in
// ascending k order (ties: the lower index, as the unsplit scan).
template <typename T, int RB>
__device__ __forceinline__ void exact_few_body(const T* __restrict__ X, int64_t ldx, int D,
                                               const T* __restrict__ C, int K,
                                               int32_t* __restrict__ labels,
                                               T* __restrict__ mind,
                                               const int32_t* __restrict__ rowidx, int n,
                                               T* __restrict__ part_d, int* __restrict__ part_k,
                                               char* few_smem, T (*s_c)[257],
                                               T (*s_rb)[EXACT_FEW_RB],
                                               int (*s_rk)[EXACT_FEW_RB]) {
  constexpr int KT = 256, DC = 32;
  // the row group's rows, staged once (D <= EXACT_FEW_MAXD, zero-padded to the chunk): a
  // per-chunk slice had put two dependent global loads (index, row) on every chunk; in
  // dynamic LDS sized by the launch (Dp x EXACT_FEW_RB): a static D = 1024 image (64 KiB
  // in fp64) had left room for one workgroup per CU
  T(*s_x)[RB] = reinterpret_cast<T(*)[RB]>(few_smem);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // (k0, dc) chunks in one flat sequence; the next chunk's centroid slice (16-B loads when
  // rows allow) and row values are loaded into registers while the current one is computed
  constexpr int VEC = 16 / (int)sizeof(T), VPR = DC / VEC, NV = KT * DC / VEC / 256;
  typedef T vecT __attribute__((ext_vector_type(VEC)));
  const int nd = (D + DC - 1) / DC, nkc = (K + KT - 1) / KT;
  const bool vec_ok = D % VEC == 0 && ((uintptr_t)C % 16) == 0;
  vecT cv[NV];
  const int Dp = nd * DC;
  const int S = part_d ? exact_few_splits(n, nkc, (int)gridDim.x, RB) : 1;
  const int kcs = (nkc + S - 1) / S;  // 256-centroid chunks per split
  const int64_t items = (int64_t)((n + RB - 1) / RB) * S;
  auto load = [&](int64_t r0, int ci) __attribute__((always_inline)) {
    const int k0 = (ci / nd) * KT, dc = (ci % nd) * DC;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int e = tid + 256 * i, r = e / VPR, d = dc + (e % VPR) * VEC;
      const T* src = C + (int64_t)(k0 + r) * D + d;
      if (k0 + r < K && vec_ok && d + VEC <= D) {
        cv[i] = *reinterpret_cast<const vecT*>(src);
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) cv[i][j] = (k0 + r < K && d + j < D) ? src[j] : (T)0;
      }
    }
  };
  for (int64_t item = blockIdx.x; item < items; item += gridDim.x) {
    const int64_t r0 = (item / S) * RB;
    const int sp = (int)(item % S);
    const int c0 = sp * kcs * nd;  // this split's (k0, dc) chunk range
    const int c1 = min(nkc, (sp + 1) * kcs) * nd;
    if (c0 >= c1) continue;  // uniform per workgroup
    T best[RB];
    int bk[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      best[i] = (T)INFINITY;
      bk[i] = 0;
    }
    T acc[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) acc[i] = (T)0;
    load(r0, c0);
    __syncthreads();  // the previous group's reads of s_x are done
    for (int e = tid; e < RB * Dp; e += 256) {
      const int r = e / Dp, d = e % Dp;
      const int64_t row = r0 + r;
      s_x[d][r] = (row < n && d < D) ? X[(int64_t)rowidx[row] * ldx + d] : (T)0;
    }
    for (int ci = c0; ci < c1; ++ci) {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int e = tid + 256 * i, r = e / VPR, d = (e % VPR) * VEC;
#pragma unroll
        for (int j = 0; j < VEC; ++j) s_c[d + j][r] = cv[i][j];
      }
      __syncthreads();
      if (ci + 1 < c1) load(r0, ci + 1);
      const int dc = (ci % nd) * DC;
#pragma unroll 4
      for (int d = 0; d < DC; ++d) {
        const T c = s_c[d][tid];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const T df = s_x[dc + d][i] - c;
          acc[i] = fma(df, df, acc[i]);
        }
      }
      if (ci % nd == nd - 1) {  // a 256-centroid chunk is complete
        const int k = (ci / nd) * KT + tid;
        if (k < K) {
#pragma unroll
          for (int i = 0; i < RB; ++i)
            if (acc[i] < best[i]) {  // ascending k per thread: strict < keeps the first
              best[i] = acc[i];
              bk[i] = k;
            }
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) acc[i] = (T)0;
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const T ob = __shfl_xor(best[i], o, 64);
        const int ok = __shfl_xor(bk[i], o, 64);
        if (ob < best[i] || (ob == best[i] && ok < bk[i])) {
          best[i] = ob;
          bk[i] = ok;
        }
      }
      if (lane == 0) {
        s_rb[w][i] = best[i];
        s_rk[w][i] = bk[i];
      }
    }
    __syncthreads();
    if (tid < RB && r0 + tid < n) {
      T b = s_rb[0][tid];
      int k = s_rk[0][tid];
#pragma unroll
      for (int v = 1; v < 4; ++v)
        if (s_rb[v][tid] < b || (s_rb[v][tid] == b && s_rk[v][tid] < k)) {
          b = s_rb[v][tid];
          k = s_rk[v][tid];
        }
      if (S > 1) {
        part_d[(r0 + tid) * S + sp] = b;
        part_k[(r0 + tid) * S + sp] = k;
      } else {
        const int64_t orow = rowidx[r0 + tid];
        labels[orow] = k;
        if (mind) mind[orow] = b;
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void assign_exact_few_kernel(const T* __restrict__ X, int64_t ldx,
                                                               int D, const T* __restrict__ C, int K,
                                                               int32_t* __restrict__ labels,
                                                               T* __restrict__ mind,
                                                               const int32_t* __restrict__ rowidx,
                                                               const int* __restrict__ nptr,
                                                               T* __restrict__ part_d,
                                                               int* __restrict__ part_k,
                                                               int force_rb) {
  extern __shared__ __attribute__((aligned(16))) char few_smem[];
  __shared__ T s_c[32][257];
  __shared__ T s_rb[4][EXACT_FEW_RB];
  __shared__ int s_rk[4][EXACT_FEW_RB];
  const int n = *nptr;
  if (n > EXACT_FEW_MAX) return;  // assign_exact_kernel has them
  const int rb = exact_few_rb(n, force_rb);  // uniform: every workgroup reads the same n
  if (rb == 1)
    exact_few_body<T, 1>(X, ldx, D, C, K, labels, mind, rowidx, n, part_d, part_k, few_smem, s_c, s_rb, s_rk);
  else if (rb == 2)
    exact_few_body<T, 2>(X, ldx, D, C, K, labels, mind, rowidx, n, part_d, part_k, few_smem, s_c, s_rb, s_rk);
  else if (rb == 4)
    exact_few_body<T, 4>(X, ldx, D, C, K, labels, mind, rowidx, n, part_d, part_k, few_smem, s_c, s_rb, s_rk);
  else
    exact_few_body<T, EXACT_FEW_RB>(X, ldx, D, C, K, labels, mind, rowidx, n, part_d, part_k, few_smem, s_c, s_rb, s_rk);
}

template <typename T>
__global__ __launch_bounds__(256) void exact_few_merge_kernel(int K, int few_grid,
                                                              int32_t* __restrict__ labels,
                                                              T* __restrict__ mind,
                                                              const int32_t* __restrict__ rowidx,
                                                              const int* __restrict__ nptr,
                                                              const T* __restrict__ part_d,
                                                              const int* __restrict__ part_k,
                                                              int force_rb) {
  const int n = *nptr;
  if (n > EXACT_FEW_MAX) return;
  exact_few_merge_rows<T>(K, few_grid, n, force_rb, labels, mind, rowidx, part_d, part_k);
}

// split scratch of the few-rows re-scan, one per device (allocated on first use, before
// any graph capture: the engines run an eager step first)
static void* few_parts(int dtype_bytes) {
  static void* bufs[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!bufs[dev]) {
    void* p = nullptr;
    if (hipMalloc(&p, (size_t)EXACT_FEW_PARTS * (8 + 4)) != hipSuccess) return nullptr;
    bufs[dev] = p;
  }
  (void)dtype_bytes;
  return bufs[dev];
}

int tdc_assign_exact(int dtype, const void* X, int64_t N, int64_t ldx, int D, const void* C, int K,
                     int32_t* labels, void* mind, int num_cus, hipStream_t s,
                     const int32_t* rowidx, const int* nptr) {
  if (N <= 0) return 0;
  const bool few = nptr && D <= EXACT_FEW_MAXD;
  // K split: the grid covers the row groups of up to EXACT_FEW_MAX rows or, when fewer are
  // listed, their 256-centroid chunks (a few hundred workgroups either way); two workgroups
  // per CU: the listed count is read on the device, the few busy workgroups split their row
  // groups over K (exact_few_splits), the rest leave at once
  const int64_t fb = (int64_t)(num_cus > 0 ? num_cus : 256) * 2;
  char* parts = nullptr;
  int* part_k = nullptr;
  // with N > EXACT_FEW_MAX the tiled launch below also runs (and returns at once when the
  // listed rows were few): it does the K-split merge then, one launch fewer per step
  const bool tiled = !few || N > EXACT_FEW_MAX;
  if (few) {
    if (!rowidx) return (int)hipErrorInvalidValue;
    // both launches read the listed count; exactly one of them has work
    const int dpad = (D + 31) / 32 * 32;
    const size_t few_lds = (size_t)dpad * EXACT_FEW_RB * (dtype == TDC_F64 ? 8 : 4);
    parts = (char*)few_parts(dtype == TDC_F64 ? 8 : 4);
    if (!parts) return (int)hipErrorOutOfMemory;
    part_k = (int*)(parts + (size_t)EXACT_FEW_PARTS * 8);
    const int mb = (EXACT_FEW_PARTS + 255) / 256;
    if (dtype == TDC_F32) {
      hipLaunchKernelGGL(assign_exact_few_kernel<float>, dim3((unsigned)fb), dim3(256), few_lds, s,
                         (const float*)X, ldx, D, (const float*)C, K, labels, (float*)mind, rowidx,
                         nptr, (float*)parts, part_k, 0);
      TDC_CHECK_LAUNCH();
      if (!tiled)
        hipLaunchKernelGGL(exact_few_merge_kernel<float>, dim3((unsigned)mb), dim3(256), 0, s, K,
                           (int)fb, labels, (float*)mind, rowidx, nptr, (const float*)parts,
                           (const int*)part_k, 0);
    } else if (dtype == TDC_F64) {
      hipLaunchKernelGGL(assign_exact_few_kernel<double>, dim3((unsigned)fb), dim3(256), few_lds, s,
                         (const double*)X, ldx, D, (const double*)C, K, labels, (double*)mind,
                         rowidx, nptr, (double*)parts, part_k, 0);
      TDC_CHECK_LAUNCH();
      if (!tiled)
        hipLaunchKernelGGL(exact_few_merge_kernel<double>, dim3((unsigned)mb), dim3(256), 0, s, K,
                           (int)fb, labels, (double*)mind, rowidx, nptr, (const double*)parts,
                           (const int*)part_k, 0);
    } else {
      return (int)hipErrorInvalidValue;
    }
    TDC_CHECK_LAUNCH();
    if (!tiled) return 0;
  }
  const int64_t rows_per_tile = 16 * (dtype == TDC_F64 ? ExactCfg<double>::MR : ExactCfg<float>::MR);
  int64_t blocks = (N + rows_per_tile - 1) / rows_per_tile;
  // grid-stride over row tiles with the blocks resident at once (no partial 2nd round)
  static const int res32 = resident_blocks(assign_exact_kernel<float>, 256);
  static const int res64 = resident_blocks(assign_exact_kernel<double>, 256);
  const int64_t resident = dtype == TDC_F64 ? res64 : res32;
  if (blocks > resident) blocks = resident;
  if (dtype == TDC_F32)
    hipLaunchKernelGGL(assign_exact_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const float*)X, N, ldx, D, (const float*)C, K, labels, (float*)mind,
                       rowidx, nptr, few ? EXACT_FEW_MAX : -1, (int)fb, (const float*)parts,
                       (const int*)part_k);
  else if (dtype == TDC_F64)
    hipLaunchKernelGGL(assign_exact_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const double*)X, N, ldx, D, (const double*)C, K, labels, (double*)mind,
                       rowidx, nptr, few ? EXACT_FEW_MAX : -1, (int)fb, (const double*)parts,
                       (const int*)part_k);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  return 0;
}

int tdc_assign_simt(int dtype, const void* X, int64_t N, int64_t ldx, int D, const void* C,
                    int K, int32_t* labels, void* mind, hipStream_t s) {
  if (N <= 0) return 0;
  const dim3 grid((unsigned)((N + 255) / 256));
#define TDC_AS(T, DM)                                                                      \
  if (D <= DM) {                                                                           \
    hipLaunchKernelGGL((assign_simt_kernel<T, DM>), grid, dim3(256), 0, s, (const T*)X, N, \
                       ldx, D, (const T*)C, K, labels, (T*)mind);                          \
    TDC_CHECK_LAUNCH();                                                                    \
    return 0;                                                                              \
  }
  if (dtype == TDC_F32) {
    TDC_AS(float, 4) TDC_AS(float, 8) TDC_AS(float, 16) TDC_AS(float, 32) TDC_AS(float, 64)
  } else if (dtype == TDC_F64) {
    TDC_AS(double, 4) TDC_AS(double, 8) TDC_AS(double, 16) TDC_AS(double, 32)
  }
#undef TDC_AS
  return (int)hipErrorInvalidValue;
}

namespace {
template <typename XT, typename ACC, int VEC>
int launch_update(const void* X, int64_t N, int64_t ldx, int D, int DS, const int32_t* labels,
                  int K, void* sums, void* counts, int num_cus, hipStream_t s) {
  const int nslices = (D + DS - 1) / DS;
  const size_t lds = (size_t)K * (DS + 1) * sizeof(typename LdsT<XT>::type) + (size_t)K * sizeof(int);
  const int blocks_per_cu = lds <= 40 * 1024 ? 4 : (lds <= 80 * 1024 ? 2 : 1);
  const int tpr = DS / VEC, rpi = 256 / tpr;
  int64_t target_chunks = (int64_t)num_cus * blocks_per_cu / nslices;
  if (target_chunks < 1) target_chunks = 1;
  const int64_t max_chunks = (N + rpi - 1) / rpi;
  int64_t chunks = target_chunks < max_chunks ? target_chunks : max_chunks;
  if (chunks < 1) chunks = 1;
  const int64_t rpb = (N + chunks - 1) / chunks;
  chunks = (N + rpb - 1) / rpb;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)update_lds_kernel<XT, ACC, VEC>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL((update_lds_kernel<XT, ACC, VEC>), dim3((unsigned)(chunks * nslices)),
                     dim3(256), lds, s, (const XT*)X, N, ldx, D, DS, labels, K, (ACC*)sums,
                     (ACC*)counts, nslices, rpb);
  TDC_CHECK_LAUNCH();
  return 0;
}

template <typename ACC>
int dispatch_update(int x_dtype, const void* X, int64_t N, int64_t ldx, int D,
                    const int32_t* labels, int K, void* sums, void* counts, int num_cus,
                    hipStream_t s) {
  // slice width: largest power of two (<= next_pow2(D), <= 256) whose LDS image fits 140 KB
  const size_t es = (x_dtype == TDC_F64) ? 8 : 4;
  auto bytes = [&](int ds) { return (size_t)K * (ds + 1) * es + (size_t)K * 4; };
  int dmax = 1;
  while (dmax < D && dmax < 256) dmax <<= 1;
  int DS = dmax;
  while (DS > 1 && bytes(DS) > 140 * 1024) DS >>= 1;
  if (bytes(DS) > 140 * 1024) return (int)hipErrorInvalidValue;
  // prefer two blocks per CU when it only costs half the slice width
  if (DS >= 16 && bytes(DS) > 80 * 1024 && bytes(DS / 2) <= 80 * 1024) DS >>= 1;
  const bool aligned = ((uintptr_t)X % 16 == 0);
  if (x_dtype == TDC_BF16) {
    if (aligned && D % 4 == 0 && ldx % 4 == 0 && DS >= 4)
      return launch_update<__bf16, ACC, 4>(X, N, ldx, D, DS, labels, K, sums, counts, num_cus, s);
    return launch_update<__bf16, ACC, 1>(X, N, ldx, D, DS, labels, K, sums, counts, num_cus, s);
  }
  if (x_dtype == TDC_F32) {
    if (aligned && D % 4 == 0 && ldx % 4 == 0 && DS >= 4)
      return launch_update<float, ACC, 4>(X, N, ldx, D, DS, labels, K, sums, counts, num_cus, s);
    return launch_update<float, ACC, 1>(X, N, ldx, D, DS, labels, K, sums, counts, num_cus, s);
  }
  if (x_dtype == TDC_F64) {
    if (aligned && D % 2 == 0 && ldx % 2 == 0 && DS >= 2)
      return launch_update<double, ACC, 2>(X, N, ldx, D, DS, labels, K, sums, counts, num_cus, s);
    return launch_update<double, ACC, 1>(X, N, ldx, D, DS, labels, K, sums, counts, num_cus, s);
  }
  return (int)hipErrorInvalidValue;
}
}  // namespace

int tdc_update_lds(int x_dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                   const int32_t* labels, int K, void* sums, void* counts, int num_cus,
                   hipStream_t s) {
  if (N <= 0) return 0;
  if (acc_dtype == TDC_F64)
    return dispatch_update<double>(x_dtype, X, N, ldx, D, labels, K, sums, counts, num_cus, s);
  return dispatch_update<float>(x_dtype, X, N, ldx, D, labels, K, sums, counts, num_cus, s);
}
