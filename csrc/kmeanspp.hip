// N7: k-means++ seeding step on the device.
//
// Reference: sklearn's private `k_means_._init_centroids(..., 'k-means++')` on a host copy
// of every batch (`scripts/distribuitedClustering.py:82,191`).  Greedy k-means++ adds one
// center per step: draw T candidates with probability ~ D^2, keep the candidate that
// minimises the potential sum_i min(D^2_i, ||x_i - c_t||^2), then update D^2.  The torch
// formulation materialises a [T, N] distance matrix and re-reads X T+1 times per step;
// here one pass over X scores all T candidates (exact-difference distances against the
// candidates held in LDS, fp64 potentials per block -> one atomic per candidate per
// block), and a second pass applies the winner (mode 1) and returns the new potential.
#include "kernels.h"
#include "tdc_common.h"

namespace tdc {

constexpr int KPP_TMAX = 16;

template <typename DT, typename XT> __device__ __forceinline__ DT kpp_cvt(XT v) { return (DT)v; }
template <> __device__ __forceinline__ float kpp_cvt<float, __bf16>(__bf16 v) { return (float)v; }
template <> __device__ __forceinline__ double kpp_cvt<double, __bf16>(__bf16 v) { return (double)(float)v; }

template <typename XT, typename DT, int TPR>
__global__ __launch_bounds__(256) void kpp_step_kernel(const XT* __restrict__ X, int64_t N,
                                                       int64_t ldx, int D,
                                                       const DT* __restrict__ cand, int T,
                                                       DT* __restrict__ closest, int mode,
                                                       double* __restrict__ pots) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  DT* s_c = reinterpret_cast<DT*>(smem_raw);          // [T][D]
  __shared__ double s_pot[4][KPP_TMAX];
  const int tid = threadIdx.x;
  for (int i = tid; i < T * D; i += 256) s_c[i] = cand[i];
  __syncthreads();
  constexpr int G = 64 / TPR;  // rows per wave-instruction
  const int lane = tid & 63, w = tid >> 6;
  const int g = lane / TPR, t = lane % TPR;
  double pot[KPP_TMAX];
#pragma unroll
  for (int c = 0; c < KPP_TMAX; ++c) pot[c] = 0.0;
  const int64_t rows_per_block = 4 * G;
  for (int64_t r0 = (int64_t)blockIdx.x * rows_per_block; r0 < N;
       r0 += (int64_t)gridDim.x * rows_per_block) {
    const int64_t row = r0 + w * G + g;
    const bool ok = row < N;
    DT acc[KPP_TMAX];
#pragma unroll
    for (int c = 0; c < KPP_TMAX; ++c) acc[c] = 0;
    if (ok) {
      const XT* xr = X + row * ldx;
      for (int d = t; d < D; d += TPR) {
        const DT xv = kpp_cvt<DT, XT>(xr[d]);
#pragma unroll
        for (int c = 0; c < KPP_TMAX; ++c) {
          if (c < T) {
            const DT df = xv - s_c[c * D + d];
            acc[c] = fma(df, df, acc[c]);
          }
        }
      }
    }
    // reduce over the TPR lanes of the row
#pragma unroll
    for (int c = 0; c < KPP_TMAX; ++c) {
      if (c < T) {
#pragma unroll
        for (int o = TPR / 2; o > 0; o >>= 1) acc[c] += __shfl_xor(acc[c], o, 64);
      }
    }
    if (ok && t == 0) {
      const DT old = closest[row];
      if (mode == 0) {
#pragma unroll
        for (int c = 0; c < KPP_TMAX; ++c)
          if (c < T) pot[c] += (double)(acc[c] < old ? acc[c] : old);
      } else {
        const DT nv = acc[0] < old ? acc[0] : old;
        closest[row] = nv;
        pot[0] += (double)nv;
      }
    }
  }
  const int nt = mode == 0 ? T : 1;
#pragma unroll
  for (int c = 0; c < KPP_TMAX; ++c) {
    if (c < nt) {
      double v = wave_sum(pot[c]);
      if (lane == 0) s_pot[w][c] = v;
    }
  }
  __syncthreads();
  if (tid < nt) atomicAdd(&pots[tid], s_pot[0][tid] + s_pot[1][tid] + s_pot[2][tid] + s_pot[3][tid]);
}

template <typename XT, typename DT>
int launch_kpp(const void* X, int64_t N, int64_t ldx, int D, const void* cand, int T,
               void* closest, int mode, double* pots, int num_cus, hipStream_t s) {
  const size_t lds = sizeof(DT) * (size_t)T * D;
  if (lds > 64 * 1024) return (int)hipErrorInvalidValue;
  int64_t blocks = (int64_t)num_cus * 8;
#define TDC_KPP(TPRV)                                                                          \
  {                                                                                            \
    const int64_t per = 4 * (64 / TPRV);                                                       \
    const int64_t need = (N + per - 1) / per;                                                  \
    hipLaunchKernelGGL((kpp_step_kernel<XT, DT, TPRV>), dim3((unsigned)(need < blocks ? need : blocks)), \
                       dim3(256), lds, s, (const XT*)X, N, ldx, D, (const DT*)cand, T,         \
                       (DT*)closest, mode, pots);                                              \
  }
  if (D <= 8) TDC_KPP(1)
  else if (D <= 64) TDC_KPP(8)
  else TDC_KPP(16)
#undef TDC_KPP
  TDC_CHECK_LAUNCH();
  return 0;
}

}  // namespace tdc

using namespace tdc;

int tdc_kpp_step(int x_dtype, int d_dtype, const void* X, int64_t N, int64_t ldx, int D,
                 const void* cand, int T, void* closest, int mode, double* pots, int num_cus,
                 hipStream_t s) {
  if (N <= 0) return 0;
  if (T < 1 || T > KPP_TMAX || (mode == 1 && T != 1)) return (int)hipErrorInvalidValue;
  if (d_dtype == TDC_F64) {
    if (x_dtype == TDC_F64) return launch_kpp<double, double>(X, N, ldx, D, cand, T, closest, mode, pots, num_cus, s);
    if (x_dtype == TDC_F32) return launch_kpp<float, double>(X, N, ldx, D, cand, T, closest, mode, pots, num_cus, s);
    if (x_dtype == TDC_BF16) return launch_kpp<__bf16, double>(X, N, ldx, D, cand, T, closest, mode, pots, num_cus, s);
  } else if (d_dtype == TDC_F32) {
    if (x_dtype == TDC_F32) return launch_kpp<float, float>(X, N, ldx, D, cand, T, closest, mode, pots, num_cus, s);
    if (x_dtype == TDC_BF16) return launch_kpp<__bf16, float>(X, N, ldx, D, cand, T, closest, mode, pots, num_cus, s);
  }
  return (int)hipErrorInvalidValue;
}
