// N3: centroid finalize + next-iteration operand prep, one wave per centroid row.
//
// Reference (scripts/distribuitedClustering.py:257-263): on /cpu:0, AddN of the tower
// partials, Tile/Reshape of the counts, Div, Transpose, Assign.  Here every rank runs this
// on its replicated copy right after the all-reduce:
//   c_k = sums_k / count_k            (empty cluster: keep | NaN (reference) | zero)
//   shift = max_k ||c_k - c_k_old||^2  (for the optional tolerance stop)
// and, for the bf16 MFMA assignment, writes its operands in the same pass:
//   Cm2[k] = -2 * bf16(c_k)   (exact scaling), cnorm[k] = ||bf16(c_k)||^2 (fp32),
//   pad rows k >= K: Cm2 = 0, cnorm = 3e38 (never selected).
#include <algorithm>

#include "tdc_common.h"
#include "kernels.h"

namespace tdc {

// One wave per centroid row, rows strided over a grid of at most MAX_BLOCKS blocks; the
// shift max is reduced per block (LDS) so the single-address atomicMax runs once per
// block instead of once per row (4096 same-address atomics cost ~40 us).
constexpr int MAX_BLOCKS = 256;

// shift values are >= 0 or NaN: as unsigned bit patterns every NaN orders above every
// finite value, so an integer max keeps a NaN shift NaN (a float fmax would drop it)
__device__ __forceinline__ void block_max_shift(unsigned sh, float* shift) {
  __shared__ unsigned s_sh[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) sh = max(sh, (unsigned)__shfl_xor((int)sh, o, 64));
  if ((threadIdx.x & 63) == 0) s_sh[threadIdx.x >> 6] = sh;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned m = max(max(s_sh[0], s_sh[1]), max(s_sh[2], s_sh[3]));
    if (m != 0u) atomicMax(reinterpret_cast<unsigned*>(shift), m);
  }
}

template <typename ACC, typename CT>
__global__ __launch_bounds__(256) void finalize_kernel(const ACC* __restrict__ sums,
                                                       const ACC* __restrict__ counts, int K,
                                                       int D, CT* __restrict__ C, int policy,
                                                       float* __restrict__ shift,
                                                       __bf16* __restrict__ Cm2,
                                                       float* __restrict__ cnorm, int Kp, int DP,
                                                       float* __restrict__ drift,
                                                       float* __restrict__ maxdrift) {
  const int lane = threadIdx.x & 63;
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  unsigned shmax = 0u, dmax = 0u;
  for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < rows; k += gridDim.x * 4) {
    if (k >= K) {
      if (Cm2)
        for (int d = lane; d < DP; d += 64) Cm2[(int64_t)k * DP + d] = (__bf16)0.f;
      if (cnorm && lane == 0) cnorm[k] = 3.0e38f;
      continue;
    }
    float sh = 0.f, nrm = 0.f, dsq = 0.f;
    ACC cnt = sums ? counts[k] : (ACC)1;
    const int dend = Cm2 ? (DP > D ? DP : D) : D;
    for (int d = lane; d < dend; d += 64) {
      if (d < D) {
        const CT old = C[(int64_t)k * D + d];
        CT nw = old;
        if (sums) {
          if (cnt > (ACC)0) {
            nw = (CT)(sums[(int64_t)k * D + d] / cnt);
          } else if (policy == 1) {
            nw = (CT)NAN;
          } else if (policy == 2) {
            nw = (CT)0;
          }
          C[(int64_t)k * D + d] = nw;
          const float df = (float)nw - (float)old;
          sh += df * df;
          if (drift) {  // movement in the assignment kernels' own (bf16) coordinates
            // a centroid that was already NaN can never win the argmin: leave it out
            // (drift 0) instead of forcing every row to re-assign on every later step;
            // one that comes back from NaN moved arbitrarily far (drift +inf)
            const float nb = (float)(__bf16)(float)nw, ob = (float)(__bf16)(float)old;
            const float e = isnan(ob) ? (isnan(nb) ? 0.f : INFINITY) : nb - ob;
            dsq = fmaf(e, e, dsq);
          }
        }
        if (Cm2) {
          const __bf16 b = (__bf16)(float)nw;
          const float bf = (float)b;
          Cm2[(int64_t)k * DP + d] = (__bf16)(-2.f * bf);
          nrm = fmaf(bf, bf, nrm);
        }
      } else if (Cm2 && d < DP) {
        Cm2[(int64_t)k * DP + d] = (__bf16)0.f;
      }
    }
    if (sums && shift) shmax = max(shmax, __float_as_uint(wave_sum(sh)));
    if (sums && drift) {
      const float dk = sqrtf(wave_sum(dsq));  // NaN (poisoned centroid) stays NaN
      if (lane == 0) drift[k] = dk;
      dmax = max(dmax, __float_as_uint(dk));
    }
    if (cnorm) {
      nrm = wave_sum(nrm);
      if (lane == 0) cnorm[k] = nrm;
    }
  }
  if (sums && shift) block_max_shift(shmax, shift);
  if (sums && maxdrift) {
    __syncthreads();  // block_max_shift's LDS slots are reused
    block_max_shift(dmax, maxdrift);
  }
}

template <typename ACC, typename CT>
int launch_finalize(const void* sums, const void* counts, int K, int D, void* C, int policy,
                    float* shift, void* Cm2, float* cnorm, int Kp, int DP, hipStream_t s,
                    float* drift, float* maxdrift) {
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  if (rows <= 0) return 0;  // an rsag rank with no centroid rows of its own: nothing to do
  const int blocks = std::min((rows + 3) / 4, MAX_BLOCKS);
  hipLaunchKernelGGL((finalize_kernel<ACC, CT>), dim3((unsigned)blocks), dim3(256), 0,
                     s, (const ACC*)sums, (const ACC*)counts, K, D, (CT*)C, policy, shift,
                     (__bf16*)Cm2, cnorm, Kp, DP, drift, maxdrift);
  TDC_CHECK_LAUNCH();
  return 0;
}

// Mini-batch (Sculley) centre update, one wave per centroid row:
//   n_k > 0:  c_k <- (v_k c_k + S_k) / (v_k + n_k),  v_k <- v_k + n_k   (fp64 arithmetic)
//   n_k = 0:  c_k unchanged
// shift = max over updated k of ||c_k - c_k_old||^2, plus the bf16 operand prep of the
// next assignment -- one launch instead of ~15 small fp64 elementwise kernels.
template <typename ACC, typename CT>
__global__ __launch_bounds__(256) void sculley_kernel(const ACC* __restrict__ sums,
                                                      const ACC* __restrict__ counts, int K, int D,
                                                      CT* __restrict__ C, double* __restrict__ v,
                                                      float* __restrict__ shift,
                                                      __bf16* __restrict__ Cm2,
                                                      float* __restrict__ cnorm, int Kp, int DP) {
  const int lane = threadIdx.x & 63;
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  unsigned shmax = 0u;
  for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < rows; k += gridDim.x * 4) {
    if (k >= K) {
      if (Cm2)
        for (int d = lane; d < DP; d += 64) Cm2[(int64_t)k * DP + d] = (__bf16)0.f;
      if (cnorm && lane == 0) cnorm[k] = 3.0e38f;
      continue;
    }
    const double n = (double)counts[k];
    const double vk = v[k];
    const double inv = n > 0.0 ? 1.0 / (vk + n) : 0.0;
    float sh = 0.f, nrm = 0.f;
    const int dend = Cm2 ? (DP > D ? DP : D) : D;
    for (int d = lane; d < dend; d += 64) {
      if (d < D) {
        const CT old = C[(int64_t)k * D + d];
        CT nw = old;
        if (n > 0.0) {
          nw = (CT)((vk * (double)old + (double)sums[(int64_t)k * D + d]) * inv);
          C[(int64_t)k * D + d] = nw;
          const float df = (float)nw - (float)old;
          sh += df * df;
        }
        if (Cm2) {
          const __bf16 b = (__bf16)(float)nw;
          const float bf = (float)b;
          Cm2[(int64_t)k * DP + d] = (__bf16)(-2.f * bf);
          nrm = fmaf(bf, bf, nrm);
        }
      } else if (Cm2 && d < DP) {
        Cm2[(int64_t)k * DP + d] = (__bf16)0.f;
      }
    }
    if (shift) shmax = max(shmax, __float_as_uint(wave_sum(sh)));
    if (cnorm) {
      nrm = wave_sum(nrm);
      if (lane == 0) cnorm[k] = nrm;
    }
    if (lane == 0) v[k] = vk + n;  // every lane read v[k] above (wave lockstep)
  }
  if (shift) block_max_shift(shmax, shift);
}

template <typename ACC, typename CT>
int launch_sculley(const void* sums, const void* counts, int K, int D, void* C, double* v,
                   float* shift, void* Cm2, float* cnorm, int Kp, int DP, hipStream_t s) {
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  const int blocks = std::min((rows + 3) / 4, MAX_BLOCKS);
  hipLaunchKernelGGL((sculley_kernel<ACC, CT>), dim3((unsigned)blocks), dim3(256), 0, s,
                     (const ACC*)sums, (const ACC*)counts, K, D, (CT*)C, v, shift, (__bf16*)Cm2,
                     cnorm, Kp, DP);
  TDC_CHECK_LAUNCH();
  return 0;
}

}  // namespace tdc

using namespace tdc;

int tdc_sculley_update(int acc_dtype, int c_dtype, const void* sums, const void* counts, int K,
                       int D, void* C, double* v, float* shift, void* Cm2, float* cnorm, int Kp,
                       int DP, hipStream_t s) {
  if (acc_dtype == TDC_F64 && c_dtype == TDC_F32)
    return launch_sculley<double, float>(sums, counts, K, D, C, v, shift, Cm2, cnorm, Kp, DP, s);
  if (acc_dtype == TDC_F32 && c_dtype == TDC_F32)
    return launch_sculley<float, float>(sums, counts, K, D, C, v, shift, Cm2, cnorm, Kp, DP, s);
  if (acc_dtype == TDC_F64 && c_dtype == TDC_F64)
    return launch_sculley<double, double>(sums, counts, K, D, C, v, shift, Cm2, cnorm, Kp, DP, s);
  if (acc_dtype == TDC_F32 && c_dtype == TDC_F64)
    return launch_sculley<float, double>(sums, counts, K, D, C, v, shift, Cm2, cnorm, Kp, DP, s);
  return (int)hipErrorInvalidValue;
}

int tdc_finalize(int acc_dtype, int c_dtype, const void* sums, const void* counts, int K, int D,
                 void* C, int policy, float* shift, void* Cm2, float* cnorm, int Kp, int DP,
                 hipStream_t s, float* drift, float* maxdrift) {
  if (acc_dtype == TDC_F64 && c_dtype == TDC_F32)
    return launch_finalize<double, float>(sums, counts, K, D, C, policy, shift, Cm2, cnorm, Kp, DP, s,
                                         drift, maxdrift);
  if (acc_dtype == TDC_F32 && c_dtype == TDC_F32)
    return launch_finalize<float, float>(sums, counts, K, D, C, policy, shift, Cm2, cnorm, Kp, DP, s,
                                         drift, maxdrift);
  if (acc_dtype == TDC_F64 && c_dtype == TDC_F64)
    return launch_finalize<double, double>(sums, counts, K, D, C, policy, shift, Cm2, cnorm, Kp, DP, s,
                                         drift, maxdrift);
  if (acc_dtype == TDC_F32 && c_dtype == TDC_F64)
    return launch_finalize<float, double>(sums, counts, K, D, C, policy, shift, Cm2, cnorm, Kp, DP, s,
                                         drift, maxdrift);
  return (int)hipErrorInvalidValue;
}
