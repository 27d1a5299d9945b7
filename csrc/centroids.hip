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
#include <type_traits>

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

// One centroid row k (one wave, lane-strided features): c_k = rowsum(d) / cnt with the
// empty-cluster policy, its shift^2 / drift contributions, and the bf16 operand prep of
// the next assignment.  have_sums == false: operand prep only (C unchanged).  rowsum(d)
// is called once for every d < D by the lane owning d.
template <typename S, typename CT, typename F>
__device__ __forceinline__ void finalize_row(int k, int D, bool have_sums, S cnt, F&& rowsum,
                                             CT* __restrict__ C, int policy,
                                             __bf16* __restrict__ Cm2, float* __restrict__ cnorm,
                                             int DP, bool want_shift, float* __restrict__ drift,
                                             unsigned& shmax, unsigned& dmax) {
  const int lane = threadIdx.x & 63;
  float sh = 0.f, nrm = 0.f, dsq = 0.f;
  const int dend = Cm2 ? (DP > D ? DP : D) : D;
  for (int d = lane; d < dend; d += 64) {
    if (d < D) {
      const CT old = C[(int64_t)k * D + d];
      CT nw = old;
      if (have_sums) {
        const auto sv = rowsum(d);
        if (cnt > (S)0) {
          nw = (CT)(sv / cnt);
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
  if (have_sums && want_shift) shmax = max(shmax, __float_as_uint(wave_sum(sh)));
  if (have_sums && drift) {
    const float dk = sqrtf(wave_sum(dsq));  // NaN (poisoned centroid) stays NaN
    if (lane == 0) drift[k] = dk;
    dmax = max(dmax, __float_as_uint(dk));
  }
  if (cnorm) {
    nrm = wave_sum(nrm);
    if (lane == 0) cnorm[k] = nrm;
  }
}

// padding rows k >= K of the assign operands: zero -2c, a norm that never wins
__device__ __forceinline__ void pad_row(int k, __bf16* __restrict__ Cm2, float* __restrict__ cnorm,
                                        int DP) {
  const int lane = threadIdx.x & 63;
  if (Cm2)
    for (int d = lane; d < DP; d += 64) Cm2[(int64_t)k * DP + d] = (__bf16)0.f;
  if (cnorm && lane == 0) cnorm[k] = 3.0e38f;
}

template <typename ACC, typename CT>
__global__ __launch_bounds__(256) void finalize_kernel(const ACC* __restrict__ sums,
                                                       const ACC* __restrict__ counts, int K,
                                                       int D, CT* __restrict__ C, int policy,
                                                       float* __restrict__ shift,
                                                       __bf16* __restrict__ Cm2,
                                                       float* __restrict__ cnorm, int Kp, int DP,
                                                       float* __restrict__ drift,
                                                       float* __restrict__ maxdrift,
                                                       double inv_scale) {
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  unsigned shmax = 0u, dmax = 0u;
  for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < rows; k += gridDim.x * 4) {
    if (k >= K) {
      pad_row(k, Cm2, cnorm, DP);
      continue;
    }
    if constexpr (std::is_same<ACC, long long>::value) {
      // fixed-point sums (the deterministic update): value = sum / scale
      const double cnt = sums ? (double)counts[k] : 1.0;
      finalize_row(k, D, sums != nullptr, cnt,
                   [&](int d) { return (double)sums[(int64_t)k * D + d] * inv_scale; }, C,
                   policy, Cm2, cnorm, DP, shift != nullptr, drift, shmax, dmax);
    } else {
      const ACC cnt = sums ? counts[k] : (ACC)1;
      finalize_row(k, D, sums != nullptr, cnt,
                   [&](int d) { return sums[(int64_t)k * D + d]; }, C, policy, Cm2, cnorm, DP,
                   shift != nullptr, drift, shmax, dmax);
    }
  }
  if (sums && shift) block_max_shift(shmax, shift);
  if (sums && maxdrift) {
    __syncthreads();  // block_max_shift's LDS slots are reused
    block_max_shift(dmax, maxdrift);
  }
}

// Delta-update finalize (update_sorted.hip, delta_* kernels): G = [sums K*D | counts K]
// fp64 running totals of the current assignment, replicated on every rank.  The step's
// all-reduced buffer holds the DELTAS of a delta step (G += buf) or the full partials of
// a full step (G = buf); the centroids are then G's means.  Block 0 also picks the mode
// of the next step (kernels.h TDC_DC_*): full every `refresh` steps, or when this step
// moved more than theta_n rows globally (the all-reduced moved slot, identical on every
// rank); and accumulates stats = [moved rows, steps with a valid prev, full steps, steps].
template <typename ACC, typename CT>
__global__ __launch_bounds__(256) void finalize_delta_kernel(
    const ACC* __restrict__ dsums, const ACC* __restrict__ dcounts,
    const float* __restrict__ cnt_hi, const float* __restrict__ cnt_lo,
    const ACC* __restrict__ moved, double* __restrict__ G, int K, int D, CT* __restrict__ C,
    int policy, float* __restrict__ shift, __bf16* __restrict__ Cm2, float* __restrict__ cnorm,
    int Kp, int DP, int* __restrict__ ctrl, double* __restrict__ stats, int refresh,
    double theta_n, double inv_scale) {
  const int lane = threadIdx.x & 63;
  const bool full = ctrl[TDC_DC_MODE] != 0;
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  double* Gc = G + (int64_t)K * D;
  unsigned shmax = 0u, dmax = 0u;
  for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < rows; k += gridDim.x * 4) {
    if (k >= K) {
      pad_row(k, Cm2, cnorm, DP);
      continue;
    }
    const double dc = cnt_hi ? (double)cnt_hi[k] * 4096.0 + (double)cnt_lo[k] : (double)dcounts[k];
    const double gc = (full ? 0.0 : Gc[k]) + dc;  // every lane reads before lane 0 writes
    finalize_row(k, D, true, gc,
                 [&](int d) {
                   const int64_t e = (int64_t)k * D + d;
                   const double g = (full ? 0.0 : G[e]) + (double)dsums[e] * inv_scale;
                   G[e] = g;
                   return g;
                 },
                 C, policy, Cm2, cnorm, DP, shift != nullptr, nullptr, shmax, dmax);
    if (lane == 0) Gc[k] = gc;
  }
  if (shift) block_max_shift(shmax, shift);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // only this thread touches NEXT / PREVOK / ITER / stats (every block reads MODE)
    const int it = ctrl[TDC_DC_ITER] + 1;
    const bool prev_ok = ctrl[TDC_DC_PREVOK] != 0;
    const double m = moved ? (double)*moved : 0.0;
    const bool next_full = (refresh > 0 && it % refresh == 0) || (prev_ok && m > theta_n);
    ctrl[TDC_DC_ITER] = it;
    ctrl[TDC_DC_NEXT] = next_full ? 1 : 0;
    ctrl[TDC_DC_PREVOK] = 1;
    if (stats) {
      stats[0] += prev_ok ? m : 0.0;
      stats[1] += prev_ok ? 1.0 : 0.0;
      stats[2] += full ? 1.0 : 0.0;
      stats[3] += 1.0;
    }
  }
}

template <typename ACC, typename CT>
int launch_finalize_delta(const void* dsums, const void* dcounts, const float* cnt_hi,
                          const float* cnt_lo, const void* moved, double* G, int K, int D, void* C,
                          int policy, float* shift, void* Cm2, float* cnorm, int Kp, int DP,
                          int* ctrl, double* stats, int refresh, double theta_n, hipStream_t s,
                          double inv_scale) {
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  const int blocks = std::max(1, std::min((rows + 3) / 4, MAX_BLOCKS));
  hipLaunchKernelGGL((finalize_delta_kernel<ACC, CT>), dim3((unsigned)blocks), dim3(256), 0, s,
                     (const ACC*)dsums, (const ACC*)dcounts, cnt_hi, cnt_lo, (const ACC*)moved, G,
                     K, D, (CT*)C, policy, shift, (__bf16*)Cm2, cnorm, Kp, DP, ctrl, stats,
                     refresh, theta_n, inv_scale);
  TDC_CHECK_LAUNCH();
  return 0;
}

template <typename ACC, typename CT>
int launch_finalize(const void* sums, const void* counts, int K, int D, void* C, int policy,
                    float* shift, void* Cm2, float* cnorm, int Kp, int DP, hipStream_t s,
                    float* drift, float* maxdrift, double inv_scale = 1.0) {
  const int rows = Cm2 ? (Kp > K ? Kp : K) : K;
  if (rows <= 0) return 0;  // an rsag rank with no centroid rows of its own: nothing to do
  const int blocks = std::min((rows + 3) / 4, MAX_BLOCKS);
  hipLaunchKernelGGL((finalize_kernel<ACC, CT>), dim3((unsigned)blocks), dim3(256), 0,
                     s, (const ACC*)sums, (const ACC*)counts, K, D, (CT*)C, policy, shift,
                     (__bf16*)Cm2, cnorm, Kp, DP, drift, maxdrift, inv_scale);
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
                 hipStream_t s, float* drift, float* maxdrift, double fixed_scale) {
  if (acc_dtype == TDC_I64) {
    if (!(fixed_scale > 0.0)) return (int)hipErrorInvalidValue;
    if (c_dtype == TDC_F32)
      return launch_finalize<long long, float>(sums, counts, K, D, C, policy, shift, Cm2, cnorm,
                                               Kp, DP, s, drift, maxdrift, 1.0 / fixed_scale);
    if (c_dtype == TDC_F64)
      return launch_finalize<long long, double>(sums, counts, K, D, C, policy, shift, Cm2, cnorm,
                                                Kp, DP, s, drift, maxdrift, 1.0 / fixed_scale);
    return (int)hipErrorInvalidValue;
  }
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

int tdc_delta_finalize(int acc_dtype, int c_dtype, const void* dsums, const void* dcounts,
                       const float* cnt_hi, const float* cnt_lo, const void* moved, double* G,
                       int K, int D, void* C, int policy, float* shift, void* Cm2, float* cnorm,
                       int Kp, int DP, int* ctrl, double* stats, int refresh, double theta_n,
                       hipStream_t s, double fixed_scale) {
  if (acc_dtype == TDC_I64 && !(fixed_scale > 0.0)) return (int)hipErrorInvalidValue;
  const double inv = acc_dtype == TDC_I64 ? 1.0 / fixed_scale : 1.0;
#define TDC_FD(A, T)                                                                        \
  return launch_finalize_delta<A, T>(dsums, dcounts, cnt_hi, cnt_lo, moved, G, K, D, C, policy, \
                                     shift, Cm2, cnorm, Kp, DP, ctrl, stats, refresh, theta_n, s, \
                                     inv)
  if (acc_dtype == TDC_I64 && c_dtype == TDC_F32) TDC_FD(long long, float);
  if (acc_dtype == TDC_I64 && c_dtype == TDC_F64) TDC_FD(long long, double);
  if (acc_dtype == TDC_F64 && c_dtype == TDC_F32) TDC_FD(double, float);
  if (acc_dtype == TDC_F32 && c_dtype == TDC_F32) TDC_FD(float, float);
  if (acc_dtype == TDC_F64 && c_dtype == TDC_F64) TDC_FD(double, double);
  if (acc_dtype == TDC_F32 && c_dtype == TDC_F64) TDC_FD(float, double);
#undef TDC_FD
  return (int)hipErrorInvalidValue;
}
