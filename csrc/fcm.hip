// N4/N5: fused Fuzzy C-Means tower for small K x D (the reference's FCM configs:
// D=5, K<=15, fp64; image segmentation D=3, K=3).
//
// Reference op chain per GPU per iteration (scripts/distribuitedClustering.py:108-137):
//   Tile x2, Sub, Square, Sum, Sqrt  -> d [N,K]
//   Pow(d, -2/(M-1)), Transpose, Sum, Div -> u [K,N]
//   IsNan/Select (NaN -> 0), Pow(u, M) -> W
//   MatMul(W, X) [K,D], Sum(W, 1) [K]           (+ CPU argmax label pass :141)
// Here ONE kernel reads each point once and keeps sum_i w_ki x_i and sum_i w_ki in
// VGPRs (static register tiles), then reduces wave -> LDS -> one global atomic per
// output per block.  d^(-2/(m-1)) = (d^2)^(-1/(m-1)) and u^m use transcendental-free
// forms for the common fuzzifiers (m = 2, 3, 5; integer m by binary powering) and
// exp2/log2 otherwise; the argmax label comes for free.
//
// nan_to_zero = 1 reproduces the reference guard (a point ON a centroid gets zero
// membership everywhere, :125-126); 0 gives the correct one-hot membership.
#include "tdc_common.h"
#include "kernels.h"
#include "fcm_math.h"

namespace tdc {

// labels may be null (the fit's final label pass writes them).  FM: compile-time fuzzifier
// form (fcm_math.h fm_t / fm_w: m = 2, m = 5, any m) -- a runtime switch per centroid
// inlined K copies of every form and their divergent branches into the row loop.
// LPR lanes share a row, lane part p owning clusters p*KL .. p*KL+KL-1 (see
// lloyd_small_kernel): the row normaliser, the on-centroid count and the argmax meet by
// lane swaps.
template <typename T, typename ACC, int KL, int DMAX, int FM, int LPR>
__global__ __launch_bounds__(256) void fcm_small_kernel(
    const T* __restrict__ X, int64_t N, int64_t ldx, int D, const T* __restrict__ C, int K,
    T expo, T m, int nan_to_zero, int32_t* __restrict__ labels, ACC* __restrict__ wx,
    ACC* __restrict__ ws) {
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
  T wsum[KL];
#pragma unroll
  for (int k = 0; k < KL; ++k) {
    wsum[k] = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) acc[k][d] = 0;
  }
  const T inf = (T)INFINITY;
  // grid-stride, ping-pong prefetch of the row's next row (see lloyd_small_kernel)
  auto row = [&](T (&x)[DMAX], int64_t r) {
    row_mask(D, x);
    // larger / split tiles: centroids re-read from LDS every row (see lloyd_small_kernel)
    if constexpr (KL >= 8 || LPR > 1) asm volatile("" ::: "memory");
    T t[KL];
    T tsum = 0;
    int nzero = 0;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      const int k = part * KL + j;
      t[j] = (T)0;
      if (LPR > 1 || k < K) {  // LPR == 1: wave-uniform skip
        T dd = 0;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) {
          const T df = x[d] - sc[j * DMAX + d];
          dd = fma(df, df, dd);
        }
        const T tk = fm_t<FM>(dd, expo);
        const bool on = k < K;
        t[j] = !on ? (T)0 : (dd == (T)0 ? inf : tk);
        nzero += (on && dd == (T)0);
        tsum += t[j];
      }
    }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) {
      tsum += __shfl_xor(tsum, o, 64);
      nzero += __shfl_xor(nzero, o, 64);
    }
    // memberships u_k, argmax label, weights w_k = u_k^m (all in t[]); a row past N
    // (the prefetch's clamped duplicate) gets zero weight
    const bool valid = r < N;
    int best = 0;
    T bu = (T)-1;
    const T inv = valid ? (T)1 / tsum : (T)0;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      const int k = part * KL + j;
      if (LPR > 1 || k < K) {
        T u;
        if (nzero == 0) {
          u = t[j] * inv;
        } else if (nan_to_zero || !valid) {
          u = (T)0;  // inf/inf = NaN -> 0 and finite/inf = 0  (reference guard)
        } else {
          u = (t[j] == inf) ? (T)1 / (T)nzero : (T)0;
        }
        if (k < K && u > bu) {
          bu = u;
          best = k;
        }
        t[j] = (u > (T)0) ? fm_w<FM>(u, m) : (T)0;
      }
    }
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) {  // argmax over the row's lanes, first index on ties
      const T ou = __shfl_xor(bu, o, 64);
      const int ob = __shfl_xor(best, o, 64);
      if (ou > bu || (ou == bu && ob < best)) {
        bu = ou;
        best = ob;
      }
    }
    if (labels && valid && part == 0) labels[r] = best;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      if (LPR > 1 || part * KL + j < K) {
        wsum[j] += t[j];
#pragma unroll
        for (int d = 0; d < DMAX; ++d) acc[j][d] = fma(t[j], x[d], acc[j][d]);
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

  const int lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int j = 0; j < KL; ++j) {
#pragma unroll
    for (int d = 0; d <= DMAX; ++d) {
      T v = (d < DMAX) ? acc[j][d] : wsum[j];
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
    if (v == (T)0) continue;
    if (d == DMAX) atomic_add(&ws[k], (ACC)v);
    else atomic_add(&wx[k * D + d], (ACC)v);
  }
}

template <typename T, typename ACC, int KL, int DMAX, int FM, int LPR>
int launch_fcm_fm(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K, double m,
                  int nan_to_zero, int32_t* labels, void* wx, void* ws, hipStream_t s) {
  // exactly the blocks the GPU holds at once (see launch_small, csrc/lloyd_simt.hip)
  static const int resident =
      resident_blocks(fcm_small_kernel<T, ACC, KL, DMAX, FM, LPR>, 256);
  int64_t g = (N * LPR + 255) / 256;
  if (g < 1) g = 1;
  if (g > resident) g = resident;
  hipLaunchKernelGGL((fcm_small_kernel<T, ACC, KL, DMAX, FM, LPR>), dim3((unsigned)g),
                     dim3(256), 0, s, (const T*)X, N, ldx, D, (const T*)C, K,
                     (T)(-1.0 / (m - 1.0)), (T)m, nan_to_zero, labels, (ACC*)wx, (ACC*)ws);
  TDC_CHECK_LAUNCH();
  return 0;
}

template <typename T, typename ACC, int KL, int DMAX, int LPR>
int launch_fcm(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K, double m,
               int nan_to_zero, int32_t* labels, void* wx, void* ws, hipStream_t s) {
  switch (fcm_fm(m)) {
    case 2:
      return launch_fcm_fm<T, ACC, KL, DMAX, 2, LPR>(X, N, ldx, D, C, K, m, nan_to_zero, labels,
                                                     wx, ws, s);
    case 5:
      return launch_fcm_fm<T, ACC, KL, DMAX, 5, LPR>(X, N, ldx, D, C, K, m, nan_to_zero, labels,
                                                     wx, ws, s);
    default:
      return launch_fcm_fm<T, ACC, KL, DMAX, 0, LPR>(X, N, ldx, D, C, K, m, nan_to_zero, labels,
                                                     wx, ws, s);
  }
}

template <typename T, typename ACC>
int dispatch_fcm(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K, double m,
                 int nz, int32_t* labels, void* wx, void* ws, hipStream_t s) {
#define TDC_FCM(KL, DM, LPR)                                                                 \
  if (K <= (KL) * (LPR) && D <= DM)                                                          \
    return launch_fcm<T, ACC, KL, DM, LPR>(X, N, ldx, D, C, K, m, nz, labels, wx, ws, s);
  TDC_FCM(4, 4, 1)
  if (D == 5) {  // the reference's own configs (D = 5, K in {3, 6, 9, 12, 15}): exact tiles
    TDC_FCM(4, 5, 1)
    TDC_FCM(4, 5, 2)
    TDC_FCM(6, 5, 2)
    TDC_FCM(8, 5, 2)
    TDC_FCM(8, 5, 4)  // K <= 32: four lanes per row (the tower took 8.7x longer at K=32)
    TDC_FCM(8, 5, 8)  // K <= 64: eight
  }
  TDC_FCM(4, 8, 1)
  TDC_FCM(8, 4, 1)
  TDC_FCM(8, 8, 1)
  TDC_FCM(16, 4, 1)
  if constexpr (sizeof(T) == 4) {
    TDC_FCM(16, 8, 1)
    TDC_FCM(32, 4, 1)
  }
#undef TDC_FCM
  return (int)hipErrorInvalidValue;
}

}  // namespace tdc

using namespace tdc;

int tdc_fcm_small_supported(int dtype, int K, int D) {
  if (dtype == TDC_F32) return (K <= 16 && D <= 8) || (K <= 32 && D <= 4) || (K <= 64 && D == 5);
  if (dtype == TDC_F64) return (K <= 8 && D <= 8) || (K <= 16 && D <= 5) || (K <= 64 && D == 5);
  return 0;
}

int tdc_fcm_small(int dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                  const void* C, int K, double m, int nan_to_zero, int32_t* labels, void* wx,
                  void* ws, hipStream_t s) {
  if (N <= 0) return 0;
  if (dtype == TDC_F32) {
    if (acc_dtype == TDC_F64)
      return dispatch_fcm<float, double>(X, N, ldx, D, C, K, m, nan_to_zero, labels, wx, ws, s);
    return dispatch_fcm<float, float>(X, N, ldx, D, C, K, m, nan_to_zero, labels, wx, ws, s);
  }
  if (dtype == TDC_F64)
    return dispatch_fcm<double, double>(X, N, ldx, D, C, K, m, nan_to_zero, labels, wx, ws, s);
  return (int)hipErrorInvalidValue;
}
