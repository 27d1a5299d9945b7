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

// labels may be null (the fit's final label pass writes them).
template <typename T, typename ACC, int KMAX, int DMAX>
__global__ __launch_bounds__(256) void fcm_small_kernel(
    const T* __restrict__ X, int64_t N, int64_t ldx, int D, const T* __restrict__ C, int K,
    T expo, T m, int pmode, int mint, int nan_to_zero, int32_t* __restrict__ labels,
    ACC* __restrict__ wx, ACC* __restrict__ ws) {
  __shared__ T s_c[KMAX * DMAX];
  __shared__ T s_red[4][KMAX * (DMAX + 1)];
  const int tid = threadIdx.x;
  for (int i = tid; i < KMAX * DMAX; i += 256) {
    const int k = i / DMAX, d = i % DMAX;
    s_c[i] = (k < K && d < D) ? C[k * D + d] : (T)0;
  }
  __syncthreads();

  T acc[KMAX][DMAX];
  T wsum[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    wsum[k] = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) acc[k][d] = 0;
  }
  const T inf = (T)INFINITY;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + tid; i < N; i += stride) {
    T x[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) x[d] = (d < D) ? X[i * ldx + d] : (T)0;
    T t[KMAX];
    T tsum = 0;
    int nzero = 0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      T dd = 0;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const T df = x[d] - s_c[k * DMAX + d];
        dd = fma(df, df, dd);
      }
      const bool on = (k < K);
      t[k] = !on ? (T)0 : (dd == (T)0 ? inf : fcm_t(dd, expo, pmode));
      nzero += (on && dd == (T)0);
      tsum += t[k];
    }
    // memberships u_k, argmax label, weights w_k = u_k^m (all in t[])
    int best = 0;
    T bu = (T)-1;
    const T inv = (T)1 / tsum;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      T u;
      if (nzero == 0) {
        u = t[k] * inv;
      } else if (nan_to_zero) {
        u = (T)0;  // inf/inf = NaN -> 0 and finite/inf = 0  (reference guard)
      } else {
        u = (t[k] == inf) ? (T)1 / (T)nzero : (T)0;
      }
      if (k < K && u > bu) {
        bu = u;
        best = k;
      }
      t[k] = (u > (T)0) ? fcm_w(u, m, mint) : (T)0;
    }
    if (labels) labels[i] = best;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      wsum[k] += t[k];
#pragma unroll
      for (int d = 0; d < DMAX; ++d) acc[k][d] = fma(t[k], x[d], acc[k][d]);
    }
  }

  const int lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
#pragma unroll
    for (int d = 0; d <= DMAX; ++d) {
      T v = (d < DMAX) ? acc[k][d] : wsum[k];
      v = wave_sum(v);
      if (lane == 0) s_red[w][k * (DMAX + 1) + d] = v;
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

template <typename T, typename ACC, int KMAX, int DMAX>
int launch_fcm(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K, double m,
               int nan_to_zero, int32_t* labels, void* wx, void* ws, hipStream_t s) {
  // exactly the blocks the GPU holds at once (see launch_small, csrc/lloyd_simt.hip)
  static const int resident = resident_blocks(fcm_small_kernel<T, ACC, KMAX, DMAX>, 256);
  int64_t g = (N + 255) / 256;
  if (g < 1) g = 1;
  if (g > resident) g = resident;
  const T expo = (T)(-1.0 / (m - 1.0));
  const int pmode = m == 2.0 ? 1 : (m == 3.0 ? 2 : (m == 5.0 ? 3 : 0));
  const int mint = (m == (double)(int)m && m >= 1.0 && m <= 16.0) ? (int)m : 0;
  hipLaunchKernelGGL((fcm_small_kernel<T, ACC, KMAX, DMAX>), dim3((unsigned)g), dim3(256), 0, s,
                     (const T*)X, N, ldx, D, (const T*)C, K, expo, (T)m, pmode, mint, nan_to_zero,
                     labels, (ACC*)wx, (ACC*)ws);
  TDC_CHECK_LAUNCH();
  return 0;
}

template <typename T, typename ACC>
int dispatch_fcm(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K, double m,
                 int nz, int32_t* labels, void* wx, void* ws, hipStream_t s) {
#define TDC_FCM(KM, DM)                                                                    \
  if (K <= KM && D <= DM)                                                                  \
    return launch_fcm<T, ACC, KM, DM>(X, N, ldx, D, C, K, m, nz, labels, wx, ws, s);
  TDC_FCM(4, 4)
  TDC_FCM(4, 6)  // the reference's own configs: D = 5, K <= 4
  TDC_FCM(4, 8)
  TDC_FCM(8, 4)
  TDC_FCM(8, 8)
  TDC_FCM(16, 4)
  if constexpr (sizeof(T) == 4) {
    TDC_FCM(16, 8)
    TDC_FCM(32, 4)
  } else {
    TDC_FCM(16, 5)
  }
#undef TDC_FCM
  return (int)hipErrorInvalidValue;
}

}  // namespace tdc

using namespace tdc;

int tdc_fcm_small_supported(int dtype, int K, int D) {
  if (dtype == TDC_F32) return (K <= 16 && D <= 8) || (K <= 32 && D <= 4);
  if (dtype == TDC_F64) return (K <= 8 && D <= 8) || (K <= 16 && D <= 5);
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

// ------------------------------------------------------------------------------------
// N4 for large K*D (HipGemmFCM, ops/__init__.py): the GEMM terms run on hipBLASLt and this
// kernel is the whole elementwise middle of the FCM tower (`distribuitedClustering.py:
// 117-148`), one wave per row, in place on G = ||c||^2 - 2 x.c [rows, K] (fp32):
//   d2 = max(G + ||x||^2, 0);  t = d2^(-1/(m-1)) (= d^(-2/(m-1)));  u = t / sum_k t
//   nan_to_zero: NaN (a row on a centroid: inf/inf) -> 0, else the one-hot of the zero
//   distances;  G <- w = u^m;  labels = argmax_k u (first index on ties).
// Two sweeps over the row (t is stored in G by the first); the row stays in L2.
// ------------------------------------------------------------------------------------
namespace tdc {

// NV > 0: the row is held in registers (NV values per lane, K <= 64*NV): one read and one
// write of G.  NV == 0: any K, t is stored in G between the two sweeps.
// cc (nullable): ||c||^2 added here (G then holds only -2 x.c, so the GEMM needs no
// broadcast bias copy).  colsum (nullable, zeroed by the caller): += sum over rows of w
// (the FCM denominators); a lane owns columns lane + 64v across all the rows its wave
// visits, so NV > 0 flushes one atomic per column per wave.
template <int NV>
__global__ __launch_bounds__(256) void fcm_rows_kernel(float* __restrict__ G, int64_t rows, int K,
                                                       const float* __restrict__ xx,
                                                       const float* __restrict__ cc, float m,
                                                       int nan_to_zero,
                                                       int32_t* __restrict__ labels,
                                                       float* __restrict__ colsum) {
  const int lane = threadIdx.x & 63;
  const float e = -1.0f / (m - 1.0f);
  constexpr int NR = NV > 0 ? NV : 1;
  float ccr[NR], csum[NR];
#pragma unroll
  for (int v = 0; v < NR; ++v) {
    const int k = v * 64 + lane;
    ccr[v] = (NV > 0 && cc && k < K) ? cc[k] : 0.f;
    csum[v] = 0.f;
  }
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows;
       row += (int64_t)gridDim.x * 4) {  // wave-uniform
    float* g = G + row * (int64_t)K;
    const float x2 = xx[row];
    float sum = 0.f, best = INFINITY;
    int bk = 0, nzero = 0;
    float tr[NR];
    auto visit = [&](int k, float gv) __attribute__((always_inline)) {
      const float d2 = fmaxf(gv + x2, 0.f);
      const float t = exp2f(log2f(d2) * e);  // d2 = 0 -> +inf
      sum += t;
      nzero += d2 == 0.f;
      if (d2 < best) { best = d2; bk = k; }  // lane-local: ascending k, first wins
      return t;
    };
    if constexpr (NV > 0) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int k = v * 64 + lane;
        tr[v] = k < K ? g[k] : 0.f;
      }
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int k = v * 64 + lane;
        if (k < K) tr[v] = visit(k, tr[v] + ccr[v]);
      }
    } else {
      for (int k = lane; k < K; k += 64) g[k] = visit(k, g[k] + (cc ? cc[k] : 0.f));
    }
    sum = wave_sum(sum);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int ok = __shfl_xor(bk, o, 64);
      if (ob < best || (ob == best && ok < bk)) { best = ob; bk = ok; }
      nzero += __shfl_xor(nzero, o, 64);
    }
    // on-centroid row (sum = inf): u = inf/inf = NaN on the zero distances, 0 elsewhere
    const bool oncen = nzero > 0;
    const float inv = 1.0f / sum;
    const float onehot = oncen ? 1.0f / (float)nzero : 0.f;
    auto weight = [&](float t) __attribute__((always_inline)) {
      float u;
      if (!oncen) u = t * inv;
      else if (nan_to_zero) u = 0.f;
      else u = isinf(t) ? onehot : 0.f;
      return u > 0.f ? exp2f(log2f(u) * m) : 0.f;
    };
    if constexpr (NV > 0) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int k = v * 64 + lane;
        if (k < K) {
          const float w = weight(tr[v]);
          g[k] = w;
          csum[v] += w;
        }
      }
    } else {
      for (int k = lane; k < K; k += 64) {
        const float w = weight(g[k]);
        g[k] = w;
        if (colsum && w != 0.f) atomicAdd(colsum + k, w);
      }
    }
    // argmax u = argmin d2; an all-zero row (nan_to_zero on a centroid) -> index 0
    if (lane == 0) labels[row] = (oncen && nan_to_zero) ? 0 : bk;
  }
  if constexpr (NV > 0) {
    if (colsum) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int k = v * 64 + lane;
        if (k < K && csum[v] != 0.f) atomicAdd(colsum + k, csum[v]);
      }
    }
  }
}

}  // namespace tdc

int tdc_fcm_rows(float* G, int64_t rows, int K, const float* xx, const float* cc, float m,
                 int nan_to_zero, int32_t* labels, float* colsum, hipStream_t s) {
  if (rows <= 0) return 0;
  // persistent waves, exactly the blocks resident at once (every block the same row
  // count, so a larger grid would leave a partial second round); the column-sum flush is
  // one atomic per column per block
  const int64_t want = (rows + 3) / 4;
#define TDC_FR(NVV)                                                                           \
  do {                                                                                        \
    static const int res = resident_blocks(tdc::fcm_rows_kernel<NVV>, 256);                   \
    const dim3 grid((unsigned)(want < res ? want : res));                                     \
    hipLaunchKernelGGL(tdc::fcm_rows_kernel<NVV>, grid, dim3(256), 0, s, G, rows, K, xx, cc,  \
                       m, nan_to_zero, labels, colsum);                                       \
  } while (0)
  if (K <= 256) TDC_FR(4);
  else if (K <= 1024) TDC_FR(16);
  else if (K <= 2048) TDC_FR(32);
  else TDC_FR(0);
#undef TDC_FR
  TDC_CHECK_LAUNCH();
  return 0;
}
