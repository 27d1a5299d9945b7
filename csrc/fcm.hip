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
