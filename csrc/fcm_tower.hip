// N4/N5 for any K x D (fp32 / fp64): the Fuzzy C-Means tower as two native passes.
//
// Reference per GPU per iteration (scripts/distribuitedClustering.py:108-137): the [N,K,D]
// difference tiles -> d -> t = d^(-2/(m-1)) -> u = t / sum_k t -> NaN -> 0 -> W = u^m ->
// W X (cuBLAS DGEMM) and sum(W).  fcm_small (fcm.hip) fuses all of it for tiny K x D in
// registers; past that the [K, D] partials no longer fit one thread, so the tower splits
// into two kernels, both on exact difference-form distances (the reference's arithmetic):
//
//   fcm_stats  (one sweep over all K per row)   rowinfo_i, label_i = argmax_k u_ik
//   fcm_accum  (block = 64-centroid tile x row range)
//              recompute d2 for its tile, w_ik = (t_ik * rowinfo_i)^m, and the tile's
//              sum_i w_ik x_i / sum_i w_ik in registers; one atomic per output per block
//
// rowinfo encodes the row normaliser and the on-centroid cases (d2 = 0 -> t = inf):
//   > 0  : 1 / sum_k t_ik                       u_ik = t_ik * rowinfo_i
//   == 0 : every membership 0  (nan_to_zero on a centroid: inf/inf = NaN -> 0, :125-126)
//   < 0  : -nzero, u = 1/nzero on the zero-distance centroids (the correct one-hot limit)
//
// Tiles: R rows x 64 centroids per block, 256 threads as 16 x 16 with a (R/16) x 4
// register micro-tile; X rows are staged whole in LDS (reused by the W^T X product), the
// centroids in 16-feature chunks.
#include "tdc_common.h"
#include "kernels.h"
#include "fcm_math.h"

namespace tdc {
namespace {

constexpr int KT = 64;   // centroids per tile
// feature chunk of the centroid staging: 16, or DMAX itself for the narrow tiles (a fixed
// 16 made the D <= 8 tiles do twice the work of their feature count)
template <int DMAX> struct Chunk { static constexpr int DC = DMAX < 16 ? DMAX : 16; };

template <typename T>
struct FcmParam {
  T expo, m;
  int pmode, mint, nz;
};

// FM: compile-time fuzzifier form (fcm_math.h fm_t / fm_w; 2, 5 or any m)
template <int FM, typename T>
__device__ __forceinline__ T fcm_weight(T d2, T info, const FcmParam<T>& p) {
  T u;
  if (info > (T)0) u = fm_t<FM>(d2, p.expo) * info;
  else if (info == (T)0) return (T)0;
  else u = (d2 == (T)0) ? (T)-1 / info : (T)0;
  return u > (T)0 ? fm_w<FM>(u, p.m) : (T)0;
}

// d2 of the block's R rows (s_x, staged) against centroids [k0, k0 + 64): acc[i][j] is row
// ty + 16 i, centroid k0 + tx + 16 j.  Ends with a barrier-free read of s_c, so callers
// sync before the next staging.
template <typename T, int DMAX, int R>
__device__ __forceinline__ void tile_d2(T (*s_x)[DMAX + 1], T (*s_c)[Chunk<DMAX>::DC + 1],
                                        const T* __restrict__ C, int K, int D, int k0,
                                        T (&acc)[R / 16][4]) {
  constexpr int RM = R / 16;
  constexpr int DC = Chunk<DMAX>::DC;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (T)0;
  for (int dc = 0; dc < D; dc += DC) {
    __syncthreads();
    for (int e = tid; e < KT * DC; e += 256) {
      const int kk = e / DC, d = e % DC;
      s_c[kk][d] = (k0 + kk < K && dc + d < D) ? C[(int64_t)(k0 + kk) * D + dc + d] : (T)0;
    }
    __syncthreads();
#pragma unroll 4
    for (int d = 0; d < DC; ++d) {
      if (dc + d >= DMAX) break;
      T xv[RM], cv[4];
#pragma unroll
      for (int i = 0; i < RM; ++i) xv[i] = s_x[ty + 16 * i][dc + d];
#pragma unroll
      for (int j = 0; j < 4; ++j) cv[j] = s_c[tx + 16 * j][d];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const T df = xv[i] - cv[j];
          acc[i][j] = fma(df, df, acc[i][j]);
        }
    }
  }
}

template <typename T, int DMAX, int R>
__device__ __forceinline__ void stage_x(const T* __restrict__ X, int64_t N, int64_t ldx, int D,
                                        int64_t r0, T (*s_x)[DMAX + 1]) {
  for (int e = threadIdx.x; e < R * DMAX; e += 256) {
    const int r = e / DMAX, d = e % DMAX;
    s_x[r][d] = (r0 + r < N && d < D) ? X[(r0 + r) * ldx + d] : (T)0;
  }
}

template <typename T, int DMAX, int R, int FM>
__global__ __launch_bounds__(256) void fcm_stats_kernel(const T* __restrict__ X, int64_t N,
                                                        int64_t ldx, int D,
                                                        const T* __restrict__ C, int K,
                                                        FcmParam<T> p, int32_t* __restrict__ labels,
                                                        T* __restrict__ rowinfo) {
  constexpr int RM = R / 16;
  __shared__ T s_x[R][DMAX + 1];
  __shared__ T s_c[KT][Chunk<DMAX>::DC + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const T inf = (T)INFINITY;
  for (int64_t r0 = (int64_t)blockIdx.x * R; r0 < N; r0 += (int64_t)gridDim.x * R) {
    __syncthreads();
    stage_x<T, DMAX, R>(X, N, ldx, D, r0, s_x);
    T S[RM], best[RM];
    int bk[RM], nzc[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      S[i] = (T)0;
      best[i] = inf;
      bk[i] = 0;
      nzc[i] = 0;
    }
    for (int k0 = 0; k0 < K; k0 += KT) {
      T acc[RM][4];
      tile_d2<T, DMAX, R>(s_x, s_c, C, K, D, k0, acc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + tx + 16 * j;
        if (k >= K) continue;
#pragma unroll
        for (int i = 0; i < RM; ++i) {
          const T d2 = acc[i][j];
          const T t = fm_t<FM>(d2, p.expo);
          S[i] += d2 == (T)0 ? inf : t;
          nzc[i] += d2 == (T)0;
          if (d2 < best[i]) {  // ascending k per thread: the first minimum wins
            best[i] = d2;
            bk[i] = k;
          }
        }
      }
    }
    // the 16 threads of a row group (tx) hold disjoint centroid residues
#pragma unroll
    for (int i = 0; i < RM; ++i) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        S[i] += __shfl_xor(S[i], o, 64);
        nzc[i] += __shfl_xor(nzc[i], o, 64);
        const T ob = __shfl_xor(best[i], o, 64);
        const int ok = __shfl_xor(bk[i], o, 64);
        if (ob < best[i] || (ob == best[i] && ok < bk[i])) {
          best[i] = ob;
          bk[i] = ok;
        }
      }
      const int64_t row = r0 + ty + 16 * i;
      if (tx == 0 && row < N) {
        const bool on = nzc[i] > 0;
        labels[row] = (on && p.nz) ? 0 : bk[i];
        rowinfo[row] = on ? (p.nz ? (T)0 : -(T)nzc[i]) : (T)1 / S[i];
      }
    }
  }
}

template <typename T, typename ACC, int DMAX, int R, int FM>
__global__ __launch_bounds__(256) void fcm_accum_kernel(const T* __restrict__ X, int64_t N,
                                                        int64_t ldx, int D,
                                                        const T* __restrict__ C, int K,
                                                        FcmParam<T> p,
                                                        const T* __restrict__ rowinfo,
                                                        int64_t rows_per_split, int nkt,
                                                        ACC* __restrict__ wx, ACC* __restrict__ ws) {
  constexpr int RM = R / 16;
  constexpr int QD = DMAX >= 16 ? DMAX / 16 : 1;
  __shared__ T s_x[R][DMAX + 1];
  __shared__ T s_c[KT][Chunk<DMAX>::DC + 1];
  __shared__ T s_w[R][KT + 1];
  __shared__ T s_info[R];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int k0 = (int)(blockIdx.x % nkt) * KT;
  const int64_t a = (int64_t)(blockIdx.x / nkt) * rows_per_split;
  const int64_t b = min(N, a + rows_per_split);
  // W^T X micro-tile: centroids ko..ko+3, features tx + 16 q
  const int ko = ty * 4;
  ACC out[4][QD];
  T wsp[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    wsp[c] = (T)0;
#pragma unroll
    for (int q = 0; q < QD; ++q) out[c][q] = (ACC)0;
  }
  for (int64_t r0 = a; r0 < b; r0 += R) {
    __syncthreads();
    stage_x<T, DMAX, R>(X, b, ldx, D, r0, s_x);
    if (tid < R) s_info[tid] = (r0 + tid < b) ? rowinfo[r0 + tid] : (T)0;
    T acc[RM][4];
    tile_d2<T, DMAX, R>(s_x, s_c, C, K, D, k0, acc);  // its first barrier covers s_info
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const T info = s_info[ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const T w = (k0 + tx + 16 * j < K) ? fcm_weight<FM>(acc[i][j], info, p) : (T)0;
        s_w[ty + 16 * i][tx + 16 * j] = w;
        wsp[j] += w;
      }
    }
    __syncthreads();
    for (int r = 0; r < R; ++r) {
      T wv[4], xv[QD];
#pragma unroll
      for (int c = 0; c < 4; ++c) wv[c] = s_w[r][ko + c];
#pragma unroll
      for (int q = 0; q < QD; ++q) xv[q] = s_x[r][(tx + 16 * q) < DMAX ? tx + 16 * q : 0];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int q = 0; q < QD; ++q) out[c][q] = fma((ACC)wv[c], (ACC)xv[q], out[c][q]);
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int k = k0 + ko + c;
    if (k >= K) continue;
#pragma unroll
    for (int q = 0; q < QD; ++q) {
      const int d = tx + 16 * q;
      if (d < D && out[c][q] != (ACC)0) atomic_add(&wx[(int64_t)k * D + d], out[c][q]);
    }
  }
  // column sums: reduce the 16 row groups (ty) of each centroid through LDS
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) s_w[ty][tx + 16 * j] = wsp[j];
  __syncthreads();
  if (tid < KT && k0 + tid < K) {
    ACC s = 0;
    for (int t = 0; t < 16; ++t) s += (ACC)s_w[t][tid];
    if (s != (ACC)0) atomic_add(&ws[k0 + tid], s);
  }
}

template <typename T>
FcmParam<T> make_param(double m, int nan_to_zero) {
  FcmParam<T> p;
  p.expo = (T)(-1.0 / (m - 1.0));
  p.m = (T)m;
  p.pmode = fcm_pmode(m);
  p.mint = fcm_mint(m);
  p.nz = nan_to_zero;
  return p;
}

template <typename T, int DMAX>
int launch_stats(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K, double m,
                 int nz, int32_t* labels, void* rowinfo, int num_cus, hipStream_t s) {
  constexpr int R = (sizeof(T) == 8 && DMAX > 128) ? 16 : 32;
  int64_t tiles = (N + R - 1) / R;
  int64_t blocks = tiles < (int64_t)num_cus * 8 ? tiles : (int64_t)num_cus * 8;
#define TDC_LS(FMV)                                                                            \
  hipLaunchKernelGGL((fcm_stats_kernel<T, DMAX, R, FMV>), dim3((unsigned)blocks), dim3(256), 0, s, \
                     (const T*)X, N, ldx, D, (const T*)C, K, make_param<T>(m, nz), labels,       \
                     (T*)rowinfo)
  switch (fcm_fm(m)) {
    case 2: TDC_LS(2); break;
    case 5: TDC_LS(5); break;
    default: TDC_LS(0);
  }
#undef TDC_LS
  TDC_CHECK_LAUNCH();
  return 0;
}

template <typename T, typename ACC, int DMAX>
int launch_accum(const void* X, int64_t N, int64_t ldx, int D, const void* C, int K, double m,
                 int nz, const void* rowinfo, void* wx, void* ws, int num_cus, hipStream_t s) {
  constexpr int R = (sizeof(T) == 8 && DMAX > 128) ? 16 : 32;
  const int nkt = (K + KT - 1) / KT;
  const int64_t tiles = (N + R - 1) / R;
  int64_t splits = ((int64_t)num_cus * 8 + nkt - 1) / nkt;
  if (splits > tiles) splits = tiles;
  if (splits < 1) splits = 1;
  const int64_t rps = ((tiles + splits - 1) / splits) * R;
  splits = (N + rps - 1) / rps;
#define TDC_LA(FMV)                                                                            \
  hipLaunchKernelGGL((fcm_accum_kernel<T, ACC, DMAX, R, FMV>), dim3((unsigned)(splits * nkt)),   \
                     dim3(256), 0, s, (const T*)X, N, ldx, D, (const T*)C, K,                   \
                     make_param<T>(m, nz), (const T*)rowinfo, rps, nkt, (ACC*)wx, (ACC*)ws)
  switch (fcm_fm(m)) {
    case 2: TDC_LA(2); break;
    case 5: TDC_LA(5); break;
    default: TDC_LA(0);
  }
#undef TDC_LA
  TDC_CHECK_LAUNCH();
  return 0;
}

template <typename T>
int dispatch_tower(int pass, const void* X, int64_t N, int64_t ldx, int D, const void* C, int K,
                   double m, int nz, int32_t* labels, void* rowinfo, void* wx, void* ws,
                   int num_cus, hipStream_t s) {
#define TDC_TOWER(DM)                                                                         \
  if (D <= DM) {                                                                              \
    if (pass == 0) return launch_stats<T, DM>(X, N, ldx, D, C, K, m, nz, labels, rowinfo,     \
                                              num_cus, s);                                    \
    return launch_accum<T, double, DM>(X, N, ldx, D, C, K, m, nz, rowinfo, wx, ws, num_cus, s); \
  }
  TDC_TOWER(8)
  TDC_TOWER(16)
  TDC_TOWER(32)
  TDC_TOWER(64)
  TDC_TOWER(128)
  TDC_TOWER(256)
#undef TDC_TOWER
  return (int)hipErrorInvalidValue;
}

}  // namespace
}  // namespace tdc

using namespace tdc;

int tdc_fcm_tower(int pass, int dtype, const void* X, int64_t N, int64_t ldx, int D, const void* C,
                  int K, double m, int nan_to_zero, int32_t* labels, void* rowinfo, void* wx,
                  void* ws, int num_cus, hipStream_t s) {
  if (N <= 0 || K <= 0) return 0;
  if (D < 1 || D > 256) return (int)hipErrorInvalidValue;
  if (dtype == TDC_F64)
    return dispatch_tower<double>(pass, X, N, ldx, D, C, K, m, nan_to_zero, labels, rowinfo, wx, ws,
                                  num_cus, s);
  if (dtype == TDC_F32)
    return dispatch_tower<float>(pass, X, N, ldx, D, C, K, m, nan_to_zero, labels, rowinfo, wx, ws,
                                 num_cus, s);
  return (int)hipErrorInvalidValue;
}
