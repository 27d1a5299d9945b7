// N4/N5 for any D (fp32 / fp64): the Fuzzy C-Means tower past the register / LDS budgets
// of fcm_tower.hip (D <= 256) and fcm_mfma.hip (D <= 128).
//
// Reference per GPU per iteration (scripts/distribuitedClustering.py:108-137): [N,K,D]
// difference tiles -> d -> t = d^(-2/(m-1)) -> u = t / sum_k t -> NaN -> 0 -> W = u^m ->
// MatMul(W, X) (cuBLAS DGEMM) and Sum(W).  At large D a row no longer fits a thread's
// registers, so the tower runs over row chunks of the shard with the [rows, K] block in
// HBM (the only intermediate), three native kernels per chunk:
//
//   fcm_wide_d2   exact difference-form d2 (the reference's arithmetic, no GEMM
//                 cancellation): 128-row x 128-centroid tiles, features staged through LDS
//                 feature-major in 32-wide chunks (LDS use independent of D), MR x 8 register
//                 micro-tiles, fp32 on packed math (csrc/lloyd_simt.hip assign_exact's tile)
//   fcm_wide_rows one wave per row: sum_k t, the on-centroid count and argmin d2 (the label),
//                 then w = u^m written over d2 in place (rowinfo semantics of fcm_tower.hip:
//                 NaN -> 0 on a centroid, or the one-hot limit)
//   fcm_wide_wtx  W^T X and sum W: 64-centroid x 64-feature output tiles over a row range,
//                 32-row W / X slabs through LDS, 4 x 4 fp64 micro-tiles, one atomic per
//                 output per block
//
// The chunk is sized by the caller (ops.HipWideFCM: 2^27 elements of [rows, K]).
#include "tdc_common.h"
#include "kernels.h"
#include "fcm_math.h"

namespace tdc {
namespace {

typedef float wf32x2 __attribute__((ext_vector_type(2)));

// x - c for a centroid pair c with x broadcast from one half of a row pair (VOP3P op_sel)
__device__ __forceinline__ wf32x2 wpk_sub_lo(wf32x2 xp, wf32x2 c) {
  wf32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]"
      : "=v"(r) : "v"(xp), "v"(c));
  return r;
}
__device__ __forceinline__ wf32x2 wpk_sub_hi(wf32x2 xp, wf32x2 c) {
  wf32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]"
      : "=v"(r) : "v"(xp), "v"(c));
  return r;
}

template <typename T> struct WideCfg { static constexpr int MR = 8; };
template <> struct WideCfg<double> { static constexpr int MR = 4; };

// G[r, k] = sum_d (x_rd - c_kd)^2 for rows [0, M) (grid.x) x centroids (grid.y, 128 each)
template <typename T>
__global__ __launch_bounds__(256) void fcm_wide_d2_kernel(const T* __restrict__ X, int64_t M,
                                                          int64_t ldx, int D,
                                                          const T* __restrict__ C, int K,
                                                          T* __restrict__ G) {
  constexpr int MR = WideCfg<T>::MR;
  constexpr int R = 16 * MR, KT = 128, DC = 32;
  constexpr int PX = R + 4, PC = KT + 4;
  constexpr bool F32 = sizeof(T) == 4;
  __shared__ __attribute__((aligned(16))) T s_x[DC][PX];
  __shared__ __attribute__((aligned(16))) T s_c[DC][PC];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int k0 = (int)blockIdx.y * KT;
  typename std::conditional<F32, wf32x2[MR][4], double[MR][8]>::type acc;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < (F32 ? 4 : 8); ++j) {
      if constexpr (F32) acc[i][j] = wf32x2{0.f, 0.f};
      else acc[i][j] = 0.0;
    }
  for (int dc = 0; dc < D; dc += DC) {
    __syncthreads();
    for (int e = tid; e < R * DC; e += 256) {
      const int r = e / DC, d = e % DC;
      s_x[d][r] = (r0 + r < M && dc + d < D) ? X[(r0 + r) * ldx + dc + d] : (T)0;
    }
    for (int e = tid; e < KT * DC; e += 256) {
      const int r = e / DC, d = e % DC;
      s_c[d][r] = (k0 + r < K && dc + d < D) ? C[(int64_t)(k0 + r) * D + dc + d] : (T)0;
    }
    __syncthreads();
#pragma unroll 2
    for (int d = 0; d < DC; ++d) {
      if constexpr (F32) {
        const wf32x2* xs = reinterpret_cast<const wf32x2*>(&s_x[d][ty * MR]);
        const wf32x2* cs = reinterpret_cast<const wf32x2*>(&s_c[d][tx * 8]);
        wf32x2 xp[MR / 2], c2[4];
#pragma unroll
        for (int m = 0; m < MR / 2; ++m) xp[m] = xs[m];
#pragma unroll
        for (int j = 0; j < 4; ++j) c2[j] = cs[j];
#pragma unroll
        for (int m = 0; m < MR / 2; ++m)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const wf32x2 d0 = wpk_sub_lo(xp[m], c2[j]);
            const wf32x2 d1 = wpk_sub_hi(xp[m], c2[j]);
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
  for (int i = 0; i < MR; ++i) {
    const int64_t row = r0 + ty * MR + i;
    if (row >= M) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = k0 + tx * 8 + j;
      if (k < K) {
        T v;
        if constexpr (F32) v = acc[i][j >> 1][j & 1];
        else v = acc[i][j];
        G[row * (int64_t)K + k] = v;
      }
    }
  }
}

// one wave per row: d2 -> rowinfo (fcm_tower.hip semantics) -> label, then w in place
template <typename T, int FM>
__global__ __launch_bounds__(256) void fcm_wide_rows_kernel(T* __restrict__ G, int64_t M, int K,
                                                            T expo, T m, int nz, int write_w,
                                                            int32_t* __restrict__ labels) {
  const int lane = threadIdx.x & 63;
  const T inf = (T)INFINITY;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < M;
       row += (int64_t)gridDim.x * 4) {  // wave-uniform
    T* g = G + row * (int64_t)K;
    T S = (T)0, best = inf;
    int bk = 0, nzc = 0;
    for (int k = lane; k < K; k += 64) {  // ascending per lane: the first minimum wins
      const T d2 = g[k];
      if (d2 == (T)0) ++nzc;
      else S += fm_t<FM>(d2, expo);
      if (d2 < best) {
        best = d2;
        bk = k;
      }
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      S += __shfl_xor(S, o, 64);
      nzc += __shfl_xor(nzc, o, 64);
      const T ob = __shfl_xor(best, o, 64);
      const int ok = __shfl_xor(bk, o, 64);
      if (ob < best || (ob == best && ok < bk)) {
        best = ob;
        bk = ok;
      }
    }
    const bool on = nzc > 0;
    // > 0: 1 / sum t;  == 0: every membership 0 (NaN -> 0);  < 0: one-hot over the zeros
    const T info = on ? (nz ? (T)0 : -(T)nzc) : (T)1 / S;
    if (lane == 0) labels[row] = (on && nz) ? 0 : bk;
    if (!write_w) continue;
    for (int k = lane; k < K; k += 64) {
      const T d2 = g[k];
      T u;
      if (info > (T)0) u = fm_t<FM>(d2, expo) * info;
      else if (info == (T)0) u = (T)0;
      else u = (d2 == (T)0) ? (T)-1 / info : (T)0;
      g[k] = u > (T)0 ? fm_w<FM>(u, m) : (T)0;
    }
  }
}

// wx[k, d] += sum_r W[r, k] x[r, d]; ws[k] += sum_r W[r, k] (blocks of feature tile 0)
template <typename T>
__global__ __launch_bounds__(256) void fcm_wide_wtx_kernel(const T* __restrict__ W,
                                                           const T* __restrict__ X, int64_t M,
                                                           int64_t ldx, int D, int K, int nkt,
                                                           int ndt, int64_t rows_per_split,
                                                           double* __restrict__ wx,
                                                           double* __restrict__ ws) {
  constexpr int TK = 64, TD = 64, RB = 32;
  __shared__ T s_w[RB][TK + 1];
  __shared__ T s_x[RB][TD + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int kt = (int)(blockIdx.x % nkt);
  const int dt = (int)((blockIdx.x / nkt) % ndt);
  const int64_t split = blockIdx.x / ((int64_t)nkt * ndt);
  const int k0 = kt * TK, d0 = dt * TD;
  const int64_t a = split * rows_per_split;
  const int64_t b = min(M, a + rows_per_split);
  double out[4][4] = {};
  double wsum = 0.0;
  for (int64_t r0 = a; r0 < b; r0 += RB) {
    __syncthreads();
    for (int e = tid; e < RB * TK; e += 256) {
      const int r = e / TK, c = e % TK;
      s_w[r][c] = (r0 + r < b && k0 + c < K) ? W[(r0 + r) * (int64_t)K + k0 + c] : (T)0;
    }
    for (int e = tid; e < RB * TD; e += 256) {
      const int r = e / TD, c = e % TD;
      s_x[r][c] = (r0 + r < b && d0 + c < D) ? X[(r0 + r) * ldx + d0 + c] : (T)0;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < RB; ++r) {
      double wv[4], xv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        wv[i] = (double)s_w[r][ty + 16 * i];
        xv[i] = (double)s_x[r][tx + 16 * i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) out[i][j] = fma(wv[i], xv[j], out[i][j]);
    }
    if (dt == 0 && tid < TK) {
      for (int r = 0; r < RB; ++r) wsum += (double)s_w[r][tid];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + ty + 16 * i;
    if (k >= K) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d = d0 + tx + 16 * j;
      if (d < D && out[i][j] != 0.0) atomicAdd(&wx[(int64_t)k * D + d], out[i][j]);
    }
  }
  if (dt == 0 && tid < TK && k0 + tid < K && wsum != 0.0) atomicAdd(&ws[k0 + tid], wsum);
}

template <typename T>
int launch_wide(int pass, const void* X, int64_t M, int64_t ldx, int D, const void* C, int K,
                double m, int nz, void* G, int32_t* labels, double* wx, double* ws, int num_cus,
                hipStream_t s) {
  if (pass == 0) {
    constexpr int R = 16 * WideCfg<T>::MR;
    const dim3 grid((unsigned)((M + R - 1) / R), (unsigned)((K + 127) / 128));
    hipLaunchKernelGGL(fcm_wide_d2_kernel<T>, grid, dim3(256), 0, s, (const T*)X, M, ldx, D,
                       (const T*)C, K, (T*)G);
    TDC_CHECK_LAUNCH();
    return 0;
  }
  if (pass == 1 || pass == 3) {  // 3: labels only (label pass), G keeps d2
    const T expo = (T)(-1.0 / (m - 1.0));
    const int64_t want = (M + 3) / 4;
    const dim3 grid((unsigned)(want < (int64_t)num_cus * 16 ? want : (int64_t)num_cus * 16));
    const int ww = pass == 1;
#define TDC_WR(FMV)                                                                            \
  hipLaunchKernelGGL((fcm_wide_rows_kernel<T, FMV>), grid, dim3(256), 0, s, (T*)G, M, K, expo, \
                     (T)m, nz, ww, labels)
    switch (fcm_fm(m)) {
      case 2: TDC_WR(2); break;
      case 5: TDC_WR(5); break;
      default: TDC_WR(0);
    }
#undef TDC_WR
    TDC_CHECK_LAUNCH();
    return 0;
  }
  // pass 2: W^T X
  const int nkt = (K + 63) / 64, ndt = (D + 63) / 64;
  const int64_t tiles = (M + 31) / 32;
  int64_t splits = ((int64_t)num_cus * 4 + (int64_t)nkt * ndt - 1) / ((int64_t)nkt * ndt);
  if (splits > tiles) splits = tiles;
  if (splits < 1) splits = 1;
  const int64_t rps = ((tiles + splits - 1) / splits) * 32;
  splits = (M + rps - 1) / rps;
  hipLaunchKernelGGL(fcm_wide_wtx_kernel<T>, dim3((unsigned)(splits * nkt * ndt)), dim3(256), 0, s,
                     (const T*)G, (const T*)X, M, ldx, D, K, nkt, ndt, rps, wx, ws);
  TDC_CHECK_LAUNCH();
  return 0;
}

}  // namespace
}  // namespace tdc

using namespace tdc;

int tdc_fcm_wide(int pass, int dtype, const void* X, int64_t M, int64_t ldx, int D, const void* C,
                 int K, double m, int nan_to_zero, void* G, int32_t* labels, double* wx, double* ws,
                 int num_cus, hipStream_t s) {
  if (M <= 0 || K <= 0) return 0;
  if (D < 1 || pass < 0 || pass > 3) return (int)hipErrorInvalidValue;
  if (dtype == TDC_F64)
    return launch_wide<double>(pass, X, M, ldx, D, C, K, m, nan_to_zero, G, labels, wx, ws,
                               num_cus, s);
  if (dtype == TDC_F32)
    return launch_wide<float>(pass, X, M, ldx, D, C, K, m, nan_to_zero, G, labels, wx, ws,
                              num_cus, s);
  return (int)hipErrorInvalidValue;
}
