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
// fp64 runs the two GEMM-shaped passes on the f64 matrix cores instead
// (fcm_wide_d2_f64m_kernel: the expansion ||x||^2 + ||c||^2 - 2 x.c with a rigorous zero
// floor; fcm_wide_wtx_f64m_kernel), see below.
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

// ---------------------------------------------------------------------------------------
// fp64 on the matrix cores (v_mfma_f64_16x16x4_f64): the reference's per-GPU DGEMM
// (`MatMul(MU, X)`, scripts/distribuitedClustering.py:133) and its distances as GEMMs.
// On MI355X the f64 MFMA runs at the f64 vector FMA rate, so what it buys is the
// instruction count: one MFMA is 1024 multiply-adds (a wave-wide v_fma_f64 is 64), the
// distance becomes the GEMM expansion ||x||^2 + ||c||^2 - 2 x.c (one product per element
// and feature instead of a subtract + FMA), and the W^T X partials stay in 16 accumulator
// tiles per wave (no per-output LDS traffic).  128 x 128 output tiles, 4 waves (2 x 2) of
// 4 x 4 16x16 MFMA tiles each, 16-deep stages double-buffered through LDS.
// f64 16x16x4 lane maps (cdna_hip_programming.md §3): A[i = l&15][k = l>>4],
// B[k = l>>4][j = l&15], C/D: col = l&15, row = (l>>4) + 4 reg.
// ---------------------------------------------------------------------------------------
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int F64T = 128;  // output tile edge
// reduction depth per LDS stage: 16 in the distance pass, 32 in W^T X (half its register-
// staged stores and barriers per MFMA, 46.3 -> 43.9 ms per D=768 step; the distance pass
// went 40.9 -> 44.1 ms at 32, profiles/fcm_fp64_d768_kernel_stats_r05l.txt)
constexpr int F64S_D = 16;
constexpr int F64S_W = 32;

// G[r, k] = d2 for rows [0, M) x centroids (grid: XCD-grouped (row tile, centroid tile)).
// The norms are summed from the staged tiles (the kernel sees every feature of its rows
// and centroids).  The expansion's rounding is at most (3D + 4) 2^-53 (||x|| + ||c||)^2 for
// any summation order; a d2 below that bound is indistinguishable from 0 and stored as 0,
// so a point on a centroid keeps the difference form's exact zero (the on-centroid rule
// of fcm_wide_rows: NaN -> 0 or one-hot).
__global__ __launch_bounds__(256, 1) void fcm_wide_d2_f64m_kernel(
    const double* __restrict__ X, int64_t M, int64_t ldx, int D, const double* __restrict__ C,
    int K, int nct, double* __restrict__ G) {
  constexpr int PX = F64S_D + 2;  // 144-B rows: each 32-lane half of a b64 fragment read covers 64 banks once
  __shared__ double s_x[2][F64T * PX];
  __shared__ double s_c[2][F64T * PX];
  __shared__ double s_xn[F64T], s_cn[F64T];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  int64_t L = blockIdx.x;
  {
    const int64_t per = (int64_t)gridDim.x / 8;
    if (per * 8 == (int64_t)gridDim.x) L = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const int ct = (int)(L % nct);
  const int64_t r0 = (L / nct) * F64T;
  const int k0 = ct * F64T;
  // staging: thread t loads F64S_D / 4 features (chunk t & 3) of rows (t >> 2) and (t >> 2) + 64
  constexpr int FPT = F64S_D / 4;
  const int srow = tid >> 2, sch = (tid & 3) * FPT;
  const double* xr[2];
  const double* cr[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t rr = min(r0 + srow + 64 * j, M - 1);
    const int kk = min(k0 + srow + 64 * j, K - 1);
    xr[j] = X + rr * ldx;
    cr[j] = C + (int64_t)kk * D;
  }
  double vx[2][FPT], vc[2][FPT];
  double nx[2] = {0.0, 0.0}, nc[2] = {0.0, 0.0};
  auto load = [&](int st) __attribute__((always_inline)) {
    const int d0 = st * F64S_D + sch;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < FPT; ++e) {
        const bool ok = d0 + e < D;
        vx[j][e] = ok ? xr[j][d0 + e] : 0.0;
        vc[j][e] = ok ? cr[j][d0 + e] : 0.0;
      }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < FPT; ++e) {
        s_x[buf][(srow + 64 * j) * PX + sch + e] = vx[j][e];
        s_c[buf][(srow + 64 * j) * PX + sch + e] = vc[j][e];
        nx[j] = fma(vx[j][e], vx[j][e], nx[j]);
        nc[j] = fma(vc[j][e], vc[j][e], nc[j]);
      }
  };
  f64x4 acc[4][4];
#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int nst = (D + F64S_D - 1) / F64S_D;
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) load(st + 1);
    const double* sx = s_x[buf] + (wr * 64 + fr) * PX + fk;
    const double* sc = s_c[buf] + (wc * 64 + fr) * PX + fk;
#pragma unroll
    for (int kk = 0; kk < F64S_D / 4; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = sx[t * 16 * PX + kk * 4];
        b[t] = sc[t * 16 * PX + kk * 4];
      }
#pragma unroll
      for (int ti = 0; ti < 4; ++ti)
#pragma unroll
        for (int tj = 0; tj < 4; ++tj)
          acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ti], b[tj], acc[ti][tj], 0, 0, 0);
    }
    if (st + 1 < nst) store(buf ^ 1);  // its previous contents were read before the last barrier
    __syncthreads();
  }
  // norms: the four chunk threads of a row are lanes t, t^1, t^2, t^3 of one wave
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    nx[j] += __shfl_xor(nx[j], 1, 64);
    nx[j] += __shfl_xor(nx[j], 2, 64);
    nc[j] += __shfl_xor(nc[j], 1, 64);
    nc[j] += __shfl_xor(nc[j], 2, 64);
    if ((tid & 3) == 0) {
      s_xn[srow + 64 * j] = nx[j];
      s_cn[srow + 64 * j] = nc[j];
    }
  }
  __syncthreads();
  const double eb = (double)(3 * D + 4) * 0x1p-53;
#pragma unroll
  for (int tj = 0; tj < 4; ++tj) {
    const int kl = wc * 64 + tj * 16 + fr;
    const int k = k0 + kl;
    const double cn = s_cn[kl];
#pragma unroll
    for (int ti = 0; ti < 4; ++ti)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = wr * 64 + ti * 16 + fk + 4 * q;
        const int64_t row = r0 + rl;
        if (row < M && k < K) {
          const double xn = s_xn[rl];
          const double d2 = xn + cn - 2.0 * acc[ti][tj][q];
          const double s = sqrt(xn) + sqrt(cn);
          G[row * (int64_t)K + k] = d2 <= eb * s * s ? 0.0 : d2;
        }
      }
  }
}

// wx[k, d] += sum_r W[r, k] x[r, d] over one split's rows (128 x 128 output tile per block);
// ws[k] += sum_r W[r, k] (feature-tile-0 blocks); one fp64 atomic per output per block
// WT >= 0: G holds t (fcm_f64_tstats_kernel) and w = fm_w<WT>(t * rowinfo) is formed while
// staging (rowinfo < 0: one-hot over the row's t = inf, == 0: all zero); WT < 0: G holds w
template <int WT, int NW = 4>
__global__ __launch_bounds__(NW * 64, 1) void fcm_wide_wtx_f64m_kernel(
    const double* __restrict__ W, const double* __restrict__ X, int64_t M, int64_t ldx, int D,
    int K, int nkt, int ndt, int64_t rows_per_split, double* __restrict__ wx,
    double* __restrict__ ws, const double* __restrict__ rowinfo = nullptr, double m = 2.0) {
  // NW = 4: 2 x 2 waves of 64 x 64 outputs (acc[4][4]: one wave per SIMD); NW = 8: 4 x 2
  // waves of 32 x 64 (acc[2][4]: two waves per SIMD, one hides the other's staging / barrier)
  constexpr int NT = NW * 64;
  constexpr int WRN = NW / 2, TI = F64T / WRN / 16;
  constexpr int PW = F64T + 16;  // 1152-B rows (= 128 mod 256): the two 16-lane groups of a
                                 // b64 fragment read fall on disjoint bank halves
  __shared__ double s_w[2][F64S_W * PW];
  __shared__ double s_x[2][F64S_W * PW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  // XCD-aware order: the nkt x ndt tile blocks of one row split are consecutive on one XCD,
  // so its W and X rows come from HBM once into that XCD's L2
  int64_t L = blockIdx.x;
  {
    const int64_t per = (int64_t)gridDim.x / 8;
    if (per * 8 == (int64_t)gridDim.x) L = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  const int kt = (int)(L % nkt);
  const int dt = (int)((L / nkt) % ndt);
  const int64_t split = L / ((int64_t)nkt * ndt);
  const int k0 = kt * F64T, d0 = dt * F64T;
  const int64_t a = split * rows_per_split;
  const int64_t b = min(M, a + rows_per_split);
  // staging: thread t loads 8 consecutive columns (t & 15) * 8 of stage rows (t >> 4) + j NT/16
  constexpr int RPT = F64S_W * 16 / NT;
  const int srow = tid >> 4, scol = (tid & 15) * 8;
  double vw[RPT][8], vx[RPT][8], vi[RPT];
  // loads only (issued at a stage's start, consumed by store() after its MFMAs, so their
  // latency hides under them); the t -> w transform runs in store()
  auto load = [&](int64_t rs) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int64_t r = rs + srow + (NT / 16) * j;
      const bool rok = r < b;
      if constexpr (WT >= 0) vi[j] = rok ? rowinfo[r] : 0.0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + scol + e, d = d0 + scol + e;
        vw[j][e] = (rok && k < K) ? W[r * (int64_t)K + k] : 0.0;
        vx[j][e] = (rok && d < D) ? X[r * ldx + d] : 0.0;
      }
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < RPT; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        double v = vw[j][e];
        if constexpr (WT >= 0) {
          const double info = vi[j];
          const double u = info > 0.0 ? v * info : (info < 0.0 && v == (double)INFINITY ? -1.0 / info : 0.0);
          v = u > 0.0 ? fm_w<WT>(u, m) : 0.0;
        }
        s_w[buf][(srow + (NT / 16) * j) * PW + scol + e] = v;
        s_x[buf][(srow + (NT / 16) * j) * PW + scol + e] = vx[j][e];
      }
  };
  f64x4 acc[TI][4];
#pragma unroll
  for (int ti = 0; ti < TI; ++ti)
#pragma unroll
    for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = f64x4{0.0, 0.0, 0.0, 0.0};
  double wsum = 0.0;
  if (a < b) {
    load(a);
    store(0);
  }
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  int buf = 0;
  for (int64_t rs = a; rs < b; rs += F64S_W) {
    const bool more = rs + F64S_W < b;
    if (more) load(rs + F64S_W);
    const double* sw = s_w[buf] + fk * PW + wr * (TI * 16) + fr;
    const double* sx = s_x[buf] + fk * PW + wc * 64 + fr;
#pragma unroll
    for (int kk = 0; kk < F64S_W / 4; ++kk) {
      double av[TI], bv[4];
#pragma unroll
      for (int t = 0; t < TI; ++t) av[t] = sw[kk * 4 * PW + t * 16];
#pragma unroll
      for (int t = 0; t < 4; ++t) bv[t] = sx[kk * 4 * PW + t * 16];
#pragma unroll
      for (int ti = 0; ti < TI; ++ti)
#pragma unroll
        for (int tj = 0; tj < 4; ++tj)
          acc[ti][tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ti], bv[tj], acc[ti][tj], 0, 0, 0);
    }
    // sum_r W[r, k]: stage s of the split goes to feature tile s % ndt, all waves (thread t:
    // column t & 127, rows of group t >> 7) -- one tile's waves alone carried it
    if ((int)(((rs - a) / F64S_W) % ndt) == dt) {
      constexpr int RG = F64S_W / (NT / 128);
#pragma unroll
      for (int r = 0; r < RG; ++r) wsum += s_w[buf][((tid >> 7) * RG + r) * PW + (tid & 127)];
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int ti = 0; ti < TI; ++ti)
#pragma unroll
    for (int tj = 0; tj < 4; ++tj) {
      const int d = d0 + wc * 64 + tj * 16 + fr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = k0 + wr * (TI * 16) + ti * 16 + fk + 4 * q;
        const double v = acc[ti][tj][q];
        if (k < K && d < D && v != 0.0) atomicAdd(&wx[(int64_t)k * D + d], v);
      }
    }
  if (k0 + (tid & 127) < K && wsum != 0.0) atomicAdd(&ws[k0 + (tid & 127)], wsum);
}

// ---------------------------------------------------------------------------------------
// fp64 FCM with the row statistics fused into the distance GEMM (round 6): the separate
// row pass (fcm_wide_rows: read G, write w in place -- 2 x 8 B per element, 39 ms of a
// 206 ms step at N=10M, D=128, K=1024) is gone.
//   fcm_f64_tstats  one block = 128 rows x ALL centroid tiles (looped): per tile the f64-MFMA
//                   distance expansion, then t = d2^(-1/(m-1)) (+inf on a centroid) written
//                   to G, and the row's sum_k t, zero count and (d2, k) minimum carried
//                   across tiles (16-lane DPP butterflies, one owner lane per row); at the
//                   end rowinfo (fcm_wide_rows semantics) and the label
//   fcm_wide_wtx_f64m_kernel<FM>  W^T X with w = (t * rowinfo)^m formed while staging
// 8 waves x (16 rows x 128 centroids, acc[8]): a row's 128 tile columns live in one wave, and
// the block fits two waves per SIMD; lane (fr, fk) holds rows fk + 4 q, columns 16 tj + fr.
// ---------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
// one butterfly step over the 16 lanes of a DPP row: sum s, count z, min (d, k) by (d, k)
template <int CTRL>
__device__ __forceinline__ void row_step(double& s, int& z, double& d, int& k) {
  s += dpp_f64<CTRL>(s);
  z += dpp_i32<CTRL>(z);
  const double od = dpp_f64<CTRL>(d);
  const int ok = dpp_i32<CTRL>(k);
  const bool take = od < d || (od == d && ok < k);
  d = take ? od : d;
  k = take ? ok : k;
}

template <int FM>
__global__ __launch_bounds__(512, 1) void fcm_f64_tstats_kernel(
    const double* __restrict__ X, int64_t M, int64_t ldx, int D, const double* __restrict__ C,
    int K, int nct, double expo, int nz, double* __restrict__ G, double* __restrict__ rowinfo,
    int32_t* __restrict__ labels) {
  constexpr int PX = F64S_D + 2;
  __shared__ double s_x[2][F64T * PX];
  __shared__ double s_c[2][F64T * PX];
  __shared__ double s_xn[F64T], s_cn[F64T], s_cs[F64T];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;  // 8 waves x 16 rows
  const int64_t r0 = (int64_t)blockIdx.x * F64T;
  constexpr int FPT = F64S_D / 4;
  const int srow = tid >> 2, sch = (tid & 3) * FPT;  // staging: one X row + one C row
  const double* xr = X + min(r0 + srow, M - 1) * ldx;
  const int fr = lane & 15, fk = lane >> 4;
  const int nst = (D + F64S_D - 1) / F64S_D;
  const double eb = (double)(3 * D + 4) * 0x1p-53;
  // per-row state, owner lane fr = q of row 16 w + fk + 4 q (fr < 4)
  double st_s = 0.0, st_d = INFINITY;
  int st_z = 0, st_k = 0;
  double vx[FPT], vc[FPT];
  auto load_c = [&](const double* cr, int st) __attribute__((always_inline)) {
    const int d0 = st * F64S_D + sch;
#pragma unroll
    for (int e = 0; e < FPT; ++e) {
      const bool ok = d0 + e < D;
      vx[e] = ok ? xr[d0 + e] : 0.0;
      vc[e] = ok ? cr[d0 + e] : 0.0;
    }
  };
  load_c(C + (int64_t)min(srow, K - 1) * D, 0);
  for (int ct = 0; ct < nct; ++ct) {
    const int k0 = ct * F64T;
    const double* cr = C + (int64_t)min(k0 + srow, K - 1) * D;
    // the next tile's first stage is loaded during this tile's last one, so its latency
    // hides under those MFMAs and this tile's epilogue
    const double* crn = C + (int64_t)min(k0 + F64T + srow, K - 1) * D;
    double nx = 0.0, nc = 0.0;
    auto load = [&](int st) __attribute__((always_inline)) { load_c(cr, st); };
    auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
      for (int e = 0; e < FPT; ++e) {
        s_x[buf][srow * PX + sch + e] = vx[e];
        s_c[buf][srow * PX + sch + e] = vc[e];
        nx = fma(vx[e], vx[e], nx);
        nc = fma(vc[e], vc[e], nc);
      }
    };
    f64x4 acc[8];
#pragma unroll
    for (int tj = 0; tj < 8; ++tj) acc[tj] = f64x4{0.0, 0.0, 0.0, 0.0};
    store(0);  // stage 0 of this tile (loaded before the loop / during the previous tile)
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      const int buf = st & 1;
      if (st + 1 < nst) load(st + 1);
      else if (ct + 1 < nct) load_c(crn, 0);
      const double* sx = s_x[buf] + (w * 16 + fr) * PX + fk;
      const double* sc = s_c[buf] + fr * PX + fk;
#pragma unroll
      for (int kk = 0; kk < F64S_D / 4; ++kk) {
        const double a = sx[kk * 4];
        double b[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) b[t] = sc[t * 16 * PX + kk * 4];
#pragma unroll
        for (int tj = 0; tj < 8; ++tj)
          acc[tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[tj], acc[tj], 0, 0, 0);
      }
      if (st + 1 < nst) store(buf ^ 1);
      __syncthreads();
    }
    // norms: the four chunk threads of a row are lanes t, t^1, t^2, t^3 of one wave
    nx += __shfl_xor(nx, 1, 64);
    nx += __shfl_xor(nx, 2, 64);
    nc += __shfl_xor(nc, 1, 64);
    nc += __shfl_xor(nc, 2, 64);
    if ((tid & 3) == 0) {
      if (ct == 0) s_xn[srow] = nx;
      s_cn[srow] = nc;
      s_cs[srow] = sqrt(nc);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rl = w * 16 + fk + 4 * q;
      const int64_t row = r0 + rl;
      const double xn = s_xn[rl], xs = sqrt(xn);
      double s = 0.0, bd = INFINITY;
      int z = 0, bk = 0;
#pragma unroll
      for (int tj = 0; tj < 8; ++tj) {
        const int kl = tj * 16 + fr, k = k0 + kl;
        const double d2 = xn + s_cn[kl] - 2.0 * acc[tj][q];
        const double sb = xs + s_cs[kl];
        const bool zero = d2 <= eb * sb * sb;
        const double t = zero ? (double)INFINITY : fm_t<FM>(d2, expo);
        if (k < K) {
          if (row < M) G[row * (int64_t)K + k] = t;
          const double dd = zero ? 0.0 : d2;
          z += zero ? 1 : 0;
          s += zero ? 0.0 : t;
          if (dd < bd) {  // ascending k per lane: the first minimum wins
            bd = dd;
            bk = k;
          }
        }
      }
      row_step<0xB1>(s, z, bd, bk);   // quad_perm [1,0,3,2]: lane ^ 1
      row_step<0x4E>(s, z, bd, bk);   // quad_perm [2,3,0,1]: lane ^ 2
      row_step<0x141>(s, z, bd, bk);  // row_half_mirror: quads 0 <-> 1, 2 <-> 3
      row_step<0x140>(s, z, bd, bk);  // row_mirror: halves of the 16-lane row
      if (fr == q) {
        st_s += s;
        st_z += z;
        if (bd < st_d || (bd == st_d && bk < st_k)) {
          st_d = bd;
          st_k = bk;
        }
      }
    }
    __syncthreads();  // s_cn / the stage buffers are rewritten by the next tile
  }
  if (fr < 4) {
    const int64_t row = r0 + w * 16 + fk + 4 * fr;
    if (row < M) {
      const bool on = st_z > 0;
      // > 0: 1 / sum t;  == 0: every membership 0 (NaN -> 0);  < 0: one-hot over the zeros
      rowinfo[row] = on ? (nz ? 0.0 : -(double)st_z) : 1.0 / st_s;
      labels[row] = (on && nz) ? 0 : st_k;
    }
  }
}

// row splits of the fp64 W^T X pass: one 256-thread block per CU at a time, so the grid
// (splits x tiles blocks) should fill whole rounds of num_cus blocks -- 11 splits x 48
// tiles at D = 768, K = 1024 ran 2.06 rounds, i.e. three; pick the split count in
// [base, 4 base] with the least rounds x rows per block
inline int64_t wtx_f64_splits(int64_t stages, int64_t tiles, int num_cus) {
  int64_t base = ((int64_t)num_cus * 2 + tiles - 1) / tiles;
  if (base < 1) base = 1;
  int64_t best = base;
  double best_cost = 1e300;
  for (int64_t sp = base; sp <= 4 * base && sp <= stages; ++sp) {
    const int64_t rounds = (sp * tiles + num_cus - 1) / num_cus;
    const double cost = (double)rounds * (double)((stages + sp - 1) / sp) * (1.0 + 1e-3 * sp);
    if (cost < best_cost) {
      best_cost = cost;
      best = sp;
    }
  }
  return best < stages ? best : (stages > 0 ? stages : 1);
}

template <typename T>
int launch_wide(int pass, const void* X, int64_t M, int64_t ldx, int D, const void* C, int K,
                double m, int nz, void* G, int32_t* labels, double* wx, double* ws, int num_cus,
                hipStream_t s) {
  if constexpr (sizeof(T) == 8) {
    // fp64: both GEMM-shaped passes on the f64 matrix cores
    if (pass == 0) {
      const int nct = (K + F64T - 1) / F64T;
      const int64_t nb = ((M + F64T - 1) / F64T) * nct;
      hipLaunchKernelGGL(fcm_wide_d2_f64m_kernel, dim3((unsigned)nb), dim3(256), 0, s,
                         (const double*)X, M, ldx, D, (const double*)C, K, nct, (double*)G);
      TDC_CHECK_LAUNCH();
      return 0;
    }
    if (pass == 2) {
      const int nkt = (K + F64T - 1) / F64T, ndt = (D + F64T - 1) / F64T;
      const int64_t stages = (M + F64S_W - 1) / F64S_W;
      int64_t splits = wtx_f64_splits(stages, (int64_t)nkt * ndt, num_cus);
      const int64_t rps = ((stages + splits - 1) / splits) * F64S_W;
      splits = (M + rps - 1) / rps;
      hipLaunchKernelGGL(fcm_wide_wtx_f64m_kernel<-1>, dim3((unsigned)(splits * nkt * ndt)), dim3(256),
                         0, s, (const double*)G, (const double*)X, M, ldx, D, K, nkt, ndt, rps,
                         wx, ws);
      TDC_CHECK_LAUNCH();
      return 0;
    }
  }
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

int launch_f64t(int pass, const double* X, int64_t M, int64_t ldx, int D, const double* C, int K,
                double m, int nz, double* G, double* rowinfo, int32_t* labels, double* wx,
                double* ws, int num_cus, hipStream_t s) {
  const int fm = fcm_fm(m);
  if (pass == 0) {
    const int nct = (K + F64T - 1) / F64T;
    const dim3 grid((unsigned)((M + F64T - 1) / F64T));
    const double expo = -1.0 / (m - 1.0);
#define TDC_TS(FMV)                                                                             \
  hipLaunchKernelGGL((fcm_f64_tstats_kernel<FMV>), grid, dim3(512), 0, s, X, M, ldx, D, C, K, nct, \
                     expo, nz, G, rowinfo, labels)
    switch (fm) {
      case 2: TDC_TS(2); break;
      case 5: TDC_TS(5); break;
      default: TDC_TS(0);
    }
#undef TDC_TS
    TDC_CHECK_LAUNCH();
    return 0;
  }
  const int nkt = (K + F64T - 1) / F64T, ndt = (D + F64T - 1) / F64T;
  const int64_t stages = (M + F64S_W - 1) / F64S_W;
  int64_t splits = wtx_f64_splits(stages, (int64_t)nkt * ndt, num_cus);
  const int64_t rps = ((stages + splits - 1) / splits) * F64S_W;
  splits = (M + rps - 1) / rps;
#define TDC_WT(FMV)                                                                               \
  hipLaunchKernelGGL((fcm_wide_wtx_f64m_kernel<FMV, 8>), dim3((unsigned)(splits * nkt * ndt)), dim3(512), \
                     0, s, G, X, M, ldx, D, K, nkt, ndt, rps, wx, ws, rowinfo, m)
  switch (fm) {
    case 2: TDC_WT(2); break;
    case 5: TDC_WT(5); break;
    default: TDC_WT(0);
  }
#undef TDC_WT
  TDC_CHECK_LAUNCH();
  return 0;
}

}  // namespace
}  // namespace tdc

using namespace tdc;

int tdc_fcm_f64t(int pass, const double* X, int64_t M, int64_t ldx, int D, const double* C, int K,
                 double m, int nan_to_zero, double* G, double* rowinfo, int32_t* labels, double* wx,
                 double* ws, int num_cus, hipStream_t s) {
  if (M <= 0 || K <= 0) return 0;
  if (D < 1 || pass < 0 || pass > 1 || m <= 1.0) return (int)hipErrorInvalidValue;
  return launch_f64t(pass, X, M, ldx, D, C, K, m, nan_to_zero, G, rowinfo, labels, wx, ws, num_cus,
                     s);
}

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
