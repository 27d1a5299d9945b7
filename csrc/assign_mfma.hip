// N1/N6: fused squared-L2 distance + row argmin on CDNA4 matrix cores (bf16 in, fp32 acc).
//
// Replaces the reference K-Means tower's O(N*K*D) materialisation
// (Tile x2 -> Sub -> Square -> Sum -> ArgMin, scripts/distribuitedClustering.py:221-234)
// and the CPU label pass (:255,282) with ONE kernel that never writes the [N, K]
// distance matrix:
//
//   score[k, i] = ||c_k||^2 - 2 x_i . c_k      (= d2[i,k] - ||x_i||^2)
//
// computed as an MFMA GEMM with the centroids as the A operand (pre-scaled by -2,
// exact in bf16) and the points as the B operand, accumulator INITIALISED with
// ||c_k||^2, so the epilogue needs no FMA at all.  Operands are "swapped"
// (C . X^T instead of X . C^T) so that in the 32x32 accumulator a lane owns ONE
// point (column = lane & 31) and 16 centroid rows in registers: the row argmin is
// an in-register min, not a cross-lane reduction.  The centroid index rides in
// the 5 low mantissa bits of each score (2^-18 relative perturbation, far below
// bf16 input rounding), so a whole 32x32 tile is reduced with and_or + min only.
//
// Layout / schedule (one 256-thread workgroup = 4 waves):
//   * each wave holds P x 32 points as bf16 B fragments in VGPRs for the whole
//     K loop (loaded once, straight from HBM: X is read exactly once);
//   * centroids stream through LDS in 64-row stages (double-buffered, register
//     staged: loads of stage t+1 are issued before the MFMAs of stage t and
//     written after them), XOR-swizzled so every ds_read_b128 lane group hits
//     16 distinct 16-byte slots (conflict-free);
//   * feature order inside a k-step is permuted (lane half h covers features
//     [h*DP/2, (h+1)*DP/2)); A and B use the same map, so the dot product is
//     unchanged and each lane's B loads are contiguous.
#include "tdc_common.h"
#include "kernels.h"

namespace tdc {

constexpr int BN = 64;           // centroids per LDS stage = 2 MFMA row tiles of 32
constexpr float BIG = 3.0e38f;   // pad-centroid norm (finite so bit tricks stay NaN-free)

template <int DP>
__device__ __forceinline__ int swz(int r, int c) {
  constexpr int CPR = DP / 8;              // 16-byte chunks per centroid row
  constexpr int G = CPR < 16 ? CPR : 16;   // chunks per 256-byte LDS bank row
  constexpr int RPB = 16 / G;              // rows sharing a bank row
  return c ^ ((r / RPB) & (G - 1));
}

template <int DP, int P>
__global__ __launch_bounds__(256, 2) void assign_mfma_bf16_kernel(
    const __bf16* __restrict__ X, int64_t N, int64_t ldx, const __bf16* __restrict__ Cm2,
    const float* __restrict__ cnorm, int ntiles, int32_t* __restrict__ labels,
    float* __restrict__ mind) {
  constexpr int CPR = DP / 8;
  constexpr int KS = DP / 16;
  constexpr int HALF = DP / 2;
  constexpr int STAGE = BN * DP;
  constexpr int CHUNKS = BN * CPR;
  constexpr int CPT = (CHUNKS + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 s_c[2 * STAGE];
  __shared__ __attribute__((aligned(16))) float s_n[2 * BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int r = lane & 31;
  const int h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * (4 * P * 32) + (int64_t)w * (P * 32);

  // ---- point fragments: resident in VGPRs for the whole centroid loop ----
  bf16x8 bq[P][KS];
  float xn[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    int64_t row = pbase + p * 32 + r;
    if (row >= N) row = N - 1;
    const bf16x8* src = reinterpret_cast<const bf16x8*>(X + row * ldx + h * HALF);
    float s = 0.f;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      bq[p][kk] = src[kk];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = (float)bq[p][kk][j];
        s = fmaf(f, f, s);
      }
    }
    xn[p] = s + __shfl_xor(s, 32, 64);
  }

  // ---- centroid stage staging (global -> regs -> swizzled LDS) ----
  uint4 pre[CPT];
  float npre = 0.f;
  // stage 0 straight into buffer 0
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int q = tid + i * 256;
    if (CHUNKS % 256 == 0 || q < CHUNKS) {
      const int row = q / CPR, c = q % CPR;
      *reinterpret_cast<uint4*>(s_c + row * DP + swz<DP>(row, c) * 8) =
          *reinterpret_cast<const uint4*>(Cm2 + (int64_t)row * DP + c * 8);
    }
  }
  if (tid < BN) s_n[tid] = cnorm[tid];
  __syncthreads();

  float best[P];
  int bt[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    best[p] = 3.4e38f;
    bt[p] = 0;
  }

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    // issue the next stage's loads now; they land under this stage's MFMAs
    // (the last iteration re-loads the final stage: no branch, no reader)
    const int tn = (t + 1 < ntiles) ? t + 1 : t;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int q = tid + i * 256;
      if (CHUNKS % 256 == 0 || q < CHUNKS) {
        const int row = q / CPR, c = q % CPR;
        pre[i] = *reinterpret_cast<const uint4*>(Cm2 + ((int64_t)tn * BN + row) * DP + c * 8);
      }
    }
    if (tid < BN) npre = cnorm[tn * BN + tid];

    const __bf16* cs = s_c + buf * STAGE;
    const float* ns = s_n + buf * BN;
    f32x16 acc[2][P];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      // accumulator row (centroid) of register i: (i&3) + 8*(i>>2) + 4*h
      const f32x4 n0 = *reinterpret_cast<const f32x4*>(ns + q * 32 + 4 * h);
      const f32x4 n1 = *reinterpret_cast<const f32x4*>(ns + q * 32 + 8 + 4 * h);
      const f32x4 n2 = *reinterpret_cast<const f32x4*>(ns + q * 32 + 16 + 4 * h);
      const f32x4 n3 = *reinterpret_cast<const f32x4*>(ns + q * 32 + 24 + 4 * h);
      f32x16 init;
      init[0] = n0[0]; init[1] = n0[1]; init[2] = n0[2]; init[3] = n0[3];
      init[4] = n1[0]; init[5] = n1[1]; init[6] = n1[2]; init[7] = n1[3];
      init[8] = n2[0]; init[9] = n2[1]; init[10] = n2[2]; init[11] = n2[3];
      init[12] = n3[0]; init[13] = n3[1]; init[14] = n3[2]; init[15] = n3[3];
#pragma unroll
      for (int p = 0; p < P; ++p) acc[q][p] = init;
    }
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int c = h * (CPR / 2) + kk;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(cs + r * DP + swz<DP>(r, c) * 8);
      const bf16x8 a1 =
          *reinterpret_cast<const bf16x8*>(cs + (32 + r) * DP + swz<DP>(32 + r, c) * 8);
#pragma unroll
      for (int p = 0; p < P; ++p) {
        acc[0][p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[p][kk], acc[0][p], 0, 0, 0);
        acc[1][p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq[p][kk], acc[1][p], 0, 0, 0);
      }
    }
    // epilogue: embed the (tile, register) id in the low 5 mantissa bits, then min
#pragma unroll
    for (int p = 0; p < P; ++p) {
      float m = 3.4e38f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float v =
              __uint_as_float((__float_as_uint(acc[q][p][i]) & ~31u) | (unsigned)(q * 16 + i));
          m = __builtin_fminf(m, v);
        }
      }
      if (m < best[p]) {
        best[p] = m;
        bt[p] = t;
      }
    }
    {
      __bf16* dst = s_c + (buf ^ 1) * STAGE;
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int q = tid + i * 256;
        if (CHUNKS % 256 == 0 || q < CHUNKS) {
          const int row = q / CPR, c = q % CPR;
          *reinterpret_cast<uint4*>(dst + row * DP + swz<DP>(row, c) * 8) = pre[i];
        }
      }
      if (tid < BN) s_n[(buf ^ 1) * BN + tid] = npre;
    }
    __syncthreads();
  }

  // ---- combine the two lane halves (same point, disjoint centroid rows) ----
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const float ob = __shfl_xor(best[p], 32, 64);
    const int obt = __shfl_xor(bt[p], 32, 64);
    const unsigned e0 = __float_as_uint(best[p]) & 31u, e1 = __float_as_uint(ob) & 31u;
    const int l0 = bt[p] * BN + (int)(e0 >> 4) * 32 + (int)(e0 & 3) + 8 * (int)((e0 & 15) >> 2) + 4 * h;
    const int l1 = obt * BN + (int)(e1 >> 4) * 32 + (int)(e1 & 3) + 8 * (int)((e1 & 15) >> 2) + 4 * (1 - h);
    const float v0 = __uint_as_float(__float_as_uint(best[p]) & ~31u);
    const float v1 = __uint_as_float(__float_as_uint(ob) & ~31u);
    const bool other = (v1 < v0) || (v1 == v0 && l1 < l0);
    const int64_t row = pbase + p * 32 + r;
    if (h == 0 && row < N) {
      labels[row] = other ? l1 : l0;
      if (mind) mind[row] = fmaxf((other ? v1 : v0) + xn[p], 0.f);
    }
  }
}

}  // namespace tdc

using namespace tdc;

int tdc_assign_mfma_bf16(const void* X, int64_t N, int64_t ldx, int DP, const void* Cm2,
                         const float* cnorm, int Kp, int32_t* labels, float* mind,
                         hipStream_t stream) {
  if (N <= 0) return 0;
  if (Kp % BN != 0) return (int)hipErrorInvalidValue;
  const int ntiles = Kp / BN;
  const __bf16* x = (const __bf16*)X;
  const __bf16* c = (const __bf16*)Cm2;
  switch (DP) {
#define TDC_CASE(DPV, PV)                                                                    \
  case DPV: {                                                                                \
    const int64_t per = 4 * PV * 32;                                                         \
    dim3 grid((unsigned)((N + per - 1) / per));                                              \
    hipLaunchKernelGGL((assign_mfma_bf16_kernel<DPV, PV>), grid, dim3(256), 0, stream, x, N, \
                       ldx, c, cnorm, ntiles, labels, mind);                                 \
    break;                                                                                   \
  }
    TDC_CASE(32, 4)
    TDC_CASE(64, 4)
    TDC_CASE(128, 2)
    TDC_CASE(256, 1)
#undef TDC_CASE
    default:
      return (int)hipErrorInvalidValue;
  }
  TDC_CHECK_LAUNCH();
  return 0;
}
