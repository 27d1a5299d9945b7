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
#include <stdlib.h>

#include "assign_mfma_impl.h"
#include "kernels.h"

using namespace tdc;

int tdc_assign_mfma_bf16(const void* X, int64_t N, int64_t ldx, int DP, const void* Cm2,
                         const float* cnorm, int Kp, int32_t* labels, float* mind,
                         hipStream_t stream) {
  if (N <= 0) return 0;
  if (Kp % BN != 0) return (int)hipErrorInvalidValue;
  const int ntiles = Kp / BN;
  const __bf16* x = (const __bf16*)X;
  const __bf16* c = (const __bf16*)Cm2;
  // LDS-DMA ring, 4 waves x P x 16 points per workgroup (ring3: 16x16x32 MFMA, tag-in-
  // mantissa argmin).  The schedule variants measured against it (ring / ring2 schedules,
  // ablations, WAVES/P/QT/NST sweeps: docs/PERF_NOTES.md) are instantiated by the harnesses
  // in tools/, not selectable here.
  if (DP == 64 || DP == 128 || DP == 256) {
    const int64_t per = 4 * 4 * 16;
    dim3 grid((unsigned)((N + per - 1) / per));
    if (DP == 64) {
      // D=64: P=8 point tiles per wave (the register footprint of D=128's P=4) and 128-row
      // stages: 1.74 -> 1.60 ms at N=4M, K=4096 (TDC_RING3_D64 sweep)
      const int64_t per8 = 4 * 8 * 16;
      const dim3 grid8((unsigned)((N + per8 - 1) / per8));
      if (Kp % 128 == 0)
        hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<64, 8, 3, 4, 8>), grid8, dim3(256), 0,
                           stream, x, N, ldx, c, cnorm, Kp / 128, labels, mind);
      else
        hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<64, 8, 3, 4, 4>), grid8, dim3(256), 0,
                           stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind);
    } else if (DP == 128 && N >= (1 << 20)) {
      // shards from 1M rows: P=8 point tiles per wave (512 points per workgroup, two waves
      // per SIMD) halve the ring refill per point; NST=2.  1.93-1.95 -> 1.91 ms at the
      // headline shape (profiles/assign_ring3_ablation_r02.txt).  With the builtin LDS-DMA
      // (256 VGPRs) P=4 had won below ~4M rows (profiles/ring3_p4_vs_p8_*_r03.txt); with
      // the saddr-form DMA (244 VGPRs) P=8 wins at every strong-scaling shard size:
      // 0.247-0.251 vs 0.254-0.255 ms at 1.25M (the 8-GPU share of the headline),
      // 0.484-0.493 vs 0.498-0.502 at 2.5M, 0.948-0.959 vs 0.978-0.989 at 5M
      // (profiles/ring3_p8_threshold_r03.txt).  Below 1M rows P=4 keeps twice the
      // workgroups.
      const int64_t per8 = 4 * 8 * 16;
      hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 8, 2, 4, 4>),
                         dim3((unsigned)((N + per8 - 1) / per8)), dim3(256), 0, stream, x, N, ldx,
                         c, cnorm, Kp / 64, labels, mind);
    } else if (DP == 128) {
      hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 4, 3, 4, 4>), grid, dim3(256), 0,
                         stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind);
    } else
      hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<256, 4, 2, 4, 4>), grid, dim3(256), 0,
                         stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind);
    TDC_CHECK_LAUNCH();
    return 0;
  }
  if (DP != 32) return (int)hipErrorInvalidValue;
  // D <= 32: the 32x32x16 ring2 schedule, 4 waves x 4 tiles of 32 points
  const int64_t per = 4 * 4 * 32;
  hipLaunchKernelGGL((assign_mfma_bf16_ring2_kernel<32, 4, 3, 4, 2>), dim3((unsigned)((N + per - 1) / per)),
                     dim3(256), 0, stream, x, N, ldx, c, cnorm, ntiles, labels, mind);
  TDC_CHECK_LAUNCH();
  return 0;
}

// Indexed rows (mini-batches): point i is row rowidx[i] of X; always the ring3 schedule.
int tdc_assign_mfma_bf16_indexed(const void* X, const int32_t* rowidx, int64_t N, int64_t ldx,
                                 int DP, const void* Cm2, const float* cnorm, int Kp,
                                 int32_t* labels, float* mind, hipStream_t stream) {
  if (N <= 0) return 0;
  if (Kp % 64 != 0 || rowidx == nullptr) return (int)hipErrorInvalidValue;
  const __bf16* x = (const __bf16*)X;
  const __bf16* c = (const __bf16*)Cm2;
  const dim3 grid((unsigned)((N + 255) / 256));
  const dim3 grid8((unsigned)((N + 511) / 512));
  if (DP == 64 && Kp % 128 == 0)  // as in tdc_assign_mfma_bf16
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<64, 8, 3, 4, 8>), grid8, dim3(256), 0,
                       stream, x, N, ldx, c, cnorm, Kp / 128, labels, mind, rowidx);
  else if (DP == 64)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<64, 8, 3, 4, 4>), grid8, dim3(256), 0,
                       stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind, rowidx);
  else if (DP == 128)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 4, 3, 4, 4>), grid, dim3(256), 0,
                       stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind, rowidx);
  else if (DP == 256)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<256, 4, 2, 4, 4>), grid, dim3(256), 0,
                       stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind, rowidx);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  return 0;
}

// Top-2 distances (labels, d1 = min squared distance, d2 = second smallest); rowidx
// nullable (indexed rows as above).  Feeds the bounds of models/bounded.py.
int tdc_assign_mfma_bf16_top2(const void* X, const int32_t* rowidx, int64_t N, int64_t ldx,
                              int DP, const void* Cm2, const float* cnorm, int Kp,
                              int32_t* labels, float* mind, float* mind2, hipStream_t stream) {
  if (N <= 0) return 0;
  if (Kp % 64 != 0 || mind == nullptr || mind2 == nullptr) return (int)hipErrorInvalidValue;
  const __bf16* x = (const __bf16*)X;
  const __bf16* c = (const __bf16*)Cm2;
  const dim3 grid((unsigned)((N + 255) / 256));
  const dim3 grid8((unsigned)((N + 511) / 512));
  if (DP == 64)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<64, 8, 3, 4, 4, true>), grid8, dim3(256), 0,
                       stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind, rowidx, mind2);
  else if (DP == 128)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<128, 4, 3, 4, 4, true>), grid, dim3(256), 0,
                       stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind, rowidx, mind2);
  else if (DP == 256)
    hipLaunchKernelGGL((assign_mfma_bf16_ring3_kernel<256, 4, 2, 4, 4, true>), grid, dim3(256), 0,
                       stream, x, N, ldx, c, cnorm, Kp / 64, labels, mind, rowidx, mind2);
  else
    return (int)hipErrorInvalidValue;
  TDC_CHECK_LAUNCH();
  return 0;
}
