// Host-side launcher API of the tdc HIP kernels (raw pointers + stream; no torch
// dependency, so the kernels compile with hipcc alone and the torch bindings with g++).
// Every launcher returns 0 or a hipError_t code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// dtype codes shared with the bindings
enum TdcDtype { TDC_F32 = 0, TDC_F64 = 1, TDC_BF16 = 2, TDC_FP8 = 3, TDC_I64 = 4 };
// TDC_I64 as an accumulation dtype = fixed point (the deterministic update): partial sums
// of round-toward-zero(x * fixed_scale) in int64 (fixed_scale a power of two chosen by the
// caller so that every |sum| < 2^62); integer sums do not depend on the order of the
// atomics, so the update (and the all-reduce of int64) is bitwise reproducible.

// N1/N6  bf16 MFMA distance + argmin. X [N, ldx] bf16 (first DP columns used, DP in
// {32,64,128,256}), Cm2 [Kp, DP] bf16 = -2*c, cnorm [Kp] fp32 (pad rows: 0 / 3e38),
// Kp % 64 == 0.  labels int32 [N]; mind fp32 [N] (nullable) = min squared distance.
int tdc_assign_mfma_bf16(const void* X, int64_t N, int64_t ldx, int DP, const void* Cm2,
                         const float* cnorm, int Kp, int32_t* labels, float* mind,
                         hipStream_t stream);
// Same, point i = row rowidx[i] of X (mini-batches without a gathered copy); DP 64/128/256.
int tdc_assign_mfma_bf16_indexed(const void* X, const int32_t* rowidx, int64_t N, int64_t ldx,
                                 int DP, const void* Cm2, const float* cnorm, int Kp,
                                 int32_t* labels, float* mind, hipStream_t stream);

// Same, with the second-smallest squared distance too (mind, mind2 required); rowidx
// nullable.  DP 64/128/256.
int tdc_assign_mfma_bf16_top2(const void* X, const int32_t* rowidx, int64_t N, int64_t ldx,
                              int DP, const void* Cm2, const float* cnorm, int Kp,
                              int32_t* labels, float* mind, float* mind2, hipStream_t stream);

// Bounds-based pruning (bounds.hip).  filter: ub[i] += drift[labels[i]], lb[i] -= maxdrift
// (device scalar); rows that may change label (ub * (1 + slack) >= lb) are appended to
// active (int32) with count (device int, zeroed by the caller).
int tdc_bounds_filter(const int32_t* labels, int64_t N, float* ub, float* lb, const float* drift,
                      const float* maxdrift, float slack, int32_t* active, int* count,
                      hipStream_t stream);
// scatter: for the M active rows (M read from count on the device, up to cap): new label
// blab[j], bounds from the top-2 squared distances d1/d2; rows whose label changed are
// appended to moved_idx / moved_old / moved_new with mcount (zeroed by the caller).
int tdc_bounds_scatter(const int32_t* active, const int* count, int64_t cap,
                       const int32_t* blab, const float* d1, const float* d2, int32_t* labels,
                       float* ub, float* lb, int32_t* moved_idx, int32_t* moved_old,
                       int32_t* moved_new, int* mcount, hipStream_t stream);

// N1 for fp32 / fp64 data on the matrix cores (assign_x3.hip): bf16x3 scores + top-3 argmin;
// rows whose winner the error bound tau(DP) cannot certify are listed in amb (int32 [3 cap]:
// int2 {row, runner-up} two-candidate entries | int32 rows for a full re-scan; counts in
// amb_count [2]) for tdc_x3_recheck.
//   split: rows of src (f32/f64 [rows, ld], d valid columns) -> hi/lo bf16 [rows, DP] of v
//          (of -2v when neg2; rows >= valid are zero, norm BIG) + norm [rows] = ||v||^2 and
//          nhl (nullable, float2 [rows]) = (||hi||^2, ||lo||^2);
//   prep : cstat [3] = max over the K rows of (cnorm, ||hi||^2, ||lo||^2), amb_count [2] = 0
//          (before every assignment);
//   assign (DP in 32/64/128/256, Kp % 64 == 0 -- % 32 at DP 256): labels, optional mind;
//   rows  (wide D): top-3 over a chunk's raw d2 block G [M, K] (tdc_fcm_mfma_wide pass 1),
//          xx [M] = ||x||^2, list rows offset by row0;
//   recheck: exact difference form in the data's dtype (X/C both f32 or f64, D <= 1024);
//   prefilter (DP 64/128/256): one bf16 product (xh . th) with top-2 and a per-row bound
//          (xnhl nullable: the rows' split norms from split, for the row's own ||xl||):
//          labels of the certified rows, the others listed in pre (count *npre, zeroed by
//          prep with nzero = 3 into amb_count[2]) for assign's listed mode (rowidx / nrows:
//          point i is row rowidx[i], count read on the device; est_rows > 0 sizes the launch
//          for that many rows, with a grid-stride launch for any overflow).
int tdc_x3_split(int src_dtype, const void* src, int64_t rows, int64_t valid, int d, int64_t ld,
                 int DP, int neg2, void* hi, void* lo, float* norm, float* nhl, hipStream_t stream,
                 const void* shift = nullptr);  // shift: [d] of src's dtype, subtracted first
int tdc_x3_prep(const float* cnorm, const float* nhl, int K, float* cstat, int* amb_count,
                hipStream_t stream, int nzero = 2);
int tdc_x3_prefilter(const void* Xh, int64_t N, int DP, const void* Ch, const float* cnorm, int Kp,
                     const float* cstat, int32_t* labels, int32_t* pre, int* npre,
                     hipStream_t stream, const float* xnhl = nullptr);
int tdc_assign_x3(const void* Xh, const void* Xl, int64_t N, int DP, const void* Ch, const void* Cl,
                  const float* cnorm, int Kp, const float* cstat, int32_t* labels,
                  float* mind, int32_t* amb, int64_t cap, int* amb_count, hipStream_t stream,
                  const int32_t* rowidx = nullptr, const int* nrows = nullptr,
                  int64_t est_rows = -1);
int tdc_x3_rows(const float* G, int64_t M, int K, int64_t row0, const float* xx, const float* cstat,
                int DP, int32_t* labels, int32_t* amb, int64_t cap, int* amb_count,
                hipStream_t stream);
int tdc_x3_recheck(int dtype, const void* X, int64_t ldx, int D, const void* C, int K,
                   int32_t* labels, const int32_t* amb, int64_t cap, const int* amb_count,
                   int num_cus, hipStream_t stream);

// N1 (exact)  SIMT difference-form assignment for fp32/fp64, any K, D <= 64.
int tdc_assign_simt(int dtype, const void* X, int64_t N, int64_t ldx, int D, const void* C,
                    int K, int32_t* labels, void* mind, hipStream_t stream);

// N1 (exact, any D)  difference-form tiled assignment (fp32 / fp64), LDS use independent of D.
// rowidx (nullable): launch row i is row rowidx[i] (labels / mind too); nptr (nullable): the
// row count read from the device (N is then the capacity sizing the grid).
int tdc_assign_exact(int dtype, const void* X, int64_t N, int64_t ldx, int D, const void* C, int K,
                     int32_t* labels, void* mind, int num_cus, hipStream_t stream,
                     const int32_t* rowidx = nullptr, const int* nptr = nullptr);

// Fused small-K Lloyd step (assign + per-cluster sums/counts in registers), fp32/fp64.
// Returns hipErrorInvalidValue if (K, D) exceeds the compiled register tiles.
int tdc_lloyd_small(int dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                    const void* C, int K, int32_t* labels, void* mind, void* sums,
                    void* counts, hipStream_t stream);
int tdc_lloyd_small_supported(int dtype, int K, int D);

// N2  LDS-privatised, D-sliced per-cluster sums/counts. sums [K, D], counts [K] must be
// zeroed by the caller (accumulated with global atomics).  x_dtype: f32/f64/bf16.
int tdc_update_lds(int x_dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                   const int32_t* labels, int K, void* sums, void* counts, int num_cus,
                   hipStream_t stream);

// N2 (large K x D): counting sort by label + segmented row gather-sum.  work: int32
// workspace of tdc_update_sorted_workspace(N, K) elements.  Its histogram part must be zero
// on entry: work_clean != 0 says it is (a workspace zero-filled when allocated and only
// used by these calls, which leave it zeroed); work_clean == 0 clears it first.  sums/counts are accumulated (caller
// zeroes them once per pass); zero_first (nullable, zero_bytes a multiple of 4) is cleared
// by the first kernel before anything accumulates -- the caller's zero fill of the
// all-reduce buffer without a launch of its own.
// rowidx (nullable): labels[i] belongs to row rowidx[i] of X (N = number of labels).
// cnt_hi / cnt_lo (nullable, fp32 [K]): the exact count split of an fp32 all-reduce
// buffer, hi += c >> 12, lo += c & 4095 (each term stays an integer below 2^24, so the
// fp32 all-reduce sums them exactly; count = 4096 hi + lo up to 2^36).
// acc_dtype TDC_I64: fixed-point sums (fixed_scale) and int64 counts.
int tdc_update_sorted(int x_dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                      const int32_t* labels, int K, void* sums, void* counts, int* work,
                      int num_cus, hipStream_t stream, const int32_t* rowidx = nullptr,
                      float* cnt_hi = nullptr, float* cnt_lo = nullptr,
                      void* zero_first = nullptr, int64_t zero_bytes = 0,
                      double fixed_scale = 0.0, int work_clean = 0);
int64_t tdc_update_sorted_workspace(int64_t N, int K);

// N4/N5  fused small-K Fuzzy C-Means tower: sum_i w_ki x_i, sum_i w_ki, argmax labels.
int tdc_fcm_small(int dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                  const void* C, int K, double m, int nan_to_zero, int32_t* labels, void* wx,
                  void* ws, hipStream_t stream);
int tdc_fcm_small_supported(int dtype, int K, int D);

// N4/N5 for any K and D <= 256 (fp32 / fp64, exact difference-form distances), two passes:
// pass 0 (stats): labels = argmax_k u, rowinfo [N] (X dtype) = 1/sum_k t (> 0), 0 (all
// memberships 0: nan_to_zero on a centroid) or -nzero (one-hot over the zero distances);
// pass 1 (accum): wx [K, D] += sum_i w_ik x_i, ws [K] += sum_i w_ik (fp64, accumulated).
int tdc_fcm_tower(int pass, int dtype, const void* X, int64_t N, int64_t ldx, int D, const void* C,
                  int K, double m, int nan_to_zero, int32_t* labels, void* rowinfo, void* wx,
                  void* ws, int num_cus, hipStream_t stream);

// N4/N5 for any D (fp32 / fp64, exact difference form) over a row chunk of M rows with the
// [M, K] block G (X dtype) in HBM: pass 0: G = d2; pass 1: labels = argmax u and G <- w =
// u^m in place (rowinfo semantics as tdc_fcm_tower); pass 3: labels only (G keeps d2);
// pass 2: wx [K, D] += W^T X, ws [K] += sum W (fp64, accumulated).
int tdc_fcm_wide(int pass, int dtype, const void* X, int64_t M, int64_t ldx, int D, const void* C,
                 int K, double m, int nan_to_zero, void* G, int32_t* labels, double* wx, double* ws,
                 int num_cus, hipStream_t stream);

// N4/N5 on MFMA (fp32 FCM, large K x D): hi/lo bf16 operands.  split_rows: fp32 rows
// [rows, ld] (d valid columns, rows >= valid are zero padding) -> hi/lo bf16 [rows, DP]
// (of -2v when neg2) + norm [rows] = ||v||^2 (nullable).  fcm_mfma pass 0: labels +
// rowinfo (fp32, as tdc_fcm_tower); pass 1: wx [K, D] / ws [K] (fp64) += W^T X / sum W.
// DP in {32, 64, 128}; Ch/Cl/cc have Kp rows (Kp % 128 == 0).
// shift (nullable, fp32 [d]) is subtracted from every row first.
int tdc_fcm_split_rows(const float* src, int64_t rows, int64_t valid, int d, int64_t ld, int DP,
                       int neg2, const float* shift, void* hi, void* lo, float* norm,
                       hipStream_t stream);
// work: fp32 [tdc_fcm_mfma_workspace(...)] per-block partial slabs of pass 1; shift
// (nullable, fp32 [D]): the vector subtracted from rows and centroids at the split, added
// back as shift * sum w in the reduction.
// rowinfo holds rowinfo_len floats: [N] row statistics, and from DP = 64, when rowinfo_len >=
// tdc_fcm_mfma_rowinfo_len(N, DP), each row's two corrected nearest d2 after them (16-byte
// aligned float4 {d2a, d2b, la, lb}); with them pass 1 runs one-product distances.
// Xr (nullable, pass 1 with the fix-up rows): the shard's own bf16 rows [N, DP], unshifted,
// zero padded -- W^T X then takes them as its one operand (bf16 data only: exact products).
int tdc_fcm_mfma(int pass, const void* Xh, const void* Xl, const void* Xr, const float* xx,
                 int64_t N, int DP, int D, const void* Ch, const void* Cl, const float* cc, int K,
                 int Kp, double m, int nan_to_zero, int32_t* labels, float* rowinfo,
                 int64_t rowinfo_len, double* wx, double* ws, float* work, const float* shift,
                 int num_cus, hipStream_t stream);
int64_t tdc_fcm_mfma_workspace(int64_t N, int K, int Kp, int DP, int num_cus);
int64_t tdc_fcm_mfma_rowinfo_len(int64_t N, int DP);
// Wide D (DP in 128 ... 1024, multiples of 128), over a chunk of M rows with the [M, K]
// block G (fp32): pass 0: G = d2 (hi/lo MFMA, distances within 2^-16 ||x||^2 of a centroid
// stored as 0, the on-centroid rule of tdc_fcm_wide pass 1, which then turns G into w);
// pass 2: wx [K, D] / ws [K] (fp64) += W^T X / sum W through per-split slabs in work (fp32
// [tdc_fcm_mfma_wide_workspace]); shift as tdc_fcm_mfma.  Xh/Xl/Ch/Cl/cc as tdc_fcm_mfma
// with Kp % 128 == 0.
int tdc_fcm_mfma_wide(int pass, const void* Xh, const void* Xl, const float* xx, int64_t M,
                      int DP, int D, const void* Ch, const void* Cl, const float* cc, int K,
                      int Kp, float* G, float* work, const float* shift, double* wx, double* ws,
                      int num_cus, hipStream_t stream);
int64_t tdc_fcm_mfma_wide_workspace(int64_t M, int Kp, int DP, int num_cus);
// fp64 FCM, row statistics fused into the f64-MFMA distance pass (fcm_wide.hip), over a chunk
// of M rows with G [M, K] fp64: pass 0: G = t = d2^(-1/(m-1)) (+inf on a centroid), rowinfo
// [M] (fcm_wide_rows semantics: 1/sum t, 0 or -zeros on a centroid) and labels [M]; pass 1:
// wx [K, D] / ws [K] += W^T X / sum W with w = (t * rowinfo)^m formed while staging.
int tdc_fcm_f64t(int pass, const double* X, int64_t M, int64_t ldx, int D, const double* C, int K,
                 double m, int nan_to_zero, double* G, double* rowinfo, int32_t* labels, double* wx,
                 double* ws, int num_cus, hipStream_t stream);

// N3  finalize: C = sums/counts (empty policy), max shift^2 -> shift (float, atomic max),
// optional bf16 prep of the next assignment (Cm2 [Kp, DP] = -2*bf16(c), cnorm [Kp]).
// sums == nullptr: prep only (C unchanged).
// policy: 0 keep, 1 nan, 2 zero.
// drift (nullable, [K]) = ||bf16(c_new) - bf16(c_old)|| per centroid, maxdrift (nullable,
// zeroed by the caller) = its max: the centroid movement the bounds of bounded Lloyd need.
// acc_dtype TDC_I64: fixed-point sums (divided by fixed_scale) and int64 counts.
int tdc_finalize(int acc_dtype, int c_dtype, const void* sums, const void* counts, int K,
                 int D, void* C, int policy, float* shift, void* Cm2, float* cnorm, int Kp,
                 int DP, hipStream_t stream, float* drift = nullptr, float* maxdrift = nullptr,
                 double fixed_scale = 0.0);

// Mini-batch (Sculley) update: n = counts[k] > 0 -> C[k] = (v[k] C[k] + sums[k]) / (v[k] + n),
// v[k] += n (v fp64 [K]); shift (nullable, zeroed by the caller) = max ||dC_k||^2 over the
// updated k; optional bf16 prep of the next assignment as in tdc_finalize.
int tdc_sculley_update(int acc_dtype, int c_dtype, const void* sums, const void* counts, int K,
                       int D, void* C, double* v, float* shift, void* Cm2, float* cnorm, int Kp,
                       int DP, hipStream_t stream);

// N1 wide-D / fp8 (assign_bigd.hip).  dtype TDC_BF16: X bf16 rows (ldx elements), Cm2
// bf16 [Kp, DP] = -2c, DP in {384,512}.  dtype TDC_FP8: X e4m3 bytes (ldx bytes),
// Xs E8M0 [N, DP/32]; Cm2 = quantised -2c with scales Cs [Kp, DP/32]; DP in {256..1024}/256.
// cnorm [Kp] (pad 3e38), xnorm [N] (for mind).  Kp % 32 == 0.  The K loop is split into
// groups of kg_tiles*32 centroids (0 = one group); with >1 group keys (uint64 [N], all
// ones on entry; reset on exit) merges the group winners.
// labels2 / mind2 (fp8, one K-group): also the runner-up centroid and its distance.
int tdc_assign_bigd(int dtype, const void* X, const void* Xs, int64_t N, int64_t ldx, int DP,
                    const void* Cm2, const void* Cs, const float* cnorm, int Kp, int kg_tiles,
                    const float* xnorm, int32_t* labels, float* mind, unsigned long long* keys,
                    hipStream_t stream, int32_t* labels2 = nullptr, float* mind2 = nullptr);
// Near-tie re-check of a top-2 assignment: where d2 - d1 <= tau * d2, recompute both
// distances exactly (fp32, difference form) from X (bf16 / f32 rows) and C (fp32 [K, D])
// and swap the label if the runner-up is closer.  flips (nullable) counts the swaps.
int tdc_recheck_top2(int x_dtype, const void* X, int64_t N, int64_t ldx, int D, const float* C,
                     int32_t* labels, const int32_t* labels2, const float* d1, const float* d2,
                     float tau, int* flips, hipStream_t stream);
int tdc_assign_bigd_supported(int dtype, int DP);

// N8 fp8 quantiser: rows of X (f32/f64/bf16, d valid columns, ldx elements) -> Q e4m3
// [rows, DP] + E8M0 block scales S [rows, DP/32] + norm[rows] = ||dequant||^2.
// neg2 != 0: centroid operand (-2c; norm of +c).  Rows >= valid are padding.
int tdc_quant_fp8(int src_dtype, const void* X, int64_t rows, int64_t valid, int d, int64_t ldx,
                  int DP, int neg2, void* Q, void* S, float* norm, hipStream_t stream);

// N7 k-means++ step (kmeanspp.hip).  cand [T, D] (d_dtype, T <= 16), closest [N] (d_dtype).
// mode 0: pots[t] += sum_i min(closest_i, ||x_i - cand_t||^2) for every candidate;
// mode 1 (T == 1): closest_i = min(closest_i, ||x_i - cand_0||^2), pots[0] += sum closest.
// pots is fp64 and accumulated (caller zeroes it).
int tdc_kpp_step(int x_dtype, int d_dtype, const void* X, int64_t N, int64_t ldx, int D,
                 const void* cand, int T, void* closest, int mode, double* pots, int num_cus,
                 hipStream_t s);

// ---- delta update of plain Lloyd (update_sorted.hip delta_*, centroids.hip) ----
// ctrl: int32 [TDC_DC_WORDS] device words shared by the step's kernels and the host.
enum TdcDeltaCtrl {
  TDC_DC_NEXT = 0,    // mode of the upcoming step: 0 delta, 1 full (finalize; host on reset)
  TDC_DC_MODE = 1,    // mode of the running step (set by the scan for the kernels after it)
  TDC_DC_MOVED = 2,   // rows whose label changed in the running step (diff kernel)
  TDC_DC_EVENTS = 3,  // perm entries of the running step
  TDC_DC_PREVOK = 4,  // prev[] holds the previous step's labels (host reset: 0)
  TDC_DC_ITER = 5,    // steps since the last reset
  TDC_DC_WORDS = 16
};
constexpr int TDC_DELTA_MAX_K = 65536;      // labels packed in 16 bits in the moved list
constexpr int TDC_DELTA_MAX_BLOCKS = 1024;  // per-block moved-list slots in the workspace
// One local update of a Lloyd step in the mode ctrl[NEXT] says: labels (this step's
// assignment) vs prev (the previous one; prev = labels on return) -> sums / counts (the
// step's all-reduce buffer views: deltas of the moved rows, or full partials), the exact
// count split as tdc_update_sorted (signed), moved (nullable, acc dtype [1]) += rows that
// changed label.  work: int32 [tdc_delta_workspace(N, K)]; work_clean as
// tdc_update_sorted (its two histograms zero on entry, left zero).  K <= TDC_DELTA_MAX_K,
// N < 2^30.
int tdc_delta_update(int x_dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                     const int32_t* labels, int32_t* prev, int K, void* sums, void* counts,
                     int* work, int* ctrl, int num_cus, hipStream_t stream, float* cnt_hi,
                     float* cnt_lo, void* moved, void* zero_first, int64_t zero_bytes,
                     double fixed_scale = 0.0, int work_clean = 0);
int64_t tdc_delta_workspace(int64_t N, int K);
// The step's finalize: G (fp64 [K*D + K] totals) += or = the all-reduced buffer (by
// ctrl[MODE]), C = G means (policy as tdc_finalize), optional bf16 operand prep, shift;
// picks ctrl[NEXT] (full every `refresh` steps (0: never) or when moved > theta_n) and
// accumulates stats (nullable, fp64 [4]: moved rows, steps with a valid prev, full steps,
// steps).
int tdc_delta_finalize(int acc_dtype, int c_dtype, const void* dsums, const void* dcounts,
                       const float* cnt_hi, const float* cnt_lo, const void* moved, double* G,
                       int K, int D, void* C, int policy, float* shift, void* Cm2, float* cnorm,
                       int Kp, int DP, int* ctrl, double* stats, int refresh, double theta_n,
                       hipStream_t stream, double fixed_scale = 0.0);
