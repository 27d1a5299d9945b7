// N2 (large K x D): per-cluster sums via counting sort + segmented gather-sum.
//
// When K x D does not fit LDS (K=1024 x D=128 fp32 = 512 KB; K=65536 x D=768 = 201 MB)
// the LDS histogram of update_lds would need D-slices and one flush of K x D_slice
// global atomics per block, and its label -> row load chain is latency bound.  Instead:
//
//   1. hist     : labels -> per-cluster counts (LDS histogram per block, one global
//                 atomic per non-empty bin per block)
//   2. scan     : exclusive prefix sum -> segment offsets; counts also added (acc dtype)
//                 straight into the all-reduce buffer
//   3. scatter  : counting-sort the point indices by label: one pass per block over its
//                 whole range (LDS histogram, one returning atomic per bin to reserve the
//                 block's sub-range, LDS cursors); K > 16384: global cursor atomics
//   4. segsum   : each wave walks a contiguous range of the sorted index, gathers whole
//                 rows (16 B per lane, a row per 16/32/64 lanes), accumulates in fp32
//                 registers and flushes with global atomics only at segment boundaries
//                 (~1-3 flushes per wave instead of one atomic per element).
//
// X is read exactly once (as whole-row gathers); labels twice; the permutation once.
#include <stdlib.h>

#include <algorithm>

#include "tdc_common.h"
#include "kernels.h"

namespace tdc {

constexpr int LDS_HIST_MAX_K = 16384;
constexpr int64_t ZERO_WORDS_PER_BLOCK = 16384;  // 1024 threads x one 16-B store each, x4

// Clear words [0, n) of z with 16-B stores when z is 16-B aligned (a torch allocation or a
// view at its start), from thread t of T; the caller's grid covers n / ZERO_WORDS_PER_BLOCK
// blocks at least (the fill no longer runs on the few blocks a small row range needs).
__device__ __forceinline__ void zero_fill(uint32_t* __restrict__ z, int64_t n, int64_t t,
                                          int64_t T) {
  int64_t done = 0;
  if (((uintptr_t)z & 15) == 0) {
    uint4* z4 = reinterpret_cast<uint4*>(z);
    const int64_t n4 = n >> 2;
    for (int64_t w = t; w < n4; w += T) z4[w] = make_uint4(0u, 0u, 0u, 0u);
    done = n4 << 2;
  }
  for (int64_t w = done + t; w < n; w += T) z[w] = 0u;
}

template <int NT>
__global__ __launch_bounds__(NT) void hist_kernel(const int32_t* __restrict__ labels, int64_t N,
                                                  int K, int* __restrict__ cnt,
                                                  int64_t per_block, uint32_t* __restrict__ zero,
                                                  int64_t zero_words) {
  extern __shared__ int s_h[];
  const int tid = threadIdx.x;
  // the caller's accumulation buffer (the all-reduce buffer of the step), cleared here
  // instead of by a separate fill launch: scan / segsum accumulate into it only after
  // this kernel has finished
  if (zero_words) zero_fill(zero, zero_words, (int64_t)blockIdx.x * NT + tid, (int64_t)gridDim.x * NT);
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = min(N, r0 + per_block);
  if (r0 >= N) return;  // a block of the zero fill only (block-uniform)
  const bool lds = K <= LDS_HIST_MAX_K;
  if (lds) {
    for (int k = tid; k < K; k += NT) s_h[k] = 0;
    __syncthreads();
  }
  int64_t i = r0 + tid;
  for (; i + 3 * NT < r1; i += 4 * NT) {
    const int a = labels[i], b = labels[i + NT], c = labels[i + 2 * NT], d = labels[i + 3 * NT];
    if (lds) {
      if ((unsigned)a < (unsigned)K) atomicAdd(s_h + a, 1);
      if ((unsigned)b < (unsigned)K) atomicAdd(s_h + b, 1);
      if ((unsigned)c < (unsigned)K) atomicAdd(s_h + c, 1);
      if ((unsigned)d < (unsigned)K) atomicAdd(s_h + d, 1);
    } else {
      if ((unsigned)a < (unsigned)K) atomicAdd(cnt + a, 1);
      if ((unsigned)b < (unsigned)K) atomicAdd(cnt + b, 1);
      if ((unsigned)c < (unsigned)K) atomicAdd(cnt + c, 1);
      if ((unsigned)d < (unsigned)K) atomicAdd(cnt + d, 1);
    }
  }
  for (; i < r1; i += NT) {
    const int a = labels[i];
    if ((unsigned)a < (unsigned)K) atomicAdd(lds ? s_h + a : cnt + a, 1);
  }
  if (lds) {
    __syncthreads();
    for (int k = tid; k < K; k += NT)
      if (s_h[k]) atomicAdd(cnt + k, s_h[k]);
  }
}

// Inclusive prefix sum of one value per thread over a 1024-thread block: within each
// wave by shuffles (no barrier), then over the 16 wave totals by wave 0 (two barriers in
// all; the Hillis-Steele form over LDS took 20).
__device__ __forceinline__ int block_inclusive_scan_1024(int s) {
  __shared__ int s_wave[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (lane == 63) s_wave[wv] = inc;
  __syncthreads();
  if (wv == 0) {
    int t = lane < 16 ? s_wave[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int v = __shfl_up(t, o, 64);
      if (lane >= o) t += v;
    }
    if (lane < 16) s_wave[lane] = t;  // inclusive totals of waves 0..lane
  }
  __syncthreads();
  return inc + (wv > 0 ? s_wave[wv - 1] : 0);
}

// single block, 1024 threads: offsets[0..K] (exclusive), cursor = offsets, counts_acc = cnt
template <typename ACC>
__global__ __launch_bounds__(1024) void scan_kernel(int* __restrict__ cnt, int K,
                                                    int* __restrict__ offsets,
                                                    int* __restrict__ cursor,
                                                    ACC* __restrict__ counts_acc,
                                                    float* __restrict__ cnt_hi,
                                                    float* __restrict__ cnt_lo) {
  const int tid = threadIdx.x;
  const int per = (K + 1023) / 1024;
  const int k0 = tid * per, k1 = min(K, k0 + per);
  int s = 0;
  for (int k = k0; k < k1; ++k) s += cnt[k];
  const int inc = block_inclusive_scan_1024(s);
  int run = inc - s;  // exclusive prefix of this thread's range
  for (int k = k0; k < k1; ++k) {
    const int c = cnt[k];
    cnt[k] = 0;  // the histogram is left zeroed for the next call (no memset launch)
    offsets[k] = run;
    cursor[k] = run;
    if (counts_acc) counts_acc[k] += (ACC)c;  // accumulate: streamed chunks add up
    if (cnt_hi && c) {  // exact split for the fp32 all-reduce (kernels.h)
      cnt_hi[k] += (float)(c >> 12);
      cnt_lo[k] += (float)(c & 4095);
    }
    run += c;
  }
  if (tid == 1023) offsets[K] = inc;
}

// block-aggregated counting-sort scatter: perm[offset[label] + rank] = i
__global__ __launch_bounds__(256) void scatter_kernel(const int32_t* __restrict__ labels, int64_t N,
                                                      int K, int* __restrict__ cursor,
                                                      int32_t* __restrict__ perm,
                                                      int64_t per_block,
                                                      const int32_t* __restrict__ rowidx) {
  constexpr int R = 16;  // labels per thread per pass (4096 per block pass)
  extern __shared__ int s_mem[];
  int* s_cnt = s_mem;
  int* s_base = s_mem + K;
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = min(N, r0 + per_block);
  const bool agg = K <= 4096;
  for (int64_t p0 = r0; p0 < r1; p0 += 256 * R) {
    int lab[R], rank[R];
    if (agg) {
      for (int k = tid; k < K; k += 256) s_cnt[k] = 0;
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int64_t i = p0 + j * 256 + tid;
      lab[j] = (i < r1) ? labels[i] : -1;
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      rank[j] = -1;
      if ((unsigned)lab[j] < (unsigned)K)
        rank[j] = agg ? atomicAdd(s_cnt + lab[j], 1) : atomicAdd(cursor + lab[j], 1);
    }
    if (agg) {
      __syncthreads();
      for (int k = tid; k < K; k += 256) {
        const int c = s_cnt[k];
        s_base[k] = c ? atomicAdd(cursor + k, c) : 0;
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if (rank[j] >= 0) {
        const int pos = agg ? s_base[lab[j]] + rank[j] : rank[j];
        const int64_t i = p0 + j * 256 + tid;
        perm[pos] = rowidx ? rowidx[i] : (int32_t)i;
      }
    }
    if (agg) __syncthreads();
  }
}

// ---- one-pass block scatter for K <= LDS_HIST_MAX_K ----
// Each block takes a contiguous label range: LDS histogram of the range, ONE returning
// global atomic per non-empty bin to reserve the block's sub-range of that segment, then
// the scatter with LDS cursors.  (The per-4096-label passes of scatter_kernel reserved
// once per bin per pass: ~5x more global atomics at N=10M, K=1024.)
template <int NT>
__global__ __launch_bounds__(NT) void bscatter_kernel(const int32_t* __restrict__ labels, int64_t N,
                                                       int K, int* __restrict__ cursor,
                                                       int32_t* __restrict__ perm, int64_t per_block,
                                                       const int32_t* __restrict__ rowidx,
                                                       int parts) {
  // perm holds X row numbers: i itself, or rowidx[i] for an indexed (mini-batch) pass
#define TDC_ROW(ii) (rowidx ? rowidx[ii] : (int32_t)(ii))
  extern __shared__ int s_mem[];
  int* s_cnt = s_mem;
  int* s_cur = s_mem + K;
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = min(N, r0 + per_block);
  for (int k = tid; k < K; k += NT) s_cnt[k] = 0;
  __syncthreads();
  int64_t i = r0 + tid;
  for (; i + 3 * NT < r1; i += 4 * NT) {
    const int a0 = labels[i], a1 = labels[i + NT], a2 = labels[i + 2 * NT], a3 = labels[i + 3 * NT];
    if ((unsigned)a0 < (unsigned)K) atomicAdd(s_cnt + a0, 1);
    if ((unsigned)a1 < (unsigned)K) atomicAdd(s_cnt + a1, 1);
    if ((unsigned)a2 < (unsigned)K) atomicAdd(s_cnt + a2, 1);
    if ((unsigned)a3 < (unsigned)K) atomicAdd(s_cnt + a3, 1);
  }
  for (; i < r1; i += NT) {
    const int a0 = labels[i];
    if ((unsigned)a0 < (unsigned)K) atomicAdd(s_cnt + a0, 1);
  }
  __syncthreads();
  for (int k = tid; k < K; k += NT) {
    const int c = s_cnt[k];
    s_cur[k] = c ? atomicAdd(cursor + k, c) : 0;
  }
  __syncthreads();
  // The scatter runs in `parts` passes over bin ranges [p K / parts, (p + 1) K / parts):
  // the block re-reads its (L2-resident) labels, and the perm lines it is writing at any
  // time span 1/parts of the bins, so the partial-line stores of the XCD's blocks combine
  // in its L2 instead of thrashing it.
  for (int part = 0; part < parts; ++part) {
    const unsigned lo = (unsigned)((int64_t)K * part / parts);
    const unsigned n = (unsigned)((int64_t)K * (part + 1) / parts) - lo;
    i = r0 + tid;
    for (; i + 3 * NT < r1; i += 4 * NT) {
      const int a0 = labels[i], a1 = labels[i + NT], a2 = labels[i + 2 * NT], a3 = labels[i + 3 * NT];
      if ((unsigned)a0 - lo < n) perm[atomicAdd(s_cur + a0, 1)] = TDC_ROW(i);
      if ((unsigned)a1 - lo < n) perm[atomicAdd(s_cur + a1, 1)] = TDC_ROW(i + NT);
      if ((unsigned)a2 - lo < n) perm[atomicAdd(s_cur + a2, 1)] = TDC_ROW(i + 2 * NT);
      if ((unsigned)a3 - lo < n) perm[atomicAdd(s_cur + a3, 1)] = TDC_ROW(i + 3 * NT);
    }
    for (; i < r1; i += NT) {
      const int a0 = labels[i];
      if ((unsigned)a0 - lo < n) perm[atomicAdd(s_cur + a0, 1)] = TDC_ROW(i);
    }
  }
#undef TDC_ROW
}

// Per-element accumulator conversion: fp32 / fp64 partials, or fixed point (the
// deterministic update): v * 2^S rounded to the NEAREST integer (ties to even: unbiased, so
// the rounding of the many small elements of a feature far below max|x| averages out
// instead of drifting toward zero) in int64, whose sums are exact and therefore independent
// of the order the atomics land in.  The scale is a power of two, so v * scale is exact;
// |sum| < 2^62 by the caller's choice of S (ops.fixed_point_scale).
//   bf16 / fp32 rows: |v * scale| <= 2^30 by the scale's contract, so the conversion is a
//     v_rndne + v_cvt_i32 (+ sign extension) instead of an emulated float -> int64;
//   fp64 rows: the scale only bounds the sums (a step ~2^30 x finer, near the fp64 ulp of
//     the data), converted by the int64 round-to-nearest.
template <typename AT> __device__ __forceinline__ AT acc_cvt(float v, float scale) {
  if constexpr (std::is_same<AT, long long>::value) return (long long)__float2int_rn(v * scale);
  else return (AT)v;
}
template <typename AT> __device__ __forceinline__ AT acc_cvt(double v, double scale) {
  if constexpr (std::is_same<AT, long long>::value) return __double2ll_rn(v * scale);
  else return (AT)v;
}

// Split load / accumulate (so a batch of row loads can be in flight before any add).  sg
// is 0 or 0x80000000 (a delta update's subtracted rows), XOR-ed into every element's sign
// bit: one VALU per element on top of the conversion, folded away when sg is 0.
template <typename XT, int VEC> struct RowRaw;
template <> struct RowRaw<__bf16, 8> {
  typedef uint4 raw_t;
  typedef float sc_t;
  __device__ static raw_t load(const __bf16* p) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  template <typename AT>
  __device__ static void add(const raw_t& t, unsigned sg, AT (&a)[8], float sc) {
    a[0] += acc_cvt<AT>(__uint_as_float((t.x << 16) ^ sg), sc);
    a[1] += acc_cvt<AT>(__uint_as_float((t.x & 0xffff0000u) ^ sg), sc);
    a[2] += acc_cvt<AT>(__uint_as_float((t.y << 16) ^ sg), sc);
    a[3] += acc_cvt<AT>(__uint_as_float((t.y & 0xffff0000u) ^ sg), sc);
    a[4] += acc_cvt<AT>(__uint_as_float((t.z << 16) ^ sg), sc);
    a[5] += acc_cvt<AT>(__uint_as_float((t.z & 0xffff0000u) ^ sg), sc);
    a[6] += acc_cvt<AT>(__uint_as_float((t.w << 16) ^ sg), sc);
    a[7] += acc_cvt<AT>(__uint_as_float((t.w & 0xffff0000u) ^ sg), sc);
  }
};
template <> struct RowRaw<float, 4> {
  typedef float4 raw_t;
  typedef float sc_t;
  __device__ static raw_t load(const float* p) { return *reinterpret_cast<const float4*>(p); }
  template <typename AT>
  __device__ static void add(const raw_t& t, unsigned sg, AT (&a)[4], float sc) {
    a[0] += acc_cvt<AT>(__uint_as_float(__float_as_uint(t.x) ^ sg), sc);
    a[1] += acc_cvt<AT>(__uint_as_float(__float_as_uint(t.y) ^ sg), sc);
    a[2] += acc_cvt<AT>(__uint_as_float(__float_as_uint(t.z) ^ sg), sc);
    a[3] += acc_cvt<AT>(__uint_as_float(__float_as_uint(t.w) ^ sg), sc);
  }
};
template <> struct RowRaw<double, 2> {
  typedef double2 raw_t;
  typedef double sc_t;
  __device__ static raw_t load(const double* p) { return *reinterpret_cast<const double2*>(p); }
  template <typename AT>
  __device__ static void add(const raw_t& t, unsigned sg, AT (&a)[2], double sc) {
    const long long s = (long long)sg << 32;
    a[0] += acc_cvt<AT>(__longlong_as_double(__double_as_longlong(t.x) ^ s), sc);
    a[1] += acc_cvt<AT>(__longlong_as_double(__double_as_longlong(t.y) ^ s), sc);
  }
};

// one element per lane (unaligned rows / odd widths)
template <typename XT> struct RowLoad1 {
  typedef typename std::conditional<sizeof(XT) == 8, double, float>::type acc_t;
  typedef acc_t sc_t;
  template <typename AT>
  __device__ static void add(const XT* p, unsigned sg, AT (&a)[1], sc_t sc) {
    const acc_t v = (acc_t)p[0];
    a[0] += acc_cvt<AT>(sg ? -v : v, sc);
  }
};

// perm entries of a delta update carry the sign in bit 31 (row numbers are < 2^31)
constexpr unsigned PERM_NEG = 0x80000000u;
// moved-list row words (delta shards have < 2^30 rows): out-of-range label flags
constexpr unsigned LIDX_NO_NEW = 0x80000000u, LIDX_NO_OLD = 0x40000000u, LIDX_ROW = 0x3fffffffu;
// segment offsets staged in LDS by the segsum kernel up to this many entries (32 KiB)
constexpr int SEG_LDS_OFF_MAX = 8193;
// delta update: K up to which the diff / scatter kernels keep their two K-int tables in
// LDS (64 KiB); above it they use the global histograms / cursors directly
constexpr int DELTA_LDS_K = 8192;

// each wave: rows [a, b) of the sorted permutation; TPR lanes per row, G = 64/TPR rows
// in flight per wave-instruction, columns [c0, c0 + TPR*VEC) per pass.
// SIGNED (delta updates): a perm entry with PERM_NEG set subtracts its row.  nptr
// (nullable): the entry count lives on the device (delta updates decide it there); the
// waves then split it evenly themselves (at least 64 entries each, the rest exit).
// ACC = long long: fixed-point partials (v * scale in int64, the deterministic update).
template <typename XT, typename ACC, int VEC, int TPR, bool SIGNED = false>
__global__ __launch_bounds__(256) void segsum_kernel(const XT* __restrict__ X, int64_t ldx, int D,
                                                     const int32_t* __restrict__ perm,
                                                     const int* __restrict__ offsets, int K,
                                                     int64_t N, ACC* __restrict__ sums,
                                                     int64_t rows_per_wave,
                                                     const int* __restrict__ nptr,
                                                     double fixed_scale) {
  // fp64 data -> fp64 partials, else fp32; fixed point -> int64
  typedef typename std::conditional<std::is_same<ACC, long long>::value, long long,
                                    typename RowLoad1<XT>::acc_t>::type AT;
  typedef typename RowLoad1<XT>::sc_t SC;
  const SC sc = (SC)fixed_scale;
  constexpr int G = 64 / TPR;
  constexpr int U = 8;  // rows per group in flight
  const int lane = threadIdx.x & 63;
  const int g = lane / TPR, t = lane % TPR;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (nptr) {
    // a delta step's events: few, spread over many short segments (a wave pays one HBM
    // round trip per segment it walks), so they go to as many waves as the grid has, at
    // least 4 each -- not 64: at 150 events a 64-event wave walked ~30 segments (31 us);
    // 4 / 8 / 16: 12.4 / 14.2 / 17.8 us at the 1.25M-row shard, 29.2 / 28.5 / 28.1 us at
    // 10M rows (profiles/segsum_minrows_ab_r04za.txt)
    N = *nptr;
    const int64_t waves = (int64_t)gridDim.x * 4;
    rows_per_wave = (N + waves - 1) / waves;
    if (rows_per_wave < 4) rows_per_wave = 4;
  }
  const int64_t a = wave * rows_per_wave;
  if ((int64_t)blockIdx.x * 4 * rows_per_wave >= N) return;  // block-uniform: nothing to sum
  // The segment offsets (just written by the scan, mostly in another XCD's L2) go to LDS
  // with one coalesced read per block: the binary search below and every segment change
  // were chains of dependent global loads per wave (a 39 us delta step at ~50K entries).
  extern __shared__ int s_off[];
  const bool lds_off = K + 1 <= SEG_LDS_OFF_MAX;  // the launch sizes the dynamic LDS to match
  if (lds_off) {
    for (int i = threadIdx.x; i <= K; i += blockDim.x) s_off[i] = offsets[i];
    __syncthreads();
  }
  const int* __restrict__ off = lds_off ? s_off : offsets;
  if (a >= N) return;
  const int64_t b = min(N, a + rows_per_wave);
  // segment containing a: largest k with offsets[k] <= a
  int lo = 0, hi = K;  // invariant offsets[lo] <= a < offsets[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= a) lo = mid; else hi = mid;
  }
  for (int c0 = 0; c0 < D; c0 += TPR * VEC) {
    const int col = c0 + t * VEC;
    const bool colok = col < D;
    int k = lo;
    int64_t kend = off[k + 1];
    AT acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = 0;
#define TDC_FLUSH(KK)                                                                 \
  do {                                                                                \
    if (colok) {                                                                      \
      _Pragma("unroll") for (int e = 0; e < VEC; ++e) if (col + e < D && acc[e] != (AT)0) \
          atomic_add(&sums[(int64_t)(KK) * D + col + e], (ACC)acc[e]);                \
    }                                                                                 \
    _Pragma("unroll") for (int e = 0; e < VEC; ++e) acc[e] = 0;                       \
  } while (0)
    int64_t j = a + g;
    if constexpr (VEC > 1) {
      // One software-pipelined loop over wave-uniform batches [p, pe): a batch never
      // straddles a segment boundary, all U row gathers of a batch are in flight at once
      // and the permutation entries of the next batch load while they are.  When a batch
      // closes a segment the G row-groups of the wave are summed with cross-lane
      // shuffles and only group 0 issues the atomics: short segments (mini-batches,
      // large K) used to flush from every group into the same addresses, a G-way
      // same-address conflict inside each atomic instruction.
      typedef typename RowRaw<XT, VEC>::raw_t raw_t;
      int64_t p = a;
      int64_t knext = k + 1 < K ? off[k + 2] : N;
      int64_t pe = min(min(b, kend), p + U * G);
      int32_t nidx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = p + g + u * G;
        nidx[u] = r < pe ? perm[r] : 0;
      }
      while (p < b) {
        raw_t xv[U];
        unsigned sg[U];
        if (colok) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            sg[u] = SIGNED ? (unsigned)nidx[u] & PERM_NEG : 0u;
            const int64_t row = SIGNED ? (int64_t)((unsigned)nidx[u] & ~PERM_NEG) : (int64_t)nidx[u];
            if (p + g + u * G < pe) xv[u] = RowRaw<XT, VEC>::load(X + row * ldx + col);
          }
        }
        const bool closes = pe == kend || pe == b;  // wave-uniform
        int kn = k;
        int64_t kendn = kend, knextn = knext;
        if (pe == kend) {
          do {  // next non-empty segment (the boundary after it is prefetched)
            ++kn;
            kendn = knextn;
            knextn = kn + 1 < K ? off[kn + 2] : N;
          } while (kendn <= pe && kn + 1 < K);
        }
        const int64_t pn = pe;
        const int64_t pen = min(min(b, kendn), pn + U * G);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t r = pn + g + u * G;
          nidx[u] = r < pen ? perm[r] : 0;
        }
        if (colok) {
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (p + g + u * G < pe)
              RowRaw<XT, VEC>::template add<AT>(xv[u], SIGNED ? sg[u] : 0u, acc, sc);
        }
        if (closes) {
#pragma unroll
          for (int off = TPR; off < 64; off <<= 1)
#pragma unroll
            for (int e = 0; e < VEC; ++e) acc[e] += __shfl_xor(acc[e], off, 64);
          // every group now holds the segment's sums: group g adds elements e0 + g, so
          // each atomic wave-instruction covers up to 64 distinct columns (Guideline 12:
          // few, wide atomic instructions) instead of VEC instructions of TPR lanes
#pragma unroll
          for (int e0 = 0; e0 < VEC; e0 += G) {
            const int e = e0 + g;
            AT v = 0;
#pragma unroll
            for (int q = 0; q < VEC; ++q) v = (q == e) ? acc[q] : v;
            if (colok && e < VEC && col + e < D && v != (AT)0)
              atomic_add(&sums[(int64_t)k * D + col + e], (ACC)v);
          }
#pragma unroll
          for (int e = 0; e < VEC; ++e) acc[e] = 0;
        }
        k = kn;
        kend = kendn;
        knext = knextn;
        p = pn;
        pe = pen;
      }
      (void)j;
    } else {
      // fast path: U rows of this group all inside the current segment
      while (j < b) {
        if (j + (U - 1) * G < min(b, kend)) {
          int32_t idx[U];
#pragma unroll
          for (int u = 0; u < U; ++u) idx[u] = perm[j + u * G];
          if (colok) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const unsigned e = (unsigned)idx[u];
              RowLoad1<XT>::template add<AT>(X + (int64_t)(SIGNED ? e & ~PERM_NEG : e) * ldx + col,
                                             SIGNED ? e & PERM_NEG : 0u, acc, sc);
            }
          }
          j += U * G;
        } else {
          while (j >= kend) {
            TDC_FLUSH(k);
            ++k;
            kend = off[k + 1];
          }
          const int32_t idx = perm[j];
          if (colok) {
            const unsigned e = (unsigned)idx;
            RowLoad1<XT>::template add<AT>(X + (int64_t)(SIGNED ? e & ~PERM_NEG : e) * ldx + col,
                                           SIGNED ? e & PERM_NEG : 0u, acc, sc);
          }
          j += G;
        }
      }
    }
    TDC_FLUSH(k);
  }
#undef TDC_FLUSH
}


// ---- delta update (plain Lloyd after its first step; models/kmeans.py) ----
//
// Between two Lloyd steps only the rows whose label changed move their contribution from
// one cluster total to another.  The engine keeps the totals G (fp64, replicated) and the
// previous step's labels prev[]; a delta step sums +x into the new and -x out of the old
// cluster of every moved row (a counting sort of 2M signed events + the signed segmented
// gather-sum), all-reduces those deltas, and the finalize adds them to G.  A full step
// (the first one, every `refresh` steps, or after a step that moved more than theta N
// rows) sums every row instead and the finalize replaces G.  The choice is made ON THE
// DEVICE by the previous step's finalize (from the all-reduced moved count, so every rank
// makes the same one): no host sync, and the step stays capturable in a hipGraph.  Both
// modes run the same four kernels; each reads the mode from ctrl (kernels.h TDC_DC_*).
//
//   diff    : labels vs prev -> prev = labels; per-block list of moved rows (idx, old|new),
//             LDS-appended (no global atomic per row); LDS histograms of the events
//             (delta: +1 at new, +1 at old; full: +1 at every label) and signed counts
//   scan    : offsets of the events, signed counts into the all-reduce buffer, moved count
//             into its slot, mode of this step for the kernels after it
//   scatter : counting-sort placement of the events (delta: the list, full: every row)
//   segsum  : signed segmented gather-sum of the rows (segsum_kernel<..., SIGNED>)
// V4: 8 consecutive rows per thread by 16-B loads (labels / prev 16-B aligned, block
// ranges multiples of 8): twice the bytes in flight of the 4-strided scalar form, which
// was latency-bound (80 MB in 22 us at 10M rows)
template <int NT, bool V4>
__global__ __launch_bounds__(NT) void delta_diff_kernel(
    const int32_t* __restrict__ labels, int32_t* __restrict__ prev, int64_t N, int K,
    int* __restrict__ ctrl, int* __restrict__ cnt_ev, int* __restrict__ cnt_sg,
    int* __restrict__ blk_cnt, int32_t* __restrict__ lidx, uint32_t* __restrict__ lpair,
    int64_t per_block, uint32_t* __restrict__ zero, int64_t zero_words) {
  extern __shared__ int s_h[];  // [K] events | [K] signed counts (delta steps), K <= DELTA_LDS_K
  __shared__ int s_cur;         // this block's moved-list cursor
  const int tid = threadIdx.x, lane = tid & 63;
  // the step's all-reduce buffer, cleared before anything accumulates into it (scan and
  // segsum run after this kernel)
  if (zero_words) zero_fill(zero, zero_words, (int64_t)blockIdx.x * NT + tid, (int64_t)gridDim.x * NT);
  if ((int64_t)blockIdx.x * per_block >= N) return;  // a block of the zero fill only
  const bool full = ctrl[TDC_DC_NEXT] != 0;
  // large K: the histograms are the global ones (a delta step touches few bins)
  const bool lds = K <= DELTA_LDS_K;
  int* h_ev = lds ? s_h : cnt_ev;
  int* h_sg = lds ? s_h + K : cnt_sg;
  if (lds)
    for (int k = tid; k < (full ? K : 2 * K); k += NT) s_h[k] = 0;
  if (tid == 0) s_cur = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = min(N, r0 + per_block);
  constexpr int R = V4 ? 8 : 4;  // rows per thread per chunk
  for (int64_t c0 = r0; c0 < r1; c0 += (int64_t)R * NT) {  // block-uniform trip count
    int nw[R], od[R];
    if constexpr (V4) {
      const int64_t i0 = c0 + (int64_t)R * tid;
#pragma unroll
      for (int q = 0; q < R / 4; ++q) {
        const int64_t iq = i0 + 4 * q;
        if (iq + 3 < r1) {
          const int4 a = *reinterpret_cast<const int4*>(labels + iq);
          const int4 b = *reinterpret_cast<const int4*>(prev + iq);
          nw[4 * q] = a.x; nw[4 * q + 1] = a.y; nw[4 * q + 2] = a.z; nw[4 * q + 3] = a.w;
          od[4 * q] = b.x; od[4 * q + 1] = b.y; od[4 * q + 2] = b.z; od[4 * q + 3] = b.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int64_t i = iq + e;
            nw[4 * q + e] = od[4 * q + e] = 0;
            if (i < r1) {
              nw[4 * q + e] = labels[i];
              od[4 * q + e] = prev[i];
            }
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const int64_t i = c0 + (int64_t)j * NT + tid;
        nw[j] = od[j] = 0;
        if (i < r1) {
          nw[j] = labels[i];
          od[j] = prev[i];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int64_t i = V4 ? c0 + (int64_t)R * tid + j : c0 + (int64_t)j * NT + tid;
      const bool ok = i < r1;
      const bool mv = ok && nw[j] != od[j];
      if (mv) prev[i] = nw[j];
      const bool nok = (unsigned)nw[j] < (unsigned)K, ook = (unsigned)od[j] < (unsigned)K;
      if (full) {
        if (ok && nok) atomicAdd(h_ev + nw[j], 1);
      } else if (mv) {
        if (nok) { atomicAdd(h_ev + nw[j], 1); atomicAdd(h_sg + nw[j], 1); }
        if (ook) { atomicAdd(h_ev + od[j], 1); atomicSub(h_sg + od[j], 1); }
      }
      // append: one LDS atomic per wave and row slot, positions by mbcnt of the ballot
      const unsigned long long mask = __ballot(mv);
      if (mask) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&s_cur, (int)__popcll(mask));
        base = __shfl(base, 0, 64);
        if (mv && !full) {
          const int pos = base + (int)__builtin_amdgcn_mbcnt_hi(
                                     (unsigned)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
          // labels travel in 16 bits (K <= 65536, where every 16-bit value is a label), so
          // an out-of-range label (none counted by the histograms above) is flagged in the
          // row word instead: bit 31 = no event at the new cluster, bit 30 = none at the old
          lidx[r0 + pos] = (int32_t)((uint32_t)i | (nok ? 0u : LIDX_NO_NEW) | (ook ? 0u : LIDX_NO_OLD));
          lpair[r0 + pos] = (((uint32_t)od[j] & 0xffffu) << 16) | ((uint32_t)nw[j] & 0xffffu);
        }
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    blk_cnt[blockIdx.x] = s_cur;
    if (s_cur) atomicAdd(ctrl + TDC_DC_MOVED, s_cur);  // one global atomic per block
  }
  if (lds)
    for (int k = tid; k < K; k += NT) {
      if (h_ev[k]) atomicAdd(cnt_ev + k, h_ev[k]);
      if (!full && h_sg[k]) atomicAdd(cnt_sg + k, h_sg[k]);
    }
}

// single block, 1024 threads: event offsets / cursors, the step's signed counts into the
// all-reduce buffer (acc dtype, plus the exact hi/lo split: hi = c >> 12 is a floor for
// negative c, so 4096 hi + lo == c still holds), the moved count into its slot
template <typename ACC>
__global__ __launch_bounds__(1024) void delta_scan_kernel(int* __restrict__ cnt_ev,
                                                          int* __restrict__ cnt_sg, int K,
                                                          int* __restrict__ offsets,
                                                          int* __restrict__ cursor,
                                                          int* __restrict__ ctrl,
                                                          ACC* __restrict__ counts_acc,
                                                          float* __restrict__ cnt_hi,
                                                          float* __restrict__ cnt_lo,
                                                          ACC* __restrict__ mslot) {
  const int tid = threadIdx.x;
  const bool full = ctrl[TDC_DC_NEXT] != 0;
  const int per = (K + 1023) / 1024;
  const int k0 = tid * per, k1 = min(K, k0 + per);
  int s = 0;
  for (int k = k0; k < k1; ++k) s += cnt_ev[k];
  const int inc = block_inclusive_scan_1024(s);
  int run = inc - s;
  for (int k = k0; k < k1; ++k) {
    const int e = cnt_ev[k];
    const int c = full ? e : cnt_sg[k];
    cnt_ev[k] = 0;  // both histograms are left zeroed for the next step
    cnt_sg[k] = 0;
    offsets[k] = run;
    cursor[k] = run;
    if (counts_acc) counts_acc[k] += (ACC)c;
    if (cnt_hi && c) {
      cnt_hi[k] += (float)(c >> 12);
      cnt_lo[k] += (float)(c & 4095);
    }
    run += e;
  }
  if (tid == 1023) {
    offsets[K] = inc;
    ctrl[TDC_DC_EVENTS] = inc;
  }
  if (tid == 0) {
    ctrl[TDC_DC_MODE] = full ? 1 : 0;
    const int m = ctrl[TDC_DC_MOVED];
    ctrl[TDC_DC_MOVED] = 0;
    if (mslot) *mslot += (ACC)m;
  }
}

// counting-sort placement of the step's events: a full step places every row (as
// bscatter_kernel, with the same bin-range passes), a delta step the entries of its
// block's moved list, each twice: row at its new cluster, row | PERM_NEG at its old one
template <int NT>
__global__ __launch_bounds__(NT) void delta_scatter_kernel(
    const int32_t* __restrict__ labels, int64_t N, int K, const int* __restrict__ ctrl,
    const int* __restrict__ blk_cnt, const int32_t* __restrict__ lidx,
    const uint32_t* __restrict__ lpair, int* __restrict__ cursor, int32_t* __restrict__ perm,
    int64_t per_block, int parts) {
  extern __shared__ int s_mem[];
  int* s_cnt = s_mem;
  int* s_cur = s_mem + K;
  const int tid = threadIdx.x;
  const bool full = ctrl[TDC_DC_MODE] != 0;
  const int64_t r0 = (int64_t)blockIdx.x * per_block;
  const int64_t r1 = full ? min(N, r0 + per_block) : r0 + blk_cnt[blockIdx.x];
  if (r0 >= r1) return;  // block-uniform: nothing moved in this block's rows
  if (K > DELTA_LDS_K) {
    // large K: one returning global cursor atomic per event (no block aggregation)
    if (full) {
      for (int64_t i = r0 + tid; i < r1; i += NT) {
        const int a = labels[i];
        if ((unsigned)a < (unsigned)K) perm[atomicAdd(cursor + a, 1)] = (int32_t)i;
      }
    } else {
      for (int64_t i = r0 + tid; i < r1; i += NT) {
        const uint32_t pr = lpair[i];
        const unsigned nw = pr & 0xffffu, od = pr >> 16;
        const uint32_t li = (uint32_t)lidx[i];
        const int32_t row = (int32_t)(li & LIDX_ROW);
        if (!(li & LIDX_NO_NEW) && nw < (unsigned)K) perm[atomicAdd(cursor + nw, 1)] = row;
        if (!(li & LIDX_NO_OLD) && od < (unsigned)K)
          perm[atomicAdd(cursor + od, 1)] = (int32_t)((uint32_t)row | PERM_NEG);
      }
    }
    return;
  }
  for (int k = tid; k < K; k += NT) s_cnt[k] = 0;
  __syncthreads();
  if (full) {
    for (int64_t i = r0 + tid; i < r1; i += NT) {
      const int a = labels[i];
      if ((unsigned)a < (unsigned)K) atomicAdd(s_cnt + a, 1);
    }
  } else {
    for (int64_t i = r0 + tid; i < r1; i += NT) {
      const uint32_t pr = lpair[i];
      const unsigned nw = pr & 0xffffu, od = pr >> 16;
      const uint32_t li = (uint32_t)lidx[i];
      if (!(li & LIDX_NO_NEW) && nw < (unsigned)K) atomicAdd(s_cnt + nw, 1);
      if (!(li & LIDX_NO_OLD) && od < (unsigned)K) atomicAdd(s_cnt + od, 1);
    }
  }
  __syncthreads();
  for (int k = tid; k < K; k += NT) {
    const int c = s_cnt[k];
    s_cur[k] = c ? atomicAdd(cursor + k, c) : 0;
  }
  __syncthreads();
  if (full) {
    for (int part = 0; part < parts; ++part) {
      const unsigned lo = (unsigned)((int64_t)K * part / parts);
      const unsigned n = (unsigned)((int64_t)K * (part + 1) / parts) - lo;
      for (int64_t i = r0 + tid; i < r1; i += NT) {
        const int a = labels[i];
        if ((unsigned)a - lo < n) perm[atomicAdd(s_cur + a, 1)] = (int32_t)i;
      }
    }
  } else {
    for (int64_t i = r0 + tid; i < r1; i += NT) {
      const uint32_t pr = lpair[i];
      const unsigned nw = pr & 0xffffu, od = pr >> 16;
      const uint32_t li = (uint32_t)lidx[i];
      const int32_t row = (int32_t)(li & LIDX_ROW);
      if (!(li & LIDX_NO_NEW) && nw < (unsigned)K) perm[atomicAdd(s_cur + nw, 1)] = row;
      if (!(li & LIDX_NO_OLD) && od < (unsigned)K)
        perm[atomicAdd(s_cur + od, 1)] = (int32_t)((uint32_t)row | PERM_NEG);
    }
  }
}

}  // namespace tdc

using namespace tdc;

namespace {

template <typename XT, typename ACC, int VEC, bool SIGNED>
int launch_segsum(const void* X, int64_t ldx, int D, const int32_t* perm, const int* offsets,
                  int K, int64_t N, void* sums, int num_cus, hipStream_t s,
                  const int* nptr, double fixed_scale) {
  const int lanes_needed = (D + VEC - 1) / VEC;
  (void)num_cus;
  const size_t lds = K + 1 <= SEG_LDS_OFF_MAX ? sizeof(int) * (size_t)(K + 1) : 0;
  // every wave gets the same row count, so the grid is exactly the waves resident at once
  // (8 blocks per CU asked for 8 waves per SIMD where the kernel fits 5: a second, partial
  // round of blocks).  With nptr (entry count on the device, at most N) the grid is sized
  // for N and the waves re-split the actual count.
#define TDC_SEG(TPRV)                                                                       \
  do {                                                                                      \
    static const int64_t res = resident_blocks(segsum_kernel<XT, ACC, VEC, TPRV, SIGNED>, 256); \
    int64_t waves = res * 4;                                                                \
    int64_t rpw = (N + waves - 1) / waves;                                                  \
    if (rpw < 64) rpw = 64; /* small N (mini-batches, moved rows) */                        \
    waves = (N + rpw - 1) / rpw;                                                            \
    const dim3 grid((unsigned)((waves + 3) / 4));                                           \
    hipLaunchKernelGGL((segsum_kernel<XT, ACC, VEC, TPRV, SIGNED>), grid, dim3(256), lds, s, \
                       (const XT*)X, ldx, D, perm, offsets, K, N, (ACC*)sums, rpw, nptr,    \
                       fixed_scale);                                                        \
  } while (0)
  if (lanes_needed <= 4) TDC_SEG(4);
  else if (lanes_needed <= 8) TDC_SEG(8);
  else if (lanes_needed <= 16) TDC_SEG(16);
  else if (lanes_needed <= 32) TDC_SEG(32);
  else TDC_SEG(64);
#undef TDC_SEG
  TDC_CHECK_LAUNCH();
  return 0;
}

template <typename ACC, bool SIGNED = false>
int dispatch_segsum(int x_dtype, const void* X, int64_t ldx, int D, const int32_t* perm,
                    const int* offsets, int K, int64_t N, void* sums, int num_cus, hipStream_t s,
                    const int* nptr = nullptr, double fixed_scale = 0.0) {
  const bool a16 = ((uintptr_t)X % 16) == 0;
#define TDC_SEGD(T, V)                                                                     \
  return launch_segsum<T, ACC, V, SIGNED>(X, ldx, D, perm, offsets, K, N, sums, num_cus, s, \
                                          nptr, fixed_scale)
  if (x_dtype == TDC_BF16) {
    if (a16 && D % 8 == 0 && ldx % 8 == 0) TDC_SEGD(__bf16, 8);
    TDC_SEGD(__bf16, 1);
  }
  if (x_dtype == TDC_F32) {
    if (a16 && D % 4 == 0 && ldx % 4 == 0) TDC_SEGD(float, 4);
    TDC_SEGD(float, 1);
  }
  if (x_dtype == TDC_F64) {
    if (a16 && D % 2 == 0 && ldx % 2 == 0) TDC_SEGD(double, 2);
    TDC_SEGD(double, 1);
  }
#undef TDC_SEGD
  return (int)hipErrorInvalidValue;
}

}  // namespace

int tdc_update_sorted(int x_dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                      const int32_t* labels, int K, void* sums, void* counts, int* work,
                      int num_cus, hipStream_t s, const int32_t* rowidx, float* cnt_hi,
                      float* cnt_lo, void* zero_first, int64_t zero_bytes, double fixed_scale,
                      int work_clean) {
  if (zero_bytes % 4 != 0 || (zero_bytes > 0 && zero_first == nullptr))
    return (int)hipErrorInvalidValue;
  if (acc_dtype != TDC_F32 && acc_dtype != TDC_F64 && acc_dtype != TDC_I64)
    return (int)hipErrorInvalidValue;
  if (acc_dtype == TDC_I64 && !(fixed_scale > 0.0)) return (int)hipErrorInvalidValue;
  if (N <= 0) {
    if (zero_bytes && hipMemsetAsync(zero_first, 0, (size_t)zero_bytes, s) != hipSuccess)
      return (int)hipErrorUnknown;
    return 0;
  }
  if (N >= (int64_t)1 << 31) return (int)hipErrorInvalidValue;
  // workspace layout (ints): cnt[K] | offsets[K+1] | cursor[K] | perm[N]; cnt is zero on
  // entry (a zero-filled workspace) and the scan leaves it zero
  int* cnt = work;
  int* offsets = cnt + K;
  int* cursor = offsets + K + 1;
  int32_t* perm = cursor + K;
  if (!work_clean && hipMemsetAsync(cnt, 0, sizeof(int) * (size_t)K, s) != hipSuccess)
    return (int)hipErrorUnknown;
  {
    // one 1024-thread block per CU: a quarter of the global flush atomics of 4 x 256-thread
    // blocks per CU (each block adds its whole LDS histogram into cnt)
    int64_t blocks = (int64_t)num_cus;
    int64_t per = (N + blocks - 1) / blocks;
    if (per < 4096) per = 4096;
    blocks = (N + per - 1) / per;
    // extra blocks for a large zero fill next to a small row range (they only clear)
    blocks = std::max(blocks, (zero_bytes / 4 + ZERO_WORDS_PER_BLOCK - 1) / ZERO_WORDS_PER_BLOCK);
    const size_t lds = K <= LDS_HIST_MAX_K ? sizeof(int) * (size_t)K : 0;
    hipLaunchKernelGGL(hist_kernel<1024>, dim3((unsigned)blocks), dim3(1024), lds, s, labels, N, K,
                       cnt, per, static_cast<uint32_t*>(zero_first), zero_bytes / 4);
    TDC_CHECK_LAUNCH();
  }
  if (acc_dtype == TDC_F64)
    hipLaunchKernelGGL(scan_kernel<double>, dim3(1), dim3(1024), 0, s, cnt, K, offsets, cursor,
                       (double*)counts, cnt_hi, cnt_lo);
  else if (acc_dtype == TDC_I64)
    hipLaunchKernelGGL(scan_kernel<long long>, dim3(1), dim3(1024), 0, s, cnt, K, offsets,
                       cursor, (long long*)counts, cnt_hi, cnt_lo);
  else
    hipLaunchKernelGGL(scan_kernel<float>, dim3(1), dim3(1024), 0, s, cnt, K, offsets, cursor,
                       (float*)counts, cnt_hi, cnt_lo);
  TDC_CHECK_LAUNCH();
  if (K <= LDS_HIST_MAX_K) {
    // one 1024-thread block per CU: 16 waves keep the LDS-rank -> store chains in flight
    // (2 x 256-thread blocks per CU measured 122 us at N=10M, K=1024); still one
    // reservation atomic per non-empty bin per block
    // (fewer, fuller blocks at small N -- 1, 4, 8 or 16 labels per bin per block at
    // N=1.25M, K=1024 -- measured the same: the per-block K-bin passes are not the cost)
    int64_t blocks = (int64_t)num_cus;
    int64_t per = (N + blocks - 1) / blocks;
    if (per < 4096) per = 4096;
    blocks = (N + per - 1) / per;
    // bin-range passes: the XCD's 32 blocks each write ~per/K entries into each of K perm
    // segments; with K=1024 at N=10M that is ~5 MB of lines in flight per XCD (4 MB L2)
    const int parts = K >= 512 && per >= 8 * (int64_t)K ? 2 : 1;
    hipLaunchKernelGGL(bscatter_kernel<1024>, dim3((unsigned)blocks), dim3(1024),
                       2 * sizeof(int) * (size_t)K, s, labels, N, K, cursor, perm, per, rowidx,
                       parts);
    TDC_CHECK_LAUNCH();
  } else {
    int64_t blocks = (int64_t)num_cus * 4;
    int64_t per = (N + blocks - 1) / blocks;
    per = ((per + 4095) / 4096) * 4096;
    blocks = (N + per - 1) / per;
    hipLaunchKernelGGL(scatter_kernel, dim3((unsigned)blocks), dim3(256), 0, s, labels, N, K,
                       cursor, perm, per, rowidx);
    TDC_CHECK_LAUNCH();
  }
  if (acc_dtype == TDC_F64)
    return dispatch_segsum<double>(x_dtype, X, ldx, D, perm, offsets, K, N, sums, num_cus, s);
  if (acc_dtype == TDC_I64)
    return dispatch_segsum<long long>(x_dtype, X, ldx, D, perm, offsets, K, N, sums, num_cus, s,
                                      nullptr, fixed_scale);
  return dispatch_segsum<float>(x_dtype, X, ldx, D, perm, offsets, K, N, sums, num_cus, s);
}

int64_t tdc_update_sorted_workspace(int64_t N, int K) { return 3 * (int64_t)K + 1 + N; }


int64_t tdc_delta_workspace(int64_t N, int K) {
  return 4 * (int64_t)K + 1 + TDC_DELTA_MAX_BLOCKS + 4 * N;
}

int tdc_delta_update(int x_dtype, int acc_dtype, const void* X, int64_t N, int64_t ldx, int D,
                     const int32_t* labels, int32_t* prev, int K, void* sums, void* counts,
                     int* work, int* ctrl, int num_cus, hipStream_t s, float* cnt_hi,
                     float* cnt_lo, void* moved, void* zero_first, int64_t zero_bytes,
                     double fixed_scale, int work_clean) {
  if (zero_bytes % 4 != 0 || (zero_bytes > 0 && zero_first == nullptr))
    return (int)hipErrorInvalidValue;
  if (acc_dtype == TDC_I64 && !(fixed_scale > 0.0)) return (int)hipErrorInvalidValue;
  // events are < 2N and perm entries carry the sign in bit 31; lpair packs 16-bit labels
  if (K <= 0 || K > TDC_DELTA_MAX_K || N >= ((int64_t)1 << 30)) return (int)hipErrorInvalidValue;
  if (acc_dtype != TDC_F32 && acc_dtype != TDC_F64 && acc_dtype != TDC_I64)
    return (int)hipErrorInvalidValue;
  // workspace (ints): cnt_ev[K] | cnt_sg[K] | offsets[K+1] | cursor[K] | blk_cnt[MAXB] |
  // lidx[N] | lpair[N] | perm[2N]; the histograms are zero on entry and left zero
  int* cnt_ev = work;
  int* cnt_sg = cnt_ev + K;
  int* offsets = cnt_sg + K;
  int* cursor = offsets + K + 1;
  int* blk_cnt = cursor + K;
  int32_t* lidx = blk_cnt + TDC_DELTA_MAX_BLOCKS;
  uint32_t* lpair = reinterpret_cast<uint32_t*>(lidx + N);
  int32_t* perm = reinterpret_cast<int32_t*>(lpair + N);
  if (!work_clean && hipMemsetAsync(cnt_ev, 0, 2 * sizeof(int) * (size_t)K, s) != hipSuccess)
    return (int)hipErrorUnknown;
  // one 1024-thread block per CU over contiguous row ranges (the diff and scatter kernels
  // share this geometry: block b's moved list lives at [b * per, b * per + blk_cnt[b]))
  int64_t blocks = std::max(1, std::min(num_cus, TDC_DELTA_MAX_BLOCKS));
  int64_t per = (N + blocks - 1) / blocks;
  if (per < 4096) per = 4096;
  per = (per + 7) / 8 * 8;  // block ranges start 32-B aligned (the V4 diff kernel)
  blocks = N > 0 ? (N + per - 1) / per : 0;
  const bool v4 = (((uintptr_t)labels | (uintptr_t)prev) & 15) == 0;
  const size_t lds = K <= DELTA_LDS_K ? 2 * sizeof(int) * (size_t)K : 0;
  if (blocks > 0) {
    const int64_t gblocks =
        std::max(blocks, (zero_bytes / 4 + ZERO_WORDS_PER_BLOCK - 1) / ZERO_WORDS_PER_BLOCK);
    if (v4)
      hipLaunchKernelGGL((delta_diff_kernel<1024, true>), dim3((unsigned)gblocks), dim3(1024), lds,
                         s, labels, prev, N, K, ctrl, cnt_ev, cnt_sg, blk_cnt, lidx, lpair, per,
                         static_cast<uint32_t*>(zero_first), zero_bytes / 4);
    else
      hipLaunchKernelGGL((delta_diff_kernel<1024, false>), dim3((unsigned)gblocks), dim3(1024), lds,
                         s, labels, prev, N, K, ctrl, cnt_ev, cnt_sg, blk_cnt, lidx, lpair, per,
                         static_cast<uint32_t*>(zero_first), zero_bytes / 4);
    TDC_CHECK_LAUNCH();
  } else if (zero_bytes && hipMemsetAsync(zero_first, 0, (size_t)zero_bytes, s) != hipSuccess) {
    return (int)hipErrorUnknown;
  }
  if (acc_dtype == TDC_F64)
    hipLaunchKernelGGL(delta_scan_kernel<double>, dim3(1), dim3(1024), 0, s, cnt_ev, cnt_sg, K,
                       offsets, cursor, ctrl, (double*)counts, cnt_hi, cnt_lo, (double*)moved);
  else if (acc_dtype == TDC_I64)
    hipLaunchKernelGGL(delta_scan_kernel<long long>, dim3(1), dim3(1024), 0, s, cnt_ev, cnt_sg,
                       K, offsets, cursor, ctrl, (long long*)counts, cnt_hi, cnt_lo,
                       (long long*)moved);
  else
    hipLaunchKernelGGL(delta_scan_kernel<float>, dim3(1), dim3(1024), 0, s, cnt_ev, cnt_sg, K,
                       offsets, cursor, ctrl, (float*)counts, cnt_hi, cnt_lo, (float*)moved);
  TDC_CHECK_LAUNCH();
  if (blocks == 0) return 0;
  const int parts = K >= 512 && per >= 8 * (int64_t)K ? 2 : 1;
  hipLaunchKernelGGL(delta_scatter_kernel<1024>, dim3((unsigned)blocks), dim3(1024), lds, s,
                     labels, N, K, ctrl, blk_cnt, lidx, lpair, cursor, perm, per, parts);
  TDC_CHECK_LAUNCH();
  // grid sized for a full step (N events); a delta step re-splits its 2M events on device
  if (acc_dtype == TDC_F64)
    return dispatch_segsum<double, true>(x_dtype, X, ldx, D, perm, offsets, K, N, sums, num_cus,
                                         s, ctrl + TDC_DC_EVENTS);
  if (acc_dtype == TDC_I64)
    return dispatch_segsum<long long, true>(x_dtype, X, ldx, D, perm, offsets, K, N, sums,
                                            num_cus, s, ctrl + TDC_DC_EVENTS, fixed_scale);
  return dispatch_segsum<float, true>(x_dtype, X, ldx, D, perm, offsets, K, N, sums, num_cus, s,
                                      ctrl + TDC_DC_EVENTS);
}
