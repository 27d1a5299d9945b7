// Membership arithmetic shared by the FCM kernels (fcm.hip, fcm_tower.hip, fcm_mfma.hip).
// Reference op chain: scripts/distribuitedClustering.py:117-129 (Sqrt, Pow(d, -2/(M-1)),
// row normalise, NaN -> 0, Pow(u, M)).
#pragma once
#include "tdc_common.h"

namespace tdc {

__device__ __forceinline__ float tdc_exp2(float v) { return exp2f(v); }
__device__ __forceinline__ double tdc_exp2(double v) { return exp2(v); }
__device__ __forceinline__ float tdc_log2(float v) { return log2f(v); }
__device__ __forceinline__ double tdc_log2(double v) { return log2(v); }

// t = (d^2)^expo, expo = -1/(m-1).  pmode picks a transcendental-free form for the common
// fuzzifiers: 1: m=2 (1/d2), 2: m=3 (1/sqrt d2), 3: m=5 (the reference's m = D = 5:
// 1/sqrt(sqrt d2)); 0: exp2(expo * log2 d2).
__device__ __forceinline__ float fcm_rcp(float v) { return __builtin_amdgcn_rcpf(v); }
__device__ __forceinline__ double fcm_rcp(double v) { return 1.0 / v; }

// fp32: v_rcp_f32 (1 ulp) instead of the IEEE division sequence; fp64 stays exact
template <typename T>
__device__ __forceinline__ T fcm_t(T dd, T expo, int pmode) {
  switch (pmode) {
    case 1: return fcm_rcp(dd);
    case 2: return rsqrt(dd);          // one rsqrt instead of sqrt + divide
    case 3: return rsqrt(sqrt(dd));
    default: return tdc_exp2(tdc_log2(dd) * expo);
  }
}

// dd^(-1/P) for finite dd > 0, P in {1, 2, 4}, fp64 to a few ulp: the exponent is split
// off (dd = r 2^(P q), r in [0.5, 2^P)), r^(-1/P) is seeded in fp32 (~1e-7) and refined by
// two Newton steps on y^-P = r, y <- y ((P+1) - r y^P) / P.  ~16 fp64 operations and no
// branches, against ~40 for the correctly rounded divide / sqrt / rsqrt sequences.
// dd = 0 gives NaN: callers select +inf for on-centroid rows before using it.
template <int P>
__device__ __forceinline__ double root_rcp(double dd) {
  static_assert(P == 1 || P == 2 || P == 4, "root_rcp: P in {1, 2, 4}");
  const int e = __builtin_amdgcn_frexp_exp(dd);
  const int q = P == 1 ? e : (P == 2 ? (e >> 1) : (e >> 2));  // floor(e / P)
  const double r = __builtin_amdgcn_ldexp(dd, -P * q);
  const float rf = (float)r;
  double y;
  if constexpr (P == 1) y = (double)__builtin_amdgcn_rcpf(rf);
  else if constexpr (P == 2) y = (double)__builtin_amdgcn_rsqf(rf);
  else y = (double)__builtin_amdgcn_rsqf(__builtin_amdgcn_sqrtf(rf));  // raw v_sqrt_f32: a seed
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    if constexpr (P == 1) {
      y = y * fma(-r, y, 2.0);
    } else if constexpr (P == 2) {
      y = y * fma(-r, y * y, 3.0) * 0.5;
    } else {
      const double y2 = y * y;
      y = y * fma(-r, y2 * y2, 5.0) * 0.25;
    }
  }
  return __builtin_amdgcn_ldexp(y, -q);
}

// Compile-time fuzzifier forms (the fused small-K kernel): FM = 2 (m = 2), 5 (m = 5, the
// reference's m = D = 5 configs) or 0 (any m: exp2 / log2).  t = (d^2)^(-1/(m-1)), w = u^m.
template <int FM>
__device__ __forceinline__ float fm_t(float dd, float expo) {
  if constexpr (FM == 2) return __builtin_amdgcn_rcpf(dd);
  else if constexpr (FM == 5) return __builtin_amdgcn_rsqf(__builtin_sqrtf(dd));
  else return exp2f(log2f(dd) * expo);
}
// 1 / dd in fp64 for finite dd > 0: the v_rcp_f64 estimate refined by two Newton steps
// (5 fp64 operations against root_rcp<1>'s ~9), with root_rcp's exponent split kept for
// dd whose reciprocal leaves the normal range
__device__ __forceinline__ double rcp_f64_nr(double dd) {
  double y = __builtin_amdgcn_rcp(dd);
  y = fma(y, fma(-dd, y, 1.0), y);
  y = fma(y, fma(-dd, y, 1.0), y);
  return (dd > 0x1p-1000 && dd < 0x1p1000) ? y : root_rcp<1>(dd);
}

template <int FM>
__device__ __forceinline__ double fm_t(double dd, double expo) {
  if constexpr (FM == 2) return rcp_f64_nr(dd);
  else if constexpr (FM == 5) return root_rcp<4>(dd);
  else return exp2(log2(dd) * expo);
}
template <int FM, typename T>
__device__ __forceinline__ T fm_w(T u, T m) {
  if constexpr (FM == 2) {
    return u * u;
  } else if constexpr (FM == 5) {
    const T u2 = u * u;
    return u2 * u2 * u;
  } else {
    return u > (T)0 ? tdc_exp2(m * tdc_log2(u)) : (T)0;
  }
}
inline int fcm_fm(double m) { return m == 2.0 ? 2 : (m == 5.0 ? 5 : 0); }

// w = u^m: binary powering for integer m in [1, 16] (mint), else exp2(m log2 u)
template <typename T>
__device__ __forceinline__ T fcm_w(T u, T m, int mint) {
  if (mint > 0) {
    T r = (mint & 1) ? u : (T)1;
    T b = u;
#pragma unroll
    for (int e = mint >> 1; e > 0; e >>= 1) {
      b = b * b;
      if (e & 1) r = r * b;
    }
    return r;
  }
  return u > (T)0 ? tdc_exp2(m * tdc_log2(u)) : (T)0;
}

// pmode / mint of a fuzzifier m (host side): see fcm_t / fcm_w
inline int fcm_pmode(double m) { return m == 2.0 ? 1 : (m == 3.0 ? 2 : (m == 5.0 ? 3 : 0)); }
inline int fcm_mint(double m) { return (m == (double)(int)m && m >= 1.0 && m <= 16.0) ? (int)m : 0; }

}  // namespace tdc
