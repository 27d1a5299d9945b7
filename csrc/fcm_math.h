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
