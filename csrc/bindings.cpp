// torch.ops.tdc.* custom ops over the HIP launchers in kernels.h.
// Out-parameter style (no allocation inside an op) so an iteration can be captured into
// a HIP graph and so the engine owns every buffer (one packed comm buffer per run).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <mutex>
#include <unordered_map>

#include "kernels.h"

namespace {

// PyTorch-ROCm exposes HIP devices as device type "cuda" ("masquerading"): use the
// masquerading guard/stream so we launch on exactly torch.cuda.current_stream().
hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DevGuard = at::hip::HIPGuardMasqueradingAsCUDA;

int num_cus(int dev) {
  static std::mutex mu;
  static std::unordered_map<int, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
    v = 256;
  cache[dev] = v;
  return v;
}

int dcode(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return TDC_F32;
    case at::kDouble: return TDC_F64;
    case at::kBFloat16: return TDC_BF16;
    case at::kLong: return TDC_I64;  // fixed-point accumulation (deterministic update)
    default: TORCH_CHECK(false, "tdc: unsupported dtype ", t);
  }
  return -1;
}

void check(int err, const char* what) {
  TORCH_CHECK(err == 0, "tdc: ", what, " failed: ", hipGetErrorString((hipError_t)err),
              " (code ", err, ")");
}

void check_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "tdc: ", name, " must be a GPU tensor");
}

void* opt_ptr(const std::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}

void check_rows(const at::Tensor& X, const char* name) {
  TORCH_CHECK(X.dim() == 2, "tdc: ", name, " must be 2-D");
  TORCH_CHECK(X.stride(1) == 1, "tdc: ", name, " rows must be contiguous");
}

// ------------------------------------------------------------------------------------
void assign_bf16(const at::Tensor& X, const at::Tensor& Cm2, const at::Tensor& cnorm,
                 at::Tensor& labels, const std::optional<at::Tensor>& mind) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 && Cm2.scalar_type() == at::kBFloat16,
              "tdc.assign_bf16: X and Cm2 must be bfloat16");
  TORCH_CHECK(cnorm.scalar_type() == at::kFloat && labels.scalar_type() == at::kInt,
              "tdc.assign_bf16: cnorm fp32, labels int32");
  TORCH_CHECK(Cm2.is_contiguous() && cnorm.is_contiguous() && labels.is_contiguous(),
              "tdc.assign_bf16: Cm2/cnorm/labels must be contiguous");
  const int64_t N = X.size(0);
  const int DP = (int)Cm2.size(1);
  const int Kp = (int)Cm2.size(0);
  TORCH_CHECK(DP == 32 || DP == 64 || DP == 128 || DP == 256,
              "tdc.assign_bf16: padded dim must be 32/64/128/256, got ", DP);
  TORCH_CHECK(X.size(1) >= DP, "tdc.assign_bf16: X has fewer columns than Cm2");
  TORCH_CHECK(X.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(X.data_ptr()) % 16) == 0,
              "tdc.assign_bf16: X rows must be 16-byte aligned");
  TORCH_CHECK(Kp % 64 == 0 && cnorm.numel() >= Kp, "tdc.assign_bf16: Kp must be a multiple of 64");
  TORCH_CHECK(labels.numel() >= N, "tdc.assign_bf16: labels too small");
  float* md = nullptr;
  if (mind.has_value() && mind->defined()) {
    TORCH_CHECK(mind->scalar_type() == at::kFloat && mind->numel() >= N && mind->is_contiguous(),
                "tdc.assign_bf16: mind must be fp32 [N]");
    md = mind->data_ptr<float>();
  }
  const DevGuard guard(X.device());
  check(tdc_assign_mfma_bf16(X.data_ptr(), N, X.stride(0), DP, Cm2.data_ptr(),
                             cnorm.data_ptr<float>(), Kp, labels.data_ptr<int32_t>(), md,
                             cur_stream()),
        "assign_bf16");
}

void assign_simt(const at::Tensor& X, const at::Tensor& C, at::Tensor& labels,
                 const std::optional<at::Tensor>& mind) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous(), "tdc.assign_simt: C");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.numel() >= X.size(0), "tdc.assign_simt: labels");
  const DevGuard guard(X.device());
  check(tdc_assign_simt(dcode(X.scalar_type()), X.data_ptr(), X.size(0), X.stride(0),
                        (int)C.size(1), C.data_ptr(), (int)C.size(0), labels.data_ptr<int32_t>(),
                        opt_ptr(mind), cur_stream()),
        "assign_simt");
}

void assign_exact(const at::Tensor& X, const at::Tensor& C, at::Tensor& labels,
                  const std::optional<at::Tensor>& mind) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kFloat || X.scalar_type() == at::kDouble,
              "tdc.assign_exact: X fp32/fp64");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous() && C.dim() == 2 &&
                  C.size(1) == X.size(1), "tdc.assign_exact: C [K, D] in the X dtype");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= X.size(0),
              "tdc.assign_exact: labels int32 [N]");
  if (mind.has_value() && mind->defined())
    TORCH_CHECK(mind->scalar_type() == X.scalar_type() && mind->is_contiguous() &&
                    mind->numel() >= X.size(0), "tdc.assign_exact: mind [N] in the X dtype");
  const DevGuard guard(X.device());
  check(tdc_assign_exact(dcode(X.scalar_type()), X.data_ptr(), X.size(0), X.stride(0),
                         (int)X.size(1), C.data_ptr(), (int)C.size(0), labels.data_ptr<int32_t>(),
                         opt_ptr(mind), num_cus(X.device().index()), cur_stream()),
        "assign_exact");
}

bool lloyd_small_supported(at::ScalarType dtype, int64_t K, int64_t D) {
  if (dtype != at::kFloat && dtype != at::kDouble) return false;
  return tdc_lloyd_small_supported(dcode(dtype), (int)K, (int)D) != 0;
}

void lloyd_small(const at::Tensor& X, const at::Tensor& C, const std::optional<at::Tensor>& labels,
                 const std::optional<at::Tensor>& mind, at::Tensor& sums, at::Tensor& counts) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous() && X.size(1) == C.size(1),
              "tdc.lloyd_small: C");
  TORCH_CHECK(sums.scalar_type() == counts.scalar_type(), "tdc.lloyd_small: sums/counts dtype");
  TORCH_CHECK(sums.is_contiguous() && counts.is_contiguous(), "tdc.lloyd_small: contiguity");
  TORCH_CHECK(sums.numel() == C.numel() && counts.numel() == C.size(0),
              "tdc.lloyd_small: sums [K, D] / counts [K]");
  const int64_t n = X.size(0);
  if (labels) TORCH_CHECK(labels->numel() >= n && labels->is_contiguous(), "tdc.lloyd_small: labels");
  if (mind) TORCH_CHECK(mind->numel() >= n && mind->is_contiguous(), "tdc.lloyd_small: mind");
  const DevGuard guard(X.device());
  check(tdc_lloyd_small(dcode(X.scalar_type()), dcode(sums.scalar_type()), X.data_ptr(), n,
                        X.stride(0), (int)C.size(1), C.data_ptr(), (int)C.size(0),
                        labels ? labels->data_ptr<int32_t>() : nullptr, opt_ptr(mind),
                        sums.data_ptr(), counts.data_ptr(), cur_stream()),
        "lloyd_small");
}

void update(const at::Tensor& X, const at::Tensor& labels, at::Tensor& sums, at::Tensor& counts) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous(), "tdc.update: labels int32");
  TORCH_CHECK(sums.dim() == 2 && sums.is_contiguous() && counts.is_contiguous(), "tdc.update: sums");
  TORCH_CHECK(sums.scalar_type() == counts.scalar_type() && sums.scalar_type() != at::kLong,
              "tdc.update: sums/counts dtype (fp32/fp64; fixed point runs the sorted update)");
  TORCH_CHECK(X.size(1) >= sums.size(1), "tdc.update: X narrower than sums");
  TORCH_CHECK(labels.numel() >= X.size(0), "tdc.update: labels shorter than X");
  TORCH_CHECK(counts.numel() >= sums.size(0), "tdc.update: counts shorter than K");
  const DevGuard guard(X.device());
  check(tdc_update_lds(dcode(X.scalar_type()), dcode(sums.scalar_type()), X.data_ptr(), X.size(0),
                       X.stride(0), (int)sums.size(1), labels.data_ptr<int32_t>(),
                       (int)sums.size(0), sums.data_ptr(), counts.data_ptr(),
                       num_cus(X.device().index()), cur_stream()),
        "update");
}

int64_t update_sorted_workspace(int64_t N, int64_t K) { return tdc_update_sorted_workspace(N, (int)K); }

// exact count split (kernels.h): both or neither, fp32 [>= K]
void check_split(const std::optional<at::Tensor>& hi, const std::optional<at::Tensor>& lo,
                 int64_t K, const char* op) {
  const bool h = hi.has_value() && hi->defined(), l = lo.has_value() && lo->defined();
  TORCH_CHECK(h == l, "tdc.", op, ": cnt_hi and cnt_lo go together");
  if (!h) return;
  for (const auto* t : {&hi, &lo})
    TORCH_CHECK((*t)->scalar_type() == at::kFloat && (*t)->is_contiguous() && (*t)->numel() >= K,
                "tdc.", op, ": cnt_hi/cnt_lo must be contiguous fp32 [K]");
}

// int64 sums = fixed point: each element is truncated to (int32)(x * fixed_scale), so the
// caller's scale must keep max|x| * fixed_scale <= 2^30 (ops.fixed_point_scale does; the
// hardware conversion saturates beyond it) and max|x| * N * fixed_scale < 2^63.
void check_fixed(const at::Tensor& sums, double fixed_scale, const char* op) {
  if (sums.scalar_type() == at::kLong)
    TORCH_CHECK(fixed_scale > 0.0, "tdc.", op, ": int64 (fixed-point) sums need fixed_scale > 0");
}

void update_sorted(const at::Tensor& X, const at::Tensor& labels, at::Tensor& sums,
                   at::Tensor& counts, at::Tensor& work, const std::optional<at::Tensor>& cnt_hi,
                   const std::optional<at::Tensor>& cnt_lo,
                   const std::optional<at::Tensor>& zero_first, double fixed_scale,
                   bool work_clean) {
  check_fixed(sums, fixed_scale, "update_sorted");
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= X.size(0),
              "tdc.update_sorted: labels int32 [N]");
  TORCH_CHECK(sums.dim() == 2 && sums.is_contiguous() && counts.is_contiguous(), "tdc.update_sorted: sums");
  TORCH_CHECK(sums.scalar_type() == counts.scalar_type() && counts.numel() >= sums.size(0),
              "tdc.update_sorted: counts");
  TORCH_CHECK(X.size(1) >= sums.size(1), "tdc.update_sorted: X narrower than sums");
  TORCH_CHECK(work.scalar_type() == at::kInt && work.is_contiguous() &&
                  work.numel() >= tdc_update_sorted_workspace(X.size(0), (int)sums.size(0)),
              "tdc.update_sorted: workspace too small");
  check_split(cnt_hi, cnt_lo, sums.size(0), "update_sorted");
  int64_t zbytes = 0;
  if (zero_first.has_value() && zero_first->defined()) {
    TORCH_CHECK(zero_first->is_contiguous() && zero_first->device() == X.device() &&
                    (zero_first->numel() * zero_first->element_size()) % 4 == 0,
                "tdc.update_sorted: zero_first must be a contiguous device buffer of 4-byte words");
    zbytes = zero_first->numel() * zero_first->element_size();
  }
  const DevGuard guard(X.device());
  check(tdc_update_sorted(dcode(X.scalar_type()), dcode(sums.scalar_type()), X.data_ptr(),
                          X.size(0), X.stride(0), (int)sums.size(1), labels.data_ptr<int32_t>(),
                          (int)sums.size(0), sums.data_ptr(), counts.data_ptr(),
                          work.data_ptr<int>(), num_cus(X.device().index()), cur_stream(),
                          nullptr, static_cast<float*>(opt_ptr(cnt_hi)),
                          static_cast<float*>(opt_ptr(cnt_lo)), opt_ptr(zero_first), zbytes,
                          fixed_scale, work_clean ? 1 : 0),
        "update_sorted");
}

bool fcm_small_supported(at::ScalarType dtype, int64_t K, int64_t D) {
  if (dtype != at::kFloat && dtype != at::kDouble) return false;
  return tdc_fcm_small_supported(dcode(dtype), (int)K, (int)D) != 0;
}

void fcm_small(const at::Tensor& X, const at::Tensor& C, double m, bool nan_to_zero,
               const std::optional<at::Tensor>& labels, at::Tensor& wx, at::Tensor& ws) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous() && X.size(1) == C.size(1),
              "tdc.fcm_small: C");
  TORCH_CHECK(wx.scalar_type() == ws.scalar_type() && wx.is_contiguous() && ws.is_contiguous(),
              "tdc.fcm_small: wx/ws");
  TORCH_CHECK(wx.numel() == C.numel() && ws.numel() == C.size(0), "tdc.fcm_small: wx [K, D] / ws [K]");
  const int64_t n = X.size(0);
  if (labels) TORCH_CHECK(labels->numel() >= n && labels->is_contiguous(), "tdc.fcm_small: labels");
  const DevGuard guard(X.device());
  check(tdc_fcm_small(dcode(X.scalar_type()), dcode(wx.scalar_type()), X.data_ptr(), n,
                      X.stride(0), (int)C.size(1), C.data_ptr(), (int)C.size(0), m,
                      nan_to_zero ? 1 : 0, labels ? labels->data_ptr<int32_t>() : nullptr,
                      wx.data_ptr(), ws.data_ptr(), cur_stream()),
        "fcm_small");
}

void fcm_tower_stats(const at::Tensor& X, const at::Tensor& C, double m, bool nan_to_zero,
                     at::Tensor& labels, at::Tensor& rowinfo) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kFloat || X.scalar_type() == at::kDouble,
              "tdc.fcm_tower_stats: X fp32/fp64");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous() && C.dim() == 2 &&
                  C.size(1) == X.size(1), "tdc.fcm_tower_stats: C [K, D] in the X dtype");
  TORCH_CHECK(X.size(1) >= 1 && X.size(1) <= 256, "tdc.fcm_tower_stats: D must be 1..256");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= X.size(0),
              "tdc.fcm_tower_stats: labels int32 [N]");
  TORCH_CHECK(rowinfo.scalar_type() == X.scalar_type() && rowinfo.is_contiguous() &&
                  rowinfo.numel() >= X.size(0), "tdc.fcm_tower_stats: rowinfo [N] in the X dtype");
  TORCH_CHECK(m > 1.0, "tdc.fcm_tower_stats: fuzzifier must be > 1");
  const DevGuard guard(X.device());
  check(tdc_fcm_tower(0, dcode(X.scalar_type()), X.data_ptr(), X.size(0), X.stride(0),
                      (int)X.size(1), C.data_ptr(), (int)C.size(0), m, nan_to_zero ? 1 : 0,
                      labels.data_ptr<int32_t>(), rowinfo.data_ptr(), nullptr, nullptr,
                      num_cus(X.device().index()), cur_stream()),
        "fcm_tower_stats");
}

void fcm_tower_accum(const at::Tensor& X, const at::Tensor& C, double m, bool nan_to_zero,
                     const at::Tensor& rowinfo, at::Tensor& wx, at::Tensor& ws) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kFloat || X.scalar_type() == at::kDouble,
              "tdc.fcm_tower_accum: X fp32/fp64");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous() && C.dim() == 2 &&
                  C.size(1) == X.size(1), "tdc.fcm_tower_accum: C [K, D] in the X dtype");
  TORCH_CHECK(X.size(1) >= 1 && X.size(1) <= 256, "tdc.fcm_tower_accum: D must be 1..256");
  TORCH_CHECK(rowinfo.scalar_type() == X.scalar_type() && rowinfo.is_contiguous() &&
                  rowinfo.numel() >= X.size(0), "tdc.fcm_tower_accum: rowinfo [N]");
  TORCH_CHECK(wx.scalar_type() == at::kDouble && ws.scalar_type() == at::kDouble &&
                  wx.is_contiguous() && ws.is_contiguous() && wx.numel() == C.numel() &&
                  ws.numel() == C.size(0), "tdc.fcm_tower_accum: wx [K, D] / ws [K] fp64");
  TORCH_CHECK(m > 1.0, "tdc.fcm_tower_accum: fuzzifier must be > 1");
  const DevGuard guard(X.device());
  check(tdc_fcm_tower(1, dcode(X.scalar_type()), X.data_ptr(), X.size(0), X.stride(0),
                      (int)X.size(1), C.data_ptr(), (int)C.size(0), m, nan_to_zero ? 1 : 0,
                      nullptr, const_cast<void*>(rowinfo.data_ptr()), wx.data_ptr(), ws.data_ptr(),
                      num_cus(X.device().index()), cur_stream()),
        "fcm_tower_accum");
}

// pass 0: G = d2 of the chunk X against C; 1: labels + G <- w; 3: labels only; 2: wx/ws +=
void fcm_wide(int64_t pass, const at::Tensor& X, const at::Tensor& C, double m, bool nan_to_zero,
              at::Tensor& G, const std::optional<at::Tensor>& labels,
              const std::optional<at::Tensor>& wx, const std::optional<at::Tensor>& ws) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kFloat || X.scalar_type() == at::kDouble,
              "tdc.fcm_wide: X fp32/fp64");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous() && C.dim() == 2 &&
                  C.size(1) == X.size(1), "tdc.fcm_wide: C [K, D] in the X dtype");
  const int64_t M = X.size(0), K = C.size(0);
  TORCH_CHECK(G.scalar_type() == X.scalar_type() && G.is_contiguous() && G.numel() >= M * K,
              "tdc.fcm_wide: G [M, K] in the X dtype");
  TORCH_CHECK(m > 1.0, "tdc.fcm_wide: fuzzifier must be > 1");
  int32_t* lab = nullptr;
  if (pass == 1 || pass == 3) {
    TORCH_CHECK(labels.has_value() && labels->defined() && labels->scalar_type() == at::kInt &&
                    labels->is_contiguous() && labels->numel() >= M,
                "tdc.fcm_wide: labels int32 [M]");
    lab = labels->data_ptr<int32_t>();
  }
  double *pwx = nullptr, *pws = nullptr;
  if (pass == 2) {
    TORCH_CHECK(wx.has_value() && ws.has_value() && wx->scalar_type() == at::kDouble &&
                    ws->scalar_type() == at::kDouble && wx->is_contiguous() &&
                    ws->is_contiguous() && wx->numel() == C.numel() && ws->numel() == K,
                "tdc.fcm_wide: wx [K, D] / ws [K] fp64");
    pwx = wx->data_ptr<double>();
    pws = ws->data_ptr<double>();
  }
  TORCH_CHECK(pass >= 0 && pass <= 3, "tdc.fcm_wide: pass 0..3");
  const DevGuard guard(X.device());
  check(tdc_fcm_wide((int)pass, dcode(X.scalar_type()), X.data_ptr(), M, X.stride(0),
                     (int)X.size(1), C.data_ptr(), (int)K, m, nan_to_zero ? 1 : 0, G.data_ptr(),
                     lab, pwx, pws, num_cus(X.device().index()), cur_stream()),
        "fcm_wide");
}

// fp64 FCM with fused row statistics (kernels.h tdc_fcm_f64t): pass 0 G = t, rowinfo,
// labels; pass 1 wx / ws += W^T X / sum W with w from G and rowinfo
void fcm_f64t(int64_t pass, const at::Tensor& X, const at::Tensor& C, double m, bool nan_to_zero,
              at::Tensor& G, at::Tensor& rowinfo, const std::optional<at::Tensor>& labels,
              const std::optional<at::Tensor>& wx, const std::optional<at::Tensor>& ws) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kDouble, "tdc.fcm_f64t: X fp64");
  TORCH_CHECK(C.scalar_type() == at::kDouble && C.is_contiguous() && C.dim() == 2 &&
                  C.size(1) == X.size(1), "tdc.fcm_f64t: C [K, D] fp64");
  const int64_t M = X.size(0), K = C.size(0);
  TORCH_CHECK(G.scalar_type() == at::kDouble && G.is_contiguous() && G.numel() >= M * K,
              "tdc.fcm_f64t: G [M, K] fp64");
  TORCH_CHECK(rowinfo.scalar_type() == at::kDouble && rowinfo.is_contiguous() &&
                  rowinfo.numel() >= M, "tdc.fcm_f64t: rowinfo fp64 [M]");
  TORCH_CHECK(m > 1.0, "tdc.fcm_f64t: fuzzifier must be > 1");
  TORCH_CHECK(pass == 0 || pass == 1, "tdc.fcm_f64t: pass 0 or 1");
  int32_t* lab = nullptr;
  double *pwx = nullptr, *pws = nullptr;
  if (pass == 0) {
    TORCH_CHECK(labels.has_value() && labels->defined() && labels->scalar_type() == at::kInt &&
                    labels->is_contiguous() && labels->numel() >= M,
                "tdc.fcm_f64t: labels int32 [M]");
    lab = labels->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(wx.has_value() && ws.has_value() && wx->scalar_type() == at::kDouble &&
                    ws->scalar_type() == at::kDouble && wx->is_contiguous() &&
                    ws->is_contiguous() && wx->numel() == C.numel() && ws->numel() == K,
                "tdc.fcm_f64t: wx [K, D] / ws [K] fp64");
    pwx = wx->data_ptr<double>();
    pws = ws->data_ptr<double>();
  }
  const DevGuard guard(X.device());
  check(tdc_fcm_f64t((int)pass, X.data_ptr<double>(), M, X.stride(0), (int)X.size(1),
                     C.data_ptr<double>(), (int)K, m, nan_to_zero ? 1 : 0, G.data_ptr<double>(),
                     rowinfo.data_ptr<double>(), lab, pwx, pws, num_cus(X.device().index()),
                     cur_stream()),
        "fcm_f64t");
}

// the row pass of the wide towers alone (G [M, K] of d2 -> labels, and w in place)
void fcm_wide_rows(at::Tensor& G, int64_t K, double m, bool nan_to_zero, at::Tensor& labels,
                   bool write_w) {
  check_cuda(G, "G");
  TORCH_CHECK((G.scalar_type() == at::kFloat || G.scalar_type() == at::kDouble) &&
                  G.is_contiguous() && G.dim() == 2 && G.size(1) == K,
              "tdc.fcm_wide_rows: G [M, K] fp32/fp64");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() &&
                  labels.numel() >= G.size(0), "tdc.fcm_wide_rows: labels int32 [M]");
  TORCH_CHECK(m > 1.0, "tdc.fcm_wide_rows: fuzzifier must be > 1");
  const DevGuard guard(G.device());
  check(tdc_fcm_wide(write_w ? 1 : 3, dcode(G.scalar_type()), nullptr, G.size(0), 0, 1, nullptr,
                     (int)K, m, nan_to_zero ? 1 : 0, G.data_ptr(), labels.data_ptr<int32_t>(),
                     nullptr, nullptr, num_cus(G.device().index()), cur_stream()),
        "fcm_wide_rows");
}

int64_t fcm_mfma_wide_workspace(const at::Tensor& like, int64_t M, int64_t Kp, int64_t DP) {
  return tdc_fcm_mfma_wide_workspace(M, (int)Kp, (int)DP, num_cus(like.device().index()));
}

void fcm_mfma_wide(int64_t pass, const at::Tensor& Xh, const at::Tensor& Xl, const at::Tensor& xx,
                   const at::Tensor& Ch, const at::Tensor& Cl, const at::Tensor& cc, int64_t K,
                   int64_t D, at::Tensor& G, const std::optional<at::Tensor>& work,
                   const std::optional<at::Tensor>& shift, const std::optional<at::Tensor>& wx,
                   const std::optional<at::Tensor>& ws) {
  check_cuda(Xh, "Xh");
  const int64_t M = Xh.size(0), DP = Xh.size(1), Kp = Ch.size(0);
  for (const at::Tensor* t : {&Xh, &Xl, &Ch, &Cl})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 2 &&
                    t->size(1) == DP, "tdc.fcm_mfma_wide: hi/lo operands bf16 [rows, DP]");
  TORCH_CHECK(Xl.size(0) == M && Cl.size(0) == Kp, "tdc.fcm_mfma_wide: hi/lo row counts");
  TORCH_CHECK(DP % 128 == 0 && DP >= 128 && DP <= 1024 && Kp % 128 == 0 && Kp >= K && D <= DP,
              "tdc.fcm_mfma_wide: DP in 128..1024 (x128), Kp % 128 == 0");
  TORCH_CHECK(xx.scalar_type() == at::kFloat && xx.is_contiguous() && xx.numel() >= M &&
                  cc.scalar_type() == at::kFloat && cc.is_contiguous() && cc.numel() >= Kp,
              "tdc.fcm_mfma_wide: norms fp32");
  TORCH_CHECK(G.scalar_type() == at::kFloat && G.is_contiguous() && G.numel() >= M * K,
              "tdc.fcm_mfma_wide: G fp32 [M, K]");
  float* wk = nullptr;
  double *pwx = nullptr, *pws = nullptr;
  if (pass == 2) {
    TORCH_CHECK(work.has_value() && work->defined() && work->scalar_type() == at::kFloat &&
                    work->is_contiguous() &&
                    work->numel() >= tdc_fcm_mfma_wide_workspace(M, (int)Kp, (int)DP,
                                                                 num_cus(Xh.device().index())),
                "tdc.fcm_mfma_wide: workspace fp32 too small");
    TORCH_CHECK(wx.has_value() && ws.has_value() && wx->scalar_type() == at::kDouble &&
                    ws->scalar_type() == at::kDouble && wx->is_contiguous() &&
                    ws->is_contiguous() && wx->numel() == K * D && ws->numel() == K,
                "tdc.fcm_mfma_wide: wx [K, D] / ws [K] fp64");
    wk = work->data_ptr<float>();
    pwx = wx->data_ptr<double>();
    pws = ws->data_ptr<double>();
    if (shift.has_value() && shift->defined())
      TORCH_CHECK(shift->scalar_type() == at::kFloat && shift->numel() >= D,
                  "tdc.fcm_mfma_wide: shift fp32 [D]");
  } else {
    TORCH_CHECK(pass == 0 || pass == 1,
                "tdc.fcm_mfma_wide: pass 0 (distances, on-centroid floor), 1 (raw distances) or 2 (W^T X)");
  }
  const DevGuard guard(Xh.device());
  check(tdc_fcm_mfma_wide((int)pass, Xh.data_ptr(), Xl.data_ptr(), xx.data_ptr<float>(), M,
                          (int)DP, (int)D, Ch.data_ptr(), Cl.data_ptr(), cc.data_ptr<float>(),
                          (int)K, (int)Kp, G.data_ptr<float>(), wk,
                          static_cast<const float*>(opt_ptr(shift)), pwx, pws,
                          num_cus(Xh.device().index()), cur_stream()),
        "fcm_mfma_wide");
}

void fcm_split_rows(const at::Tensor& src, int64_t valid, int64_t neg2, at::Tensor& hi,
                    at::Tensor& lo, const std::optional<at::Tensor>& norm,
                    const std::optional<at::Tensor>& shift) {
  check_cuda(src, "src");
  TORCH_CHECK(src.scalar_type() == at::kFloat && src.dim() == 2 && src.stride(1) == 1,
              "tdc.fcm_split_rows: src fp32 rows");
  TORCH_CHECK(hi.scalar_type() == at::kBFloat16 && lo.scalar_type() == at::kBFloat16 &&
                  hi.is_contiguous() && lo.is_contiguous() && hi.dim() == 2 &&
                  hi.sizes() == lo.sizes(), "tdc.fcm_split_rows: hi/lo bf16 [rows, DP]");
  const int64_t rows = hi.size(0);
  const int DP = (int)hi.size(1);
  TORCH_CHECK(src.size(1) <= DP && valid <= rows && valid <= src.size(0),
              "tdc.fcm_split_rows: shapes");
  if (norm.has_value() && norm->defined())
    TORCH_CHECK(norm->scalar_type() == at::kFloat && norm->is_contiguous() && norm->numel() >= rows,
                "tdc.fcm_split_rows: norm fp32 [rows]");
  if (shift.has_value() && shift->defined())
    TORCH_CHECK(shift->scalar_type() == at::kFloat && shift->is_contiguous() &&
                    shift->numel() >= src.size(1), "tdc.fcm_split_rows: shift fp32 [d]");
  const DevGuard guard(src.device());
  check(tdc_fcm_split_rows(src.data_ptr<float>(), rows, valid, (int)src.size(1), src.stride(0), DP,
                           (int)neg2, static_cast<const float*>(opt_ptr(shift)), hi.data_ptr(),
                           lo.data_ptr(),
                           static_cast<float*>(opt_ptr(norm)), cur_stream()),
        "fcm_split_rows");
}

void check_mfma_fcm(const at::Tensor& Xh, const at::Tensor& Xl, const at::Tensor& xx,
                    const at::Tensor& Ch, const at::Tensor& Cl, const at::Tensor& cc, int64_t K,
                    double m, const char* op) {
  check_cuda(Xh, "Xh");
  for (const at::Tensor* t : {&Xh, &Xl, &Ch, &Cl})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 2,
                "tdc.", op, ": hi/lo operands must be contiguous bf16 [rows, DP]");
  const int64_t DP = Xh.size(1);
  TORCH_CHECK(DP == 32 || DP == 64 || DP == 128, "tdc.", op, ": DP must be 32/64/128");
  TORCH_CHECK(Xl.sizes() == Xh.sizes() && Ch.size(1) == DP && Cl.sizes() == Ch.sizes(),
              "tdc.", op, ": operand shapes");
  TORCH_CHECK(Ch.size(0) % 128 == 0 && Ch.size(0) >= K && K > 0, "tdc.", op, ": Kp % 128, Kp >= K");
  TORCH_CHECK(xx.scalar_type() == at::kFloat && xx.is_contiguous() && xx.numel() >= Xh.size(0),
              "tdc.", op, ": xx fp32 [N]");
  TORCH_CHECK(cc.scalar_type() == at::kFloat && cc.is_contiguous() && cc.numel() >= Ch.size(0),
              "tdc.", op, ": cc fp32 [Kp]");
  TORCH_CHECK(m > 1.0, "tdc.", op, ": fuzzifier must be > 1");
}

void fcm_mfma_stats(const at::Tensor& Xh, const at::Tensor& Xl, const at::Tensor& xx,
                    const at::Tensor& Ch, const at::Tensor& Cl, const at::Tensor& cc, int64_t K,
                    double m, bool nan_to_zero, at::Tensor& labels, at::Tensor& rowinfo) {
  check_mfma_fcm(Xh, Xl, xx, Ch, Cl, cc, K, m, "fcm_mfma_stats");
  const int64_t N = Xh.size(0);
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= N,
              "tdc.fcm_mfma_stats: labels int32 [N]");
  TORCH_CHECK(rowinfo.scalar_type() == at::kFloat && rowinfo.is_contiguous() && rowinfo.numel() >= N,
              "tdc.fcm_mfma_stats: rowinfo fp32 [N]");
  const DevGuard guard(Xh.device());
  check(tdc_fcm_mfma(0, Xh.data_ptr(), Xl.data_ptr(), nullptr, xx.data_ptr<float>(), N, (int)Xh.size(1), 0,
                     Ch.data_ptr(), Cl.data_ptr(), cc.data_ptr<float>(), (int)K, (int)Ch.size(0),
                     m, nan_to_zero ? 1 : 0, labels.data_ptr<int32_t>(), rowinfo.data_ptr<float>(),
                     rowinfo.numel(), nullptr, nullptr, nullptr, nullptr,
                     num_cus(Xh.device().index()), cur_stream()),
        "fcm_mfma_stats");
}

void fcm_mfma_accum(const at::Tensor& Xh, const at::Tensor& Xl, const at::Tensor& xx,
                    const at::Tensor& rowinfo, const at::Tensor& Ch, const at::Tensor& Cl,
                    const at::Tensor& cc, int64_t K, double m, bool nan_to_zero, at::Tensor& wx,
                    at::Tensor& ws, at::Tensor& work, const std::optional<at::Tensor>& shift,
                    const std::optional<at::Tensor>& Xr) {
  check_mfma_fcm(Xh, Xl, xx, Ch, Cl, cc, K, m, "fcm_mfma_accum");
  if (Xr.has_value() && Xr->defined())
    TORCH_CHECK(Xr->scalar_type() == at::kBFloat16 && Xr->is_contiguous() &&
                    Xr->sizes() == Xh.sizes(),
                "tdc.fcm_mfma_accum: Xr bf16 [N, DP] like Xh");
  const int nc = num_cus(Xh.device().index());
  TORCH_CHECK(work.scalar_type() == at::kFloat && work.is_contiguous() &&
                  work.numel() >= tdc_fcm_mfma_workspace(Xh.size(0), (int)K, (int)Ch.size(0),
                                                         (int)Xh.size(1), nc),
              "tdc.fcm_mfma_accum: work fp32 [fcm_mfma_workspace(...)]");
  const int64_t N = Xh.size(0);
  TORCH_CHECK(rowinfo.scalar_type() == at::kFloat && rowinfo.is_contiguous() && rowinfo.numel() >= N,
              "tdc.fcm_mfma_accum: rowinfo fp32 [N]");
  TORCH_CHECK(wx.scalar_type() == at::kDouble && ws.scalar_type() == at::kDouble &&
                  wx.is_contiguous() && ws.is_contiguous() && wx.dim() == 2 && wx.size(0) == K &&
                  wx.size(1) <= Xh.size(1) && ws.numel() == K,
              "tdc.fcm_mfma_accum: wx [K, D] / ws [K] fp64");
  const DevGuard guard(Xh.device());
  check(tdc_fcm_mfma(1, Xh.data_ptr(), Xl.data_ptr(), opt_ptr(Xr), xx.data_ptr<float>(), N, (int)Xh.size(1),
                     (int)wx.size(1), Ch.data_ptr(), Cl.data_ptr(), cc.data_ptr<float>(), (int)K,
                     (int)Ch.size(0), m, nan_to_zero ? 1 : 0, nullptr,
                     const_cast<float*>(rowinfo.data_ptr<float>()), rowinfo.numel(), wx.data_ptr<double>(),
                     ws.data_ptr<double>(), work.data_ptr<float>(),
                     static_cast<const float*>(opt_ptr(shift)), nc, cur_stream()),
        "fcm_mfma_accum");
}

int64_t fcm_mfma_workspace(const at::Tensor& like, int64_t N, int64_t K, int64_t Kp, int64_t DP) {
  return tdc_fcm_mfma_workspace(N, (int)K, (int)Kp, (int)DP, num_cus(like.device().index()));
}

int64_t fcm_mfma_rowinfo_len(const at::Tensor& like, int64_t N, int64_t DP) {
  (void)like;
  return tdc_fcm_mfma_rowinfo_len(N, (int)DP);
}

void finalize(const std::optional<at::Tensor>& sums, const std::optional<at::Tensor>& counts,
              at::Tensor& C, int64_t policy, const std::optional<at::Tensor>& shift,
              const std::optional<at::Tensor>& Cm2, const std::optional<at::Tensor>& cnorm,
              const std::optional<at::Tensor>& drift, const std::optional<at::Tensor>& maxdrift,
              double fixed_scale) {
  check_cuda(C, "C");
  TORCH_CHECK(C.is_contiguous() && C.dim() == 2, "tdc.finalize: C");
  const int K = (int)C.size(0), D = (int)C.size(1);
  int acc = TDC_F64;
  if (sums.has_value() && sums->defined()) {
    TORCH_CHECK(counts.has_value() && counts->defined(), "tdc.finalize: counts required");
    TORCH_CHECK(sums->is_contiguous() && sums->numel() == (int64_t)K * D, "tdc.finalize: sums");
    TORCH_CHECK(counts->scalar_type() == sums->scalar_type(), "tdc.finalize: counts dtype");
    check_fixed(*sums, fixed_scale, "finalize");
    acc = dcode(sums->scalar_type());
  }
  int Kp = K, DP = D;
  if (Cm2.has_value() && Cm2->defined()) {
    TORCH_CHECK(Cm2->scalar_type() == at::kBFloat16 && Cm2->is_contiguous(), "tdc.finalize: Cm2");
    TORCH_CHECK(cnorm.has_value() && cnorm->defined(), "tdc.finalize: cnorm required with Cm2");
    Kp = (int)Cm2->size(0);
    DP = (int)Cm2->size(1);
    TORCH_CHECK(Kp >= K && DP >= D, "tdc.finalize: Cm2 smaller than C");
  }
  float* sh = nullptr;
  if (shift.has_value() && shift->defined()) {
    TORCH_CHECK(shift->scalar_type() == at::kFloat, "tdc.finalize: shift fp32");
    sh = shift->data_ptr<float>();
  }
  float* dr = nullptr;
  float* mdr = nullptr;
  if (drift.has_value() && drift->defined()) {
    TORCH_CHECK(sums.has_value() && sums->defined(), "tdc.finalize: drift needs sums");
    TORCH_CHECK(drift->scalar_type() == at::kFloat && drift->numel() >= K && drift->is_contiguous(),
                "tdc.finalize: drift fp32 [K]");
    TORCH_CHECK(maxdrift.has_value() && maxdrift->defined() &&
                    maxdrift->scalar_type() == at::kFloat && maxdrift->numel() >= 1,
                "tdc.finalize: maxdrift fp32 [1] required with drift");
    dr = drift->data_ptr<float>();
    mdr = maxdrift->data_ptr<float>();
  }
  const DevGuard guard(C.device());
  check(tdc_finalize(acc, dcode(C.scalar_type()), opt_ptr(sums), opt_ptr(counts), K, D,
                     C.data_ptr(), (int)policy, sh, opt_ptr(Cm2),
                     static_cast<float*>(opt_ptr(cnorm)), Kp, DP, cur_stream(), dr, mdr,
                     fixed_scale),
        "finalize");
}

// rows of a mini-batch by index: point i of the launch is row rowidx[i] of X
void check_rowidx(const at::Tensor& X, const at::Tensor& rowidx, int64_t n, const char* op) {
  TORCH_CHECK(rowidx.scalar_type() == at::kInt && rowidx.is_contiguous() && rowidx.dim() == 1,
              "tdc.", op, ": rowidx must be contiguous int32 [B]");
  TORCH_CHECK(rowidx.numel() == n, "tdc.", op, ": rowidx/labels length mismatch");
  TORCH_CHECK(rowidx.device() == X.device(), "tdc.", op, ": rowidx on another device");
  TORCH_CHECK(X.size(0) < ((int64_t)1 << 31), "tdc.", op, ": X has >= 2^31 rows");
}

void assign_bf16_indexed(const at::Tensor& X, const at::Tensor& rowidx, const at::Tensor& Cm2,
                         const at::Tensor& cnorm, at::Tensor& labels,
                         const std::optional<at::Tensor>& mind) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 && Cm2.scalar_type() == at::kBFloat16,
              "tdc.assign_bf16_indexed: X and Cm2 must be bfloat16");
  TORCH_CHECK(cnorm.scalar_type() == at::kFloat && labels.scalar_type() == at::kInt,
              "tdc.assign_bf16_indexed: cnorm fp32, labels int32");
  TORCH_CHECK(Cm2.is_contiguous() && cnorm.is_contiguous() && labels.is_contiguous(),
              "tdc.assign_bf16_indexed: Cm2/cnorm/labels must be contiguous");
  const int64_t B = rowidx.numel();
  check_rowidx(X, rowidx, B, "assign_bf16_indexed");
  const int DP = (int)Cm2.size(1);
  const int Kp = (int)Cm2.size(0);
  TORCH_CHECK(DP == 64 || DP == 128 || DP == 256,
              "tdc.assign_bf16_indexed: padded dim must be 64/128/256, got ", DP);
  TORCH_CHECK(X.size(1) >= DP, "tdc.assign_bf16_indexed: X has fewer columns than Cm2");
  TORCH_CHECK(X.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(X.data_ptr()) % 16) == 0,
              "tdc.assign_bf16_indexed: X rows must be 16-byte aligned");
  TORCH_CHECK(Kp % 64 == 0 && cnorm.numel() >= Kp, "tdc.assign_bf16_indexed: Kp % 64");
  TORCH_CHECK(labels.numel() >= B, "tdc.assign_bf16_indexed: labels too small");
  float* md = nullptr;
  if (mind.has_value() && mind->defined()) {
    TORCH_CHECK(mind->scalar_type() == at::kFloat && mind->numel() >= B && mind->is_contiguous(),
                "tdc.assign_bf16_indexed: mind must be fp32 [B]");
    md = mind->data_ptr<float>();
  }
  const DevGuard guard(X.device());
  check(tdc_assign_mfma_bf16_indexed(X.data_ptr(), rowidx.data_ptr<int32_t>(), B, X.stride(0), DP,
                                     Cm2.data_ptr(), cnorm.data_ptr<float>(), Kp,
                                     labels.data_ptr<int32_t>(), md, cur_stream()),
        "assign_bf16_indexed");
}

void update_sorted_indexed(const at::Tensor& X, const at::Tensor& rowidx, const at::Tensor& labels,
                           at::Tensor& sums, at::Tensor& counts, at::Tensor& work,
                           const std::optional<at::Tensor>& cnt_hi,
                           const std::optional<at::Tensor>& cnt_lo, bool work_clean,
                           const std::optional<at::Tensor>& zero_first) {
  check_cuda(X, "X");
  check_rows(X, "X");
  const int64_t B = labels.numel();
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous(),
              "tdc.update_sorted_indexed: labels int32 [B]");
  check_rowidx(X, rowidx, B, "update_sorted_indexed");
  TORCH_CHECK(sums.dim() == 2 && sums.is_contiguous() && counts.is_contiguous(),
              "tdc.update_sorted_indexed: sums");
  TORCH_CHECK(sums.scalar_type() == counts.scalar_type() && counts.numel() >= sums.size(0),
              "tdc.update_sorted_indexed: counts");
  TORCH_CHECK(X.size(1) >= sums.size(1), "tdc.update_sorted_indexed: X narrower than sums");
  TORCH_CHECK(work.scalar_type() == at::kInt && work.is_contiguous() &&
                  work.numel() >= tdc_update_sorted_workspace(B, (int)sums.size(0)),
              "tdc.update_sorted_indexed: workspace too small");
  check_split(cnt_hi, cnt_lo, sums.size(0), "update_sorted_indexed");
  // zero_first (the caller's all-reduce buffer): cleared by the histogram kernel, before
  // anything accumulates into it (one fill launch fewer per mini-batch step)
  int64_t zbytes = 0;
  if (zero_first.has_value() && zero_first->defined()) {
    TORCH_CHECK(zero_first->is_contiguous() && zero_first->device() == X.device() &&
                    (zero_first->numel() * zero_first->element_size()) % 4 == 0,
                "tdc.update_sorted_indexed: zero_first must be a contiguous device buffer of 4-byte words");
    zbytes = zero_first->numel() * zero_first->element_size();
  }
  const DevGuard guard(X.device());
  check(tdc_update_sorted(dcode(X.scalar_type()), dcode(sums.scalar_type()), X.data_ptr(), B,
                          X.stride(0), (int)sums.size(1), labels.data_ptr<int32_t>(),
                          (int)sums.size(0), sums.data_ptr(), counts.data_ptr(),
                          work.data_ptr<int>(), num_cus(X.device().index()), cur_stream(),
                          rowidx.data_ptr<int32_t>(), static_cast<float*>(opt_ptr(cnt_hi)),
                          static_cast<float*>(opt_ptr(cnt_lo)), opt_ptr(zero_first), zbytes, 0.0,
                          work_clean ? 1 : 0),
        "update_sorted_indexed");
}

// ---- fp32 / fp64 assignment on the matrix cores (kernels.h tdc_x3_*) ----
void x3_split(const at::Tensor& src, int64_t valid, int64_t neg2, at::Tensor& hi, at::Tensor& lo,
              const std::optional<at::Tensor>& norm, const std::optional<at::Tensor>& nhl,
              const std::optional<at::Tensor>& shift) {
  check_cuda(src, "src");
  check_rows(src, "src");
  TORCH_CHECK(src.scalar_type() == at::kFloat || src.scalar_type() == at::kDouble,
              "tdc.x3_split: src fp32/fp64");
  TORCH_CHECK(hi.scalar_type() == at::kBFloat16 && lo.scalar_type() == at::kBFloat16 &&
                  hi.is_contiguous() && lo.is_contiguous() && hi.sizes() == lo.sizes() && hi.dim() == 2,
              "tdc.x3_split: hi/lo bf16 [rows, DP]");
  const int64_t rows = hi.size(0);
  const int DP = (int)hi.size(1);
  TORCH_CHECK(src.size(1) <= DP && valid <= rows && valid <= src.size(0), "tdc.x3_split: shapes");
  if (norm.has_value() && norm->defined())
    TORCH_CHECK(norm->scalar_type() == at::kFloat && norm->is_contiguous() && norm->numel() >= rows,
                "tdc.x3_split: norm fp32 [rows]");
  if (nhl.has_value() && nhl->defined())
    TORCH_CHECK(nhl->scalar_type() == at::kFloat && nhl->is_contiguous() && nhl->numel() >= 2 * rows,
                "tdc.x3_split: nhl fp32 [rows, 2]");
  if (shift.has_value() && shift->defined())
    TORCH_CHECK(shift->scalar_type() == src.scalar_type() && shift->is_contiguous() &&
                    shift->numel() >= src.size(1) && shift->device() == src.device(),
                "tdc.x3_split: shift [d] of src's dtype");
  const DevGuard guard(src.device());
  check(tdc_x3_split(dcode(src.scalar_type()), src.data_ptr(), rows, valid, (int)src.size(1),
                     src.stride(0), DP, (int)neg2, hi.data_ptr(), lo.data_ptr(),
                     static_cast<float*>(opt_ptr(norm)), static_cast<float*>(opt_ptr(nhl)),
                     cur_stream(), opt_ptr(shift)),
        "x3_split");
}

// amb: int32 [3 cap] (two-candidate int2 entries | full re-scan rows), amb_count int32 [2]
int64_t check_x3_state(const at::Tensor& cstat, const at::Tensor& amb, const at::Tensor& amb_count,
                       int64_t rows, const char* op) {
  TORCH_CHECK(cstat.scalar_type() == at::kFloat && cstat.numel() >= 3, "tdc.", op, ": cstat fp32 [3]");
  TORCH_CHECK(amb_count.scalar_type() == at::kInt && amb_count.numel() >= 2, "tdc.", op,
              ": amb_count int32 [2]");
  TORCH_CHECK(amb.scalar_type() == at::kInt && amb.is_contiguous() && amb.numel() % 3 == 0 &&
                  amb.numel() >= 3 * rows,
              "tdc.", op, ": amb int32 [3 * capacity >= 3 * rows]");
  return amb.numel() / 3;
}

void x3_prep(const at::Tensor& cnorm, const std::optional<at::Tensor>& nhl, int64_t K,
             at::Tensor& cstat, at::Tensor& amb_count) {
  check_cuda(cnorm, "cnorm");
  TORCH_CHECK(cnorm.scalar_type() == at::kFloat && cnorm.is_contiguous() && cnorm.numel() >= K,
              "tdc.x3_prep: cnorm fp32 [>= K]");
  if (nhl.has_value() && nhl->defined())
    TORCH_CHECK(nhl->scalar_type() == at::kFloat && nhl->numel() >= 2 * K, "tdc.x3_prep: nhl");
  TORCH_CHECK(cstat.scalar_type() == at::kFloat && cstat.numel() >= 3 &&
                  amb_count.scalar_type() == at::kInt && amb_count.numel() >= 2,
              "tdc.x3_prep: cstat fp32 [3], amb_count int32 [2]");
  const DevGuard guard(cnorm.device());
  check(tdc_x3_prep(cnorm.data_ptr<float>(), static_cast<const float*>(opt_ptr(nhl)), (int)K,
                    cstat.data_ptr<float>(), amb_count.data_ptr<int>(), cur_stream()),
        "x3_prep");
}

void x3_recheck(const at::Tensor& X, const at::Tensor& C, at::Tensor& labels, const at::Tensor& amb,
                const at::Tensor& amb_count) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kFloat || X.scalar_type() == at::kDouble, "tdc.x3_recheck: X");
  TORCH_CHECK(C.scalar_type() == X.scalar_type() && C.is_contiguous() && C.dim() == 2 &&
                  C.size(1) <= X.size(1) && C.size(1) <= 1024,
              "tdc.x3_recheck: C [K, D <= 1024] in the X dtype");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= X.size(0),
              "tdc.x3_recheck: labels int32 [N]");
  TORCH_CHECK(amb.scalar_type() == at::kInt && amb.is_contiguous() && amb.numel() % 3 == 0 &&
                  amb_count.scalar_type() == at::kInt && amb_count.numel() >= 2,
              "tdc.x3_recheck: amb int32 [3 cap], amb_count int32 [2]");
  const DevGuard guard(X.device());
  check(tdc_x3_recheck(dcode(X.scalar_type()), X.data_ptr(), X.stride(0), (int)C.size(1), C.data_ptr(),
                       (int)C.size(0), labels.data_ptr<int32_t>(), amb.data_ptr<int>(),
                       amb.numel() / 3, amb_count.data_ptr<int>(), num_cus(X.device().index()),
                       cur_stream()),
        "x3_recheck");
}

// prep (cmax, list reset) + bf16x3 assignment + exact re-check of the listed rows
void x3_assign(const at::Tensor& X, const at::Tensor& Xh, const at::Tensor& Xl, const at::Tensor& Ch,
               const at::Tensor& Cl, const at::Tensor& cnorm, const at::Tensor& cnhl,
               const at::Tensor& C, at::Tensor& labels, const std::optional<at::Tensor>& mind,
               at::Tensor& amb, at::Tensor& cstat, at::Tensor& amb_count, bool recheck,
               const std::optional<at::Tensor>& pre, const std::optional<at::Tensor>& xnhl,
               int64_t pre_est) {
  check_cuda(Xh, "Xh");
  TORCH_CHECK(Xh.scalar_type() == at::kBFloat16 && Xl.scalar_type() == at::kBFloat16 &&
                  Ch.scalar_type() == at::kBFloat16 && Cl.scalar_type() == at::kBFloat16,
              "tdc.x3_assign: hi/lo operands bf16");
  TORCH_CHECK(Xh.is_contiguous() && Xl.is_contiguous() && Ch.is_contiguous() && Cl.is_contiguous() &&
                  Xh.sizes() == Xl.sizes() && Ch.sizes() == Cl.sizes() && Xh.dim() == 2 && Ch.dim() == 2,
              "tdc.x3_assign: Xh/Xl [N, DP], Ch/Cl [Kp, DP] contiguous");
  const int64_t N = Xh.size(0);
  const int DP = (int)Xh.size(1);
  const int Kp = (int)Ch.size(0);
  TORCH_CHECK(Ch.size(1) == DP, "tdc.x3_assign: DP mismatch");
  TORCH_CHECK(DP == 32 || DP == 64 || DP == 128 || DP == 256, "tdc.x3_assign: DP 32/64/128/256");
  TORCH_CHECK(Kp % (DP == 256 ? 32 : 64) == 0 && cnorm.scalar_type() == at::kFloat &&
                  cnorm.is_contiguous() && cnorm.numel() >= Kp,
              "tdc.x3_assign: Kp % 64 (% 32 at DP 256), cnorm fp32 [Kp]");
  const int K = (int)C.size(0);
  TORCH_CHECK(K <= Kp && C.size(1) <= DP, "tdc.x3_assign: C [K <= Kp, D <= DP]");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= N,
              "tdc.x3_assign: labels int32 [N]");
  const int64_t cap = check_x3_state(cstat, amb, amb_count, N, "x3_assign");
  TORCH_CHECK(cnhl.scalar_type() == at::kFloat && cnhl.is_contiguous() && cnhl.numel() >= 2 * K,
              "tdc.x3_assign: cnhl fp32 [K, 2] (centroid hi/lo norms)");
  float* md = nullptr;
  if (mind.has_value() && mind->defined()) {
    TORCH_CHECK(mind->scalar_type() == at::kFloat && mind->numel() >= N && mind->is_contiguous(),
                "tdc.x3_assign: mind fp32 [N]");
    md = mind->data_ptr<float>();
  }
  if (recheck) {
    check_rows(X, "X");
    TORCH_CHECK(X.size(0) >= N && (X.scalar_type() == at::kFloat || X.scalar_type() == at::kDouble) &&
                    C.scalar_type() == X.scalar_type() && C.is_contiguous(),
                "tdc.x3_assign: X / C fp32 or fp64 (same dtype)");
  }
  int32_t* pl = nullptr;
  if (pre.has_value() && pre->defined()) {
    TORCH_CHECK(pre->scalar_type() == at::kInt && pre->is_contiguous() && pre->numel() >= N &&
                    amb_count.numel() >= 3 && (DP == 64 || DP == 128 || DP == 256) && md == nullptr,
                "tdc.x3_assign: pre int32 [>= N] needs amb_count int32 [3], DP 64/128/256 and no mind");
    pl = pre->data_ptr<int32_t>();
  }
  const float* xn2 = nullptr;
  if (pl && xnhl.has_value() && xnhl->defined()) {
    TORCH_CHECK(xnhl->scalar_type() == at::kFloat && xnhl->is_contiguous() && xnhl->numel() >= 2 * N,
                "tdc.x3_assign: xnhl fp32 [>= N, 2] (the rows' hi/lo norms from x3_split)");
    xn2 = xnhl->data_ptr<float>();
  }
  const DevGuard guard(Xh.device());
  hipStream_t s = cur_stream();
  int32_t* list = amb.data_ptr<int>();
  int* cnt = amb_count.data_ptr<int>();
  check(tdc_x3_prep(cnorm.data_ptr<float>(), cnhl.data_ptr<float>(), K, cstat.data_ptr<float>(),
                    cnt, s, pl ? 3 : 2),
        "x3_prep");
  if (pl)  // one-product prefilter, then the three products over the rows it could not certify
    check(tdc_x3_prefilter(Xh.data_ptr(), N, DP, Ch.data_ptr(), cnorm.data_ptr<float>(), Kp,
                           cstat.data_ptr<float>(), labels.data_ptr<int32_t>(), pl, cnt + 2, s,
                           xn2),
          "x3_prefilter");
  check(tdc_assign_x3(Xh.data_ptr(), Xl.data_ptr(), N, DP, Ch.data_ptr(), Cl.data_ptr(),
                      cnorm.data_ptr<float>(), Kp, cstat.data_ptr<float>(),
                      labels.data_ptr<int32_t>(), md, list, cap, cnt, s, pl,
                      pl ? cnt + 2 : nullptr, pre_est),
        "assign_x3");
  if (recheck)
    check(tdc_x3_recheck(dcode(X.scalar_type()), X.data_ptr(), X.stride(0), (int)C.size(1), C.data_ptr(),
                         K, labels.data_ptr<int32_t>(), list, cap, amb_count.data_ptr<int>(),
                         num_cus(X.device().index()), s),
          "x3_recheck");
}

void x3_rows(const at::Tensor& G, int64_t row0, const at::Tensor& xx, const at::Tensor& cstat,
             int64_t DP, at::Tensor& labels, at::Tensor& amb, at::Tensor& amb_count) {
  check_cuda(G, "G");
  TORCH_CHECK(G.scalar_type() == at::kFloat && G.is_contiguous() && G.dim() == 2, "tdc.x3_rows: G fp32 [M, K]");
  const int64_t M = G.size(0);
  TORCH_CHECK(xx.scalar_type() == at::kFloat && xx.numel() >= M, "tdc.x3_rows: xx fp32 [M]");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.numel() >= row0 + M, "tdc.x3_rows: labels");
  const int64_t cap = check_x3_state(cstat, amb, amb_count, row0 + M, "x3_rows");
  const DevGuard guard(G.device());
  check(tdc_x3_rows(G.data_ptr<float>(), M, (int)G.size(1), row0, xx.data_ptr<float>(),
                    cstat.data_ptr<float>(), (int)DP, labels.data_ptr<int32_t>(),
                    amb.data_ptr<int>(), cap, amb_count.data_ptr<int>(), cur_stream()),
        "x3_rows");
}

// ---- delta update of plain Lloyd (kernels.h tdc_delta_*) ----
int64_t delta_workspace(int64_t N, int64_t K) { return tdc_delta_workspace(N, (int)K); }

void check_ctrl(const at::Tensor& ctrl, const at::Tensor& like, const char* op) {
  TORCH_CHECK(ctrl.scalar_type() == at::kInt && ctrl.is_contiguous() &&
                  ctrl.numel() >= TDC_DC_WORDS && ctrl.device() == like.device(),
              "tdc.", op, ": ctrl must be int32 [", (int)TDC_DC_WORDS, "] on the data's device");
}

void delta_update(const at::Tensor& X, const at::Tensor& labels, at::Tensor& prev, at::Tensor& sums,
                  at::Tensor& counts, at::Tensor& work, at::Tensor& ctrl,
                  const std::optional<at::Tensor>& cnt_hi, const std::optional<at::Tensor>& cnt_lo,
                  const std::optional<at::Tensor>& moved, const std::optional<at::Tensor>& zero_first,
                  double fixed_scale, bool work_clean) {
  check_cuda(X, "X");
  check_fixed(sums, fixed_scale, "delta_update");
  check_rows(X, "X");
  const int64_t N = X.size(0);
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= N,
              "tdc.delta_update: labels int32 [N]");
  TORCH_CHECK(prev.scalar_type() == at::kInt && prev.is_contiguous() && prev.numel() >= N,
              "tdc.delta_update: prev int32 [N]");
  TORCH_CHECK(sums.dim() == 2 && sums.is_contiguous() && counts.is_contiguous(),
              "tdc.delta_update: sums");
  TORCH_CHECK(sums.scalar_type() == counts.scalar_type() && counts.numel() >= sums.size(0),
              "tdc.delta_update: counts");
  TORCH_CHECK(X.size(1) >= sums.size(1), "tdc.delta_update: X narrower than sums");
  const int K = (int)sums.size(0);
  TORCH_CHECK(K <= TDC_DELTA_MAX_K, "tdc.delta_update: K > ", TDC_DELTA_MAX_K);
  TORCH_CHECK(N < ((int64_t)1 << 30), "tdc.delta_update: shard has >= 2^30 rows");
  TORCH_CHECK(work.scalar_type() == at::kInt && work.is_contiguous() &&
                  work.numel() >= tdc_delta_workspace(N, K),
              "tdc.delta_update: workspace too small");
  check_ctrl(ctrl, X, "delta_update");
  check_split(cnt_hi, cnt_lo, K, "delta_update");
  if (moved.has_value() && moved->defined())
    TORCH_CHECK(moved->scalar_type() == sums.scalar_type() && moved->numel() >= 1,
                "tdc.delta_update: moved must be one element of the sums dtype");
  int64_t zbytes = 0;
  if (zero_first.has_value() && zero_first->defined()) {
    TORCH_CHECK(zero_first->is_contiguous() && zero_first->device() == X.device() &&
                    (zero_first->numel() * zero_first->element_size()) % 4 == 0,
                "tdc.delta_update: zero_first must be a contiguous device buffer of 4-byte words");
    zbytes = zero_first->numel() * zero_first->element_size();
  }
  const DevGuard guard(X.device());
  check(tdc_delta_update(dcode(X.scalar_type()), dcode(sums.scalar_type()), X.data_ptr(), N,
                         X.stride(0), (int)sums.size(1), labels.data_ptr<int32_t>(),
                         prev.data_ptr<int32_t>(), K, sums.data_ptr(), counts.data_ptr(),
                         work.data_ptr<int>(), ctrl.data_ptr<int>(), num_cus(X.device().index()),
                         cur_stream(), static_cast<float*>(opt_ptr(cnt_hi)),
                         static_cast<float*>(opt_ptr(cnt_lo)), opt_ptr(moved), opt_ptr(zero_first),
                         zbytes, fixed_scale, work_clean ? 1 : 0),
        "delta_update");
}

void delta_finalize(const at::Tensor& sums, const at::Tensor& counts,
                    const std::optional<at::Tensor>& cnt_hi, const std::optional<at::Tensor>& cnt_lo,
                    const std::optional<at::Tensor>& moved, at::Tensor& G, at::Tensor& C,
                    int64_t policy, const std::optional<at::Tensor>& shift,
                    const std::optional<at::Tensor>& Cm2, const std::optional<at::Tensor>& cnorm,
                    at::Tensor& ctrl, const std::optional<at::Tensor>& stats, int64_t refresh,
                    double theta_n, double fixed_scale) {
  check_cuda(C, "C");
  check_fixed(sums, fixed_scale, "delta_finalize");
  TORCH_CHECK(C.is_contiguous() && C.dim() == 2, "tdc.delta_finalize: C");
  const int K = (int)C.size(0), D = (int)C.size(1);
  TORCH_CHECK(sums.is_contiguous() && sums.numel() == (int64_t)K * D, "tdc.delta_finalize: sums");
  TORCH_CHECK(counts.scalar_type() == sums.scalar_type() && counts.is_contiguous() &&
                  counts.numel() >= K, "tdc.delta_finalize: counts");
  TORCH_CHECK(G.scalar_type() == at::kDouble && G.is_contiguous() &&
                  G.numel() >= (int64_t)K * D + K, "tdc.delta_finalize: G fp64 [K*D + K]");
  check_split(cnt_hi, cnt_lo, K, "delta_finalize");
  if (moved.has_value() && moved->defined())
    TORCH_CHECK(moved->scalar_type() == sums.scalar_type() && moved->numel() >= 1,
                "tdc.delta_finalize: moved");
  int Kp = K, DP = D;
  if (Cm2.has_value() && Cm2->defined()) {
    TORCH_CHECK(Cm2->scalar_type() == at::kBFloat16 && Cm2->is_contiguous(), "tdc.delta_finalize: Cm2");
    TORCH_CHECK(cnorm.has_value() && cnorm->defined(), "tdc.delta_finalize: cnorm required with Cm2");
    Kp = (int)Cm2->size(0);
    DP = (int)Cm2->size(1);
    TORCH_CHECK(Kp >= K && DP >= D, "tdc.delta_finalize: Cm2 smaller than C");
  }
  float* sh = nullptr;
  if (shift.has_value() && shift->defined()) {
    TORCH_CHECK(shift->scalar_type() == at::kFloat, "tdc.delta_finalize: shift fp32");
    sh = shift->data_ptr<float>();
  }
  double* st = nullptr;
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->scalar_type() == at::kDouble && stats->numel() >= 4 && stats->is_contiguous(),
                "tdc.delta_finalize: stats fp64 [4]");
    st = stats->data_ptr<double>();
  }
  check_ctrl(ctrl, C, "delta_finalize");
  const DevGuard guard(C.device());
  check(tdc_delta_finalize(dcode(sums.scalar_type()), dcode(C.scalar_type()), sums.data_ptr(),
                           counts.data_ptr(), static_cast<const float*>(opt_ptr(cnt_hi)),
                           static_cast<const float*>(opt_ptr(cnt_lo)), opt_ptr(moved),
                           G.data_ptr<double>(), K, D, C.data_ptr(), (int)policy, sh, opt_ptr(Cm2),
                           static_cast<float*>(opt_ptr(cnorm)), Kp, DP, ctrl.data_ptr<int>(), st,
                           (int)refresh, theta_n, cur_stream(), fixed_scale),
        "delta_finalize");
}

void sculley_update(const at::Tensor& sums, const at::Tensor& counts, at::Tensor& C, at::Tensor& v,
                    const std::optional<at::Tensor>& shift, const std::optional<at::Tensor>& Cm2,
                    const std::optional<at::Tensor>& cnorm) {
  check_cuda(C, "C");
  TORCH_CHECK(C.is_contiguous() && C.dim() == 2, "tdc.sculley_update: C");
  const int K = (int)C.size(0), D = (int)C.size(1);
  TORCH_CHECK(sums.is_contiguous() && sums.numel() == (int64_t)K * D, "tdc.sculley_update: sums");
  TORCH_CHECK(counts.scalar_type() == sums.scalar_type() && counts.numel() >= K,
              "tdc.sculley_update: counts");
  TORCH_CHECK(v.scalar_type() == at::kDouble && v.is_contiguous() && v.numel() >= K,
              "tdc.sculley_update: v must be fp64 [K]");
  int Kp = K, DP = D;
  if (Cm2.has_value() && Cm2->defined()) {
    TORCH_CHECK(Cm2->scalar_type() == at::kBFloat16 && Cm2->is_contiguous(), "tdc.sculley_update: Cm2");
    TORCH_CHECK(cnorm.has_value() && cnorm->defined(), "tdc.sculley_update: cnorm required with Cm2");
    Kp = (int)Cm2->size(0);
    DP = (int)Cm2->size(1);
    TORCH_CHECK(Kp >= K && DP >= D, "tdc.sculley_update: Cm2 smaller than C");
  }
  float* sh = nullptr;
  if (shift.has_value() && shift->defined()) {
    TORCH_CHECK(shift->scalar_type() == at::kFloat, "tdc.sculley_update: shift fp32");
    sh = shift->data_ptr<float>();
  }
  const DevGuard guard(C.device());
  check(tdc_sculley_update(dcode(sums.scalar_type()), dcode(C.scalar_type()), sums.data_ptr(),
                           counts.data_ptr(), K, D, C.data_ptr(), v.data_ptr<double>(), sh,
                           opt_ptr(Cm2), static_cast<float*>(opt_ptr(cnorm)), Kp, DP,
                           cur_stream()),
        "sculley_update");
}

void assign_bf16_top2(const at::Tensor& X, const std::optional<at::Tensor>& rowidx,
                      const at::Tensor& Cm2, const at::Tensor& cnorm, at::Tensor& labels,
                      at::Tensor& mind, at::Tensor& mind2) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 && Cm2.scalar_type() == at::kBFloat16,
              "tdc.assign_bf16_top2: X and Cm2 must be bfloat16");
  TORCH_CHECK(cnorm.scalar_type() == at::kFloat && labels.scalar_type() == at::kInt,
              "tdc.assign_bf16_top2: cnorm fp32, labels int32");
  TORCH_CHECK(Cm2.is_contiguous() && cnorm.is_contiguous() && labels.is_contiguous(),
              "tdc.assign_bf16_top2: Cm2/cnorm/labels must be contiguous");
  const bool idx = rowidx.has_value() && rowidx->defined();
  const int64_t B = idx ? rowidx->numel() : X.size(0);
  if (idx) check_rowidx(X, *rowidx, B, "assign_bf16_top2");
  const int DP = (int)Cm2.size(1);
  const int Kp = (int)Cm2.size(0);
  TORCH_CHECK(DP == 64 || DP == 128 || DP == 256, "tdc.assign_bf16_top2: DP must be 64/128/256");
  TORCH_CHECK(X.size(1) >= DP, "tdc.assign_bf16_top2: X has fewer columns than Cm2");
  TORCH_CHECK(X.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(X.data_ptr()) % 16) == 0,
              "tdc.assign_bf16_top2: X rows must be 16-byte aligned");
  TORCH_CHECK(Kp % 64 == 0 && cnorm.numel() >= Kp, "tdc.assign_bf16_top2: Kp % 64");
  TORCH_CHECK(labels.numel() >= B, "tdc.assign_bf16_top2: labels too small");
  for (const at::Tensor* m : {&mind, &mind2})
    TORCH_CHECK(m->scalar_type() == at::kFloat && m->numel() >= B && m->is_contiguous(),
                "tdc.assign_bf16_top2: mind/mind2 must be fp32 [B]");
  const DevGuard guard(X.device());
  check(tdc_assign_mfma_bf16_top2(X.data_ptr(), idx ? rowidx->data_ptr<int32_t>() : nullptr, B,
                                  X.stride(0), DP, Cm2.data_ptr(), cnorm.data_ptr<float>(), Kp,
                                  labels.data_ptr<int32_t>(), mind.data_ptr<float>(),
                                  mind2.data_ptr<float>(), cur_stream()),
        "assign_bf16_top2");
}

void bounds_filter(const at::Tensor& labels, at::Tensor& ub, at::Tensor& lb, const at::Tensor& drift,
                   const at::Tensor& maxdrift, double slack, at::Tensor& active, at::Tensor& count) {
  check_cuda(labels, "labels");
  const int64_t N = labels.numel();
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous(), "tdc.bounds_filter: labels");
  for (const at::Tensor* t : {&ub, &lb})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == N,
                "tdc.bounds_filter: ub/lb fp32 [N]");
  TORCH_CHECK(drift.scalar_type() == at::kFloat && drift.is_contiguous(), "tdc.bounds_filter: drift");
  TORCH_CHECK(maxdrift.scalar_type() == at::kFloat && maxdrift.numel() >= 1, "tdc.bounds_filter: maxdrift");
  TORCH_CHECK(active.scalar_type() == at::kInt && active.numel() >= N && active.is_contiguous(),
              "tdc.bounds_filter: active int32 [N]");
  TORCH_CHECK(count.scalar_type() == at::kInt && count.numel() >= 1, "tdc.bounds_filter: count");
  const DevGuard guard(labels.device());
  check(tdc_bounds_filter(labels.data_ptr<int32_t>(), N, ub.data_ptr<float>(), lb.data_ptr<float>(),
                          drift.data_ptr<float>(), maxdrift.data_ptr<float>(), (float)slack,
                          active.data_ptr<int32_t>(), count.data_ptr<int>(), cur_stream()),
        "bounds_filter");
}

void bounds_scatter(const at::Tensor& active, const at::Tensor& count, const at::Tensor& blab,
                    const at::Tensor& d1, const at::Tensor& d2, at::Tensor& labels, at::Tensor& ub,
                    at::Tensor& lb, at::Tensor& moved_idx, at::Tensor& moved_old,
                    at::Tensor& moved_new, at::Tensor& mcount) {
  check_cuda(labels, "labels");
  const int64_t cap = active.numel();
  TORCH_CHECK(blab.numel() >= cap && d1.numel() >= cap && d2.numel() >= cap,
              "tdc.bounds_scatter: per-active arrays shorter than active");
  TORCH_CHECK(moved_idx.numel() >= cap && moved_old.numel() >= cap && moved_new.numel() >= cap,
              "tdc.bounds_scatter: moved arrays shorter than active");
  TORCH_CHECK(ub.numel() == labels.numel() && lb.numel() == labels.numel(), "tdc.bounds_scatter: ub/lb");
  const DevGuard guard(labels.device());
  check(tdc_bounds_scatter(active.data_ptr<int32_t>(), count.data_ptr<int>(), cap,
                           blab.data_ptr<int32_t>(), d1.data_ptr<float>(), d2.data_ptr<float>(),
                           labels.data_ptr<int32_t>(), ub.data_ptr<float>(), lb.data_ptr<float>(),
                           moved_idx.data_ptr<int32_t>(), moved_old.data_ptr<int32_t>(),
                           moved_new.data_ptr<int32_t>(), mcount.data_ptr<int>(), cur_stream()),
        "bounds_scatter");
}

bool assign_bigd_supported(at::ScalarType dtype, int64_t DP) {
  const int code = dtype == at::kFloat8_e4m3fn ? TDC_FP8 : (dtype == at::kBFloat16 ? TDC_BF16 : -1);
  return code >= 0 && tdc_assign_bigd_supported(code, (int)DP) != 0;
}

// X: bf16 [N, >=DP] or float8_e4m3fn [N, DP] (with Xs uint8 [N, DP/32]).
void assign_bigd(const at::Tensor& X, const std::optional<at::Tensor>& Xs, const at::Tensor& xnorm,
                 const at::Tensor& Cm2, const std::optional<at::Tensor>& Cs,
                 const at::Tensor& cnorm, int64_t kg_tiles, at::Tensor& labels,
                 const std::optional<at::Tensor>& mind, const std::optional<at::Tensor>& keys,
                 const std::optional<at::Tensor>& labels2, const std::optional<at::Tensor>& mind2) {
  check_cuda(X, "X");
  check_rows(X, "X");
  const bool fp8 = X.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(fp8 || X.scalar_type() == at::kBFloat16, "tdc.assign_bigd: X must be bf16 or float8_e4m3fn");
  TORCH_CHECK(Cm2.scalar_type() == X.scalar_type() && Cm2.is_contiguous() && Cm2.dim() == 2,
              "tdc.assign_bigd: Cm2 dtype/contiguity");
  const int64_t N = X.size(0);
  const int DP = (int)Cm2.size(1);
  const int Kp = (int)Cm2.size(0);
  TORCH_CHECK(tdc_assign_bigd_supported(fp8 ? TDC_FP8 : TDC_BF16, DP), "tdc.assign_bigd: unsupported DP ", DP);
  TORCH_CHECK(X.size(1) >= DP && Kp % 32 == 0, "tdc.assign_bigd: shapes");
  const int64_t es = fp8 ? 1 : 2;
  TORCH_CHECK((X.stride(0) * es) % 16 == 0 && reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0,
              "tdc.assign_bigd: X rows must be 16-byte aligned");
  TORCH_CHECK(cnorm.scalar_type() == at::kFloat && cnorm.is_contiguous() && cnorm.numel() >= Kp,
              "tdc.assign_bigd: cnorm fp32 [Kp]");
  TORCH_CHECK(xnorm.scalar_type() == at::kFloat && xnorm.is_contiguous() && xnorm.numel() >= N,
              "tdc.assign_bigd: xnorm fp32 [N]");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.is_contiguous() && labels.numel() >= N,
              "tdc.assign_bigd: labels int32 [N]");
  const void* xs = nullptr;
  const void* cs = nullptr;
  if (fp8) {
    TORCH_CHECK(Xs.has_value() && Cs.has_value(), "tdc.assign_bigd: fp8 needs Xs and Cs");
    TORCH_CHECK(Xs->scalar_type() == at::kByte && Xs->is_contiguous() && Xs->numel() >= N * (DP / 32),
                "tdc.assign_bigd: Xs uint8 [N, DP/32]");
    TORCH_CHECK(Cs->scalar_type() == at::kByte && Cs->is_contiguous() && Cs->numel() >= (int64_t)Kp * (DP / 32),
                "tdc.assign_bigd: Cs uint8 [Kp, DP/32]");
    TORCH_CHECK(X.stride(0) == DP, "tdc.assign_bigd: fp8 X must be [N, DP] contiguous");
    xs = Xs->data_ptr();
    cs = Cs->data_ptr();
  }
  float* md = nullptr;
  if (mind.has_value() && mind->defined()) {
    TORCH_CHECK(mind->scalar_type() == at::kFloat && mind->numel() >= N && mind->is_contiguous(),
                "tdc.assign_bigd: mind fp32 [N]");
    md = mind->data_ptr<float>();
  }
  unsigned long long* kp = nullptr;
  if (keys.has_value() && keys->defined()) {
    TORCH_CHECK(keys->scalar_type() == at::kLong && keys->is_contiguous() && keys->numel() >= N,
                "tdc.assign_bigd: keys int64 [N]");
    kp = reinterpret_cast<unsigned long long*>(keys->data_ptr());
  }
  const int ntiles = Kp / 32;
  const int kg = (kg_tiles <= 0 || kg_tiles > ntiles) ? ntiles : (int)kg_tiles;
  TORCH_CHECK(kg == ntiles || kp != nullptr, "tdc.assign_bigd: keys required with >1 centroid group");
  int32_t* l2 = nullptr;
  float* m2 = nullptr;
  if (labels2.has_value() && labels2->defined()) {
    TORCH_CHECK(fp8 && kg == ntiles, "tdc.assign_bigd: labels2 needs fp8 and one centroid group");
    TORCH_CHECK(labels2->scalar_type() == at::kInt && labels2->numel() >= N && labels2->is_contiguous(),
                "tdc.assign_bigd: labels2 int32 [N]");
    TORCH_CHECK(mind2.has_value() && mind2->defined() && mind2->scalar_type() == at::kFloat &&
                    mind2->numel() >= N && mind2->is_contiguous() && md != nullptr,
                "tdc.assign_bigd: labels2 needs mind and mind2 fp32 [N]");
    l2 = labels2->data_ptr<int32_t>();
    m2 = mind2->data_ptr<float>();
  }
  const DevGuard guard(X.device());
  check(tdc_assign_bigd(fp8 ? TDC_FP8 : TDC_BF16, X.data_ptr(), xs, N, X.stride(0), DP, Cm2.data_ptr(),
                        cs, cnorm.data_ptr<float>(), Kp, kg, xnorm.data_ptr<float>(),
                        labels.data_ptr<int32_t>(), md, kp, cur_stream(), l2, m2),
        "assign_bigd");
}

int64_t recheck_top2(const at::Tensor& X, const at::Tensor& C, at::Tensor& labels,
                     const at::Tensor& labels2, const at::Tensor& d1, const at::Tensor& d2,
                     double tau) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(X.scalar_type() == at::kBFloat16 || X.scalar_type() == at::kFloat,
              "tdc.recheck_top2: X bf16 or fp32");
  TORCH_CHECK(C.scalar_type() == at::kFloat && C.is_contiguous() && C.dim() == 2 &&
                  X.size(1) >= C.size(1), "tdc.recheck_top2: C fp32 [K, D]");
  const int64_t N = X.size(0);
  for (const at::Tensor* t : {static_cast<const at::Tensor*>(&labels), &labels2})
    TORCH_CHECK(t->scalar_type() == at::kInt && t->numel() >= N && t->is_contiguous(),
                "tdc.recheck_top2: labels int32 [N]");
  for (const at::Tensor* t : {&d1, &d2})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() >= N && t->is_contiguous(),
                "tdc.recheck_top2: distances fp32 [N]");
  const DevGuard guard(X.device());
  auto flips = at::zeros({1}, labels.options());
  check(tdc_recheck_top2(dcode(X.scalar_type()), X.data_ptr(), N, X.stride(0), (int)C.size(1),
                         C.data_ptr<float>(), labels.data_ptr<int32_t>(),
                         labels2.data_ptr<int32_t>(), d1.data_ptr<float>(), d2.data_ptr<float>(),
                         (float)tau, flips.data_ptr<int>(), cur_stream()),
        "recheck_top2");
  return 0;  // the flip count stays on the device (no host sync in the iteration)
}

void quant_fp8(const at::Tensor& X, int64_t valid, int64_t neg2, at::Tensor& Q, at::Tensor& S,
               const std::optional<at::Tensor>& norm) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(Q.scalar_type() == at::kFloat8_e4m3fn && Q.is_contiguous() && Q.dim() == 2,
              "tdc.quant_fp8: Q float8_e4m3fn [rows, DP]");
  const int64_t rows = Q.size(0);
  const int DP = (int)Q.size(1);
  TORCH_CHECK(DP % 32 == 0 && X.size(1) <= DP, "tdc.quant_fp8: DP");
  TORCH_CHECK(valid <= X.size(0) && valid <= rows, "tdc.quant_fp8: valid rows");
  TORCH_CHECK(S.scalar_type() == at::kByte && S.is_contiguous() && S.numel() >= rows * (DP / 32),
              "tdc.quant_fp8: S uint8 [rows, DP/32]");
  float* nm = nullptr;
  if (norm.has_value() && norm->defined()) {
    TORCH_CHECK(norm->scalar_type() == at::kFloat && norm->is_contiguous() && norm->numel() >= rows,
                "tdc.quant_fp8: norm fp32 [rows]");
    nm = norm->data_ptr<float>();
  }
  const DevGuard guard(X.device());
  check(tdc_quant_fp8(dcode(X.scalar_type()), X.data_ptr(), rows, valid, (int)X.size(1), X.stride(0),
                      DP, (int)neg2, Q.data_ptr(), S.data_ptr(), nm, cur_stream()),
        "quant_fp8");
}

void kpp_step(const at::Tensor& X, const at::Tensor& cand, at::Tensor& closest, int64_t mode,
              at::Tensor& pots) {
  check_cuda(X, "X");
  check_rows(X, "X");
  TORCH_CHECK(cand.is_contiguous() && cand.dim() == 2 && cand.size(1) == X.size(1),
              "tdc.kpp_step: cand [T, D]");
  TORCH_CHECK(closest.scalar_type() == cand.scalar_type() && closest.is_contiguous() &&
                  closest.numel() >= X.size(0), "tdc.kpp_step: closest [N] in the candidate dtype");
  TORCH_CHECK(pots.scalar_type() == at::kDouble && pots.is_contiguous() && pots.numel() >= cand.size(0),
              "tdc.kpp_step: pots fp64 [T]");
  const DevGuard guard(X.device());
  check(tdc_kpp_step(dcode(X.scalar_type()), dcode(cand.scalar_type()), X.data_ptr(), X.size(0),
                     X.stride(0), (int)X.size(1), cand.data_ptr(), (int)cand.size(0),
                     closest.data_ptr(), (int)mode, pots.data_ptr<double>(),
                     num_cus(X.device().index()), cur_stream()),
        "kpp_step");
}

}  // namespace

TORCH_LIBRARY(tdc, m) {
  m.def("assign_bf16(Tensor X, Tensor Cm2, Tensor cnorm, Tensor(a!) labels, Tensor(b!)? mind) -> ()");
  m.def("assign_simt(Tensor X, Tensor C, Tensor(a!) labels, Tensor(b!)? mind) -> ()");
  m.def("assign_exact(Tensor X, Tensor C, Tensor(a!) labels, Tensor(b!)? mind) -> ()");
  m.def("lloyd_small_supported(ScalarType dtype, int K, int D) -> bool", &lloyd_small_supported);
  m.def("lloyd_small(Tensor X, Tensor C, Tensor(a!)? labels, Tensor(b!)? mind, Tensor(c!) sums, Tensor(d!) counts) -> ()");
  m.def("update(Tensor X, Tensor labels, Tensor(a!) sums, Tensor(b!) counts) -> ()");
  m.def("update_sorted_workspace(int N, int K) -> int", &update_sorted_workspace);
  m.def("update_sorted(Tensor X, Tensor labels, Tensor(a!) sums, Tensor(b!) counts, Tensor(c!) work, Tensor(d!)? cnt_hi=None, Tensor(e!)? cnt_lo=None, Tensor(f!)? zero_first=None, float fixed_scale=0.0, bool work_clean=False) -> ()");
  m.def("fcm_small_supported(ScalarType dtype, int K, int D) -> bool", &fcm_small_supported);
  m.def("fcm_small(Tensor X, Tensor C, float m, bool nan_to_zero, Tensor(a!)? labels, Tensor(b!) wx, Tensor(c!) ws) -> ()");
  m.def("fcm_tower_stats(Tensor X, Tensor C, float m, bool nan_to_zero, Tensor(a!) labels, Tensor(b!) rowinfo) -> ()");
  m.def("fcm_tower_accum(Tensor X, Tensor C, float m, bool nan_to_zero, Tensor rowinfo, Tensor(a!) wx, Tensor(b!) ws) -> ()");
  m.def("fcm_wide(int stage, Tensor X, Tensor C, float m, bool nan_to_zero, Tensor(a!) G, Tensor(b!)? labels=None, Tensor(c!)? wx=None, Tensor(d!)? ws=None) -> ()");
  m.def("fcm_wide_rows(Tensor(a!) G, int K, float m, bool nan_to_zero, Tensor(b!) labels, bool write_w) -> ()");
  m.def("fcm_f64t(int stage, Tensor X, Tensor C, float m, bool nan_to_zero, Tensor(a!) G, Tensor(b!) rowinfo, Tensor(c!)? labels=None, Tensor(d!)? wx=None, Tensor(e!)? ws=None) -> ()");
  m.def("fcm_mfma_wide_workspace(Tensor like, int M, int Kp, int DP) -> int");
  m.def("fcm_mfma_wide(int stage, Tensor Xh, Tensor Xl, Tensor xx, Tensor Ch, Tensor Cl, Tensor cc, int K, int D, Tensor(a!) G, Tensor(b!)? work=None, Tensor? shift=None, Tensor(c!)? wx=None, Tensor(d!)? ws=None) -> ()");
  m.def("fcm_split_rows(Tensor src, int valid, int neg2, Tensor(a!) hi, Tensor(b!) lo, Tensor(c!)? norm, Tensor? shift=None) -> ()");
  m.def("fcm_mfma_stats(Tensor Xh, Tensor Xl, Tensor xx, Tensor Ch, Tensor Cl, Tensor cc, int K, float m, bool nan_to_zero, Tensor(a!) labels, Tensor(b!) rowinfo) -> ()");
  m.def("fcm_mfma_accum(Tensor Xh, Tensor Xl, Tensor xx, Tensor rowinfo, Tensor Ch, Tensor Cl, Tensor cc, int K, float m, bool nan_to_zero, Tensor(a!) wx, Tensor(b!) ws, Tensor(c!) work, Tensor? shift=None, Tensor? Xr=None) -> ()");
  m.def("fcm_mfma_workspace(Tensor like, int N, int K, int Kp, int DP) -> int");
  m.def("fcm_mfma_rowinfo_len(Tensor like, int N, int DP) -> int");
  m.def("assign_bigd_supported(ScalarType dtype, int DP) -> bool", &assign_bigd_supported);
  m.def("assign_bigd(Tensor X, Tensor? Xs, Tensor xnorm, Tensor Cm2, Tensor? Cs, Tensor cnorm, int kg_tiles, Tensor(a!) labels, Tensor(b!)? mind, Tensor(c!)? keys, Tensor(d!)? labels2=None, Tensor(e!)? mind2=None) -> ()");
  m.def("recheck_top2(Tensor X, Tensor C, Tensor(a!) labels, Tensor labels2, Tensor d1, Tensor d2, float tau) -> int");
  m.def("quant_fp8(Tensor X, int valid, int neg2, Tensor(a!) Q, Tensor(b!) S, Tensor(c!)? norm) -> ()");
  m.def("kpp_step(Tensor X, Tensor cand, Tensor(a!) closest, int mode, Tensor(b!) pots) -> ()");
  m.def("finalize(Tensor? sums, Tensor? counts, Tensor(a!) C, int policy, Tensor(b!)? shift, Tensor(c!)? Cm2, Tensor(d!)? cnorm, Tensor(e!)? drift=None, Tensor(f!)? maxdrift=None, float fixed_scale=0.0) -> ()");
  m.def("assign_bf16_indexed(Tensor X, Tensor rowidx, Tensor Cm2, Tensor cnorm, Tensor(a!) labels, Tensor(b!)? mind) -> ()");
  m.def("update_sorted_indexed(Tensor X, Tensor rowidx, Tensor labels, Tensor(a!) sums, Tensor(b!) counts, Tensor(c!) work, Tensor(d!)? cnt_hi=None, Tensor(e!)? cnt_lo=None, bool work_clean=False, Tensor(f!)? zero_first=None) -> ()");
  m.def("assign_bf16_top2(Tensor X, Tensor? rowidx, Tensor Cm2, Tensor cnorm, Tensor(a!) labels, Tensor(b!) mind, Tensor(c!) mind2) -> ()");
  m.def("bounds_filter(Tensor labels, Tensor(a!) ub, Tensor(b!) lb, Tensor drift, Tensor maxdrift, float slack, Tensor(c!) active, Tensor(d!) count) -> ()");
  m.def("bounds_scatter(Tensor active, Tensor count, Tensor blab, Tensor d1, Tensor d2, Tensor(a!) labels, Tensor(b!) ub, Tensor(c!) lb, Tensor(d!) moved_idx, Tensor(e!) moved_old, Tensor(f!) moved_new, Tensor(g!) mcount) -> ()");
  m.def("delta_workspace(int N, int K) -> int", &delta_workspace);
  m.def("delta_update(Tensor X, Tensor labels, Tensor(a!) prev, Tensor(b!) sums, Tensor(c!) counts, Tensor(d!) work, Tensor(e!) ctrl, Tensor(f!)? cnt_hi=None, Tensor(g!)? cnt_lo=None, Tensor(h!)? moved=None, Tensor(i!)? zero_first=None, float fixed_scale=0.0, bool work_clean=False) -> ()");
  m.def("delta_finalize(Tensor sums, Tensor counts, Tensor? cnt_hi, Tensor? cnt_lo, Tensor? moved, Tensor(a!) G, Tensor(b!) C, int policy, Tensor(c!)? shift, Tensor(d!)? Cm2, Tensor(e!)? cnorm, Tensor(f!) ctrl, Tensor(g!)? stats, int refresh, float theta_n, float fixed_scale=0.0) -> ()");
  m.def("sculley_update(Tensor sums, Tensor counts, Tensor(a!) C, Tensor(b!) v, Tensor(c!)? shift, Tensor(d!)? Cm2, Tensor(e!)? cnorm) -> ()");
  m.def("x3_split(Tensor src, int valid, int neg2, Tensor(a!) hi, Tensor(b!) lo, Tensor(c!)? norm, Tensor(d!)? nhl=None, Tensor? shift=None) -> ()");
  m.def("x3_prep(Tensor cnorm, Tensor? nhl, int K, Tensor(a!) cstat, Tensor(b!) amb_count) -> ()");
  m.def("x3_assign(Tensor X, Tensor Xh, Tensor Xl, Tensor Ch, Tensor Cl, Tensor cnorm, Tensor cnhl, Tensor C, Tensor(a!) labels, Tensor(b!)? mind, Tensor(c!) amb, Tensor(d!) cstat, Tensor(e!) amb_count, bool recheck=True, Tensor(f!)? pre=None, Tensor? xnhl=None, int pre_est=-1) -> ()");
  m.def("x3_rows(Tensor G, int row0, Tensor xx, Tensor cstat, int DP, Tensor(a!) labels, Tensor(b!) amb, Tensor(c!) amb_count) -> ()");
  m.def("x3_recheck(Tensor X, Tensor C, Tensor(a!) labels, Tensor amb, Tensor amb_count) -> ()");
}

TORCH_LIBRARY_IMPL(tdc, CUDA, m) {
  m.impl("assign_bf16", &assign_bf16);
  m.impl("assign_simt", &assign_simt);
  m.impl("assign_exact", &assign_exact);
  m.impl("lloyd_small", &lloyd_small);
  m.impl("update", &update);
  m.impl("update_sorted", &update_sorted);
  m.impl("fcm_small", &fcm_small);
  m.impl("fcm_tower_stats", &fcm_tower_stats);
  m.impl("fcm_split_rows", &fcm_split_rows);
  m.impl("fcm_mfma_stats", &fcm_mfma_stats);
  m.impl("fcm_mfma_accum", &fcm_mfma_accum);
  m.impl("fcm_mfma_workspace", &fcm_mfma_workspace);
  m.impl("fcm_mfma_rowinfo_len", &fcm_mfma_rowinfo_len);
  m.impl("fcm_tower_accum", &fcm_tower_accum);
  m.impl("fcm_wide", &fcm_wide);
  m.impl("fcm_wide_rows", &fcm_wide_rows);
  m.impl("fcm_f64t", &fcm_f64t);
  m.impl("fcm_mfma_wide_workspace", &fcm_mfma_wide_workspace);
  m.impl("fcm_mfma_wide", &fcm_mfma_wide);
  m.impl("finalize", &finalize);
  m.impl("delta_update", &delta_update);
  m.impl("delta_finalize", &delta_finalize);
  m.impl("assign_bigd", &assign_bigd);
  m.impl("recheck_top2", &recheck_top2);
  m.impl("quant_fp8", &quant_fp8);
  m.impl("kpp_step", &kpp_step);
  m.impl("assign_bf16_indexed", &assign_bf16_indexed);
  m.impl("update_sorted_indexed", &update_sorted_indexed);
  m.impl("sculley_update", &sculley_update);
  m.impl("assign_bf16_top2", &assign_bf16_top2);
  m.impl("bounds_filter", &bounds_filter);
  m.impl("bounds_scatter", &bounds_scatter);
  m.impl("x3_split", &x3_split);
  m.impl("x3_prep", &x3_prep);
  m.impl("x3_assign", &x3_assign);
  m.impl("x3_rows", &x3_rows);
  m.impl("x3_recheck", &x3_recheck);
}
