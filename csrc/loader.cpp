// Native host-side row streamer: the MI355X-native replacement for the reference's
// tf.data streaming attempt (notebooks/batching_tests.ipynb:353-378, which hung in
// TF_ExtendGraph) and its OOM-driven host batching (scripts/distribuitedClustering.py:328-360).
//
// A RowStreamer reads row ranges of a host matrix (typically a memory-mapped .npy member
// of the input NPZ, float64 or float32, any row stride) and converts them -- in a pool of
// worker threads, off the Python thread -- into a caller-owned destination buffer
// (typically a pinned tensor) in the kernel layout: bf16, fp32 or fp64, zero-padded to
// `dp` columns.  submit() is asynchronous; wait() blocks until that slot is filled.  The
// Python side (data/stream.py) rings these pinned slots and overlaps their H2D copies with
// compute on a separate HIP stream.
#include <torch/custom_class.h>
#include <torch/extension.h>

#include <memory>

#include "row_streamer.h"

namespace {

// TorchScript custom class over tdc::RowStreamerCore (tensor checks live here)
class RowStreamer : public torch::CustomClassHolder {
 public:
  RowStreamer(int64_t src_addr, int64_t src_type, int64_t n_rows, int64_t n_cols,
              int64_t src_ld, int64_t dst_type, int64_t dp, int64_t n_threads) {
    try {
      core_ = std::make_unique<tdc::RowStreamerCore>(reinterpret_cast<const void*>(src_addr),
                                                     src_type, n_rows, n_cols, src_ld, dst_type,
                                                     dp, n_threads);
    } catch (const std::exception& e) {
      TORCH_CHECK(false, e.what());
    }
  }

  // fill dst[0:rows, 0:dp] with source rows [start, start+rows); returns a ticket
  int64_t submit(at::Tensor dst, int64_t start, int64_t rows) {
    TORCH_CHECK(!dst.is_cuda(), "RowStreamer: destination must be host memory");
    TORCH_CHECK(dst.is_contiguous() && dst.dim() == 2 && dst.size(1) == core_->dp(),
                "RowStreamer: dst [rows, dp]");
    TORCH_CHECK(dst.size(0) >= rows, "RowStreamer: dst too small");
    TORCH_CHECK(start >= 0 && rows >= 0 && start + rows <= core_->rows(),
                "RowStreamer: range out of bounds");
    TORCH_CHECK((core_->dst_type() == tdc::DST_BF16 && dst.scalar_type() == at::kBFloat16) ||
                    (core_->dst_type() == tdc::DST_F32 && dst.scalar_type() == at::kFloat) ||
                    (core_->dst_type() == tdc::DST_F64 && dst.scalar_type() == at::kDouble),
                "RowStreamer: dst dtype mismatch");
    return core_->submit(dst.data_ptr(), start, rows);
  }

  void wait(int64_t ticket) { core_->wait(ticket); }
  int64_t rows() const { return core_->rows(); }
  int64_t cols() const { return core_->cols(); }

 private:
  std::unique_ptr<tdc::RowStreamerCore> core_;
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(tdc, m) {
  m.class_<RowStreamer>("RowStreamer")
      .def(torch::init<int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t>())
      .def("submit", &RowStreamer::submit)
      .def("wait", &RowStreamer::wait)
      .def("rows", &RowStreamer::rows)
      .def("cols", &RowStreamer::cols);
}
