// Torch-free core of the native host-side row streamer (see loader.cpp for the role it
// plays): a pool of worker threads converting row ranges of a host matrix (f64 / f32, any
// row stride) into a caller-owned buffer in the kernel layout (bf16 RNE, f32 or f64,
// zero-padded to dp columns; f64 -> f64 is a row copy, so the exact fp64 kernels stream
// through the same pinned ring as the bf16 ones).  submit() is asynchronous and returns a ticket; wait(ticket) blocks until
// every piece of that submission is converted.  Kept free of torch so the thread pool can
// be built and stress-tested on its own under ThreadSanitizer / AddressSanitizer
// (tests/native/row_streamer_test.cpp, tests/test_native_sanitizers.py).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <unordered_map>
#include <vector>

namespace tdc {

inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

enum SrcType { SRC_F64 = 0, SRC_F32 = 1 };
enum DstType { DST_BF16 = 0, DST_F32 = 1, DST_F64 = 2 };

class RowStreamerCore {
 public:
  RowStreamerCore(const void* src, int64_t src_type, int64_t n_rows, int64_t n_cols,
                  int64_t src_ld, int64_t dst_type, int64_t dp, int64_t n_threads)
      : src_(static_cast<const char*>(src)), src_type_(src_type), n_rows_(n_rows),
        n_cols_(n_cols), src_ld_(src_ld), dst_type_(dst_type), dp_(dp) {
    if (src == nullptr) throw std::invalid_argument("RowStreamer: null source");
    if (src_type != SRC_F64 && src_type != SRC_F32)
      throw std::invalid_argument("RowStreamer: src must be f64/f32");
    if (dst_type != DST_BF16 && dst_type != DST_F32 && dst_type != DST_F64)
      throw std::invalid_argument("RowStreamer: dst must be bf16/f32/f64");
    if (dp < n_cols) throw std::invalid_argument("RowStreamer: padded width smaller than the row");
    const int64_t nt = n_threads > 0 ? n_threads : 4;
    for (int64_t i = 0; i < nt; ++i) workers_.emplace_back([this] { loop(); });
  }

  ~RowStreamerCore() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

  RowStreamerCore(const RowStreamerCore&) = delete;
  RowStreamerCore& operator=(const RowStreamerCore&) = delete;

  // fill out[0:rows, 0:dp] (dst layout) with source rows [start, start+rows)
  int64_t submit(void* out_ptr, int64_t start, int64_t rows) {
    if (start < 0 || rows < 0 || start + rows > n_rows_)
      throw std::out_of_range("RowStreamer: range out of bounds");
    char* out = static_cast<char*>(out_ptr);
    const int64_t ticket = next_ticket_++;
    const int64_t pieces = std::max<int64_t>(1, std::min<int64_t>((int64_t)workers_.size() * 2,
                                                                  (rows + 4095) / 4096));
    {
      std::lock_guard<std::mutex> g(mu_);
      pending_[ticket] = pieces;
      const int64_t per = (rows + pieces - 1) / pieces;
      for (int64_t p = 0; p < pieces; ++p) {
        const int64_t r0 = std::min(rows, p * per), r1 = std::min(rows, r0 + per);
        q_.push_back([=] { convert(out, start, r0, r1); finish(ticket); });
      }
    }
    cv_.notify_all();
    return ticket;
  }

  void wait(int64_t ticket) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_.find(ticket) == pending_.end(); });
  }

  int64_t rows() const { return n_rows_; }
  int64_t cols() const { return n_cols_; }
  int64_t dp() const { return dp_; }
  int64_t dst_type() const { return dst_type_; }

 private:
  void convert(char* out, int64_t start, int64_t r0, int64_t r1) {
    const size_t es = src_type_ == SRC_F64 ? 8 : 4;
    for (int64_t r = r0; r < r1; ++r) {
      const char* srow = src_ + (size_t)(start + r) * src_ld_ * es;
      if (dst_type_ == DST_BF16) {
        uint16_t* drow = reinterpret_cast<uint16_t*>(out) + (size_t)r * dp_;
        if (src_type_ == SRC_F64) {
          const double* s = reinterpret_cast<const double*>(srow);
          for (int64_t c = 0; c < n_cols_; ++c) drow[c] = f32_to_bf16_rne((float)s[c]);
        } else {
          const float* s = reinterpret_cast<const float*>(srow);
          for (int64_t c = 0; c < n_cols_; ++c) drow[c] = f32_to_bf16_rne(s[c]);
        }
        for (int64_t c = n_cols_; c < dp_; ++c) drow[c] = 0;
      } else if (dst_type_ == DST_F64) {
        double* drow = reinterpret_cast<double*>(out) + (size_t)r * dp_;
        if (src_type_ == SRC_F64) {
          std::memcpy(drow, srow, (size_t)n_cols_ * 8);
        } else {
          const float* s = reinterpret_cast<const float*>(srow);
          for (int64_t c = 0; c < n_cols_; ++c) drow[c] = (double)s[c];
        }
        for (int64_t c = n_cols_; c < dp_; ++c) drow[c] = 0.0;
      } else {
        float* drow = reinterpret_cast<float*>(out) + (size_t)r * dp_;
        if (src_type_ == SRC_F64) {
          const double* s = reinterpret_cast<const double*>(srow);
          for (int64_t c = 0; c < n_cols_; ++c) drow[c] = (float)s[c];
        } else {
          std::memcpy(drow, srow, (size_t)n_cols_ * 4);
        }
        for (int64_t c = n_cols_; c < dp_; ++c) drow[c] = 0.f;
      }
    }
  }

  void finish(int64_t ticket) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = pending_.find(ticket);
    if (it != pending_.end() && --(it->second) == 0) {
      pending_.erase(it);
      done_cv_.notify_all();
    }
  }

  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }

  const char* src_;
  int64_t src_type_, n_rows_, n_cols_, src_ld_, dst_type_, dp_;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::function<void()>> q_;
  std::unordered_map<int64_t, int64_t> pending_;
  std::atomic<int64_t> next_ticket_{0};
  bool stop_ = false;
};

}  // namespace tdc
