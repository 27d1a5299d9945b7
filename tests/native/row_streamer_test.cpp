// Stress test of tdc::RowStreamerCore (csrc/row_streamer.h) for the sanitizer builds run
// by tests/test_native_sanitizers.py: -fsanitize=thread (data races in the worker pool,
// the ticket map and the condition variables) and -fsanitize=address,undefined (bounds of
// the row conversion, padding, lifetime of queued jobs at destruction).
//
// Several caller threads submit overlapping-in-time conversions of random row ranges into
// their own buffers, wait for them in a shuffled order and check every converted value
// (bf16 round-to-nearest-even, f32 and the exact f64 copy, zero padding up to dp).  Exit code 0 = pass.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "row_streamer.h"

static float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

static int check(const std::vector<double>& src, int64_t ld, int64_t cols, int64_t dp,
                 int dst_type, const std::vector<char>& out, int64_t start, int64_t rows) {
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t c = 0; c < dp; ++c) {
      const double want = c < cols ? src[(size_t)(start + r) * ld + c] : 0.0;
      double got;
      if (dst_type == tdc::DST_BF16) {
        got = bf16_to_f32(reinterpret_cast<const uint16_t*>(out.data())[(size_t)r * dp + c]);
        if (std::fabs(got - want) > std::fabs(want) * (1.0 / 256) + 1e-30) return 1;
      } else if (dst_type == tdc::DST_F64) {
        got = reinterpret_cast<const double*>(out.data())[(size_t)r * dp + c];
        if (got != want) return 1;
      } else {
        got = reinterpret_cast<const float*>(out.data())[(size_t)r * dp + c];
        if (got != (double)(float)want) return 1;
      }
    }
  return 0;
}

int main() {
  const int64_t n = 20000, cols = 37, ld = 41, dp = 48;
  std::vector<double> src((size_t)n * ld);
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd(0.0, 3.0);
  for (auto& v : src) v = nd(rng);
  int failures = 0;
  for (int dst_type : {tdc::DST_BF16, tdc::DST_F32, tdc::DST_F64}) {
    const size_t es = dst_type == tdc::DST_BF16 ? 2 : dst_type == tdc::DST_F64 ? 8 : 4;
    for (int round = 0; round < 3; ++round) {
      tdc::RowStreamerCore rs(src.data(), tdc::SRC_F64, n, cols, ld, dst_type, dp, 4);
      std::vector<std::thread> callers;
      std::vector<int> fails(4, 0);
      for (int t = 0; t < 4; ++t)
        callers.emplace_back([&, t] {
          std::mt19937_64 g(100 * round + t);
          std::vector<std::vector<char>> bufs(6);
          std::vector<int64_t> tickets(6), starts(6), rows(6);
          for (int j = 0; j < 6; ++j) {
            rows[j] = 1 + (int64_t)(g() % 9000);
            starts[j] = (int64_t)(g() % (uint64_t)(n - rows[j] + 1));
            bufs[j].assign((size_t)rows[j] * dp * es, (char)0x5a);
            tickets[j] = rs.submit(bufs[j].data(), starts[j], rows[j]);
          }
          for (int j = 5; j >= 0; --j) {  // wait out of submission order
            rs.wait(tickets[j]);
            fails[t] += check(src, ld, cols, dp, dst_type, bufs[j], starts[j], rows[j]);
          }
        });
      for (auto& c : callers) c.join();
      for (int f : fails) failures += f;
      // jobs still queued when the pool is destroyed must not outlive their buffers:
      // submit + wait, then let the destructor join an idle pool
      std::vector<char> tail((size_t)100 * dp * es);
      rs.wait(rs.submit(tail.data(), n - 100, 100));
      failures += check(src, ld, cols, dp, dst_type, tail, n - 100, 100);
    }
  }
  bool threw = false;
  try {
    tdc::RowStreamerCore bad(src.data(), tdc::SRC_F64, n, cols, ld, tdc::DST_F32, dp, 2);
    bad.submit(nullptr, n - 10, 11);
  } catch (const std::out_of_range&) {
    threw = true;
  }
  if (!threw) ++failures;
  std::printf("row_streamer_test: %s (%d failures)\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
