// query_order.cpp — order the source queries so that every 64 consecutive queries (one wave)
// are spatially compact: a kd partition with 64-point buckets, each split on the longest axis
// of the node's bounding box at a multiple of 64 near the median (std::nth_element), and each
// 64-bucket split on down to `bucket` points (aligned lane groups of the search kernel). Buckets of
// this partition have bounded aspect ratio, unlike Z-order runs, which jump across cell
// boundaries; the wave-cooperative search scans ~the points of one bucket's neighbourhood.
#include "query_order.h"

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

namespace icp {

namespace {

struct Part {
  const double* xyz;
  int bucket;

  void run(int32_t* idx, int64_t n, int depth_threads) {
    while (n > bucket) {
      double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
      for (int64_t k = 0; k < n; k++) {
        const double* p = xyz + 3 * (int64_t)idx[k];
        for (int a = 0; a < 3; a++) {
          const double v = std::isfinite(p[a]) ? p[a] : 0.0;
          lo[a] = v < lo[a] ? v : lo[a];
          hi[a] = v > hi[a] ? v : hi[a];
        }
      }
      int ax = 0;
      for (int a = 1; a < 3; a++)
        if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
      // splits at multiples of 64 (one wave) while the range is larger than a wave, then at
      // multiples of `bucket` inside it: a wave's lanes form aligned kd sub-buckets
      const int64_t unit = n > 64 ? 64 : bucket;
      int64_t h = ((n / 2 + unit - 1) / unit) * unit;
      if (h >= n) h = n - unit;
      const double* X = xyz;
      auto key = [X, ax](int32_t i) {
        const double v = X[3 * (int64_t)i + ax];
        return std::isfinite(v) ? v : 0.0;
      };
      std::nth_element(idx, idx + h, idx + n, [&](int32_t a, int32_t b) {
        const double ka = key(a), kb = key(b);
        return ka < kb || (ka == kb && a < b);
      });
      if (depth_threads > 0) {
        std::thread t([this, idx, h, depth_threads]() { run(idx, h, depth_threads - 1); });
        run(idx + h, n - h, depth_threads - 1);
        t.join();
        return;
      }
      run(idx, h, 0);
      idx += h;
      n -= h;
    }
  }
};

}  // namespace

void kd_query_order(const double* xyz, int64_t n, int bucket, std::vector<int32_t>* perm) {
  perm->resize((size_t)n);
  for (int64_t i = 0; i < n; i++) (*perm)[i] = (int32_t)i;
  if (n <= bucket) return;
  Part p{xyz, bucket};
  unsigned hw = std::thread::hardware_concurrency();
  int levels = 0;
  while ((1u << (levels + 1)) <= (hw ? hw : 1u) && levels < 4) levels++;
  if (n < (int64_t)1 << 16) levels = 0;
  p.run(perm->data(), n, levels);
}

}  // namespace icp
