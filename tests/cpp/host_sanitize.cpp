// CPU self-test of libicp_hip.so's host-side code, built with sanitizers (csrc/Makefile targets
// asan = AddressSanitizer + UndefinedBehaviorSanitizer, tsan = ThreadSanitizer) and run by
// tests/test_sanitize.py. No HIP call is made; the sources are the product's own:
//   lasio.cpp          the LAS readers/writers on the given files (golden, truncated, garbage)
//   octree_build.cpp   the host octree builder on random, degenerate and duplicated clouds
//   query_order.cpp    the host kd query order (its worker threads)
//   svd3_impl.h        3x3 Jacobi SVD and best fit on random, singular and non-finite matrices
//   session_step.h     the session's decisions (engine.cpp's loop) on random statistic sequences
//   group_sync.h       Driver threads + LocalExchange (the multi-device context's host transport)
//                      with N members, thousands of exchanges and injected member failures
// Exit status 0 and one "ok" line when every check passed; the sanitizers abort on their findings.
//
// usage: host_sanitize [las files...]
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <unistd.h>
#include <vector>

#include "../../include/icp_las.h"
#include "../../iterativeclosestpoint_amd/csrc/group_sync.h"
#include "../../iterativeclosestpoint_amd/csrc/octree_build.h"
#include "../../iterativeclosestpoint_amd/csrc/query_order.h"
#include "../../iterativeclosestpoint_amd/csrc/session_step.h"
#include "../../iterativeclosestpoint_amd/csrc/svd3_impl.h"

static int g_fail = 0;
#define CHECK(c)                                                            \
  do {                                                                      \
    if (!(c)) {                                                             \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                             \
    }                                                                       \
  } while (0)

static std::string tmp_path(const char* tag) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), "/tmp/icp_host_sanitize_%d_%s.las", (int)getpid(), tag);
  return buf;
}

static void las_file(const char* path) {
  for (int rules : {ICP_LAS_CORE, ICP_LAS_CLI}) {
    icp_las_header h;
    const int rc = icp_las_read_header(path, rules, &h);
    if (rc != 0) continue;  // unreadable or rejected: the error path itself is what ran
    const int64_t n = h.num_points;
    // the buffer the caller sizes from the header (a garbage header may claim 4e9 points: bounded
    // by max_points, which is also the buffer capacity for both rules)
    const int64_t big = n < 100000 ? 0 : 100000;
    for (int64_t cap : {big, (int64_t)1, (n < 100000 ? n : 100000) / 2 + 1}) {
      const int64_t want = cap > 0 && cap < n ? cap : n;
      std::vector<double> xyz((size_t)(3 * (want > 0 ? want : 1)));
      const int64_t got = icp_las_read(path, rules, cap, xyz.data(), &h);
      CHECK(got <= want);  // negative: a short file is reported, not overrun
      if (got > 0) {
        const std::string a = tmp_path("core"), b = tmp_path("cli");
        CHECK(icp_las_write_core(a.c_str(), xyz.data(), got) == 0);
        CHECK(icp_las_write_cli(b.c_str(), xyz.data(), got, h.scale, h.offset) == 0);
        std::vector<double> back((size_t)(3 * got));
        CHECK(icp_las_read(a.c_str(), ICP_LAS_CORE, 0, back.data(), &h) == got);
        CHECK(icp_las_read(b.c_str(), ICP_LAS_CLI, 0, back.data(), &h) == got);
        std::remove(a.c_str());
        std::remove(b.c_str());
      }
    }
  }
}

static void octrees(std::mt19937_64& rng) {
  std::normal_distribution<double> g(0.0, 1.0);
  const int sizes[] = {1, 2, 17, 1000, 20000};
  const int params[][2] = {{1, 1}, {10, 20}, {3, 60}, {1, 0}};
  for (int n : sizes)
    for (auto& pr : params) {
      std::vector<double> xyz((size_t)(3 * n));
      for (auto& v : xyz) v = g(rng);
      if (n > 10)
        for (int i = 0; i < n / 3; i++)  // duplicates: force max-depth leaves
          for (int k = 0; k < 3; k++) xyz[3 * i + k] = xyz[k];
      icp::FlatOctree t;
      const char* why = nullptr;
      CHECK(icp::build_flat_octree(xyz.data(), n, pr[0], pr[1], &t, &why));
      CHECK((int64_t)t.pts.size() == n);
      int64_t in_leaves = 0;
      for (const auto& nd : t.nodes)
        if (nd.meta & icp::kLeafBit) in_leaves += nd.meta & ~icp::kLeafBit;
      CHECK(in_leaves == n);
    }
  std::vector<double> bad = {0.0, 0.0, 0.0, NAN, 1.0, 2.0};
  icp::FlatOctree t;
  const char* why = nullptr;
  CHECK(!icp::build_flat_octree(bad.data(), 2, 10, 20, &t, &why));
}

static void query_orders(std::mt19937_64& rng) {
  std::uniform_real_distribution<double> u(-5.0, 5.0);
  for (int n : {1, 63, 64, 65, 1000, 100000}) {
    std::vector<double> xyz((size_t)(3 * n));
    for (auto& v : xyz) v = u(rng);
    std::vector<int32_t> perm;
    icp::kd_query_order(xyz.data(), n, 8, &perm);
    CHECK((int)perm.size() == n);
    std::vector<char> seen((size_t)n, 0);
    for (int32_t p : perm) {
      CHECK(p >= 0 && p < n);
      if (p >= 0 && p < n) seen[p]++;
    }
    for (char s : seen) CHECK(s == 1);
  }
}

static void svds(std::mt19937_64& rng) {
  std::normal_distribution<double> g(0.0, 1.0);
  for (int k = 0; k < 2000; k++) {
    double H[9], U[9], S[3], V[9];
    for (auto& h : H) h = g(rng);
    if (k % 7 == 1)
      for (int i = 3; i < 9; i++) H[i] = H[i % 3] * (i / 3);  // rank one
    if (k % 11 == 2)
      for (auto& h : H) h = 0.0;
    if (k % 13 == 3) H[4] = NAN;
    icp::svd::jacobi_svd3(H, U, S, V);
    if (k % 13 != 3) CHECK(S[0] >= S[1] && S[1] >= S[2] && S[2] >= 0.0);
    double T[16];
    const double ma[3] = {g(rng), g(rng), g(rng)}, mb[3] = {g(rng), g(rng), g(rng)};
    icp::svd::best_fit_from_moments(ma, mb, H, T);
    double C[16];
    icp::svd::mat4_mul(T, T, C);
  }
}

static void sessions(std::mt19937_64& rng) {
  std::uniform_real_distribution<double> u(0.0, 1.0);
  for (int k = 0; k < 3000; k++) {
    icp::SessionCore s;
    icp::SessionParams p{k % 3 == 0 ? 0.0 : 1e-6, 1 + (int32_t)(k % 60), (int32_t)(k % 2), (int32_t)(k % 5 == 0), 0};
    icp::session_core_init(s, p.max_iterations);
    double rmse = 1.0;
    int steps = 0;
    while (!s.done && steps < 1000) {
      rmse *= (k % 4 == 0) ? 1.2 : (0.5 + u(rng));
      if (k % 17 == 5 && steps == 3) rmse = NAN;
      const int64_t valid = (k % 9 == 4 && steps == 2) ? 2 : (int64_t)1 << (20 + k % 12);
      double ma[3] = {u(rng), u(rng), u(rng)}, mb[3] = {u(rng), u(rng), u(rng)}, H[9];
      for (auto& h : H) h = u(rng) - 0.5;
      icp::session_core_step(s, p, rmse, valid, ma, mb, H);
      steps++;
    }
    CHECK(s.done && steps <= p.max_iterations);
  }
}

// The multi-device context's host transport: n members on their driver threads, exchanges of
// three records per job (as an iterate's two plus one), a member that fails before joining (it
// raises the abort flag and wakes the others, who give up), the per-job reset (icp_group.cpp
// for_members).
static void group_exchange(int n, int jobs) {
  std::atomic<int> abort{0};
  icp::LocalExchange lx;
  lx.n = n;
  lx.abort = &abort;
  std::vector<icp::ExchangeSlot> slots((size_t)n);
  std::vector<std::unique_ptr<icp::Driver>> drivers;
  for (int k = 0; k < n; k++) {
    slots[k] = icp::ExchangeSlot{&lx, k};
    drivers.push_back(std::make_unique<icp::Driver>());
  }
  std::atomic<int> bad{0};
  for (int job = 0; job < jobs; job++) {
    abort.store(0);
    lx.reset();
    const int failing = (job % 7 == 3) ? job % n : -1;
    for (int k = 0; k < n; k++) {
      drivers[k]->post([&, k, job, failing] {
        if (k == failing) {  // fails before its first exchange
          abort.store(1);
          lx.wake();
          return;
        }
        for (int r = 0; r < 3; r++) {
          double local[2] = {1000.0 * k + job, (double)r};
          std::vector<double> all((size_t)(2 * n));
          if (icp::local_exchange(&slots[k], local, 2, all.data()) != 0) {
            if (failing < 0) bad++;  // nobody failed: an exchange must not give up
            return;
          }
          for (int m = 0; m < n; m++)
            if (all[2 * m] != 1000.0 * m + job || all[2 * m + 1] != (double)r) bad++;
        }
      });
    }
    for (auto& d : drivers) d->wait();
  }
  CHECK(bad.load() == 0);
}

int main(int argc, char** argv) {
  std::mt19937_64 rng(2024);
  for (int i = 1; i < argc; i++) las_file(argv[i]);
  octrees(rng);
  query_orders(rng);
  svds(rng);
  sessions(rng);
  for (int n : {2, 3, 8}) group_exchange(n, 400);
  if (g_fail) {
    std::printf("FAILED %d checks\n", g_fail);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
