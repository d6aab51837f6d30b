// ref_bench.cpp — TEST INFRASTRUCTURE ONLY: times the REFERENCE CPU path for bench.py's
// cpu_baseline leg (kind "reference").
//
// Usage: ref_bench <target.f64> <source_sample.f64>
//   both files: raw little-endian fp64 AoS xyz.
// Builds the reference Octree over the full target (untimed: the reference builds it once per
// registration), then times ICP() from icp_registration.cpp:443-622 with max_iterations 1 and 2
// on the source sample; one reference iteration = t(2) - t(1) (cancels the octree build).
// Prints one JSON line on stdout (the reference's own cout chatter goes to /dev/null).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define main icp_reference_cli_main
#include "icp_registration.cpp"
#undef main

static std::vector<Point3D> load(const char* path) {
  std::vector<Point3D> v;
  FILE* f = std::fopen(path, "rb");
  if (!f) return v;
  std::fseek(f, 0, SEEK_END);
  long bytes = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<double> raw(bytes / 8);
  size_t got = std::fread(raw.data(), 8, raw.size(), f);
  std::fclose(f);
  v.reserve(got / 3);
  for (size_t i = 0; i + 2 < got; i += 3) v.emplace_back(raw[i], raw[i + 1], raw[i + 2]);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: ref_bench target.f64 source.f64\n");
    return 2;
  }
  PointCloud tgt, src;
  tgt.points = load(argv[1]);
  src.points = load(argv[2]);
  if (tgt.points.empty() || src.points.empty()) return 3;
  std::streambuf* old = std::cout.rdbuf();
  std::ofstream devnull("/dev/null");
  std::cout.rdbuf(devnull.rdbuf());
  double secs[2];
  for (int k = 0; k < 2; k++) {
    PointCloud s = src;
    double R[3][3], t[3];
    auto t0 = std::chrono::steady_clock::now();
    ICP(s, tgt, k + 1, 1e-300, R, t, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    secs[k] = std::chrono::duration<double>(t1 - t0).count();
  }
  std::cout.rdbuf(old);
  double iter_s = secs[1] - secs[0];
  std::printf("{\"n_source_sample\": %zu, \"n_target\": %zu, \"t_icp1_s\": %.6f, \"t_icp2_s\": %.6f, "
              "\"iter_s\": %.6f, \"mcorr_per_s\": %.6f}\n",
              src.points.size(), tgt.points.size(), secs[0], secs[1], iter_s,
              src.points.size() / iter_s / 1e6);
  return 0;
}
