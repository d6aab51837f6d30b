// Compile-and-run check of the C++ drop-in facade (include/icp_engine.hpp): the reference's
// ICPEngine / Octree / ICP() call shapes against libicp_hip.so. Built by tests/test_cpp_facade.py.
#include <cmath>
#include <cstdio>
#include <random>

#include "icp_engine.hpp"

int main() {
  std::mt19937_64 rng(5);
  std::normal_distribution<double> g(0.0, 1.0);
  icp_amd::PointCloud tgt, src;
  for (int i = 0; i < 20000; i++) tgt.points.emplace_back(8 * g(rng), 4 * g(rng), 1.5 * g(rng));
  const double a = 0.01, c = std::cos(a), s = std::sin(a);
  for (const auto& p : tgt.points) src.points.emplace_back(c * p.x + s * p.y - 0.02, -s * p.x + c * p.y + 0.01, p.z);
  icp_amd::ICPEngine engine;
  int iters = 0;
  bool ok = false;
  engine.onIterationCompleted = [&](const icp_amd::IterationResult&) { iters++; };
  engine.onFinished = [&](bool success, const std::string&) { ok = success; };
  icp_amd::ICPParameters p;
  p.tolerance = 1e-12;
  engine.setParameters(p);
  engine.registerPointClouds(&src, &tgt);
  const icp_amd::ICPResult r = engine.getResult();
  double err = 0;
  for (size_t i = 0; i < src.size(); i++)
    err = std::fmax(err, std::fabs(src.points[i].x - tgt.points[i].x) + std::fabs(src.points[i].y - tgt.points[i].y));
  icp_amd::Octree tree(tgt.points);
  const int nn = tree.findNearest(tgt.points[123]);
  std::vector<int> many = tree.findNearest(std::vector<icp_amd::Point3D>(tgt.points.begin(), tgt.points.begin() + 100));
  bool many_ok = true;
  for (int i = 0; i < 100; i++) many_ok = many_ok && many[i] == i;
  icp_amd::PointCloud src2;
  for (const auto& p2 : tgt.points) src2.points.emplace_back(p2.x + 0.01, p2.y, p2.z);
  double R[3][3], t[3];
  std::vector<icp_amd::Matrix4> hist;
  icp_amd::ICP(src2, tgt, 20, 1e-2, R, t, &hist);
  std::printf("{\"ok\": %d, \"success\": %d, \"iterations\": %d, \"history\": %zu, \"max_err\": %.3e, "
              "\"nn\": %d, \"many_ok\": %d, \"cli_transforms\": %zu}\n",
              ok, r.success, r.totalIterations, r.iterationHistory.size(), err, nn, many_ok, hist.size());
  return (ok && r.success && err < 1e-6 && nn == 123 && many_ok) ? 0 : 1;
}
