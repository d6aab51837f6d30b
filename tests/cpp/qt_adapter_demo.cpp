// Compile-and-run check of the Qt signal adapter (include/icp_engine_qt.h): connects to every
// signal of icp_amd::QtICPEngine the way RegistrationService connects to the reference engine's
// (registrationservice.cpp:208-211), runs one registration and prints what arrived as one JSON
// line. The same registration through the plain facade (icp_engine.hpp) must give the same
// transforms: the adapter only re-emits. Built by tests/test_qt_adapter.py.
//
//   qt_adapter_demo          a 20k-point registration on the GPU
//   qt_adapter_demo empty    an empty source: finished(false, ...) and no other signal (no GPU)
#include <QCoreApplication>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>

#include "icp_engine_qt.h"

int main(int argc, char** argv) {
  QCoreApplication app(argc, argv);
  const bool empty = argc > 1 && std::strcmp(argv[1], "empty") == 0;
  std::mt19937_64 rng(11);
  std::normal_distribution<double> g(0.0, 1.0);
  icp_amd::PointCloud tgt, src;
  for (int i = 0; i < 20000; i++) tgt.points.emplace_back(8 * g(rng), 4 * g(rng), 1.5 * g(rng));
  const double a = 0.01, c = std::cos(a), s = std::sin(a);
  if (!empty)
    for (const auto& p : tgt.points) src.points.emplace_back(c * p.x + s * p.y - 0.02, -s * p.x + c * p.y + 0.01, p.z);
  icp_amd::PointCloud src_plain = src;

  icp_amd::QtICPEngine engine;
  int n_started = 0, n_progress = 0, n_iter = 0, n_finished = 0, n_log = 0, last_progress = 0;
  bool ok = false;
  QString message;
  QObject::connect(&engine, &icp_amd::QtICPEngine::started, [&]() { n_started++; });
  QObject::connect(&engine, &icp_amd::QtICPEngine::progressUpdated, [&](int it, int total, double) {
    n_progress++;
    last_progress = it;
    (void)total;
  });
  QObject::connect(&engine, &icp_amd::QtICPEngine::iterationCompleted,
                   [&](const icp_amd::IterationResult&) { n_iter++; });
  QObject::connect(&engine, &icp_amd::QtICPEngine::finished, [&](bool success, const QString& m) {
    n_finished++;
    ok = success;
    message = m;
  });
  QObject::connect(&engine, &icp_amd::QtICPEngine::logMessage, [&](const QString&) { n_log++; });
  icp_amd::ICPParameters p;
  p.maxIterations = 30;
  p.tolerance = 1e-12;
  engine.setParameters(p);
  engine.registerPointClouds(&src, &tgt);
  const icp_amd::ICPResult r = engine.getResult();

  // the same registration through the facade's std::function hooks
  bool same = true;
  if (!empty) {
    icp_amd::ICPEngine plain;
    plain.setParameters(p);
    plain.registerPointClouds(&src_plain, &tgt);
    const icp_amd::ICPResult q = plain.getResult();
    same = q.success == r.success && q.totalIterations == r.totalIterations &&
           q.iterationHistory.size() == r.iterationHistory.size();
    for (int i = 0; i < 3 && same; i++) {
      same = same && q.finalT[i] == r.finalT[i];
      for (int j = 0; j < 3; j++) same = same && q.finalR[i][j] == r.finalR[i][j];
    }
    for (size_t i = 0; i < src.size() && same; i++)
      same = src.points[i].x == src_plain.points[i].x && src.points[i].y == src_plain.points[i].y &&
             src.points[i].z == src_plain.points[i].z;
  }
  std::printf("{\"started\": %d, \"progress\": %d, \"last_progress\": %d, \"iterations\": %d, \"finished\": %d, "
              "\"log\": %d, \"success\": %d, \"total_iterations\": %d, \"history\": %zu, \"same_as_facade\": %d, "
              "\"message_len\": %d}\n",
              n_started, n_progress, last_progress, n_iter, n_finished, n_log, ok ? 1 : 0, r.totalIterations,
              r.iterationHistory.size(), same ? 1 : 0, (int)message.size());
  return 0;
}
