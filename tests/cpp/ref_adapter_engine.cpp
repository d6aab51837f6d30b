// The reference's own ICPEngine (PointCloudRegistration/core/icpengine.h, unchanged) and
// PointCloud (core/pointcloud.h/.cpp, unchanged) driven exactly as RegistrationService drives them
// (registrationservice.cpp:204-212: setParameters, registerPointClouds, the five signals), with
// the class implemented by integration/icpengine_hip.cpp on libicp_hip.so instead of
// core/icpengine.cpp. Built by oracle/Makefile's refadapter target (reference sources compiled
// where they lie; test infrastructure). Prints one JSON line: signal counts, the result, the
// moved source's checksum and every iteration's transform (read through Eigen::Matrix4d).
//
//   ref_adapter_engine [N]     an N-point registration (default 20000) on the GPU
//   ref_adapter_engine stop    engine.stop() called from the 3rd iterationCompleted
//   ref_adapter_engine empty   an empty source: finished(false) only (no GPU)
#include <QCoreApplication>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>

#include "icpengine.h"
#include "pointcloud.h"

int main(int argc, char** argv) {
  QCoreApplication app(argc, argv);
  const std::string mode = argc > 1 ? argv[1] : "";
  const int n = (argc > 1 && mode != "stop" && mode != "empty") ? std::atoi(argv[1]) : 20000;
  std::mt19937_64 rng(11);
  std::normal_distribution<double> g(0.0, 1.0);
  PointCloud tgt, src;
  for (int i = 0; i < n; i++) tgt.points.emplace_back(8 * g(rng), 4 * g(rng), 1.5 * g(rng));
  const double a = 0.01, c = std::cos(a), s = std::sin(a);
  if (mode != "empty")
    for (const auto& p : tgt.points) src.points.emplace_back(c * p.x + s * p.y - 0.02, -s * p.x + c * p.y + 0.01, p.z);

  ICPEngine engine;
  int n_started = 0, n_progress = 0, n_iter = 0, n_finished = 0, n_log = 0;
  bool ok = false;
  QString message;
  QObject::connect(&engine, &ICPEngine::started, [&]() { n_started++; });
  QObject::connect(&engine, &ICPEngine::progressUpdated, [&](int, int, double) { n_progress++; });
  QObject::connect(&engine, &ICPEngine::iterationCompleted, [&](const IterationResult&) {
    if (++n_iter == 3 && mode == "stop") engine.stop();
  });
  QObject::connect(&engine, &ICPEngine::finished, [&](bool success, const QString& m) {
    n_finished++;
    ok = success;
    message = m;
  });
  QObject::connect(&engine, &ICPEngine::logMessage, [&](const QString&) { n_log++; });
  ICPParameters p;
  p.maxIterations = 30;
  p.tolerance = 1e-12;
  engine.setParameters(p);
  engine.registerPointClouds(&src, &tgt);
  const ICPResult r = engine.getResult();

  double sum = 0.0;
  for (const auto& q : src.points) sum += q.x + 2.0 * q.y + 3.0 * q.z;
  std::printf("{\"started\": %d, \"progress\": %d, \"iterations\": %d, \"finished\": %d, \"log\": %d, "
              "\"success\": %d, \"message\": \"%s\", \"result_success\": %d, \"total_iterations\": %d, "
              "\"final_rmse\": %.17g, \"final_R\": [",
              n_started, n_progress, n_iter, n_finished, n_log, ok ? 1 : 0, message.toUtf8().constData(),
              r.success ? 1 : 0, r.totalIterations, r.finalRMSE);
  for (int i = 0; i < 9; i++) std::printf("%s%.17g", i ? ", " : "", r.finalR[i / 3][i % 3]);
  std::printf("], \"final_t\": [%.17g, %.17g, %.17g], \"checksum\": %.17g, \"transforms\": [", r.finalT[0], r.finalT[1],
              r.finalT[2], sum);
  for (size_t h = 0; h < r.iterationHistory.size(); h++) {
    const Eigen::Matrix4d& T = r.iterationHistory[h].transform;
    std::printf("%s[", h ? ", " : "");
    for (int e = 0; e < 16; e++) std::printf("%s%.17g", e ? ", " : "", T(e / 4, e % 4));
    std::printf("]");
  }
  std::printf("], \"rmse\": [");
  for (size_t h = 0; h < r.iterationHistory.size(); h++) std::printf("%s%.17g", h ? ", " : "", r.iterationHistory[h].rmse);
  std::printf("]}\n");
  return 0;
}
