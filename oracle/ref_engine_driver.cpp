// ref_engine_driver.cpp — TEST INFRASTRUCTURE ONLY. A C-ABI around the reference's own core
// engine and LAS I/O, compiled from the sources where they lie:
//   /root/reference/PointCloudRegistration/core/{icpengine,octree,pointcloud,lasio}.cpp
// plus moc's output for icpengine.h, against the Qt 5.9.7 that this image carries in /opt/conda
// (oracle/Makefile target `refqt`; output oracle/_ref/libicp_ref_engine.so, git-ignored).
// Used only by tests/golden/gen_golden.py to write the engine-rule and core-LAS fixtures, and by
// the CPU tests that pin the oracle's SEM_ENGINE rules against them. Nothing here is product.
//
// Entry points replace nothing: they are the reference, called as its GUI service calls it
// (registrationservice.cpp:204-212: setParameters + registerPointClouds on one thread).
#include <QObject>
#include <QString>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "icpengine.h"
#include "lasio.h"
#include "pointcloud.h"

namespace {

PointCloud make_cloud(const double* xyz, int64_t n) {
  PointCloud c;
  c.points.resize((size_t)n);
  for (int64_t i = 0; i < n; i++) c.points[(size_t)i] = Point3D(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
  return c;
}

}  // namespace

extern "C" {

// Record layout of `hist` (doubles per record): iteration, rmse, validPoints, outlierPoints,
// transform (16, row-major), rotationAngle, translationDistance. The engine leaves the last two
// uninitialised in its convergence record (icpengine.cpp:293-301): they are written as NaN here.
constexpr int kRecDoubles = 22;

// ICPEngine::setParameters + registerPointClouds (icpengine.cpp:19-60). stop_at >= 0 calls
// ICPEngine::stop() from the progressUpdated signal of that iteration (the cross-thread stop of
// icpengine.cpp:62-66, checked at :160). Returns 1 when finished(true), 0 when finished(false),
// -1 when no finished signal came. src_out receives the (possibly rewritten) source.
int refeng_register(const double* src, int64_t n_src, const double* tgt, int64_t n_tgt, int max_iter, double tol,
                    double sigma, int max_pts, int max_depth, int stop_at, double* src_out, int32_t* total_iterations,
                    double* final_rmse, double* final_R, double* final_T, double* hist, int32_t cap, int32_t* n_hist,
                    char* message, int32_t msg_cap) {
  PointCloud s = make_cloud(src, n_src);
  PointCloud t = make_cloud(tgt, n_tgt);
  ICPEngine engine;
  ICPParameters p;
  p.maxIterations = max_iter;
  p.tolerance = tol;
  p.sigmaMultiplier = sigma;
  p.octreeMaxPoints = max_pts;
  p.octreeMaxDepth = max_depth;
  engine.setParameters(p);
  int status = -1;
  std::string msg;
  std::vector<IterationResult> recs;
  bool converged_record = false;
  QObject::connect(&engine, &ICPEngine::finished, [&](bool ok, const QString& m) {
    status = ok ? 1 : 0;
    msg = m.toUtf8().toStdString();
  });
  QObject::connect(&engine, &ICPEngine::iterationCompleted, [&](const IterationResult& r) { recs.push_back(r); });
  QObject::connect(&engine, &ICPEngine::logMessage, [&](const QString& m) {
    if (m.toUtf8().toStdString().find("收敛达到") != std::string::npos) converged_record = true;
  });
  QObject::connect(&engine, &ICPEngine::progressUpdated, [&](int iteration, int, double) {
    if (stop_at >= 0 && iteration == stop_at) engine.stop();
  });
  engine.registerPointClouds(&s, &t);
  const ICPResult res = engine.getResult();
  for (int64_t i = 0; i < n_src; i++) {
    src_out[3 * i] = s.points[(size_t)i].x;
    src_out[3 * i + 1] = s.points[(size_t)i].y;
    src_out[3 * i + 2] = s.points[(size_t)i].z;
  }
  *total_iterations = res.totalIterations;
  *final_rmse = res.finalRMSE;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) final_R[3 * r + c] = res.finalR[r][c];
    final_T[r] = res.finalT[r];
  }
  int32_t k = 0;
  for (size_t j = 0; j < recs.size() && k < cap; j++, k++) {
    const IterationResult& r = recs[j];
    double* h = hist + (size_t)kRecDoubles * k;
    h[0] = r.iteration;
    h[1] = r.rmse;
    h[2] = r.validPoints;
    h[3] = r.outlierPoints;
    for (int a = 0; a < 4; a++)
      for (int b = 0; b < 4; b++) h[4 + 4 * a + b] = r.transform(a, b);
    const bool last_of_convergence = converged_record && j + 1 == recs.size();
    h[20] = last_of_convergence ? __builtin_nan("") : r.rotationAngle;
    h[21] = last_of_convergence ? __builtin_nan("") : r.translationDistance;
  }
  *n_hist = k;
  if (message && msg_cap > 0) {
    std::strncpy(message, msg.c_str(), (size_t)msg_cap - 1);
    message[msg_cap - 1] = 0;
  }
  return status;
}

// LASIO::readLAS (lasio.cpp:7-125). Returns the point count, -1 when readLAS returns false.
int64_t refeng_read_las(const char* path, int64_t max_points, double* xyz, int64_t cap) {
  PointCloud c;
  if (!LASIO::readLAS(path, c, (size_t)max_points)) return -1;
  const int64_t n = (int64_t)c.points.size();
  for (int64_t i = 0; i < n && i < cap; i++) {
    xyz[3 * i] = c.points[(size_t)i].x;
    xyz[3 * i + 1] = c.points[(size_t)i].y;
    xyz[3 * i + 2] = c.points[(size_t)i].z;
  }
  return n;
}

// LASIO::writeLAS (lasio.cpp:127-210). The writer takes its offset and bounds from the cloud's
// minX..maxZ fields: bounds (minX, maxX, minY, maxY, minZ, maxZ) sets them as a caller left them
// (RegistrationService::saveRegisteredCloud writes the registered source with the bounds
// computed at load time, registrationservice.cpp:98, :156); null = PointCloud::computeBounds().
// Returns 1 on success.
int refeng_write_las(const char* path, const double* xyz, int64_t n, const double* bounds) {
  PointCloud c = make_cloud(xyz, n);
  if (bounds) {
    c.minX = bounds[0];
    c.maxX = bounds[1];
    c.minY = bounds[2];
    c.maxY = bounds[3];
    c.minZ = bounds[4];
    c.maxZ = bounds[5];
  } else {
    c.computeBounds();
  }
  return LASIO::writeLAS(path, c) ? 1 : 0;
}

}  // extern "C"
