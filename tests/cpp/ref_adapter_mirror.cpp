// Compile-and-run check of include/icp_ref_adapter.hpp on types laid out exactly as the
// reference's (pointcloud.h:12-65, icpengine.h:13-44): a Point3D with constructors, a PointCloud
// with its QColor / pointSize / bounds members, ICPParameters, an IterationResult whose transform
// is a column-major 4x4 with an Eigen-style m(i, j) accessor, ICPResult. The registration runs on
// the caller's own clouds (no copy) and must equal the plain facade (icp_engine.hpp) bit for bit.
// Built by tests/test_ref_adapter.py. Prints one JSON line.
//
//   ref_adapter_mirror          a 20k-point registration on the GPU, compared with the facade
//   ref_adapter_mirror stop     should_stop() turns true after the 3rd iteration: 3 records, then
//                               finished(false, cancelled)
//   ref_adapter_mirror empty    an empty source: finished(false, empty) and nothing else (no GPU)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "icp_engine.hpp"
#include "icp_ref_adapter.hpp"

namespace mirror {
struct Point3D {  // pointcloud.h:12-23
  double x, y, z;
  Point3D() : x(0), y(0), z(0) {}
  Point3D(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
};
struct QColorLike {  // QColor's members (cspec + a 5 x ushort union): only the layout matters here
  int cspec = 1;
  unsigned short ct[5] = {65535, 65535, 0, 0, 0};
};
class PointCloud {  // pointcloud.h:30-65
 public:
  size_t size() const { return points.size(); }
  bool empty() const { return points.empty(); }
  std::vector<Point3D> points;
  QColorLike color;
  float pointSize = 2.0f;
  double minX = 0, maxX = 0, minY = 0, maxY = 0, minZ = 0, maxZ = 0;

 private:
  bool m_boundsComputed = false;
};
struct Matrix4d {  // Eigen::Matrix4d's storage (column-major) and accessor
  double m[16] = {};
  double& operator()(int r, int c) { return m[4 * c + r]; }
  double operator()(int r, int c) const { return m[4 * c + r]; }
};
struct ICPParameters {  // icpengine.h:13-19
  int maxIterations = 50;
  double tolerance = 1e-6;
  double sigmaMultiplier = 3.0;
  int octreeMaxPoints = 10;
  int octreeMaxDepth = 20;
};
struct IterationResult {  // icpengine.h:24-32
  int iteration;
  double rmse;
  int validPoints;
  int outlierPoints;
  Matrix4d transform;
  double rotationAngle;
  double translationDistance;
};
struct ICPResult {  // icpengine.h:37-44
  bool success;
  int totalIterations;
  double finalRMSE;
  double finalR[3][3];
  double finalT[3];
  std::vector<IterationResult> iterationHistory;
};
}  // namespace mirror

struct Counts {
  int started = 0, progress = 0, iter = 0, finished = 0, log = 0, last_progress = 0;
  bool ok = false;
  std::string message;
};
struct Emit {
  Counts* c;
  void started() { c->started++; }
  void progress(int it, int, double) {
    c->progress++;
    c->last_progress = it;
  }
  void iteration(const mirror::IterationResult&) { c->iter++; }
  void finished(bool ok, const char* m) {
    c->finished++;
    c->ok = ok;
    c->message = m;
  }
  void log(const char*) { c->log++; }
};

// equal bits, NaN included (the reference's rotation angle, acos((trace - 1) / 2), is NaN when
// the trace of a near-identity increment rounds above 3: icpengine.cpp:361)
static bool same_d(double a, double b) { return a == b || (a != a && b != b); }

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "";
  std::mt19937_64 rng(11);
  std::normal_distribution<double> g(0.0, 1.0);
  mirror::PointCloud tgt, src;
  icp_amd::PointCloud ftgt, fsrc;
  for (int i = 0; i < 20000; i++) tgt.points.emplace_back(8 * g(rng), 4 * g(rng), 1.5 * g(rng));
  const double a = 0.01, c = std::cos(a), s = std::sin(a);
  if (mode != "empty")
    for (const auto& p : tgt.points) src.points.emplace_back(c * p.x + s * p.y - 0.02, -s * p.x + c * p.y + 0.01, p.z);
  for (const auto& p : tgt.points) ftgt.points.emplace_back(p.x, p.y, p.z);
  for (const auto& p : src.points) fsrc.points.emplace_back(p.x, p.y, p.z);
  const double* src_data = src.points.empty() ? nullptr : &src.points[0].x;

  mirror::ICPParameters p;
  p.maxIterations = 30;
  p.tolerance = 1e-12;
  mirror::ICPResult r{};
  Counts k;
  Emit e{&k};
  const std::function<bool()> stop = [&]() { return mode == "stop" && k.iter >= 3; };
  const int rc = icp_amd::ref::register_point_clouds(p, &src, &tgt, r, stop, e);

  bool same = true, in_place = src.points.empty() || &src.points[0].x == src_data;
  if (mode.empty()) {  // the same registration through the facade
    icp_amd::ICPEngine plain;
    icp_amd::ICPParameters fp;
    fp.maxIterations = p.maxIterations;
    fp.tolerance = p.tolerance;
    plain.setParameters(fp);
    plain.registerPointClouds(&fsrc, &ftgt);
    const icp_amd::ICPResult q = plain.getResult();
    same = q.success == r.success && q.totalIterations == r.totalIterations &&
           q.iterationHistory.size() == r.iterationHistory.size() && same_d(q.finalRMSE, r.finalRMSE);
    if (!same)  // what differs (stderr: the test prints it on failure)
      std::fprintf(stderr, "facade: success %d/%d iterations %d/%d history %zu/%zu rmse %.17g/%.17g\n", (int)q.success,
                   (int)r.success, q.totalIterations, r.totalIterations, q.iterationHistory.size(),
                   r.iterationHistory.size(), q.finalRMSE, r.finalRMSE);
    for (int i = 0; i < 3 && same; i++) {
      same = same && q.finalT[i] == r.finalT[i];
      for (int j = 0; j < 3; j++) same = same && q.finalR[i][j] == r.finalR[i][j];
    }
    for (size_t h = 0; h < q.iterationHistory.size() && same; h++) {
      const auto& A = q.iterationHistory[h];
      const auto& B = r.iterationHistory[h];
      same = A.iteration == B.iteration && same_d(A.rmse, B.rmse) && A.validPoints == B.validPoints &&
             A.outlierPoints == B.outlierPoints && same_d(A.rotationAngle, B.rotationAngle);
      if (!same)
        std::fprintf(stderr,
                     "facade: history %zu: iteration %d/%d rmse %.17g/%.17g valid %d/%d outliers %d/%d angle "
                     "%.17g/%.17g\n",
                     h, A.iteration, B.iteration, A.rmse, B.rmse, A.validPoints, B.validPoints, A.outlierPoints,
                     B.outlierPoints, A.rotationAngle, B.rotationAngle);
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) same = same && same_d(A.transform[i][j], B.transform(i, j));
    }
    for (size_t i = 0; i < src.size() && same; i++)
      same = src.points[i].x == fsrc.points[i].x && src.points[i].y == fsrc.points[i].y &&
             src.points[i].z == fsrc.points[i].z;
  }
  double sum = 0.0;
  for (const auto& q : src.points) sum += q.x + 2.0 * q.y + 3.0 * q.z;
  std::printf("{\"rc\": %d, \"started\": %d, \"progress\": %d, \"last_progress\": %d, \"iterations\": %d, "
              "\"finished\": %d, \"log\": %d, \"success\": %d, \"result_success\": %d, \"total_iterations\": %d, "
              "\"history\": %zu, \"same_as_facade\": %d, \"in_place\": %d, \"message\": \"%s\", \"checksum\": %.17g, "
              "\"final_R\": [",
              rc, k.started, k.progress, k.last_progress, k.iter, k.finished, k.log, k.ok ? 1 : 0, r.success ? 1 : 0,
              r.totalIterations, r.iterationHistory.size(), same ? 1 : 0, in_place ? 1 : 0, k.message.c_str(), sum);
  for (int i = 0; i < 9; i++) std::printf("%s%.17g", i ? ", " : "", r.finalR[i / 3][i % 3]);
  std::printf("], \"final_t\": [%.17g, %.17g, %.17g], \"transforms\": [", r.finalT[0], r.finalT[1], r.finalT[2]);
  for (size_t h = 0; h < r.iterationHistory.size(); h++) {
    std::printf("%s[", h ? ", " : "");
    for (int e = 0; e < 16; e++) std::printf("%s%.17g", e ? ", " : "", r.iterationHistory[h].transform(e / 4, e % 4));
    std::printf("]");
  }
  std::printf("]}\n");
  return 0;
}
