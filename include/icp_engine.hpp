// icp_engine.hpp — header-only C++ facade over libicp_hip.so with the reference's class shapes,
// so a caller of PointCloudRegistration/core can switch by changing includes and a namespace:
//
//   reference (Qt)                                   here (no Qt; callbacks instead of signals)
//   struct Point3D             pointcloud.h:12-23    icp_amd::Point3D (same layout: 3 doubles)
//   PointCloud::points         pointcloud.h:42       icp_amd::PointCloud::points
//   struct ICPParameters       icpengine.h:13-19     icp_amd::ICPParameters (same fields/defaults)
//   struct IterationResult     icpengine.h:24-32     icp_amd::IterationResult
//   struct ICPResult           icpengine.h:37-44     icp_amd::ICPResult
//   class ICPEngine            icpengine.h:51-87     icp_amd::ICPEngine (setParameters,
//                                                    getParameters, registerPointClouds, stop,
//                                                    getResult; started/progressUpdated/
//                                                    iterationCompleted/finished/logMessage hooks)
//   class Octree               octree.h:27-43        icp_amd::Octree (findNearest one / many)
//   void ICP(...)              icp_registration.cpp:443-446   icp_amd::ICP (same signature)
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "icp_engine.h"
#include "icp_hip.h"

namespace icp_amd {

struct Point3D {
  double x = 0, y = 0, z = 0;
  Point3D() = default;
  Point3D(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
};
static_assert(sizeof(Point3D) == 24, "Point3D must stay AoS xyz");

struct PointCloud {
  std::vector<Point3D> points;
  size_t size() const { return points.size(); }
  bool empty() const { return points.empty(); }
};

struct ICPParameters {
  int maxIterations = 50;
  double tolerance = 1e-6;
  double sigmaMultiplier = 3.0;
  int octreeMaxPoints = 10;
  int octreeMaxDepth = 20;
  int device = -1;  // build-only knob: HIP ordinal (-1: the calling thread's current device)
  // build-only knob: several GPUs of this process (the source sharded over them, the octree
  // replicated, RCCL per iteration); empty = `device` alone
  std::vector<int> devices;
};

struct IterationResult {
  int iteration = 0;
  double rmse = 0;
  int validPoints = 0;
  int outlierPoints = 0;
  double transform[4][4] = {};  // cumulative
  double rotationAngle = 0;
  double translationDistance = 0;
};

struct ICPResult {
  bool success = false;
  int totalIterations = 0;
  double finalRMSE = 0;
  double finalR[3][3] = {};
  double finalT[3] = {};
  std::vector<IterationResult> iterationHistory;
};

class ICPEngine {
 public:
  std::function<void()> onStarted;
  std::function<void(int, int, double)> onProgressUpdated;
  std::function<void(const IterationResult&)> onIterationCompleted;
  std::function<void(bool, const std::string&)> onFinished;
  std::function<void(const std::string&)> onLogMessage;

  void setParameters(const ICPParameters& p) { params_ = p; }
  ICPParameters getParameters() const { return params_; }
  ICPResult getResult() const { return result_; }
  // atomic: fixes the reference's plain-bool data race (icpengine.cpp:62-66, read at :160)
  void stop() { stop_.store(1); }

  // Synchronous, like ICPEngine::registerPointClouds (icpengine.cpp:24-60); rewrites
  // source->points on success.
  void registerPointClouds(PointCloud* source, const PointCloud* target) {
    result_ = ICPResult();
    stop_.store(0);
    if (!source || !target) return finish(false, "source or target cloud is null");
    if (source->empty() || target->empty()) return finish(false, "point cloud is empty");
    if (onStarted) onStarted();
    icp_params p;
    icp_params_default(&p);
    p.max_iterations = params_.maxIterations;
    p.tolerance = params_.tolerance;
    p.sigma_multiplier = params_.sigmaMultiplier;
    p.octree_max_points = params_.octreeMaxPoints;
    p.octree_max_depth = params_.octreeMaxDepth;
    p.rules = ICP_RULES_ENGINE;
    std::vector<icp_iteration_record> hist((size_t)(params_.maxIterations > 0 ? params_.maxIterations + 1 : 1));
    icp_engine_hooks hooks{};
    hooks.user = this;
    hooks.on_iteration = &ICPEngine::iterThunk;
    hooks.on_progress = &ICPEngine::progressThunk;
    hooks.on_log = &ICPEngine::logThunk;
    hooks.stop_flag = reinterpret_cast<const volatile int32_t*>(&stop_);
    icp_result r;
    std::vector<int> devs = params_.devices.empty() ? std::vector<int>{params_.device} : params_.devices;
    int rc = icp_engine_register_devices(&p, reinterpret_cast<double*>(source->points.data()), (int64_t)source->size(),
                                         reinterpret_cast<const double*>(target->points.data()),
                                         (int64_t)target->size(), (int)devs.size(), devs.data(), &r, hist.data(),
                                         (int32_t)hist.size(), &hooks);
    for (int k = 0; k < r.n_history; k++) result_.iterationHistory.push_back(convert(hist[k]));
    if (rc != ICP_HIP_OK) return finish(false, r.message);
    result_.success = true;
    result_.totalIterations = r.total_iterations;
    result_.finalRMSE = r.final_rmse;
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) result_.finalR[i][j] = r.final_R[3 * i + j];
      result_.finalT[i] = r.final_t[i];
    }
    finish(true, "registration finished");
  }

 private:
  ICPParameters params_;
  ICPResult result_;
  std::atomic<int32_t> stop_{0};
  static_assert(sizeof(std::atomic<int32_t>) == sizeof(int32_t), "lock-free int32 flag");

  static IterationResult convert(const icp_iteration_record& h) {
    IterationResult o;
    o.iteration = h.iteration;
    o.rmse = h.rmse;
    o.validPoints = h.valid_points;
    o.outlierPoints = h.outlier_points;
    for (int i = 0; i < 16; i++) o.transform[i / 4][i % 4] = h.transform[i];
    o.rotationAngle = h.rotation_angle_deg;
    o.translationDistance = h.translation_distance;
    return o;
  }
  void finish(bool ok, const std::string& msg) {
    if (onFinished) onFinished(ok, msg);
  }
  static void iterThunk(void* u, const icp_iteration_record* h) {
    auto* self = static_cast<ICPEngine*>(u);
    if (self->onIterationCompleted) self->onIterationCompleted(convert(*h));
  }
  static void progressThunk(void* u, int it, int total, double rmse) {
    auto* self = static_cast<ICPEngine*>(u);
    if (self->onProgressUpdated) self->onProgressUpdated(it, total, rmse);
  }
  static void logThunk(void* u, const char* m) {
    auto* self = static_cast<ICPEngine*>(u);
    if (self->onLogMessage) self->onLogMessage(m);
  }
};

// Octree(const std::vector<Point3D>&, int max_pts, int max_d) + findNearest (octree.h:29-32),
// engine flavour (initial best = DBL_MAX). The tree lives on the GPU.
class Octree {
 public:
  Octree(const std::vector<Point3D>& pts, int max_pts = 10, int max_d = 20, int device = 0) {
    if (icp_hip_create(&ctx_, device) != ICP_HIP_OK) throw std::runtime_error(icp_hip_last_error());
    if (!pts.empty() && icp_hip_set_target(ctx_, reinterpret_cast<const double*>(pts.data()), (int64_t)pts.size(),
                                           max_pts, max_d, ICP_RULES_ENGINE) != ICP_HIP_OK) {
      icp_hip_destroy(ctx_);
      ctx_ = nullptr;
      throw std::runtime_error(icp_hip_last_error());
    }
    empty_ = pts.empty();
  }
  ~Octree() { icp_hip_destroy(ctx_); }
  Octree(const Octree&) = delete;
  Octree& operator=(const Octree&) = delete;

  int findNearest(const Point3D& q) const {
    if (empty_) return 0;  // octree.cpp:177
    int32_t idx = 0;
    double d = 0;
    if (icp_hip_nn(ctx_, &q.x, 1, &idx, &d) != ICP_HIP_OK) throw std::runtime_error(icp_hip_last_error());
    return idx;
  }
  // Batched form (the way to use a GPU): one index per query.
  std::vector<int> findNearest(const std::vector<Point3D>& q) const {
    std::vector<int> out(q.size(), 0);
    if (empty_ || q.empty()) return out;
    std::vector<int32_t> idx(q.size());
    if (icp_hip_nn(ctx_, reinterpret_cast<const double*>(q.data()), (int64_t)q.size(), idx.data(), nullptr) !=
        ICP_HIP_OK)
      throw std::runtime_error(icp_hip_last_error());
    for (size_t i = 0; i < q.size(); i++) out[i] = idx[i];
    return out;
  }

 private:
  icp_hip_ctx* ctx_ = nullptr;
  bool empty_ = true;
};

// void ICP(PointCloud& source, const PointCloud& target, int max_iterations, double tolerance,
//          double final_R[3][3], double final_t[3], vector<Matrix4d>* iteration_transforms)
// (icp_registration.cpp:443-446); Matrix4d replaced by a row-major 4x4 array.
using Matrix4 = std::array<double, 16>;
inline void ICP(PointCloud& source, const PointCloud& target, int max_iterations, double tolerance,
                double final_R[3][3], double final_t[3], std::vector<Matrix4>* iteration_transforms,
                const std::vector<int>& devices) {
  std::vector<double> tr((size_t)(max_iterations > 0 ? max_iterations : 1) * 16);
  int32_t n = 0;
  double R[9], t[3];
  int rc = icp_cli_icp_devices(reinterpret_cast<double*>(source.points.data()), (int64_t)source.size(),
                               reinterpret_cast<const double*>(target.points.data()), (int64_t)target.size(),
                               max_iterations, tolerance, R, t, tr.data(), (int32_t)(tr.size() / 16), &n,
                               (int)devices.size(), devices.data());
  if (rc != ICP_HIP_OK) throw std::runtime_error(icp_hip_last_error());
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) final_R[i][j] = R[3 * i + j];
    final_t[i] = t[i];
  }
  if (iteration_transforms)
    for (int k = 0; k < n; k++) {
      Matrix4 m;
      for (int e = 0; e < 16; e++) m[e] = tr[16 * k + e];
      iteration_transforms->push_back(m);
    }
}
inline void ICP(PointCloud& source, const PointCloud& target, int max_iterations, double tolerance,
                double final_R[3][3], double final_t[3], std::vector<Matrix4>* iteration_transforms = nullptr,
                int device = -1) {
  ICP(source, target, max_iterations, tolerance, final_R, final_t, iteration_transforms, std::vector<int>{device});
}

}  // namespace icp_amd
