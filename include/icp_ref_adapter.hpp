// icp_ref_adapter.hpp — the GPU registration on the caller's OWN reference types, with no copy of
// the clouds: the drop-in for code that holds the reference's PointCloud / ICPParameters /
// IterationResult / ICPResult (PointCloudRegistration/core/pointcloud.h:30-65, icpengine.h:13-44)
// and consumes IterationResult::transform as an Eigen::Matrix4d (the viewer's replay,
// pointcloudviewer.cpp:86-116).
//
//   reference                                         here
//   ICPEngine::registerPointClouds(src, tgt)           icp_amd::ref::register_point_clouds(params, src,
//     icpengine.cpp:24-60, loop :117-394                  tgt, result, should_stop, sink[, devices])
//   m_params (ICPParameters, icpengine.h:13-19)        read field by field from the caller's struct
//   m_result (ICPResult, icpengine.h:37-44)            filled in place: success, totalIterations,
//                                                      finalRMSE, finalR, finalT, iterationHistory
//   IterationResult (icpengine.h:24-32)                the caller's type; transform assigned through
//                                                      m(i, j) (Eigen::Matrix4d) or m[i][j] (arrays)
//   source->points rewritten on success (:342-346)     the GPU result lands in source->points.data()
//   signals started / progressUpdated /                sink.started(), sink.progress(it, total, rmse),
//   iterationCompleted / finished / logMessage         sink.iteration(rec), sink.finished(ok, msg),
//                                                      sink.log(msg) (any object with those members)
//   m_shouldStop, checked once per iteration (:160)    should_stop(), polled after each iteration's
//                                                      hooks (the same point of the loop)
//
// Point types are checked at compile time: three contiguous doubles x, y, z (24 bytes, standard
// layout), i.e. std::vector<Point3D>::data() is the AoS xyz array the C-ABI takes. The clouds are
// handed to libicp_hip.so by pointer: nothing is converted or copied on the host (at 10M points
// the facade's assign would copy 240 MB each way). integration/icpengine_hip.cpp uses this header
// to implement the reference's own QObject class ICPEngine, so a reference build switches to the
// GPU by compiling that file instead of core/icpengine.cpp.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "icp_engine.h"
#include "icp_hip.h"

namespace icp_amd {
namespace ref {

// The reference's finished() messages (icpengine.cpp:27-32, :162, :321, :393), UTF-8.
inline const char* msg_null() { return "\u6e90\u70b9\u4e91\u6216\u76ee\u6807\u70b9\u4e91\u4e3a\u7a7a"; }
inline const char* msg_empty() { return "\u70b9\u4e91\u6570\u636e\u4e3a\u7a7a"; }
inline const char* msg_cancelled() { return "\u7528\u6237\u53d6\u6d88"; }
inline const char* msg_too_few() { return "\u6709\u6548\u70b9\u5bf9\u4e0d\u8db3"; }
inline const char* msg_success() { return "\u914d\u51c6\u6210\u529f"; }

// Layout of the caller's point type: the AoS xyz doubles of the C-ABI.
template <class P>
constexpr bool xyz24() {
  return std::is_standard_layout<P>::value && sizeof(P) == 3 * sizeof(double) &&
         std::is_same<decltype(P::x), double>::value && std::is_same<decltype(P::y), double>::value &&
         std::is_same<decltype(P::z), double>::value && offsetof(P, x) == 0 && offsetof(P, y) == sizeof(double) &&
         offsetof(P, z) == 2 * sizeof(double);
}

namespace detail {
// m(i, j) = T[4 i + j]: Eigen::Matrix4d and any type with a (row, col) accessor ...
template <class M>
auto set4(M& m, const double* T, int) -> decltype(m(0, 0) = 0.0, void()) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) m(i, j) = T[4 * i + j];
}
// ... or a double[4][4]
template <class M>
void set4(M& m, const double* T, long) {
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) m[i][j] = T[4 * i + j];
}

template <class Emit, class IterT>
struct Ctx {
  Emit* sink;
  std::vector<IterT>* history;
  const std::function<bool()>* should_stop;
  int32_t stop = 0;  // the engine's per-iteration stop flag, refreshed from should_stop()
};

template <class IterT>
IterT convert(const icp_iteration_record& h) {
  IterT o{};
  o.iteration = h.iteration;
  o.rmse = h.rmse;
  o.validPoints = h.valid_points;
  o.outlierPoints = h.outlier_points;
  set4(o.transform, h.transform, 0);
  o.rotationAngle = h.rotation_angle_deg;
  o.translationDistance = h.translation_distance;
  return o;
}
}  // namespace detail

// One registration of `source` onto `target` with the reference engine's rules (octree
// initial best DBL_MAX, relaxed iteration-0 threshold, T_cum as the result; icpengine.cpp:117-394),
// on `devices` (HIP ordinals; {-1}: the calling thread's current device; several: one process
// over several GPUs). `result` is reset and filled as m_result is; source->points is rewritten in
// place on success. Returns the icp_engine_register code (ICP_HIP_OK on success). `sink` needs
// started(), progress(int, int, double), iteration(const IterT&), finished(bool, const char*),
// log(const char*).
template <class CloudT, class ParamsT, class ResultT, class Emit>
int register_point_clouds(const ParamsT& params, CloudT* source, const CloudT* target, ResultT& result,
                          const std::function<bool()>& should_stop, Emit& sink,
                          const std::vector<int>& devices = std::vector<int>{-1}) {
  using PointT = typename std::decay<decltype(source->points[0])>::type;
  using IterT = typename decltype(result.iterationHistory)::value_type;
  static_assert(xyz24<PointT>(), "the cloud's point type must be three contiguous doubles x, y, z (Point3D)");
  if (!source || !target) {
    sink.finished(false, msg_null());
    return ICP_HIP_EINVAL;
  }
  if (source->points.empty() || target->points.empty()) {
    sink.finished(false, msg_empty());
    return ICP_HIP_EINVAL;
  }
  result = ResultT();
  sink.started();
  icp_params p;
  icp_params_default(&p);
  p.max_iterations = params.maxIterations;
  p.tolerance = params.tolerance;
  p.sigma_multiplier = params.sigmaMultiplier;
  p.octree_max_points = params.octreeMaxPoints;
  p.octree_max_depth = params.octreeMaxDepth;
  p.rules = ICP_RULES_ENGINE;
  detail::Ctx<Emit, IterT> ctx{&sink, &result.iterationHistory, &should_stop};
  ctx.stop = should_stop && should_stop() ? 1 : 0;
  icp_engine_hooks hooks{};
  hooks.user = &ctx;
  hooks.on_iteration = [](void* u, const icp_iteration_record* h) {
    auto* c = static_cast<detail::Ctx<Emit, IterT>*>(u);
    c->history->push_back(detail::convert<IterT>(*h));
    c->sink->iteration(c->history->back());
  };
  hooks.on_progress = [](void* u, int it, int total, double rmse) {
    auto* c = static_cast<detail::Ctx<Emit, IterT>*>(u);
    c->sink->progress(it, total, rmse);
    // the reference tests m_shouldStop at the top of the next iteration: the engine reads this
    // flag there too
    if (*c->should_stop && (*c->should_stop)()) c->stop = 1;
  };
  hooks.on_log = [](void* u, const char* m) { static_cast<detail::Ctx<Emit, IterT>*>(u)->sink->log(m); };
  hooks.stop_flag = &ctx.stop;
  icp_result r;
  // the history comes back through on_iteration (in order); the record array is not needed
  const std::vector<int> devs = devices.empty() ? std::vector<int>{-1} : devices;
  const int rc = icp_engine_register_devices(&p, &source->points[0].x, (int64_t)source->points.size(),
                                             &target->points[0].x, (int64_t)target->points.size(), (int)devs.size(),
                                             devs.data(), &r, nullptr, 0, &hooks);
  if (rc == ICP_ENGINE_CANCELLED) {
    sink.finished(false, msg_cancelled());
    return rc;
  }
  if (rc == ICP_ENGINE_TOO_FEW) {
    sink.finished(false, msg_too_few());
    return rc;
  }
  if (rc != ICP_HIP_OK) {
    sink.finished(false, r.message);
    return rc;
  }
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) result.finalR[i][j] = r.final_R[3 * i + j];
    result.finalT[i] = r.final_t[i];
  }
  result.success = true;
  result.totalIterations = (int)result.iterationHistory.size();
  result.finalRMSE = result.iterationHistory.empty() ? 0.0 : result.iterationHistory.back().rmse;
  sink.finished(true, msg_success());
  return ICP_HIP_OK;
}

}  // namespace ref
}  // namespace icp_amd
