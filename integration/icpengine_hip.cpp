// icpengine_hip.cpp — the reference's own class ICPEngine (PointCloudRegistration/core/icpengine.h,
// unchanged) implemented on libicp_hip.so. A reference build switches its registration to the GPU
// by compiling this file in place of core/icpengine.cpp (and linking libicp_hip.so): the header,
// the QObject, its five signals, ICPParameters / IterationResult (with its Eigen::Matrix4d) /
// ICPResult and every caller (RegistrationService, registrationservice.cpp:204-212; the viewer's
// replay of iterationHistory) stay as they are. The clouds are passed to the GPU by pointer
// (include/icp_ref_adapter.hpp): no host copy, source->points rewritten in place on success.
//
//   ICPEngine(QObject*) / ~ICPEngine()      icpengine.cpp:7-17
//   setParameters                           icpengine.cpp:19-22
//   registerPointClouds                     icpengine.cpp:24-60 (checks, started, logs) + the loop
//                                           of :117-394 on the device (icp_engine_register_devices)
//   stop                                    icpengine.cpp:62-66 (m_shouldStop, read once per
//                                           iteration at the loop's top, :160)
//
// Build (inside the reference tree): add -I<this repo>/include, compile this file instead of
// core/icpengine.cpp, link -L<this repo>/iterativeclosestpoint_amd -licp_hip. moc runs on the
// reference's icpengine.h as before. tests/test_ref_adapter.py compiles it against the
// reference's real headers (Qt 5.9.7 from the image, the vendored Eigen).
#include "icpengine.h"

#include <QString>

#include "icp_ref_adapter.hpp"

namespace {

// The engine's signals, emitted on the caller's thread as the reference emits them.
struct QtEmit {
  ICPEngine* e;
  void started() { emit e->started(); }
  void progress(int it, int total, double rmse) { emit e->progressUpdated(it, total, rmse); }
  void iteration(const IterationResult& r) { emit e->iterationCompleted(r); }
  void finished(bool ok, const char* msg) { emit e->finished(ok, QString::fromUtf8(msg)); }
  void log(const char* msg) { emit e->logMessage(QString::fromUtf8(msg)); }
};

}  // namespace

ICPEngine::ICPEngine(QObject* parent) : QObject(parent), m_source(nullptr), m_target(nullptr), m_shouldStop(false) {}

ICPEngine::~ICPEngine() {}

void ICPEngine::setParameters(const ICPParameters& params) { m_params = params; }

void ICPEngine::registerPointClouds(PointCloud* source, const PointCloud* target) {
  QtEmit emitter{this};
  if (source && target && !source->empty() && !target->empty()) {
    m_source = source;
    m_target = target;
    m_shouldStop = false;
  }
  // m_shouldStop is the reference's plain bool (its stop() races with the loop's read, as there);
  // read through volatile so each iteration sees a store from the thread that called stop()
  const std::function<bool()> should_stop = [this]() { return *const_cast<volatile bool*>(&m_shouldStop); };
  icp_amd::ref::register_point_clouds(m_params, source, target, m_result, should_stop, emitter);
}

void ICPEngine::stop() {
  m_shouldStop = true;
  emit logMessage(QString::fromUtf8("\u7528\u6237\u8bf7\u6c42\u505c\u6b62\u914d\u51c6..."));
}
