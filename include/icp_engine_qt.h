// icp_engine_qt.h — Qt signal adapter over the C++ facade (icp_engine.hpp): a QObject with the
// reference engine's slots-and-signals surface, for callers that connect to ICPEngine's signals
// (the GUI and RegistrationService, registrationservice.cpp:208-211):
//
//   reference (core/icpengine.h)                      here
//   class ICPEngine : public QObject   :51-53         icp_amd::QtICPEngine : public QObject
//   setParameters / getParameters      :58-59         same
//   registerPointClouds(src, tgt)      :62            same (synchronous, like icpengine.cpp:24-60)
//   stop()                             :63            same (atomic flag, checked once per iteration)
//   getResult()                        :66            same (icp_amd::ICPResult)
//   signal started()                   :70            before the first iteration (icpengine.cpp:42)
//   signal progressUpdated(it, total, rmse)  :71      after each iteration record (icpengine.cpp:303, :367)
//   signal iterationCompleted(result)  :72            once per iteration record (icpengine.cpp:302, :366)
//   signal finished(success, message)  :73            once per call (icpengine.cpp:27-32, :162, :321)
//   signal logMessage(message)         :74            the engine's log lines
//
// The signals are emitted from the thread that calls registerPointClouds, as the reference's are
// (it runs the loop on the caller's thread, and RegistrationService calls it from a QtConcurrent
// worker): queued connections deliver them to the GUI thread. icp_amd::IterationResult is
// registered as a metatype so it can cross threads in a queued connection.
//
// Build: add this header to the target's moc sources (CMake AUTOMOC picks it up from the target's
// headers); link Qt5::Core and libicp_hip.so. tests/test_qt_adapter.py builds it with the image's
// Qt 5.9.7 moc.
#pragma once

#include <QMetaType>
#include <QObject>
#include <QString>

#include "icp_engine.hpp"

Q_DECLARE_METATYPE(icp_amd::IterationResult)

namespace icp_amd {

class QtICPEngine : public QObject {
  Q_OBJECT

 public:
  explicit QtICPEngine(QObject* parent = nullptr) : QObject(parent) {
    qRegisterMetaType<icp_amd::IterationResult>("icp_amd::IterationResult");
    engine_.onStarted = [this]() { emit started(); };
    engine_.onProgressUpdated = [this](int it, int total, double rmse) { emit progressUpdated(it, total, rmse); };
    engine_.onIterationCompleted = [this](const IterationResult& r) { emit iterationCompleted(r); };
    engine_.onFinished = [this](bool ok, const std::string& m) { emit finished(ok, QString::fromStdString(m)); };
    engine_.onLogMessage = [this](const std::string& m) { emit logMessage(QString::fromStdString(m)); };
  }
  ~QtICPEngine() override = default;

  void setParameters(const ICPParameters& params) { engine_.setParameters(params); }
  ICPParameters getParameters() const { return engine_.getParameters(); }

  void registerPointClouds(PointCloud* source, const PointCloud* target) {
    engine_.registerPointClouds(source, target);
  }
  void stop() { engine_.stop(); }

  ICPResult getResult() const { return engine_.getResult(); }

 signals:
  void started();
  void progressUpdated(int iteration, int total, double rmse);
  void iterationCompleted(const icp_amd::IterationResult& result);
  void finished(bool success, const QString& message);
  void logMessage(const QString& message);

 private:
  ICPEngine engine_;
};

}  // namespace icp_amd
