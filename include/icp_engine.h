/*
 * icp_engine.h — C-ABI of the ICP driver in libicp_hip.so: the drop-in for the reference's
 * engine API and CLI entry point, running the device path of icp_hip.h underneath.
 *
 * Reference interfaces these entry points replace:
 *   icp_params                ICPParameters            core/icpengine.h:13-19
 *   icp_iteration_record      IterationResult          core/icpengine.h:24-32
 *   icp_result                ICPResult                core/icpengine.h:37-44
 *   icp_engine_register       ICPEngine::setParameters + registerPointClouds (+ stop via the
 *                             stop flag, signals via hooks)   core/icpengine.h:60-75,
 *                             icpengine.cpp:24-66, :117-394
 *   icp_engine_register_devices  the same over several GPUs of one process
 *   icp_engine_run            the same loop on an existing (possibly multi-GPU) context
 *   icp_cli_icp               void ICP(PointCloud&, const PointCloud&, int, double,
 *                             double[3][3], double[3], vector<Matrix4d>*)
 *                             icp_registration.cpp:443-622
 *   icp_cli_icp_devices       the same over several GPUs of one process
 *   icp_best_fit_transform    computeBestFitTransform / best_fit_transform
 *                             icpengine.cpp:76-115, icp_registration.cpp:389-440 (host)
 *   icp_jacobi_svd3           Eigen::JacobiSVD<Matrix3d> as used at icpengine.cpp:93 (host)
 *
 * Points are AoS xyz doubles (the layout of std::vector<Point3D>, pointcloud.h:12-23).
 * Matrices are row-major. Return codes are those of icp_hip.h plus ICP_ENGINE_* below.
 */
#ifndef ICP_ENGINE_H
#define ICP_ENGINE_H

#include <stdint.h>

#include "icp_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ICP_ENGINE_CANCELLED (-10)   /* stop() observed: finished(false, "用户取消")          */
#define ICP_ENGINE_TOO_FEW (-11)     /* valid pairs < 3: finished(false, "有效点对不足")       */

/* status of a finished run */
#define ICP_STATUS_MAX_ITERATIONS 0
#define ICP_STATUS_CONVERGED 1
#define ICP_STATUS_DIVERGED 2 /* rmse > 1.1 * previous (icpengine.cpp:311-314)          */
#define ICP_STATUS_TOO_FEW 3
#define ICP_STATUS_CANCELLED 4

/* flags */
#define ICP_FLAG_NO_EARLY_STOP 1 /* benchmark mode: never stop on convergence/divergence */

typedef struct icp_params {
  int32_t max_iterations;   /* 50     */
  double tolerance;         /* 1e-6   */
  double sigma_multiplier;  /* 3.0    */
  int32_t octree_max_points;/* 10     */
  int32_t octree_max_depth; /* 20     */
  int32_t rules;            /* ICP_RULES_ENGINE / ICP_RULES_CLI */
  int32_t flags;
} icp_params;

typedef struct icp_iteration_record {
  int32_t iteration;
  double rmse;
  int32_t valid_points;
  int32_t outlier_points;
  double transform[16];        /* cumulative, row-major */
  double rotation_angle_deg;   /* acos((tr-1)/2) in degrees (NaN-prone like the reference) */
  double translation_distance;
  int32_t has_transform;       /* 0 for the engine's convergence record (icpengine.cpp:293-301) */
  double mean, std, threshold;
  double increment[16];        /* this iteration's T (row-major) */
} icp_iteration_record;

typedef struct icp_result {
  int32_t success;
  int32_t status;
  int32_t total_iterations;
  double final_rmse;
  double final_R[9];
  double final_t[3];
  int32_t n_history;     /* records written (<= capacity) */
  char message[160];
} icp_result;

typedef struct icp_engine_hooks {
  void* user;
  void (*on_iteration)(void* user, const icp_iteration_record* rec); /* iterationCompleted  */
  void (*on_progress)(void* user, int iteration, int total, double rmse); /* progressUpdated */
  void (*on_log)(void* user, const char* message);                   /* logMessage          */
  const volatile int32_t* stop_flag; /* ICPEngine::stop(): checked once per iteration      */
} icp_engine_hooks;

void icp_params_default(icp_params* p);

/* Full registration on one GPU (device ordinal; -1 = the calling thread's current HIP device).
 * src is rewritten in place on success (engine rules) or always (CLI rules), as the reference. */
int icp_engine_register(const icp_params* p, double* src_xyz, int64_t n_src, const double* tgt_xyz,
                        int64_t n_tgt, int device, icp_result* res, icp_iteration_record* history,
                        int32_t history_cap, const icp_engine_hooks* hooks);

/* The same on several GPUs of this process (icp_hip_create_multi: the source sharded over the
 * devices, the octree replicated, RCCL all-gathers of the two per-iteration records when the ids
 * are distinct, an in-process host gather when they repeat). n_devices = 1 is icp_engine_register. */
int icp_engine_register_devices(const icp_params* p, double* src_xyz, int64_t n_src, const double* tgt_xyz,
                                int64_t n_tgt, int n_devices, const int* device_ids, icp_result* res,
                                icp_iteration_record* history, int32_t history_cap, const icp_engine_hooks* hooks);

/* The loop on a context that already holds target + this rank's source shard (icp_hip.h).
 * Every rank of a communicator calls it in lockstep; decisions are identical on all ranks.
 * The resident source is left transformed; fetch it with icp_hip_get_source. */
int icp_engine_run(icp_hip_ctx* ctx, const icp_params* p, icp_result* res, icp_iteration_record* history,
                   int32_t history_cap, const icp_engine_hooks* hooks);

/* Steppable form of the same loop (one call = one loop body of icpengine.cpp:159-368):
 * create on a ready context, step until *done != 0, then finish (applies the pending T and
 * fills the result). icp_engine_run == create + step* + finish. */
typedef struct icp_session icp_session;
int icp_session_create(icp_hip_ctx* ctx, const icp_params* p, const icp_engine_hooks* hooks, icp_session** out);
/* rec (optional) receives the record of this iteration when one is produced (*produced = 1). */
int icp_session_step(icp_session* s, icp_iteration_record* rec, int32_t* produced, int32_t* done);
/* Up to k steps in one call (no records returned; hooks still fire); stops early when the loop
 * is done. *steps_done = steps taken. Same as calling icp_session_step k times. */
int icp_session_step_n(icp_session* s, int32_t k, int32_t* steps_done, int32_t* done);
/* icp_session_step_n that also stores each step's host wall time (ms, steady clock; the step
 * returns when its record is on the host, so this is the whole iteration). step_ms[k]. */
int icp_session_step_n_timed(icp_session* s, int32_t k, int32_t* steps_done, int32_t* done, double* step_ms);
int icp_session_finish(icp_session* s, icp_result* res);
/* Current cumulative transform (row-major 4x4). */
void icp_session_transform(const icp_session* s, double T_cum[16]);
void icp_session_destroy(icp_session* s);

/* CLI ICP(): octree 10/20, best init 1e20, threshold mean + 3 std, final R/t = the LAST
 * INCREMENTAL transform (icp_registration.cpp:616-621), cumulative transforms appended to
 * iteration_transforms (cap x 16, row-major) when non-null. */
int icp_cli_icp(double* src_xyz, int64_t n_src, const double* tgt_xyz, int64_t n_tgt, int max_iterations,
                double tolerance, double final_R[9], double final_t[3], double* iteration_transforms,
                int32_t cap, int32_t* n_transforms, int device);

/* icp_cli_icp on several GPUs of this process (as icp_engine_register_devices). */
int icp_cli_icp_devices(double* src_xyz, int64_t n_src, const double* tgt_xyz, int64_t n_tgt, int max_iterations,
                        double tolerance, double final_R[9], double final_t[3], double* iteration_transforms,
                        int32_t cap, int32_t* n_transforms, int n_devices, const int* device_ids);

/* Host helpers (no GPU needed). */
void icp_jacobi_svd3(const double H[9], double U[9], double S[3], double V[9]);
void icp_best_fit_transform(const double* a_xyz, const double* b_xyz, int64_t n, double T[16]);
void icp_best_fit_from_stats(const icp_iter_stats* st, double T[16]);
void icp_mat4_mul(const double A[16], const double B[16], double C[16]);

#ifdef __cplusplus
}
#endif
#endif
