// engine.cpp — host ICP driver over the device path (include/icp_engine.h).
//
// The control flow is the reference loop (core/icpengine.cpp:117-394 and its CLI twin
// icp_registration.cpp:443-622), with the per-point work delegated to icp_hip_iterate:
//   iterate (apply the previous T on the device, NN, residual, 3-sigma, cull, moments)
//   -> convergence / divergence / too-few checks (icpengine.cpp:287-323)
//   -> 3x3 SVD best fit on the host (icpengine.cpp:339) -> T_cum = T * T_cum (:342)
//   -> T is applied at the start of the next iterate (or explicitly after the loop).
#include <cfloat>
#include <cstdarg>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/icp_engine.h"
#include "icp_ctx_internal.h"
#include "svd3.h"

namespace {

void set_msg(icp_result* r, const char* m) {
  std::snprintf(r->message, sizeof(r->message), "%s", m);
}

void identity(double T[16]) {
  for (int k = 0; k < 16; k++) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
}

void log_msg(const icp_engine_hooks* h, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void log_msg(const icp_engine_hooks* h, const char* fmt, ...) {
  if (!h || !h->on_log) return;
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  h->on_log(h->user, buf);
}

}  // namespace

extern "C" {

void icp_params_default(icp_params* p) {
  // ICPParameters defaults (icpengine.h:13-19)
  p->max_iterations = 50;
  p->tolerance = 1e-6;
  p->sigma_multiplier = 3.0;
  p->octree_max_points = 10;
  p->octree_max_depth = 20;
  p->rules = ICP_RULES_ENGINE;
  p->flags = 0;
}

void icp_jacobi_svd3(const double H[9], double U[9], double S[3], double V[9]) { icp::jacobi_svd3(H, U, S, V); }

void icp_mat4_mul(const double A[16], const double B[16], double C[16]) { icp::mat4_mul(A, B, C); }

void icp_best_fit_from_stats(const icp_iter_stats* st, double T[16]) {
  icp::best_fit_from_moments(st->centroid_src, st->centroid_tgt, st->H, T);
}

void icp_best_fit_transform(const double* a, const double* b, int64_t n, double T[16]) {
  double ma[3] = {0, 0, 0}, mb[3] = {0, 0, 0}, C[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (n <= 0) {
    identity(T);
    return;
  }
  for (int64_t i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) {
      ma[k] += a[3 * i + k];
      mb[k] += b[3 * i + k];
    }
  for (int k = 0; k < 3; k++) {
    ma[k] /= (double)n;
    mb[k] /= (double)n;
  }
  for (int64_t i = 0; i < n; i++)
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) C[3 * r + c] += (a[3 * i + r] - ma[r]) * (b[3 * i + c] - mb[c]);
  icp::best_fit_from_moments(ma, mb, C, T);
}

}  // extern "C"

struct icp_session {
  icp_hip_ctx* ctx = nullptr;
  icp_params p;
  icp_engine_hooks hooks;
  const icp_engine_hooks* h = nullptr;
  double T[16], Tc[16];
  double prev = 1e10;  // icpengine.cpp:156
  int no_imp = 0, iter = 0, n_hist = 0;
  bool pending = false, done = false;
  double last_rec_rmse = 0.0;
  int status = ICP_STATUS_MAX_ITERATIONS;
  int rc_final = ICP_HIP_OK;
  char message[160] = {0};
};

extern "C" {

int icp_session_create(icp_hip_ctx* ctx, const icp_params* p, const icp_engine_hooks* hooks, icp_session** out) {
  if (!ctx || !p || !out) return ICP_HIP_EINVAL;
  icp_session* s = new icp_session();
  s->ctx = ctx;
  s->p = *p;
  if (hooks) {
    s->hooks = *hooks;
    s->h = &s->hooks;
  }
  identity(s->T);
  identity(s->Tc);
  s->done = p->max_iterations <= 0;
  *out = s;
  return ICP_HIP_OK;
}

void icp_session_destroy(icp_session* s) { delete s; }

void icp_session_transform(const icp_session* s, double T_cum[16]) { std::memcpy(T_cum, s->Tc, sizeof(s->Tc)); }

static void fill_record(icp_iteration_record* h, int iter, double rmse, int32_t valid, int32_t outliers,
                        const icp_iter_stats& st) {
  std::memset(h, 0, sizeof(*h));
  h->iteration = iter + 1;
  h->rmse = rmse;
  h->valid_points = valid;
  h->outlier_points = outliers;
  h->mean = st.mean;
  h->std = st.std;
  h->threshold = st.threshold;
}

int icp_session_step(icp_session* s, icp_iteration_record* rec, int32_t* produced, int32_t* done) {
  if (!s) return ICP_HIP_EINVAL;
  if (produced) *produced = 0;
  if (s->done) {
    if (done) *done = 1;
    return ICP_HIP_OK;
  }
  const icp_params& p = s->p;
  const icp_engine_hooks* hooks = s->h;
  const bool cli = p.rules == ICP_RULES_CLI;
  const bool no_stop = (p.flags & ICP_FLAG_NO_EARLY_STOP) != 0;
  const double k_sigma = cli ? 3.0 : p.sigma_multiplier;  // CLI hard-codes 3.0 (:523)
  const int iter = s->iter;
  auto finish_step = [&](bool stop) {
    s->iter++;
    if (stop || s->iter >= p.max_iterations) s->done = true;
    if (done) *done = s->done ? 1 : 0;
    return ICP_HIP_OK;
  };
  if (hooks && hooks->stop_flag && *hooks->stop_flag) {  // icpengine.cpp:160-164
    log_msg(hooks, "registration stopped");
    s->status = ICP_STATUS_CANCELLED;
    s->rc_final = ICP_ENGINE_CANCELLED;
    std::snprintf(s->message, sizeof(s->message), "cancelled by user");
    return finish_step(true);
  }
  icp_iter_stats st;
  int rc = icp_hip_iterate(s->ctx, s->pending ? s->T : nullptr, iter, p.rules, k_sigma, &st);
  if (rc != ICP_HIP_OK) {
    s->rc_final = rc;
    std::snprintf(s->message, sizeof(s->message), "%s", icp_hip_last_error());
    finish_step(true);
    return rc;
  }
  s->pending = false;
  const double rmse = st.rmse;
  const int32_t valid = (int32_t)st.valid;
  const int32_t outliers = (int32_t)(st.n - st.valid);
  if (st.n_bad > 0) log_msg(hooks, "warning: %lld non-finite distances", (long long)st.n_bad);
  log_msg(hooks, "iteration %d: mean=%.6f std=%.6f threshold=%.6f RMSE=%.6f valid %d/%lld", iter + 1, st.mean,
          st.std, st.threshold, rmse, valid, (long long)st.n);
  // convergence (icpengine.cpp:287-309)
  const double improvement = s->prev - rmse;
  if (std::fabs(improvement) < p.tolerance) {
    s->no_imp++;
    if (s->no_imp >= 3 && !no_stop) {
      s->status = ICP_STATUS_CONVERGED;
      log_msg(hooks, "converged after %d iterations", iter + 1);
      if (!cli) {  // the engine records a final entry with T_cumulative (icpengine.cpp:293-303)
        icp_iteration_record h;
        fill_record(&h, iter, rmse, valid, outliers, st);
        std::memcpy(h.transform, s->Tc, sizeof(s->Tc));
        identity(h.increment);
        h.rotation_angle_deg = NAN;  // left uninitialised by the reference
        h.translation_distance = NAN;
        h.has_transform = 0;
        if (rec) *rec = h;
        if (produced) *produced = 1;
        if (hooks && hooks->on_iteration) hooks->on_iteration(hooks->user, &h);
        s->n_hist++;
        s->last_rec_rmse = rmse;
        if (hooks && hooks->on_progress) hooks->on_progress(hooks->user, iter + 1, p.max_iterations, rmse);
      }
      return finish_step(true);
    }
  } else {
    s->no_imp = 0;
  }
  if (rmse > s->prev * 1.1 && !no_stop) {  // icpengine.cpp:311-314
    s->status = ICP_STATUS_DIVERGED;
    log_msg(hooks, "warning: error increased, stopping");
    return finish_step(true);
  }
  s->prev = rmse;
  if (valid < 3) {  // icpengine.cpp:319-323 (engine fails) / icp_registration.cpp:567-570 (CLI breaks)
    s->status = ICP_STATUS_TOO_FEW;
    if (!cli) {
      s->rc_final = ICP_ENGINE_TOO_FEW;
      std::snprintf(s->message, sizeof(s->message), "too few valid point pairs");
    }
    return finish_step(true);
  }
  icp_best_fit_from_stats(&st, s->T);  // icpengine.cpp:339
  icp::mat4_mul(s->T, s->Tc, s->Tc);   // icpengine.cpp:342
  s->pending = true;                   // src = T * src: fused into the next iterate (or finish)
  icp_iteration_record h;
  fill_record(&h, iter, rmse, valid, outliers, st);
  std::memcpy(h.transform, s->Tc, sizeof(s->Tc));
  std::memcpy(h.increment, s->T, sizeof(s->T));
  const double* Tc = s->Tc;
  const double trace = Tc[0] + Tc[5] + Tc[10];  // icpengine.cpp:357-362
  h.rotation_angle_deg = std::acos((trace - 1.0) / 2.0) * 180.0 / M_PI;
  h.translation_distance = std::sqrt((Tc[3] * Tc[3] + Tc[7] * Tc[7]) + Tc[11] * Tc[11]);
  h.has_transform = 1;
  if (rec) *rec = h;
  if (produced) *produced = 1;
  if (hooks && hooks->on_iteration) hooks->on_iteration(hooks->user, &h);
  s->n_hist++;
  s->last_rec_rmse = rmse;
  if (hooks && hooks->on_progress) hooks->on_progress(hooks->user, iter + 1, p.max_iterations, rmse);
  return finish_step(false);
}

int icp_session_step_n(icp_session* s, int32_t k, int32_t* steps_done, int32_t* done) {
  if (!s || k < 0) return ICP_HIP_EINVAL;
  int32_t n = 0, d = 0;
  int rc = ICP_HIP_OK;
  while (n < k && !d) {
    rc = icp_session_step(s, nullptr, nullptr, &d);
    if (rc != ICP_HIP_OK) break;
    n++;
  }
  if (steps_done) *steps_done = n;
  if (done) *done = d;
  return rc;
}

int icp_session_step_n_timed(icp_session* s, int32_t k, int32_t* steps_done, int32_t* done, double* step_ms) {
  if (!s || k < 0 || (k > 0 && !step_ms)) return ICP_HIP_EINVAL;
  int32_t n = 0, d = 0;
  int rc = ICP_HIP_OK;
  auto t0 = std::chrono::steady_clock::now();
  while (n < k && !d) {
    rc = icp_session_step(s, nullptr, nullptr, &d);
    if (rc != ICP_HIP_OK) break;
    const auto t1 = std::chrono::steady_clock::now();
    step_ms[n] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    t0 = t1;
    n++;
  }
  if (steps_done) *steps_done = n;
  if (done) *done = d;
  return rc;
}

int icp_session_finish(icp_session* s, icp_result* res) {
  if (!s || !res) return ICP_HIP_EINVAL;
  std::memset(res, 0, sizeof(*res));
  res->status = s->status;
  res->total_iterations = s->n_hist;
  res->n_history = s->n_hist;
  if (s->rc_final != ICP_HIP_OK) {
    set_msg(res, s->message);
    return s->rc_final;  // cancelled / engine too-few / device error: no write-back, success = false
  }
  if (s->pending) {
    int rc = icp_hip_apply(s->ctx, s->T);
    if (rc != ICP_HIP_OK) {
      set_msg(res, icp_hip_last_error());
      return rc;
    }
    s->pending = false;
  }
  const bool cli = s->p.rules == ICP_RULES_CLI;
  // final R/t: engine = T_cumulative (icpengine.cpp:378-383); CLI = last incremental T (:616-621)
  const double* F = cli ? s->T : s->Tc;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) res->final_R[3 * r + c] = F[4 * r + c];
    res->final_t[r] = F[4 * r + 3];
  }
  res->success = 1;
  // icpengine.cpp:387 (last recorded rmse) / the CLI prints prev_error
  res->final_rmse = cli ? s->prev : (s->n_hist > 0 ? s->last_rec_rmse : 0.0);
  set_msg(res, "registration finished");
  return ICP_HIP_OK;
}

int icp_engine_run(icp_hip_ctx* ctx, const icp_params* p, icp_result* res, icp_iteration_record* hist,
                   int32_t cap, const icp_engine_hooks* hooks) {
  if (!ctx || !p || !res) return ICP_HIP_EINVAL;
  icp_session* s = nullptr;
  int rc = icp_session_create(ctx, p, hooks, &s);
  if (rc != ICP_HIP_OK) return rc;
  int32_t done = 0, n = 0;
  while (!done) {
    icp_iteration_record rec;
    int32_t produced = 0;
    rc = icp_session_step(s, &rec, &produced, &done);
    if (produced && hist && n < cap) hist[n] = rec;
    if (produced) n++;
    if (rc != ICP_HIP_OK) break;
  }
  int rc2 = icp_session_finish(s, res);
  icp_session_destroy(s);
  res->n_history = n < cap ? n : cap;
  return rc != ICP_HIP_OK ? rc : rc2;
}

int icp_engine_register(const icp_params* p, double* src, int64_t n_src, const double* tgt, int64_t n_tgt,
                        int device, icp_result* res, icp_iteration_record* hist, int32_t cap,
                        const icp_engine_hooks* hooks) {
  return icp_engine_register_devices(p, src, n_src, tgt, n_tgt, 1, &device, res, hist, cap, hooks);
}

int icp_engine_register_devices(const icp_params* p, double* src, int64_t n_src, const double* tgt, int64_t n_tgt,
                                int n_devices, const int* device_ids, icp_result* res, icp_iteration_record* hist,
                                int32_t cap, const icp_engine_hooks* hooks) {
  if (!p || !res) return ICP_HIP_EINVAL;
  std::memset(res, 0, sizeof(*res));
  if (!src || !tgt) {  // icpengine.cpp:26-29
    set_msg(res, "source or target cloud is null");
    return ICP_HIP_EINVAL;
  }
  if (n_src <= 0 || n_tgt <= 0) {  // icpengine.cpp:31-34
    set_msg(res, "point cloud is empty");
    return ICP_HIP_EINVAL;
  }
  if (n_devices < 1 || !device_ids) {
    set_msg(res, "empty device list");
    return ICP_HIP_EINVAL;
  }
  const bool cli = p->rules == ICP_RULES_CLI;
  icp_hip_ctx* ctx = nullptr;
  // one device: a plain context; several: one context over all of them (source shards, RCCL)
  int rc = n_devices == 1 ? icp_hip_create(&ctx, device_ids[0])
                          : icp_hip_create_multi(&ctx, n_devices, device_ids, nullptr, ICP_XPORT_AUTO);
  if (rc == ICP_HIP_OK)
    rc = icp_hip_set_target(ctx, tgt, n_tgt, cli ? 10 : p->octree_max_points, cli ? 20 : p->octree_max_depth,
                            p->rules);
  if (rc == ICP_HIP_OK) rc = icp_hip_set_source(ctx, src, n_src);
  if (rc != ICP_HIP_OK) {
    set_msg(res, icp_hip_last_error());
    icp_hip_destroy(ctx);
    return rc;
  }
  log_msg(hooks, "source: %lld points, target: %lld points, %d device(s)", (long long)n_src, (long long)n_tgt,
          n_devices);
  rc = icp_engine_run(ctx, p, res, hist, cap, hooks);
  // write back (icpengine.cpp:371-375): only when the engine finished; the CLI always writes
  // back what it has (icp_registration.cpp:609-613) — a CLI "too few" break is a success there.
  if (rc == ICP_HIP_OK) {
    int rc2 = icp_hip_get_source(ctx, src);
    if (rc2 != ICP_HIP_OK) {
      set_msg(res, icp_hip_last_error());
      rc = rc2;
      res->success = 0;
    }
  }
  icp_hip_destroy(ctx);
  return rc;
}

int icp_cli_icp(double* src, int64_t n_src, const double* tgt, int64_t n_tgt, int max_iterations, double tolerance,
                double final_R[9], double final_t[3], double* iteration_transforms, int32_t cap, int32_t* n_transforms,
                int device) {
  return icp_cli_icp_devices(src, n_src, tgt, n_tgt, max_iterations, tolerance, final_R, final_t, iteration_transforms,
                             cap, n_transforms, 1, &device);
}

int icp_cli_icp_devices(double* src, int64_t n_src, const double* tgt, int64_t n_tgt, int max_iterations,
                        double tolerance, double final_R[9], double final_t[3], double* iteration_transforms,
                        int32_t cap, int32_t* n_transforms, int n_devices, const int* device_ids) {
  icp_params p;
  icp_params_default(&p);
  p.max_iterations = max_iterations;
  p.tolerance = tolerance;
  p.rules = ICP_RULES_CLI;
  std::vector<icp_iteration_record> hist((size_t)(max_iterations > 0 ? max_iterations : 1));
  icp_result res;
  int rc = icp_engine_register_devices(&p, src, n_src, tgt, n_tgt, n_devices, device_ids, &res, hist.data(),
                                       (int32_t)hist.size(), nullptr);
  if (rc != ICP_HIP_OK) return rc;
  for (int k = 0; k < 9; k++) final_R[k] = res.final_R[k];
  for (int k = 0; k < 3; k++) final_t[k] = res.final_t[k];
  int32_t m = 0;
  for (int32_t k = 0; k < res.n_history; k++) {
    if (!hist[k].has_transform) continue;
    if (iteration_transforms && m < cap) std::memcpy(iteration_transforms + 16 * m, hist[k].transform, 16 * sizeof(double));
    m++;
  }
  if (n_transforms) *n_transforms = m;
  return ICP_HIP_OK;
}

}  // extern "C"
