// engine.cpp — host ICP driver over the device path (include/icp_engine.h).
//
// The control flow is the reference loop (core/icpengine.cpp:117-394 and its CLI twin
// icp_registration.cpp:443-622), with the per-point work delegated to icp_hip_iterate:
//   iterate (apply the previous T on the device, NN, residual, 3-sigma, cull, moments)
//   -> convergence / divergence / too-few checks (icpengine.cpp:287-323)
//   -> 3x3 SVD best fit on the host (icpengine.cpp:339) -> T_cum = T * T_cum (:342)
//   -> T is applied at the start of the next iterate (or explicitly after the loop).
#include <algorithm>
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
#include "session_step.h"
#include "svd3_impl.h"  // the 3x3 Jacobi SVD and best fit (host + device, Eigen JacobiSVD order)

namespace {

// iterations per device-loop batch of icp_engine_run (a registration converges in tens)
constexpr int32_t kEngineBatch = 16;

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

void icp_jacobi_svd3(const double H[9], double U[9], double S[3], double V[9]) { icp::svd::jacobi_svd3(H, U, S, V); }

void icp_mat4_mul(const double A[16], const double B[16], double C[16]) { icp::svd::mat4_mul(A, B, C); }

void icp_best_fit_from_stats(const icp_iter_stats* st, double T[16]) {
  icp::svd::best_fit_from_moments(st->centroid_src, st->centroid_tgt, st->H, T);
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
  icp::svd::best_fit_from_moments(ma, mb, C, T);
}

}  // extern "C"

struct icp_session {
  icp_hip_ctx* ctx = nullptr;
  icp_params p;
  icp_engine_hooks hooks;
  const icp_engine_hooks* h = nullptr;
  icp::SessionCore core;   // T, T_cum, prev, counters, status (session_step.h)
  icp::SessionParams sp;
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
  icp::session_core_init(s->core, p->max_iterations);
  s->sp.tolerance = p->tolerance;
  s->sp.max_iterations = p->max_iterations;
  s->sp.cli = p->rules == ICP_RULES_CLI ? 1 : 0;
  s->sp.no_stop = (p->flags & ICP_FLAG_NO_EARLY_STOP) != 0 ? 1 : 0;
  s->sp.pad = 0;
  *out = s;
  return ICP_HIP_OK;
}

void icp_session_destroy(icp_session* s) { delete s; }

void icp_session_transform(const icp_session* s, double T_cum[16]) { std::memcpy(T_cum, s->core.Tc, sizeof(s->core.Tc)); }

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

// What one iteration produced, as both loops report it: the log lines, the record of the
// iteration (icpengine.cpp:293-303, :349-366) and the hooks. T / Tc: the session's transforms
// after the iteration.
static void emit_iteration(icp_session* s, int iter, int32_t outcome, const icp_iter_stats& st, const double T[16],
                           const double Tc[16], icp_iteration_record* rec, int32_t* produced) {
  const icp_engine_hooks* hooks = s->h;
  const bool cli = s->sp.cli != 0;
  const double rmse = st.rmse;
  const int32_t valid = (int32_t)st.valid;
  const int32_t outliers = (int32_t)(st.n - st.valid);
  if (st.n_bad > 0) log_msg(hooks, "warning: %lld non-finite distances", (long long)st.n_bad);
  log_msg(hooks, "iteration %d: mean=%.6f std=%.6f threshold=%.6f RMSE=%.6f valid %d/%lld", iter + 1, st.mean,
          st.std, st.threshold, rmse, valid, (long long)st.n);
  icp_iteration_record h;
  bool have = false;
  if (outcome == icp::kStepConverged) {
    log_msg(hooks, "converged after %d iterations", iter + 1);
    if (!cli) {  // the engine records a final entry with T_cumulative (icpengine.cpp:293-303)
      fill_record(&h, iter, rmse, valid, outliers, st);
      std::memcpy(h.transform, Tc, sizeof(h.transform));
      identity(h.increment);
      h.rotation_angle_deg = NAN;  // left uninitialised by the reference
      h.translation_distance = NAN;
      h.has_transform = 0;
      have = true;
    }
  } else if (outcome == icp::kStepDiverged) {
    log_msg(hooks, "warning: error increased, stopping");
  } else if (outcome == icp::kStepTooFew) {
    if (!cli) {
      s->rc_final = ICP_ENGINE_TOO_FEW;
      std::snprintf(s->message, sizeof(s->message), "too few valid point pairs");
    }
  } else if (outcome == icp::kStepTransform) {
    fill_record(&h, iter, rmse, valid, outliers, st);
    std::memcpy(h.transform, Tc, sizeof(h.transform));
    std::memcpy(h.increment, T, sizeof(h.increment));
    const double trace = Tc[0] + Tc[5] + Tc[10];  // icpengine.cpp:357-362
    h.rotation_angle_deg = std::acos((trace - 1.0) / 2.0) * 180.0 / M_PI;
    h.translation_distance = std::sqrt((Tc[3] * Tc[3] + Tc[7] * Tc[7]) + Tc[11] * Tc[11]);
    h.has_transform = 1;
    have = true;
  }
  if (!have) return;
  if (rec) *rec = h;
  if (produced) *produced = 1;
  if (hooks && hooks->on_iteration) hooks->on_iteration(hooks->user, &h);
  if (hooks && hooks->on_progress) hooks->on_progress(hooks->user, iter + 1, s->sp.max_iterations, rmse);
}

// The cancellation check at the top of an iteration (icpengine.cpp:160-164): true if it stopped
// the session.
static bool cancelled(icp_session* s) {
  const icp_engine_hooks* hooks = s->h;
  if (!(hooks && hooks->stop_flag && *hooks->stop_flag)) return false;
  log_msg(hooks, "registration stopped");
  s->core.status = ICP_STATUS_CANCELLED;
  s->rc_final = ICP_ENGINE_CANCELLED;
  std::snprintf(s->message, sizeof(s->message), "cancelled by user");
  s->core.iter++;
  s->core.done = 1;
  return true;
}

int icp_session_step(icp_session* s, icp_iteration_record* rec, int32_t* produced, int32_t* done) {
  if (!s) return ICP_HIP_EINVAL;
  if (produced) *produced = 0;
  if (!s->core.done && !cancelled(s)) {
    const icp_params& p = s->p;
    const bool cli = p.rules == ICP_RULES_CLI;
    const double k_sigma = cli ? 3.0 : p.sigma_multiplier;  // CLI hard-codes 3.0 (:523)
    const int iter = s->core.iter;
    icp_iter_stats st;
    const int rc = icp_hip_iterate(s->ctx, s->core.pending ? s->core.T : nullptr, iter, p.rules, k_sigma, &st);
    if (rc != ICP_HIP_OK) {
      s->rc_final = rc;
      std::snprintf(s->message, sizeof(s->message), "%s", icp_hip_last_error());
      s->core.iter++;
      s->core.done = 1;
      if (done) *done = 1;
      return rc;
    }
    s->core.pending = 0;
    const int32_t outcome = icp::session_core_step(s->core, s->sp, st.rmse, st.valid, st.centroid_src,
                                                   st.centroid_tgt, st.H);
    emit_iteration(s, iter, outcome, st, s->core.T, s->core.Tc, rec, produced);
  }
  if (done) *done = s->core.done ? 1 : 0;
  return ICP_HIP_OK;
}

// Up to k iterations: on the device loop (icp_hip_loop_run, batches of up to kLoopRing) or one
// host step at a time. Records and hooks are
// emitted in iteration order either way; `hist`/`cap` collect the records, step_ms the per-step
// times (device loop: each iteration's device time; host: wall time per step).
static int session_run(icp_session* s, int32_t k, int32_t* steps_done, int32_t* done, double* step_ms,
                       icp_iteration_record* hist, int32_t cap, int32_t* n_hist) {
  int32_t n = 0;
  int rc = ICP_HIP_OK;
  const bool cli = s->p.rules == ICP_RULES_CLI;
  const double k_sigma = cli ? 3.0 : s->p.sigma_multiplier;
  // A stop flag is checked before every iteration against the hooks of the previous one
  // (icpengine.cpp:160-164; a flag raised from a progress hook stops the next iteration): such a
  // session steps on the host.
  const bool per_iteration_stop = s->h && s->h->stop_flag;
  if (icp_hip_loop_eligible(s->ctx) && !per_iteration_stop) {
    std::vector<icp::LoopRec> recs((size_t)icp_hip_ctx::kLoopRing);
    std::vector<double> ms((size_t)icp_hip_ctx::kLoopRing);
    while (n < k && !s->core.done && rc == ICP_HIP_OK) {
      const int32_t b = std::min<int32_t>(k - n, icp_hip_ctx::kLoopRing);
      rc = icp_hip_loop_run(s->ctx, &s->core, &s->sp, s->p.rules, k_sigma, b, recs.data(), ms.data());
      if (rc != ICP_HIP_OK) {
        s->rc_final = rc;
        std::snprintf(s->message, sizeof(s->message), "%s", icp_hip_last_error());
        s->core.done = 1;
        break;
      }
      for (int32_t j = 0; j < b; j++) {
        const icp::LoopRec& r = recs[j];
        if (r.outcome == icp::kStepNone) break;
        icp_iter_stats st;
        std::memset(&st, 0, sizeof(st));
        st.n = (int64_t)r.n;
        st.mean = r.mean;
        st.std = r.sd;
        st.threshold = r.thr;
        st.valid = (int64_t)r.valid;
        st.rmse = r.rmse;
        st.sum_d2 = r.sum_d2;
        st.min_d = r.dmin;
        st.max_d = r.dmax;
        st.n_bad = (int64_t)r.nbad;
        for (int q = 0; q < 3; q++) {
          st.centroid_src[q] = r.ma[q];
          st.centroid_tgt[q] = r.mb[q];
        }
        for (int q = 0; q < 9; q++) st.H[q] = r.H[q];
        icp_iteration_record h;
        int32_t produced = 0;
        emit_iteration(s, r.iter, r.outcome, st, r.T, r.Tc, &h, &produced);
        if (produced && n_hist) {
          if (hist && *n_hist < cap) hist[*n_hist] = h;
          (*n_hist)++;
        }
        if (step_ms) step_ms[n] = ms[j];
        n++;
      }
    }
  } else {
    auto t0 = std::chrono::steady_clock::now();
    while (n < k && !s->core.done) {
      icp_iteration_record h;
      int32_t produced = 0, d = 0;
      rc = icp_session_step(s, &h, &produced, &d);
      if (produced && n_hist) {
        if (hist && *n_hist < cap) hist[*n_hist] = h;
        (*n_hist)++;
      }
      if (rc != ICP_HIP_OK) break;
      if (step_ms) {
        const auto t1 = std::chrono::steady_clock::now();
        step_ms[n] = std::chrono::duration<double, std::milli>(t1 - t0).count();
        t0 = t1;
      }
      n++;
    }
  }
  if (steps_done) *steps_done = n;
  if (done) *done = s->core.done ? 1 : 0;
  return rc;
}

int icp_session_step_n(icp_session* s, int32_t k, int32_t* steps_done, int32_t* done) {
  if (!s || k < 0) return ICP_HIP_EINVAL;
  return session_run(s, k, steps_done, done, nullptr, nullptr, 0, nullptr);
}

int icp_session_step_n_timed(icp_session* s, int32_t k, int32_t* steps_done, int32_t* done, double* step_ms) {
  if (!s || k < 0 || (k > 0 && !step_ms)) return ICP_HIP_EINVAL;
  return session_run(s, k, steps_done, done, step_ms, nullptr, 0, nullptr);
}

int icp_session_finish(icp_session* s, icp_result* res) {
  if (!s || !res) return ICP_HIP_EINVAL;
  std::memset(res, 0, sizeof(*res));
  res->status = s->core.status;
  res->total_iterations = s->core.n_hist;
  res->n_history = s->core.n_hist;
  if (s->rc_final != ICP_HIP_OK) {
    set_msg(res, s->message);
    return s->rc_final;  // cancelled / engine too-few / device error: no write-back, success = false
  }
  if (s->core.pending) {
    int rc = icp_hip_apply(s->ctx, s->core.T);
    if (rc != ICP_HIP_OK) {
      set_msg(res, icp_hip_last_error());
      return rc;
    }
    s->core.pending = 0;
  }
  const bool cli = s->p.rules == ICP_RULES_CLI;
  // final R/t: engine = T_cumulative (icpengine.cpp:378-383); CLI = last incremental T (:616-621)
  const double* F = cli ? s->core.T : s->core.Tc;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) res->final_R[3 * r + c] = F[4 * r + c];
    res->final_t[r] = F[4 * r + 3];
  }
  res->success = 1;
  // icpengine.cpp:387 (last recorded rmse) / the CLI prints prev_error
  res->final_rmse = cli ? s->core.prev : (s->core.n_hist > 0 ? s->core.last_rec_rmse : 0.0);
  set_msg(res, "registration finished");
  return ICP_HIP_OK;
}

int icp_engine_run(icp_hip_ctx* ctx, const icp_params* p, icp_result* res, icp_iteration_record* hist,
                   int32_t cap, const icp_engine_hooks* hooks) {
  if (!ctx || !p || !res) return ICP_HIP_EINVAL;
  icp_session* s = nullptr;
  int rc = icp_session_create(ctx, p, hooks, &s);
  if (rc != ICP_HIP_OK) return rc;
  int32_t n = 0, done = 0, steps = 0;
  // the device loop in batches of kEngineBatch (iterations enqueued past convergence return at
  // once), else host steps
  while (!done && rc == ICP_HIP_OK) rc = session_run(s, kEngineBatch, &steps, &done, nullptr, hist, cap, &n);
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
