// session_step.h — the ICP loop's per-iteration decisions as ONE host + device function: the host
// session (engine.cpp icp_session_step) and the device-resident loop (reduce_kernels.hip, the
// iteration's last kernel) both call session_core_step, so the two loops take the same decisions
// on the same statistics and compute the same transforms bit for bit (svd3_impl.h: IEEE fp64,
// no contraction).
//
//   convergence   |prev - rmse| < tolerance three times in a row       icpengine.cpp:287-309
//                 (CLI: icp_registration.cpp:545-556)
//   divergence    rmse > 1.1 prev                                      icpengine.cpp:311-314
//   too few       fewer than 3 valid pairs                             icpengine.cpp:319-323 (CLI :567-570)
//   best fit      R = V U^T, t = mb - R ma                             icpengine.cpp:76-115, :339
//   accumulate    T_cum = T * T_cum                                    icpengine.cpp:342
#pragma once

#include <cstdint>

#include "../../include/icp_engine.h"
#include "icp_common.h"
#include "svd3_impl.h"

namespace icp {

// The session state both loops carry (engine.cpp's icp_session holds one; the device loop one in
// device memory, copied back after a batch).
struct SessionCore {
  double T[16];   // the last increment: src = T * src is still to be applied when pending
  double Tc[16];  // cumulative transform
  double prev;    // the previous iteration's RMSE (icpengine.cpp:156: 1e10)
  double last_rec_rmse;
  int32_t iter, no_imp, n_hist, pending, done, status, too_few, pad;
};

struct SessionParams {
  double tolerance;
  int32_t max_iterations;
  int32_t cli;      // ICP_RULES_CLI: no convergence record, "too few" is a break, not a failure
  int32_t no_stop;  // ICP_FLAG_NO_EARLY_STOP
  int32_t pad;
};

enum StepOutcome : int32_t {
  kStepNone = 0,       // no iteration ran (the session was done)
  kStepTransform = 1,  // a transform record (T, T_cum)
  kStepConverged = 2,  // converged: the engine records a final entry with T_cum, the CLI none
  kStepDiverged = 3,
  kStepTooFew = 4,
};

ICP_HD void session_core_init(SessionCore& s, int32_t max_iterations) {
  for (int k = 0; k < 16; k++) s.T[k] = s.Tc[k] = (k % 5 == 0) ? 1.0 : 0.0;
  s.prev = 1e10;
  s.last_rec_rmse = 0.0;
  s.iter = s.no_imp = s.n_hist = s.pending = s.too_few = s.pad = 0;
  s.done = max_iterations <= 0 ? 1 : 0;
  s.status = ICP_STATUS_MAX_ITERATIONS;
}

// One iteration's decisions on its statistics (rmse, valid pairs, centroids ma/mb, co-moment H).
// Returns the outcome; the state advances as engine.cpp's finish_step does (iter + 1, done on a
// stop or at max_iterations).
ICP_HD int32_t session_core_step(SessionCore& s, const SessionParams& p, double rmse, int64_t valid,
                                 const double ma[3], const double mb[3], const double H[9]) {
  int32_t out = kStepTransform;
  bool stop = false;
  const double improvement = s.prev - rmse;
  if (__builtin_fabs(improvement) < p.tolerance) {
    s.no_imp++;
    if (s.no_imp >= 3 && !p.no_stop) {
      s.status = ICP_STATUS_CONVERGED;
      if (!p.cli) {
        s.n_hist++;
        s.last_rec_rmse = rmse;
      }
      out = kStepConverged;
      stop = true;
    }
  } else {
    s.no_imp = 0;
  }
  if (!stop && rmse > s.prev * 1.1 && !p.no_stop) {
    s.status = ICP_STATUS_DIVERGED;
    out = kStepDiverged;
    stop = true;
  }
  if (!stop) {
    s.prev = rmse;
    if ((int64_t)valid < 3) {
      s.status = ICP_STATUS_TOO_FEW;
      if (!p.cli) s.too_few = 1;
      out = kStepTooFew;
      stop = true;
    }
  }
  if (!stop) {
    svd::best_fit_from_moments(ma, mb, H, s.T);
    svd::mat4_mul(s.T, s.Tc, s.Tc);
    s.pending = 1;
    s.n_hist++;
    s.last_rec_rmse = rmse;
  }
  s.iter++;
  if (stop || s.iter >= p.max_iterations) s.done = 1;
  return out;
}

// One iteration of the device loop as the host reads it back (pinned host memory, written by the
// iteration's last kernel): the statistics of icp_iter_stats, the outcome and the transforms.
struct LoopRec {
  double n, mean, sd, thr, valid, rmse, sum_d2, dmin, dmax, nbad;
  double ma[3], mb[3], H[9];
  double lists[3];  // exact, ball, per-lane list sizes of the search
  double T[16], Tc[16];
  int32_t outcome;  // StepOutcome (kStepNone: the session was already done)
  int32_t iter;     // the iteration index (0-based)
  int32_t pad[2];
};

}  // namespace icp
