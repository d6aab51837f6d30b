// icp_ctx_internal.h — layout of the C-ABI context (private to libicp_hip.so).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/icp_hip.h"
#include "kernels.h"

// The host-exchange callback run on a thread of its own, so that the iterate can give up on it
// at config.peer_timeout_ms (the callback is the caller's code: it cannot be interrupted, only
// abandoned). One job at a time; an abandoned job finishes on its own, and join() (comm_init,
// comm_init_host, destroy) waits for it.
struct ExchangeWorker {
  std::mutex m;
  std::condition_variable cv;
  std::thread th;
  bool job = false, done = false, quit = false;
  icp_hip_exchange_fn fn = nullptr;
  void* user = nullptr;
  std::vector<double> local, all;
  int count = 0, rc = 0;

  ExchangeWorker() {
    th = std::thread([this] {
      std::unique_lock<std::mutex> lk(m);
      while (true) {
        cv.wait(lk, [this] { return job || quit; });
        if (quit && !job) return;
        lk.unlock();
        const int r = fn(user, local.data(), count, all.data());
        lk.lock();
        rc = r;
        job = false;
        done = true;
        cv.notify_all();
      }
    });
  }
  // The callback on this rank's record; 0 = done in time (gathered in `all`), 1 = the deadline
  // passed first (the job stays with the thread).
  int run(icp_hip_exchange_fn f, void* u, const double* rec, int n, int nranks, int timeout_ms) {
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [this] { return !job; });  // an abandoned job first
    fn = f;
    user = u;
    count = n;
    local.assign(rec, rec + n);
    all.assign((size_t)n * nranks, 0.0);
    done = false;
    job = true;
    cv.notify_all();
    if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [this] { return done; })) return 1;
    return 0;
  }
  void join() {
    {
      std::lock_guard<std::mutex> lk(m);
      quit = true;
    }
    cv.notify_all();
    if (th.joinable()) th.join();
  }
  ~ExchangeWorker() { join(); }
};

struct icp_hip_ctx {
  int device = 0;
  icp_hip_config cfg{};  // explicit configuration (icp_hip_create_ex); nothing from the environment
  hipStream_t stream = nullptr;
  hipEvent_t ev_it0 = nullptr, ev_it1 = nullptr;  // set_target timing
  // per-iterate timing events, a ring over the last kTimingRing iterates:
  // [0] search start (the iterate's first launch), [1] search kernel done, [2] iterate end
  static constexpr int kTimingRing = 256;
  hipEvent_t ring[kTimingRing][3] = {};
  bool timed[kTimingRing] = {};  // the slot's search carries events (config.timing_stride)
  // the record exchange of a timed multi-rank iterate: events before / after each of the two
  // all-gathers (RCCL; created at first use), or the host clock around them (host exchange)
  hipEvent_t xring[kTimingRing][4] = {};
  int8_t xtimed[kTimingRing] = {};  // 0 not timed, 1 events (RCCL), 2 host clock
  double xhost_ms[kTimingRing] = {};
  int64_t n_iterates = 0;

  // target (replicated on every rank)
  icp::NodeRec* nodes = nullptr;
  icp::TBox* tbox = nullptr;  // tight boxes of the nodes (k_tight_boxes)
  icp::TgtPt* pts = nullptr;
  int64_t n_nodes = 0, n_leaves = 0, n_tgt = 0;
  int32_t pos0 = 0, max_depth = -1, levels = 1;
  double init_best = 1.7976931348623157e308;
  int32_t* cells = nullptr;     // per-level cell tables of the octree (octree_gpu.h)
  int cell_lmax = -1;
  double root_box[6] = {0, 0, 0, 0, 0, 0};
  int target_on_device = 0;      // octree built on the device (octree_gpu.hip) or on the host
  double target_build_ms = 0.0;  // set_target wall time on the stream (upload + build)

  // this rank's source shard, Morton order (perm[k] = caller index of slot k)
  int64_t n_src = 0;
  double *x = nullptr, *y = nullptr, *z = nullptr;
  int32_t* perm = nullptr;
  int32_t* pos = nullptr;  // leaf-order position of the match
  double* dist = nullptr;  // residual
  int32_t* fb_list = nullptr;            // exact, ball and per-lane query lists (3 x n_src)
  double* fb_u = nullptr;                // the ball list's distance guesses
  icp::WaveBox* wc_box = nullptr;        // the wave search's candidate cache (one per wave)
  float4* wc_ents = nullptr;
  uint32_t wc_gen = 1;                   // bumped by set_target / set_source (records of older
                                         // generations are never reused)
  unsigned int* fb_count = nullptr;
  unsigned int* tickets = nullptr;  // "last block done" counters of the moments and cull launches
                                    // (zero between launches: the last block resets its own)
  unsigned long long* dbg = nullptr;
  unsigned int last_lists[3] = {0, 0, 0};  // exact / ball / per-lane list sizes of the last search
  double last_wide = 0.0;  // waves whose candidate set overflowed in the last published iterate
  icp::Moments* mparts = nullptr;
  icp::CovMoments* cparts = nullptr;
  icp::WaveStat* wstat = nullptr;  // the search's per-wave covariance records (wave_stats.h)
  int last_cull_path = -1;         // IterDev::cull_mode of the last host-published iterate
  int64_t nb_mom = 0, nb_cull = 0;     // residual-moment parts, cull blocks
  bool lists_zero = true;               // fb_count is zero (reset by each iteration's publish)
  bool have_results = false;
  bool have_prev = false;  // dist[] holds residuals of the resident queries (search guess)

  // per-iteration record
  icp::IterDev* it = nullptr;
  icp::IterDev* h_it = nullptr;      // pinned, coherent: the publishing kernel stores into it
  icp::IterDev* h_it_dev = nullptr;  // its device address
  uint64_t publish_seq = 0;          // h_it->pad[3] = seq once the record is complete

  // the device-resident loop (icp_hip_loop_run): the session state on the device, its pinned
  // staging copy, and one LoopRec per iteration of a batch (pinned, written by the last kernel)
  static constexpr int kLoopRing = kTimingRing;
  icp::LoopDev* loopd = nullptr;
  icp::LoopDev* h_loop = nullptr;
  icp::LoopRec* h_ring = nullptr;
  icp::LoopRec* h_ring_dev = nullptr;
  hipEvent_t ev_batch = nullptr;  // a batch's start (its first iteration's step time)
  unsigned long long* counters = nullptr;

  // multi-GPU (comm or xfn set: every iterate runs the all-gather + rank-order merge path)
  int nranks = 1, rank = 0;
  ncclComm_t comm = nullptr;
  icp_hip_exchange_fn xfn = nullptr;  // host exchange instead of RCCL (icp_hip_comm_init_host)
  void* xuser = nullptr;
  ExchangeWorker* xworker = nullptr;  // runs xfn when config.peer_timeout_ms > 0
  icp::Moments* gm = nullptr;
  icp::CovMoments* gc = nullptr;
  // a member of a multi-device context: set when a peer member failed (the waits give up)
  const std::atomic<int>* abort = nullptr;
  bool comm_aborted = false;  // icp_hip_comm_abort: iterates fail until the next comm_init
  int inject_failure = 0;     // icp_hip_debug_inject_failure: 1 = fail before the first exchange

  // multi-device context (icp_hip_create_multi): the member contexts and their driver threads
  // (icp_group.cpp); the single-device fields above are then unused
  struct DeviceGroup* group = nullptr;
};

void icp_ctx_set_error(const char* msg);

// The device-resident loop: k iterations (k <= kLoopRing) enqueued back to back, each one's last
// kernel stepping the session on the device (session_step.h), one host wait per batch. core is
// the session state (uploaded, then updated), recs gets the k iterations' records (outcome
// kStepNone once the session finished), step_ms (optional) each iteration's device time.
// Eligible: a single-device context (RCCL communicator or none; not the host exchange) with
// config.device_loop set.
bool icp_hip_loop_eligible(const icp_hip_ctx* c);
int icp_hip_loop_run(icp_hip_ctx* c, icp::SessionCore* core, const icp::SessionParams* p, int rules, double sigma,
                     int k, icp::LoopRec* recs, double* step_ms);
// Attach a communicator created elsewhere (ncclCommInitAll of a multi-device context); the
// context owns it from then on.
int icp_ctx_attach_comm(icp_hip_ctx* c, ncclComm_t comm, int nranks, int rank);
// ncclCommAbort of the context's communicator (icp_hip_comm_abort without the argument checks)
void icp_ctx_abort_comm(icp_hip_ctx* c);
// Back to a world of one without a transport: the communicator destroyed, the exchange thread
// joined (after its callback returns), comm_aborted cleared.
void icp_ctx_drop_transport(icp_hip_ctx* c);

// The multi-device context (icp_group.cpp): every C-ABI entry point of icp_ctx.hip dispatches here
// when ctx->group is set.
void group_destroy(icp_hip_ctx* c);
int group_set_target(icp_hip_ctx* c, const double* xyz, int64_t n, int max_points, int max_depth, int rules);
int group_target_build_info(icp_hip_ctx* c, int32_t* on_device, double* build_ms);
int group_set_source(icp_hip_ctx* c, const double* xyz, int64_t n);
int group_iterate(icp_hip_ctx* c, const double* T_apply, int iter, int rules, double sigma, icp_iter_stats* out);
int group_apply(icp_hip_ctx* c, const double* T);
int group_get_source(icp_hip_ctx* c, double* xyz_out);
int group_get_correspondences(icp_hip_ctx* c, int32_t* idx_out, double* dist_out);
int group_traversal_counts(icp_hip_ctx* c, double* mean_entries, double* mean_points);
int group_cull_path(icp_hip_ctx* c, int32_t* fused);
int group_timings(icp_hip_ctx* c, int k, double* nn_ms, double* it_ms);
int group_debug_counters(icp_hip_ctx* c, uint64_t out[ICP_DBG_SLOTS]);
int group_exchange_timings(icp_hip_ctx* c, int k, double* ms);
int group_comm_info(icp_hip_ctx* c, int member, int32_t* count, int32_t* rank, int32_t* device, int32_t* transport);
int group_synchronize(icp_hip_ctx* c);
int group_inject_failure(icp_hip_ctx* c, int member, int where);
icp_hip_ctx* group_member(icp_hip_ctx* c, int k);
