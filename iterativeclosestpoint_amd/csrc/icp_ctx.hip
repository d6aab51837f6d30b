// icp_ctx.hip — the C-ABI context of libicp_hip.so (include/icp_hip.h).
//
// One context = one GPU = one HIP stream. Everything that belongs to the path lives in HBM for
// the whole registration: the linear octree (64-B node records), the leaf-ordered target
// (32-B points), the Morton-ordered source shard as SoA x/y/z, per-query match position and
// residual, block partials. Per iteration the host sees one 1 KB record (IterDev).
// Multi-GPU: each rank holds its shard of the source and a replica of the octree; the two
// per-iteration exchanges are RCCL all-gathers of one Moments / one CovMoments record, merged
// on the device in rank order, so every rank computes bitwise-identical statistics.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/icp_hip.h"
#include "../../include/icp_host.h"
#include "icp_ctx_internal.h"
#include "kernels.h"
#include "octree_build.h"
#include "octree_gpu.h"
#include "query_order.h"

using namespace icp;

// The candidate cache re-walks a wave whose stored box B+ has grown loose around its current B
// (volume ratio; at 10M with margin 16: 1.4, 1.6 and 2.3 measured slower than 1.9).

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return fail(e_ == hipErrorOutOfMemory ? ICP_HIP_ENOMEM : ICP_HIP_EDEVICE,                \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                          \
  } while (0)

#define RCCL_TRY(expr)                                                                         \
  do {                                                                                         \
    ncclResult_t r_ = (expr);                                                                  \
    if (r_ != ncclSuccess) return fail(ICP_HIP_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

template <typename T>
hipError_t dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
}

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

}  // namespace

void icp_ctx_set_error(const char* msg) { g_err = msg; }

static void free_source(icp_hip_ctx* c) {
  dfree(c->x);
  dfree(c->y);
  dfree(c->z);
  dfree(c->perm);
  dfree(c->pos);
  dfree(c->dist);
  dfree(c->fb_list);
  dfree(c->fb_u);
  dfree(c->wc_box);
  dfree(c->wc_ents);
  dfree(c->mparts);
  dfree(c->cparts);
  dfree(c->wstat);
  c->n_src = 0;
}

// No band for the next iterate's search (a new source or target): its cull pass does it all.
static hipError_t reset_band(icp_hip_ctx* c) {
  c->last_cull_path = -1;
  char* base = reinterpret_cast<char*>(c->it);
  return hipMemsetAsync(base + offsetof(IterDev, fz_lo), 0, offsetof(IterDev, cull_mode) - offsetof(IterDev, fz_lo),
                        c->stream);
}

static void free_target(icp_hip_ctx* c) {
  dfree(c->nodes);
  dfree(c->tbox);
  dfree(c->pts);
  dfree(c->cells);
  c->cell_lmax = -1;
  c->n_nodes = 0;
  c->n_tgt = 0;
}

// The search launch over the resident target with this context's configuration; the caller
// fills the query arrays and the lists.
static NNLaunch base_launch(const icp_hip_ctx* c) {
  NNLaunch a;
  std::memset(&a, 0, sizeof(a));
  a.nodes = c->nodes;
  a.tbox = c->tbox;
  a.pts = c->pts;
  a.counters = c->counters;
  a.n_nodes = (int32_t)c->n_nodes;
  a.pos0 = c->pos0;
  a.levels = c->levels;
  a.init_best = c->init_best;
  a.search = c->cfg.search;
  a.scan32 = c->cfg.scan32;
  a.cells = c->cells;
  a.cell_lmax = c->cell_lmax;
  a.join_factor = c->cfg.join_factor;
  a.ball_mode = c->cfg.ball_mode;
  a.xcd_blocks = c->cfg.xcd_blocks;
  a.scan_groups = c->cfg.scan_groups;
  a.certify_prev = c->cfg.certify_prev;
  a.dbg = c->dbg;
  for (int k = 0; k < 3; k++) {
    a.root_lo[k] = c->root_box[k];
    a.root_hi[k] = c->root_box[3 + k];
  }
  return a;
}

// Process warm-up (icp_hip_config.no_warmup = 0). HIP loads a kernel's code object and sizes the
// queue's scratch at the kernel's first launch in the process; without a warm-up that cost
// (+1.3 ms at 10M, measured: first iterate 4.15 ms cold, 2.85 ms warm) lands in the first iterate
// of the first registration. A 3-iterate registration of a small synthetic pair on a private
// context with the same search options (the same kernel instances: first-iterate descent, half
// pass, ball search, the storing and the reusing search, full and fused culls) loads them, once
// per (device, options) per process. Failures are ignored: the real context works without it.
static void warm_kernels(int device, const icp_hip_config& conf) {
  static std::mutex mu;
  static std::vector<std::pair<int, uint64_t>> done;
  const uint64_t key = (uint64_t)conf.search | (uint64_t)conf.scan_groups << 4 | (uint64_t)conf.certify_prev << 8 |
                       (uint64_t)(conf.debug_counters != 0) << 12 | (uint64_t)conf.fused_cull << 13 |
                       (uint64_t)conf.overflow_halves << 14 | (uint64_t)conf.scan32 << 15 |
                       (uint64_t)conf.candidate_cache << 16 | (uint64_t)conf.ball_mode << 17 |
                       (uint64_t)conf.wide_pass << 19;
  std::lock_guard<std::mutex> lk(mu);
  for (const auto& d : done)
    if (d.first == device && d.second == key) return;
  done.emplace_back(device, key);
  const std::string saved = g_err;
  constexpr int64_t kN = 4096;
  std::vector<double> tgt(3 * kN), src(3 * kN);
  double Ttrue[16];
  icp_synth_spec sp;
  icp_synth_default(&sp);
  icp_hip_config wc = conf;
  wc.no_warmup = 1;
  wc.timing_stride = 0;
  wc.peer_timeout_ms = 0;
  icp_hip_ctx* w = nullptr;
  if (icp_synth_pair(&sp, kN, kN, tgt.data(), src.data(), Ttrue) == 0 && icp_hip_create_ex(&w, device, &wc) == 0 &&
      icp_hip_set_target(w, tgt.data(), kN, 10, 20, ICP_RULES_ENGINE) == 0 && icp_hip_set_source(w, src.data(), kN) == 0) {
    const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    icp_iter_stats st;
    for (int k = 0; k < 3; ++k)
      if (icp_hip_iterate(w, k ? I : nullptr, k, ICP_RULES_ENGINE, 3.0, &st) != 0) break;
  }
  icp_hip_destroy(w);
  icp_ctx_set_error(saved.c_str());
}

extern "C" {

int icp_hip_device_count(int* count) {
  HIP_TRY(hipGetDeviceCount(count));
  return ICP_HIP_OK;
}

void icp_hip_config_default(icp_hip_config* cfg) {
  if (!cfg) return;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->search = ICP_SEARCH_CERTIFIED;
  cfg->scan32 = 1;
  cfg->cell_starts = 1;
  cfg->octree_builder = ICP_BUILD_AUTO;
  cfg->join_factor = 3.0;
  cfg->debug_counters = 0;
  cfg->xcd_blocks = 256;
  cfg->scan_groups = 4;
  cfg->candidate_cache = 1;
  cfg->candidate_margin = 16;
  cfg->candidate_loose = 1500;
  cfg->candidate_lead = 8;
  cfg->fused_cull = 1;
  cfg->overflow_halves = 0;
  cfg->device_loop = 0;
  cfg->timing_stride = 0;
  cfg->peer_timeout_ms = 0;
  cfg->config_version = ICP_HIP_CONFIG_VERSION;
}

int icp_hip_create(icp_hip_ctx** out, int device) { return icp_hip_create_ex(out, device, nullptr); }

int icp_hip_create_ex(icp_hip_ctx** out, int device, const icp_hip_config* cfg) {
  if (!out) return fail(ICP_HIP_EINVAL, "null out");
  *out = nullptr;
  icp_hip_config conf;
  icp_hip_config_default(&conf);
  // the version word comes first: checked before the struct is copied (a struct of another
  // header version may be shorter than this one)
  if (cfg && cfg->config_version != ICP_HIP_CONFIG_VERSION)
    return fail(ICP_HIP_EINVAL, "config: config_version is not ICP_HIP_CONFIG_VERSION (start from icp_hip_config_default "
                                "of this header)");
  if (cfg) conf = *cfg;
  for (int k = 0; k < 3; k++)
    if (conf.reserved[k] != 0) return fail(ICP_HIP_EINVAL, "config: reserved words must be zero");
  if (conf.wide_pass < 0 || conf.wide_pass > 2) return fail(ICP_HIP_EINVAL, "config: wide_pass out of [0, 2]");
  if (conf.peer_timeout_ms < 0) return fail(ICP_HIP_EINVAL, "config: peer_timeout_ms must be >= 0");
  if (conf.no_warmup != 0 && conf.no_warmup != 1) return fail(ICP_HIP_EINVAL, "config: no_warmup must be 0 or 1");
  if (conf.ball_mode < 0 || conf.ball_mode > 2) return fail(ICP_HIP_EINVAL, "config: ball_mode out of [0, 2]");
  if (conf.search != ICP_SEARCH_CERTIFIED && conf.search != ICP_SEARCH_REFERENCE)
    return fail(ICP_HIP_EINVAL, "config: unknown search");
  if (conf.octree_builder != ICP_BUILD_AUTO && conf.octree_builder != ICP_BUILD_HOST)
    return fail(ICP_HIP_EINVAL, "config: unknown octree builder");
  if (conf.scan_groups != 1 && conf.scan_groups != 2 && conf.scan_groups != 4)
    return fail(ICP_HIP_EINVAL, "config: scan_groups must be 1, 2 or 4");
  if (conf.xcd_blocks < 0 || conf.xcd_blocks > (1 << 20)) return fail(ICP_HIP_EINVAL, "config: xcd_blocks out of [0, 2^20]");
  if (conf.candidate_cache != 0 && conf.candidate_cache != 1) return fail(ICP_HIP_EINVAL, "config: candidate_cache must be 0 or 1");
  if (conf.candidate_margin < 0 || conf.candidate_margin > 1024)
    return fail(ICP_HIP_EINVAL, "config: candidate_margin out of [0, 1024]");
  if (conf.candidate_loose == 0) conf.candidate_loose = 1500;
  if (conf.candidate_loose < 100 || conf.candidate_loose > 100000)
    return fail(ICP_HIP_EINVAL, "config: candidate_loose out of [100, 100000]");
  if (conf.candidate_lead < 0 || conf.candidate_lead > 64) return fail(ICP_HIP_EINVAL, "config: candidate_lead out of [0, 64]");
  if (conf.fused_cull < 0 || conf.fused_cull > 1) return fail(ICP_HIP_EINVAL, "config: fused_cull must be 0 or 1");
  if (conf.overflow_halves != 0 && conf.overflow_halves != 1) return fail(ICP_HIP_EINVAL, "config: overflow_halves must be 0 or 1");
  if (conf.query_order != 0 && conf.query_order != 1) return fail(ICP_HIP_EINVAL, "config: query_order must be 0 or 1");
  if (conf.certify_prev < 0 || conf.certify_prev > 3) return fail(ICP_HIP_EINVAL, "config: certify_prev out of [0, 3]");
  if (conf.device_loop != 0 && conf.device_loop != 1) return fail(ICP_HIP_EINVAL, "config: device_loop must be 0 or 1");
  if (conf.timing_stride < 0) return fail(ICP_HIP_EINVAL, "config: timing_stride must be >= 0");
  if (!(conf.join_factor >= 1.0 && conf.join_factor <= 1e6))
    return fail(ICP_HIP_EINVAL, "config: join_factor out of [1, 1e6]");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0)
    return fail(ICP_HIP_EDEVICE, std::string("no HIP device available: ") + hipGetErrorString(e));
  if (device < 0) HIP_TRY(hipGetDevice(&device));
  if (device >= ndev) return fail(ICP_HIP_EINVAL, "device ordinal out of range");
  HIP_TRY(hipSetDevice(device));
  icp_hip_ctx* c = new icp_hip_ctx();
  c->device = device;
  c->cfg = conf;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(ICP_HIP_EDEVICE, "hipStreamCreate failed");
  }
  for (hipEvent_t* ev : {&c->ev_it0, &c->ev_it1}) (void)hipEventCreate(ev);
  (void)hipEventCreateWithFlags(&c->ev_batch, hipEventDisableSystemFence);
  // The per-iterate timing ring only measures elapsed times: no system-scope fence on record
  // (a default event's release writes back L2, ~5 us of GPU idle per record between kernels).
  for (auto& r : c->ring)
    for (hipEvent_t& ev : r) (void)hipEventCreateWithFlags(&ev, hipEventDisableSystemFence);
  if (dalloc(&c->it, 1) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_it), sizeof(IterDev), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_it_dev), c->h_it, 0) != hipSuccess ||
      dalloc(&c->counters, 2) != hipSuccess || dalloc(&c->fb_count, 8) != hipSuccess || dalloc(&c->loopd, 1) != hipSuccess ||
      dalloc(&c->tickets, (size_t)ticket_words()) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_loop), sizeof(LoopDev)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->h_ring), icp_hip_ctx::kLoopRing * sizeof(LoopRec),
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->h_ring_dev), c->h_ring, 0) != hipSuccess ||
      (conf.debug_counters && dalloc(&c->dbg, ICP_DBG_SLOTS) != hipSuccess)) {
    icp_hip_destroy(c);
    return fail(ICP_HIP_ENOMEM, "context allocation failed");
  }
  (void)hipMemset(c->it, 0, sizeof(IterDev));
  (void)hipMemset(c->fb_count, 0, 8 * sizeof(unsigned int));
  (void)hipMemset(c->tickets, 0, (size_t)ticket_words() * sizeof(unsigned int));
  if (c->dbg) (void)hipMemset(c->dbg, 0, ICP_DBG_SLOTS * sizeof(unsigned long long));
  std::memset(c->h_it, 0, sizeof(IterDev));
  c->lists_zero = true;
  if (!conf.no_warmup) warm_kernels(device, conf);
  *out = c;
  return ICP_HIP_OK;
}

void icp_hip_destroy(icp_hip_ctx* c) {
  if (!c) return;
  if (c->group) {
    group_destroy(c);
    delete c;
    return;
  }
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  free_source(c);
  free_target(c);
  dfree(c->it);
  dfree(c->counters);
  dfree(c->fb_count);
  dfree(c->tickets);
  dfree(c->dbg);
  dfree(c->gm);
  dfree(c->gc);
  if (c->h_it) (void)hipHostFree(c->h_it);
  dfree(c->loopd);
  if (c->h_loop) (void)hipHostFree(c->h_loop);
  if (c->h_ring) (void)hipHostFree(c->h_ring);
  if (c->ev_batch) (void)hipEventDestroy(c->ev_batch);
  icp_ctx_drop_transport(c);
  for (hipEvent_t ev : {c->ev_it0, c->ev_it1})
    if (ev) (void)hipEventDestroy(ev);
  for (auto& r : c->ring)
    for (hipEvent_t ev : r)
      if (ev) (void)hipEventDestroy(ev);
  for (auto& r : c->xring)
    for (hipEvent_t ev : r)
      if (ev) (void)hipEventDestroy(ev);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int icp_hip_get_unique_id(uint8_t out[ICP_HIP_UNIQUE_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == ICP_HIP_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  RCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
  return ICP_HIP_OK;
}

int icp_hip_comm_init(icp_hip_ctx* c, int nranks, int rank, const uint8_t id_bytes[ICP_HIP_UNIQUE_ID_BYTES]) {
  if (c && c->group) return fail(ICP_HIP_EINVAL, "a multi-device context owns its communicators");
  if (!c || !id_bytes || nranks < 1 || rank < 0 || rank >= nranks) return fail(ICP_HIP_EINVAL, "bad comm arguments");
  HIP_TRY(hipSetDevice(c->device));
  // back to a world of one first: a failure below leaves no stale transport behind
  icp_ctx_drop_transport(c);
  dfree(c->gm);
  dfree(c->gc);
  HIP_TRY(dalloc(&c->gm, (size_t)nranks));
  HIP_TRY(dalloc(&c->gc, (size_t)nranks));
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t comm = nullptr;
  RCCL_TRY(ncclCommInitRank(&comm, nranks, id, rank));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  return ICP_HIP_OK;
}

}  // extern "C"

void icp_ctx_drop_transport(icp_hip_ctx* c) {
  if (c->comm) (void)ncclCommDestroy(c->comm);
  c->comm = nullptr;
  delete c->xworker;  // waits for a callback that overran the deadline to return
  c->xworker = nullptr;
  c->comm_aborted = false;
  c->xfn = nullptr;
  c->xuser = nullptr;
  c->nranks = 1;
  c->rank = 0;
}

void icp_ctx_abort_comm(icp_hip_ctx* c) {
  if (!c->comm) return;
  (void)hipSetDevice(c->device);
  // the collectives this communicator has enqueued return (their outputs are garbage, never read:
  // the iterate that enqueued them has failed), so the stream drains
  (void)ncclCommAbort(c->comm);
  c->comm = nullptr;
  c->comm_aborted = true;
  (void)hipStreamSynchronize(c->stream);
  (void)hipGetLastError();
}

int icp_ctx_attach_comm(icp_hip_ctx* c, ncclComm_t comm, int nranks, int rank) {
  HIP_TRY(hipSetDevice(c->device));
  icp_ctx_drop_transport(c);
  dfree(c->gm);
  dfree(c->gc);
  HIP_TRY(dalloc(&c->gm, (size_t)nranks));
  HIP_TRY(dalloc(&c->gc, (size_t)nranks));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  return ICP_HIP_OK;
}

extern "C" {

int icp_hip_comm_init_host(icp_hip_ctx* c, int nranks, int rank, icp_hip_exchange_fn exchange, void* user) {
  if (c && c->group) return fail(ICP_HIP_EINVAL, "a multi-device context owns its communicators");
  if (!c || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !exchange))
    return fail(ICP_HIP_EINVAL, "bad comm arguments");
  HIP_TRY(hipSetDevice(c->device));
  icp_ctx_drop_transport(c);
  if (!exchange) return ICP_HIP_OK;  // a world of one without a transport
  dfree(c->gm);
  dfree(c->gc);
  HIP_TRY(dalloc(&c->gm, (size_t)nranks));
  HIP_TRY(dalloc(&c->gc, (size_t)nranks));
  c->xfn = exchange;
  c->xuser = user;
  c->nranks = nranks;
  c->rank = rank;
  return ICP_HIP_OK;
}

// The per-iteration all-gather of one record (count doubles) in rank order: RCCL on the compute
// stream, or the caller's host exchange (stream synchronised around the callback).
static int all_gather_record(icp_hip_ctx* c, const double* d_local, double* d_gathered, int count, hipStream_t s) {
  if (c->comm) {
    RCCL_TRY(ncclAllGather(d_local, d_gathered, (size_t)count, ncclDouble, c->comm, s));
    return ICP_HIP_OK;
  }
  std::vector<double> local((size_t)count), all((size_t)count * c->nranks);
  HIP_TRY(hipMemcpyAsync(local.data(), d_local, sizeof(double) * count, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->cfg.peer_timeout_ms > 0) {
    // the callback on the exchange thread, given up on at the deadline (it cannot be interrupted:
    // it finishes on that thread, and comm_init / comm_init_host / destroy wait for it)
    if (!c->xworker) c->xworker = new ExchangeWorker();
    if (c->xworker->run(c->xfn, c->xuser, local.data(), count, c->nranks, c->cfg.peer_timeout_ms) != 0) {
      c->comm_aborted = true;
      return fail(ICP_HIP_EEXCHANGE, "host exchange callback overran config.peer_timeout_ms (" +
                                         std::to_string(c->cfg.peer_timeout_ms) + " ms); comm_init_host again");
    }
    if (c->xworker->rc != 0) return fail(ICP_HIP_EEXCHANGE, "host exchange callback failed");
    all.swap(c->xworker->all);
  } else if (c->xfn(c->xuser, local.data(), count, all.data()) != 0) {
    return fail(ICP_HIP_EEXCHANGE, "host exchange callback failed");
  }
  HIP_TRY(hipMemcpyAsync(d_gathered, all.data(), sizeof(double) * all.size(), hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return ICP_HIP_OK;
}

int icp_hip_set_target(icp_hip_ctx* c, const double* xyz, int64_t n, int max_points, int max_depth, int rules) {
  if (!c || (!xyz && n > 0)) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return n <= 0 ? fail(ICP_HIP_EINVAL, "empty target cloud (icpengine.cpp:31-34 rejects it)")
                             : group_set_target(c, xyz, n, max_points, max_depth, rules);
  if (n <= 0) return fail(ICP_HIP_EINVAL, "empty target cloud (icpengine.cpp:31-34 rejects it)");
  if (max_depth < 0 || max_depth > 60) return fail(ICP_HIP_EINVAL, "max_depth out of range [0, 60]");
  if (n > (int64_t)0x7fffffff) return fail(ICP_HIP_EINVAL, "target size out of range (int32 indices, as the reference)");
  HIP_TRY(hipSetDevice(c->device));
  free_target(c);
  HIP_TRY(reset_band(c));
  hipEvent_t e0 = c->ev_it0, e1 = c->ev_it1;
  HIP_TRY(hipEventRecord(e0, c->stream));
  const bool on_device = max_depth <= kGpuBuildMaxDepth && c->cfg.octree_builder == ICP_BUILD_AUTO;
  if (on_device) {
    // device build straight from the uploaded AoS cloud (octree_gpu.hip)
    double* d_xyz = nullptr;
    HIP_TRY(dalloc(&d_xyz, 3 * (size_t)n));
    hipError_t e = hipMemcpyAsync(d_xyz, xyz, 3 * sizeof(double) * n, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) {
      dfree(d_xyz);
      return fail(ICP_HIP_EDEVICE, std::string("set_target upload: ") + hipGetErrorString(e));
    }
    GpuOctree t;
    std::string why;
    const int rc = gpu_build_octree(d_xyz, n, max_points, max_depth, c->stream, &t, &why);
    dfree(d_xyz);
    if (rc != 0)
      return fail(rc == 1 ? ICP_HIP_EINVAL : rc == -2 ? ICP_HIP_ENOMEM : ICP_HIP_EDEVICE, why);
    c->nodes = t.nodes;
    c->pts = t.pts;
    c->n_nodes = t.n_nodes;
    c->n_leaves = t.n_leaves;
    c->pos0 = t.pos_of_orig0;
    c->max_depth = t.max_depth;
    c->levels = t.max_inner_depth + 1 > 0 ? t.max_inner_depth + 1 : 1;
  } else {
    FlatOctree t;
    const char* why = nullptr;
    if (!build_flat_octree(xyz, n, max_points, max_depth, &t, &why)) return fail(ICP_HIP_EINVAL, why ? why : "bad target");
    HIP_TRY(dalloc(&c->nodes, t.nodes.size()));
    HIP_TRY(dalloc(&c->pts, t.pts.size()));
    HIP_TRY(hipMemcpyAsync(c->nodes, t.nodes.data(), t.nodes.size() * sizeof(NodeRec), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->pts, t.pts.data(), t.pts.size() * sizeof(TgtPt), hipMemcpyHostToDevice, c->stream));
    c->n_nodes = (int64_t)t.nodes.size();
    c->n_leaves = t.n_leaves;
    c->pos0 = t.pos_of_orig0;
    c->max_depth = t.max_depth;
    c->levels = t.max_inner_depth + 1 > 0 ? t.max_inner_depth + 1 : 1;
  }
  // separation of every target point (the previous-match certificate, certify_prev)
  if (c->cfg.certify_prev) HIP_TRY(launch_target_sep(c->nodes, c->pts, n, c->levels, c->stream));
  // after the separations (which a copy's flag overwrites: its separation is 0 either way)
  HIP_TRY(launch_mark_copies(c->pts, n, c->stream));
  HIP_TRY(dalloc(&c->tbox, (size_t)c->n_nodes));
  HIP_TRY(launch_tight_boxes(c->nodes, c->pts, c->tbox, c->n_nodes, c->max_depth, c->stream));
  // root box (host copy: the kernels' cell arithmetic starts from it) and the cell tables
  {
    NodeRec root;
    HIP_TRY(hipMemcpyAsync(&root, c->nodes, sizeof(NodeRec), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int k = 0; k < 3; k++) {
      c->root_box[k] = root.lo[k];
      c->root_box[3 + k] = root.hi[k];
    }
  }
  if (c->cfg.cell_starts && c->n_nodes < ((int64_t)1 << 26)) {
    const int lmax = cell_table_depth(c->n_leaves, c->levels - 1);
    // the tables only speed up the searches' start: without memory for them the searches start
    // from the root (identical results)
    if (dalloc(&c->cells, (size_t)cell_table_entries(lmax)) == hipSuccess) {
      HIP_TRY(build_cell_tables(c->nodes, lmax, c->cells, c->stream));
      c->cell_lmax = lmax;
    } else {
      (void)hipGetLastError();
      c->cells = nullptr;
    }
  }
  HIP_TRY(hipEventRecord(e1, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  c->target_build_ms = ms;
  c->target_on_device = on_device ? 1 : 0;
  c->n_tgt = n;
  c->init_best = (rules == ICP_RULES_CLI) ? 1e20 : DBL_MAX;  // icp_registration.cpp:201 / octree.cpp:180
  c->have_prev = false;
  c->wc_gen++;  // cached candidate lists name points of the previous tree
  c->have_results = false;
  return ICP_HIP_OK;
}

int icp_hip_target_build_info(icp_hip_ctx* c, int32_t* on_device, double* build_ms) {
  if (!c) return fail(ICP_HIP_EINVAL, "null context");
  if (c->group) return group_target_build_info(c, on_device, build_ms);
  if (!c->nodes) return fail(ICP_HIP_ENOTREADY, "target not set");
  if (on_device) *on_device = c->target_on_device;
  if (build_ms) *build_ms = c->target_build_ms;
  return ICP_HIP_OK;
}

int icp_hip_copy_target(icp_hip_ctx* c, double* box6, int32_t* first, uint32_t* meta, int32_t* depth, double* xyz,
                        int32_t* orig) {
  if (!c) return fail(ICP_HIP_EINVAL, "null context");
  if (c->group) return icp_hip_copy_target(group_member(c, 0), box6, first, meta, depth, xyz, orig);
  if (!c->nodes) return fail(ICP_HIP_ENOTREADY, "target not set");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<NodeRec> nodes((size_t)c->n_nodes);
  std::vector<TgtPt> pts((size_t)c->n_tgt);
  HIP_TRY(hipMemcpyAsync(nodes.data(), c->nodes, nodes.size() * sizeof(NodeRec), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(pts.data(), c->pts, pts.size() * sizeof(TgtPt), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < nodes.size(); i++) {
    const NodeRec& r = nodes[i];
    if (box6)
      for (int k = 0; k < 3; k++) {
        box6[6 * i + k] = r.lo[k];
        box6[6 * i + 3 + k] = r.hi[k];
      }
    if (first) first[i] = r.first;
    if (meta) meta[i] = r.meta;
    if (depth) depth[i] = r.depth;
  }
  for (size_t i = 0; i < pts.size(); i++) {
    if (xyz) {
      xyz[3 * i] = pts[i].x;
      xyz[3 * i + 1] = pts[i].y;
      xyz[3 * i + 2] = pts[i].z;
    }
    if (orig) orig[i] = pts[i].orig;
  }
  return ICP_HIP_OK;
}

int icp_hip_target_separation(icp_hip_ctx* c, float* sep_out) {
  if (!c || !sep_out) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return icp_hip_target_separation(group_member(c, 0), sep_out);
  if (!c->nodes) return fail(ICP_HIP_ENOTREADY, "target not set");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<TgtPt> pts((size_t)c->n_tgt);
  HIP_TRY(hipMemcpyAsync(pts.data(), c->pts, pts.size() * sizeof(TgtPt), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (const TgtPt& p : pts) sep_out[p.orig] = p.sep;
  return ICP_HIP_OK;
}

int icp_hip_set_source(icp_hip_ctx* c, const double* xyz, int64_t n) {
  if (!c || (!xyz && n > 0) || n < 0) return fail(ICP_HIP_EINVAL, "bad source arguments");
  if (c->group) return group_set_source(c, xyz, n);
  // the wave search addresses per-query arrays by 32-bit byte offsets (nn_device.h qat): < 2^29
  // points per shard (12 GB of coordinates; a larger cloud is sharded over a device group)
  if (n >= ((int64_t)1 << 29)) return fail(ICP_HIP_EINVAL, "source shard of 2^29 points or more");
  HIP_TRY(hipSetDevice(c->device));
  free_source(c);
  c->n_src = n;
  c->nb_mom = moments_num_parts(n);
  c->nb_cull = cull_num_blocks(n);
  HIP_TRY(dalloc(&c->x, n));
  HIP_TRY(dalloc(&c->y, n));
  HIP_TRY(dalloc(&c->z, n));
  HIP_TRY(dalloc(&c->perm, n));
  HIP_TRY(dalloc(&c->pos, n));
  HIP_TRY(dalloc(&c->dist, n));
  HIP_TRY(dalloc(&c->fb_list, 3 * (size_t)n + 64));  // exact, ball, (half, mask) pairs
  HIP_TRY(dalloc(&c->fb_u, (size_t)n));
  if (c->cfg.candidate_cache && n > 0) {
    // the cache only saves walks: without memory for it every iterate walks (identical results)
    const size_t nw = (size_t)((n + 63) / 64);
    if (dalloc(&c->wc_box, nw) == hipSuccess && dalloc(&c->wc_ents, nw * icp::kWaveCandCap) == hipSuccess) {
      HIP_TRY(hipMemsetAsync(c->wc_box, 0, nw * sizeof(icp::WaveBox), c->stream));  // generation 0: invalid
    } else {
      (void)hipGetLastError();
      dfree(c->wc_box);
      dfree(c->wc_ents);
    }
  }
  c->wc_gen++;
  HIP_TRY(dalloc(&c->mparts, (size_t)(c->nb_mom + merge_scratch_entries(c->nb_mom))));
  HIP_TRY(dalloc(&c->cparts, (size_t)(c->nb_cull + merge_scratch_entries(c->nb_cull))));
  if (n > 0 && c->cfg.fused_cull && dalloc(&c->wstat, (size_t)((n + 63) / 64)) != hipSuccess) {
    (void)hipGetLastError();  // without the records every cull is a full pass (identical results)
    dfree(c->wstat);
  }
  HIP_TRY(reset_band(c));
  if (n == 0) return ICP_HIP_OK;
  // Spatially compact query order (kd buckets of 64 = one wave): on the device from the uploaded
  // cloud (query_order_gpu.hip), or on the host (config query_order = 1)
  double* aos = nullptr;
  hipError_t e = dalloc(&aos, 3 * (size_t)n);
  if (e == hipSuccess) e = hipMemcpyAsync(aos, xyz, 3 * sizeof(double) * n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    if (c->cfg.query_order == 0) {
      e = gpu_kd_query_order(aos, n, 8, c->perm, c->stream);
    } else {
      std::vector<int32_t> perm;
      kd_query_order(xyz, n, 8, &perm);
      e = hipMemcpyAsync(c->perm, perm.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // the host order is read by the copy
    }
  }
  if (e == hipSuccess) e = launch_gather_deinterleave(aos, c->perm, c->x, c->y, c->z, n, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(aos);
  if (e != hipSuccess) return fail(ICP_HIP_EDEVICE, std::string("set_source: ") + hipGetErrorString(e));
  c->have_results = false;
  c->have_prev = false;
  return ICP_HIP_OK;
}

}  // extern "C"

// The host's wait for the device (the only wait of an iterate or of a device-loop batch): `done`
// polled in a tight loop; every 1024 polls the group's abort flag, the stream's own errors and,
// over an RCCL communicator, the communicator's asynchronous error and config.peer_timeout_ms. A
// peer process that died or a broken link leaves this rank's ncclAllGather waiting forever on the
// device: RCCL reports it as the communicator's async error, and the deadline covers what it does
// not see. Either way the communicator is aborted (the pending collective returns, the stream
// drains) and iterates fail with ERCCL until comm_init. The deadline is per iterate: `progress`
// (a count of the iterates the device has finished, e.g. a device-loop batch's published ring
// records) restarts it, so a long batch of healthy iterates is not a stalled peer. (The host
// exchange needs no deadline here: its callback ran, under its own deadline, before this wait,
// which then covers device work only.)
template <class Done, class Progress>
static int wait_device(icp_hip_ctx* c, Done done, Progress progress, const char* what) {
  hipStream_t s = c->stream;
  const bool peers = c->comm != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  uint64_t seen = progress();
  for (unsigned spin = 1; !done(); spin++) {
    if ((spin & 1023u) != 0) continue;
    const uint64_t now_p = progress();
    if (now_p != seen) {  // the device finished an iterate: the deadline starts again
      seen = now_p;
      t0 = std::chrono::steady_clock::now();
    }
    if (c->abort && c->abort->load()) return fail(ICP_HIP_EEXCHANGE, std::string(what) + ": a peer device of the group failed");
    if (c->comm) {
      ncclResult_t ae = ncclSuccess;
      if (ncclCommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
        icp_ctx_abort_comm(c);
        return fail(ICP_HIP_ERCCL, std::string(what) + ": the communicator failed (" + ncclGetErrorString(ae) +
                                       "; a peer rank died or a link broke): communicator aborted, comm_init again");
      }
    }
    if (peers && c->cfg.peer_timeout_ms > 0 &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(c->cfg.peer_timeout_ms)) {
      if (c->comm) icp_ctx_abort_comm(c);
      c->comm_aborted = true;
      return fail(ICP_HIP_ERCCL, std::string(what) + ": no record within config.peer_timeout_ms (" +
                                     std::to_string(c->cfg.peer_timeout_ms) +
                                     " ms; a peer rank stalled or died): communicator aborted, comm_init again");
    }
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess && done()) break;
    if (q == hipSuccess) return fail(ICP_HIP_EDEVICE, std::string(what) + ": stream idle but the record was not published");
    if (q != hipErrorNotReady) return fail(ICP_HIP_EDEVICE, std::string(what) + ": " + hipGetErrorString(q));
  }
  return ICP_HIP_OK;
}

// The wide pass's list: after the exact and ball lists (2 n ints) and the half list (<= 2 halves
// of every wave, two ints each: <= n / 16 + 4 ints); <= 3 entries per wave (the wave and its two
// halves), three ints each: inside the 3 n + 64 ints of fb_list.
static int32_t* wide_list(int32_t* fbl, int64_t n) { return fbl + 2 * n + n / 16 + 8; }

// config.wide_pass: 0 a source's first iterate (descent guesses: loose boxes) and any iterate after
// one with >= max(kWideAuto, waves / kWideAutoDiv) overflowing waves (surface data far from
// convergence); below that the ball search takes their queries sooner than a second launch (the
// blob's ~300 overflowing waves at 10M: a 100 us wide launch; profiles/r22/ab/ab_wide_auto.txt:
// 10M scene window +4.6 %, blob window +2.5 % against the fixed 256); 2 always
static constexpr double kWideAuto = 256.0;
#ifndef ICP_WIDE_AUTO_DIV
#define ICP_WIDE_AUTO_DIV 32
#endif
static constexpr double kWideAutoDiv = ICP_WIDE_AUTO_DIV;
static bool wide_pass_on(const icp_hip_ctx* c) {
  if (!c->cfg.scan32 || c->cfg.search != ICP_SEARCH_CERTIFIED || c->cfg.wide_pass == 1) return false;
  const double rel = (double)((c->n_src + 63) / 64) / kWideAutoDiv;
  const double thr = rel > kWideAuto ? rel : kWideAuto;
  return c->cfg.wide_pass == 2 || !c->have_prev || c->last_wide >= thr;
}

// One iterate enqueued on the context's stream, no wait. Host-driven (loop_slot < 0): the
// transform T_apply (null: none) is a kernel argument and the last kernel publishes the record
// with sequence number *seq for the host's poll. Device loop (loop_slot >= 0): the transform is
// the device session's pending increment (applied when `apply`), the last kernel steps the session
// and stores the iteration's LoopRec into ring slot loop_slot.
static int enqueue_iterate(icp_hip_ctx* c, const double* T_apply, bool apply, int iter, int rules,
                           double sigma_multiplier, int loop_slot, uint64_t* seq_out) {
  if (c->comm_aborted)
    return fail(ICP_HIP_ERCCL, "iterate: the communicator was aborted (icp_hip_comm_abort or a peer failure); comm_init again");
  hipStream_t s = c->stream;
  hipEvent_t* ev = c->ring[c->n_iterates % icp_hip_ctx::kTimingRing];
  LoopDev* loop = loop_slot >= 0 ? c->loopd : nullptr;
  NNLaunch a = base_launch(c);
  a.loop = loop;
  a.x = c->x;
  a.y = c->y;
  a.z = c->z;
  a.pos_out = c->pos;
  a.dist_out = c->dist;
  a.n = c->n_src;
  a.apply = apply ? 1 : 0;
  if (T_apply)
    for (int k = 0; k < 12; k++) a.T[k] = T_apply[k];
  a.fb_list = c->fb_list;
  a.fb_list2 = c->fb_list + c->n_src;
  // the half pass pays off where many waves overflow: the first iterate of a source (descent
  // guesses, loose boxes; ~16 % of the waves at 10M). Later iterates overflow in ~0.2 % of the
  // waves, whose queries the ball search finishes sooner than a second serial launch.
  a.fb_list3 = (c->cfg.overflow_halves && !c->have_prev) ? c->fb_list + 2 * c->n_src : nullptr;  // <= n + 64 ints
  a.fb_list4 = wide_pass_on(c) ? wide_list(c->fb_list, c->n_src) : nullptr;
  a.fb_u2 = c->fb_u;
  a.fb_count = c->fb_count;
  a.have_prev = c->have_prev ? 1 : 0;
  a.wc_box = c->wc_box;
  a.wc_ents = c->wc_ents;
  a.wc_gen = c->wc_gen;
  a.wc_margin = c->cfg.candidate_margin / 256.0;
  a.wc_loose = c->cfg.candidate_loose / 100.0;
  a.wc_lead = (double)c->cfg.candidate_lead;
  // the wave records of the fused covariance sums (the wave search only)
  a.wstat = (c->cfg.search == ICP_SEARCH_CERTIFIED && c->cfg.fused_cull) ? c->wstat : nullptr;
  a.fz = c->it;
  if (!c->lists_zero) HIP_TRY(hipMemsetAsync(c->fb_count, 0, 8 * sizeof(unsigned int), s));
  c->lists_zero = false;
  if (c->dbg) HIP_TRY(hipMemsetAsync(c->dbg, 0, ICP_DBG_SLOTS * sizeof(unsigned long long), s));
  // the search's timing events (on dispatch packets) on every timing_stride-th iterate only
  const int64_t slot = c->n_iterates % icp_hip_ctx::kTimingRing;
  const bool timed = c->cfg.timing_stride > 0 && c->n_iterates % c->cfg.timing_stride == 0;
  c->timed[slot] = timed;
  a.ev_start = timed ? ev[0] : nullptr;
  a.ev_fast_done = timed ? ev[1] : nullptr;
  HIP_TRY(launch_nn(a, s));
  // residual moments -> mean, std, threshold (no communicator: fused into the last merge level)
  const bool multi = c->comm != nullptr || c->xfn != nullptr;
  if (multi && c->inject_failure == 1) {  // testing hook: fail before joining the exchange
    c->inject_failure = 0;
    return fail(ICP_HIP_EDEVICE, "injected failure before the record exchange (icp_hip_debug_inject_failure)");
  }
  const MomentsFinalize fin{sigma_multiplier, iter, rules == ICP_RULES_ENGINE ? 1 : 0};
  CullLaunch cl;
  cl.loop = loop;
  cl.x = c->x;
  cl.y = c->y;
  cl.z = c->z;
  cl.pos = c->pos;
  cl.pts = c->pts;
  cl.it = c->it;
  cl.part = c->cparts;
  cl.n = c->n_src;
  cl.dist = c->dist;
  cl.wstat = a.wstat;
  HIP_TRY(launch_moments_tail(c->dist, c->n_src, c->mparts, loop, c->tickets, c->it, multi ? nullptr : &fin, cl, s));
  // a timed multi-rank iterate also times its two record exchanges (icp_hip_exchange_timings):
  // events around the all-gathers over RCCL, the host clock around the host exchange's callback
  c->xtimed[slot] = (int8_t)(timed && multi ? (c->comm ? 1 : 2) : 0);
  c->xhost_ms[slot] = 0.0;
  hipEvent_t* xev = c->xring[slot];
  if (c->xtimed[slot] == 1)
    for (int k = 0; k < 4; k++)
      if (!xev[k]) HIP_TRY(hipEventCreateWithFlags(&xev[k], hipEventDisableSystemFence));
  auto gather_timed = [&](int which, const double* d_local, double* d_gathered, int count) {
    if (c->xtimed[slot] == 1) HIP_TRY(hipEventRecord(xev[2 * which], s));
    const auto h0 = std::chrono::steady_clock::now();
    const int rc = all_gather_record(c, d_local, d_gathered, count, s);
    if (c->xtimed[slot] == 2)
      c->xhost_ms[slot] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
    if (rc == ICP_HIP_OK && c->xtimed[slot] == 1) HIP_TRY(hipEventRecord(xev[2 * which + 1], s));
    return rc;
  };
  if (multi) {
    const int rc = gather_timed(0, reinterpret_cast<const double*>(&c->it->m_local), reinterpret_cast<double*>(c->gm),
                                (int)(sizeof(Moments) / sizeof(double)));
    if (rc != ICP_HIP_OK) return rc;
    HIP_TRY(launch_finalize_moments(c->gm, c->nranks, c->it, fin, cl, s));
  }

  // covariance moments -> RMSE; the finished record is stored into pinned host memory (host
  // loop) or steps the device session (device loop)
  uint64_t seq = 0;
  IterPublish pub{nullptr, c->fb_count, 0.0, nullptr, nullptr};
  if (loop) {
    pub.loop = loop;
    pub.rec = c->h_ring_dev + loop_slot;
  } else {
    seq = ++c->publish_seq;
    pub.host = c->h_it_dev;
    pub.seq = (double)seq;
  }
  HIP_TRY(launch_cull_tail(cl, c->tickets + ticket_words() / 2, multi ? nullptr : &pub, s));
  if (multi) {
    const int rc = gather_timed(1, reinterpret_cast<const double*>(&c->it->c_local), reinterpret_cast<double*>(c->gc),
                                (int)(sizeof(CovMoments) / sizeof(double)));
    if (rc != ICP_HIP_OK) return rc;
    HIP_TRY(launch_finalize_cov(c->gc, c->nranks, c->it, pub, s));
  }
  HIP_TRY(hipEventRecord(ev[2], s));
  c->n_iterates++;
  c->have_prev = true;  // the next iterate's search guesses from this one's matches
  if (seq_out) *seq_out = seq;
  return ICP_HIP_OK;
}

extern "C" {

int icp_hip_iterate(icp_hip_ctx* c, const double* T_apply, int iter, int rules, double sigma_multiplier,
                    icp_iter_stats* out) {
  if (!c || !out) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return group_iterate(c, T_apply, iter, rules, sigma_multiplier, out);
  if (!c->nodes) return fail(ICP_HIP_ENOTREADY, "target not set");
  if (!c->x && c->n_src > 0) return fail(ICP_HIP_ENOTREADY, "source not set");
  HIP_TRY(hipSetDevice(c->device));
  uint64_t seq = 0;
  const int rc = enqueue_iterate(c, T_apply, T_apply != nullptr, iter, rules, sigma_multiplier, -1, &seq);
  if (rc != ICP_HIP_OK) return rc;
  // The host's only wait of the iteration: the publishing kernel stores the record with
  // system-scope stores, waits for their acknowledgement, then stores the sequence word (no
  // fence; reduce_kernels.hip finalize_cov_publish). Polling the pinned word wakes the host within
  // ~1 us; the stream is queried between polls so a device error still surfaces. The word is read
  // with acquire ordering, so the record's words are read after it.
  {
    const double want = (double)seq;
    uint64_t want_bits;
    std::memcpy(&want_bits, &want, sizeof(want));
    const uint64_t* word = reinterpret_cast<const uint64_t*>(&c->h_it->pad[3]);
    const int wrc = wait_device(
        c, [&]() { return __atomic_load_n(word, __ATOMIC_ACQUIRE) == want_bits; }, []() { return (uint64_t)0; },
        "iterate");
    if (wrc != ICP_HIP_OK) return wrc;
  }
  c->lists_zero = true;
  for (int k = 0; k < 3; k++) c->last_lists[k] = (unsigned int)c->h_it->pad[k];
  const IterDev& h = *c->h_it;
  c->last_wide = h.n_wide;
  c->last_cull_path = h.cull_mode != 0.0 ? 1 : 0;
  out->n = (int64_t)h.m_global.n;
  out->mean = h.mean;
  out->std = h.sd;
  out->threshold = h.thr;
  out->valid = (int64_t)h.c_global.n;
  out->rmse = h.rmse;
  out->sum_d2 = h.c_global.sum_d2;
  out->min_d = h.m_global.dmin;
  out->max_d = h.m_global.dmax;
  out->n_bad = (int64_t)h.m_global.nbad;
  for (int k = 0; k < 3; k++) {
    out->centroid_src[k] = h.c_global.ma[k];
    out->centroid_tgt[k] = h.c_global.mb[k];
  }
  for (int k = 0; k < 9; k++) out->H[k] = h.c_global.c[k];
  const bool cert = c->cfg.search == ICP_SEARCH_CERTIFIED;
  out->n_fallback = cert ? (int64_t)c->last_lists[0] : 0;
  out->n_lane_search = cert ? (int64_t)c->last_lists[2] : 0;
  out->n_ball_search = cert ? (int64_t)c->last_lists[1] : 0;
  c->have_results = true;
  return ICP_HIP_OK;
}

}  // extern "C"

bool icp_hip_loop_eligible(const icp_hip_ctx* c) {
  return c && !c->group && !c->xfn && c->cfg.device_loop && c->nodes && c->n_src > 0 && c->loopd;
}

int icp_hip_loop_run(icp_hip_ctx* c, icp::SessionCore* core, const icp::SessionParams* p, int rules, double sigma,
                     int k, icp::LoopRec* recs, double* step_ms) {
  if (!icp_hip_loop_eligible(c) || !core || !p || !recs || k < 0 || k > icp_hip_ctx::kLoopRing)
    return fail(ICP_HIP_EINVAL, "device loop: bad arguments");
  if (k == 0 || core->done) {
    for (int j = 0; j < k; j++) recs[j].outcome = icp::kStepNone;
    return ICP_HIP_OK;
  }
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  c->h_loop->core = *core;
  c->h_loop->p = *p;
  HIP_TRY(hipMemcpyAsync(c->loopd, c->h_loop, sizeof(LoopDev), hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(c->ev_batch, s));
  // the ring slots' outcome words, cleared to a sentinel: the batch's last kernels overwrite them
  // one iterate at a time (the host wait's progress)
  constexpr int32_t kUnset = 0x7fffffff;
  for (int j = 0; j < k; j++) __atomic_store_n(&c->h_ring[j].outcome, kUnset, __ATOMIC_RELAXED);
  const int64_t first = c->n_iterates;
  // Iteration j > 0 runs only if iteration j - 1 left the session going, i.e. produced a
  // transform: its search applies it. The first applies the session's pending increment.
  for (int j = 0; j < k; j++) {
    const int rc = enqueue_iterate(c, nullptr, j > 0 || core->pending, core->iter + j, rules, sigma, j, nullptr);
    if (rc != ICP_HIP_OK) return rc;
  }
  HIP_TRY(hipMemcpyAsync(c->h_loop, c->loopd, sizeof(LoopDev), hipMemcpyDeviceToHost, s));
  // (polled rather than hipStreamSynchronize: a batch over a communicator whose peer died would
  // otherwise wait forever)
  const int wrc = wait_device(
      c, [&]() { return hipStreamQuery(s) != hipErrorNotReady; },
      [&]() {
        uint64_t n = 0;
        for (int j = 0; j < k; j++) n += __atomic_load_n(&c->h_ring[j].outcome, __ATOMIC_RELAXED) != kUnset ? 1u : 0u;
        return n;
      },
      "device loop");
  if (wrc != ICP_HIP_OK) return wrc;
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail(ICP_HIP_EDEVICE, std::string("device loop: ") + hipGetErrorString(e));
  *core = c->h_loop->core;
  std::memcpy(recs, c->h_ring, (size_t)k * sizeof(icp::LoopRec));
  c->lists_zero = true;
  c->have_results = true;
  for (int j = k - 1; j >= 0; j--)
    if (recs[j].outcome != icp::kStepNone) {
      for (int q = 0; q < 3; q++) c->last_lists[q] = (unsigned int)recs[j].lists[q];
      c->last_wide = (double)recs[j].pad[0];
      break;
    }
  if (step_ms) {
    hipEvent_t prev = c->ev_batch;
    for (int j = 0; j < k; j++) {
      hipEvent_t end = c->ring[(first + j) % icp_hip_ctx::kTimingRing][2];
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, prev, end));
      step_ms[j] = ms;
      prev = end;
    }
  }
  return ICP_HIP_OK;
}

extern "C" {

int icp_hip_debug_counters(icp_hip_ctx* c, uint64_t out[ICP_DBG_SLOTS]) {
  if (!c || !out) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return group_debug_counters(c, out);
  std::memset(out, 0, ICP_DBG_SLOTS * sizeof(uint64_t));
  if (!c->dbg) return ICP_HIP_OK;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(out, c->dbg, ICP_DBG_SLOTS * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return ICP_HIP_OK;
}

int icp_hip_apply(icp_hip_ctx* c, const double* T) {
  if (!c || !T) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return group_apply(c, T);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(launch_apply(T, c->x, c->y, c->z, c->n_src, c->stream));
  c->have_prev = false;  // queries moved without a search: previous residuals are no guess
  HIP_TRY(hipStreamSynchronize(c->stream));
  return ICP_HIP_OK;
}

int icp_hip_get_source(icp_hip_ctx* c, double* xyz_out) {
  if (c && c->group) return xyz_out ? group_get_source(c, xyz_out) : fail(ICP_HIP_EINVAL, "null argument");
  if (!c || (!xyz_out && c->n_src > 0)) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->n_src == 0) return ICP_HIP_OK;
  HIP_TRY(hipSetDevice(c->device));
  double* aos = nullptr;
  HIP_TRY(dalloc(&aos, 3 * (size_t)c->n_src));
  hipError_t e = launch_scatter_aos(c->perm, c->x, c->y, c->z, aos, c->n_src, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(xyz_out, aos, 3 * sizeof(double) * c->n_src, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(aos);
  if (e != hipSuccess) return fail(ICP_HIP_EDEVICE, std::string("get_source: ") + hipGetErrorString(e));
  return ICP_HIP_OK;
}

int icp_hip_get_correspondences(icp_hip_ctx* c, int32_t* idx_out, double* dist_out) {
  if (!c) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return group_get_correspondences(c, idx_out, dist_out);
  if (!c->have_results) return fail(ICP_HIP_ENOTREADY, "no iteration has run on this source");
  if (c->n_src == 0) return ICP_HIP_OK;
  HIP_TRY(hipSetDevice(c->device));
  int32_t* di = nullptr;
  double* dd = nullptr;
  hipError_t e = hipSuccess;
  if (idx_out) e = dalloc(&di, c->n_src);
  if (e == hipSuccess && dist_out) e = dalloc(&dd, c->n_src);
  if (e == hipSuccess) e = launch_scatter_corr(c->perm, c->pos, c->pts, di, c->dist, dd, c->n_src, c->stream);
  if (e == hipSuccess && idx_out) e = hipMemcpyAsync(idx_out, di, sizeof(int32_t) * c->n_src, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && dist_out) e = hipMemcpyAsync(dist_out, dd, sizeof(double) * c->n_src, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(di);
  dfree(dd);
  if (e != hipSuccess) return fail(ICP_HIP_EDEVICE, std::string("get_correspondences: ") + hipGetErrorString(e));
  return ICP_HIP_OK;
}

int icp_hip_nn(icp_hip_ctx* c, const double* q, int64_t n, int32_t* idx_out, double* dist_out) {
  if (!c || n < 0 || (n > 0 && !q)) return fail(ICP_HIP_EINVAL, "bad arguments");
  if (c->group) return icp_hip_nn(group_member(c, 0), q, n, idx_out, dist_out);  // the replicated octree
  if (!c->nodes) return fail(ICP_HIP_ENOTREADY, "target not set");
  if (n == 0) return ICP_HIP_OK;
  // the wave search addresses per-query arrays by 32-bit byte offsets (nn_device.h qat): launches
  // of fewer than 2^29 queries, so larger sets go in slices (the answers are per query)
  constexpr int64_t kSlice = (int64_t)1 << 28;
  if (n > kSlice) {
    unsigned int lists[3] = {0, 0, 0};
    for (int64_t off = 0; off < n; off += kSlice) {
      const int64_t m = n - off < kSlice ? n - off : kSlice;
      const int rc = icp_hip_nn(c, q + 3 * off, m, idx_out ? idx_out + off : nullptr, dist_out ? dist_out + off : nullptr);
      if (rc != ICP_HIP_OK) return rc;
      for (int k = 0; k < 3; k++) lists[k] += c->last_lists[k];
    }
    for (int k = 0; k < 3; k++) c->last_lists[k] = lists[k];
    return ICP_HIP_OK;
  }
  HIP_TRY(hipSetDevice(c->device));
  double *aos = nullptr, *x = nullptr, *y = nullptr, *z = nullptr, *d = nullptr, *dd = nullptr;
  int32_t *pos = nullptr, *di = nullptr;
  hipError_t e = hipSuccess;
  if ((e = dalloc(&aos, 3 * (size_t)n)) == hipSuccess && (e = dalloc(&x, n)) == hipSuccess &&
      (e = dalloc(&y, n)) == hipSuccess && (e = dalloc(&z, n)) == hipSuccess && (e = dalloc(&d, n)) == hipSuccess &&
      (e = dalloc(&dd, n)) == hipSuccess && (e = dalloc(&pos, n)) == hipSuccess && (e = dalloc(&di, n)) == hipSuccess) {
    e = hipMemcpyAsync(aos, q, 3 * sizeof(double) * n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = launch_deinterleave(aos, x, y, z, n, c->stream);
    NNLaunch a = base_launch(c);
    a.x = x;
    a.y = y;
    a.z = z;
    a.pos_out = pos;
    a.dist_out = d;
    a.n = n;
    int32_t* fbl = nullptr;
    double* fbu = nullptr;
    if (e == hipSuccess) e = dalloc(&fbl, 3 * (size_t)n + 64);
    if (e == hipSuccess) e = dalloc(&fbu, (size_t)n);
    a.fb_list = fbl;
    a.fb_list2 = fbl + n;
    a.fb_list3 = c->cfg.overflow_halves ? fbl + 2 * n : nullptr;
    a.fb_list4 = c->cfg.scan32 && c->cfg.wide_pass != 1 ? wide_list(fbl, n) : nullptr;
    a.fb_u2 = fbu;
    a.fb_count = c->fb_count;
    unsigned int lists4[4] = {0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemsetAsync(c->fb_count, 0, 8 * sizeof(unsigned int), c->stream);
    c->lists_zero = false;
    if (e == hipSuccess) e = launch_nn(a, c->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(lists4, c->fb_count, 4 * sizeof(unsigned int), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    c->last_lists[0] = lists4[0] + lists4[3];  // exact: the wave search's list + the ball's DFS finishes
    c->last_lists[1] = lists4[1];
    c->last_lists[2] = lists4[2];
    dfree(fbl);
    dfree(fbu);
    if (e == hipSuccess) e = launch_scatter_corr(nullptr, pos, c->pts, di, d, dd, n, c->stream);
    if (e == hipSuccess && idx_out) e = hipMemcpyAsync(idx_out, di, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && dist_out) e = hipMemcpyAsync(dist_out, dd, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  }
  dfree(aos); dfree(x); dfree(y); dfree(z); dfree(d); dfree(dd); dfree(pos); dfree(di);
  if (e != hipSuccess) return fail(e == hipErrorOutOfMemory ? ICP_HIP_ENOMEM : ICP_HIP_EDEVICE, std::string("nn: ") + hipGetErrorString(e));
  return ICP_HIP_OK;
}

int icp_hip_traversal_counts(icp_hip_ctx* c, double* mean_entries, double* mean_points) {
  if (!c || !mean_entries || !mean_points) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return group_traversal_counts(c, mean_entries, mean_points);
  if (!c->nodes || (!c->x && c->n_src > 0)) return fail(ICP_HIP_ENOTREADY, "target/source not set");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemsetAsync(c->counters, 0, 2 * sizeof(unsigned long long), c->stream));
  NNLaunch a = base_launch(c);
  a.x = c->x;
  a.y = c->y;
  a.z = c->z;
  a.pos_out = c->pos;  // same queries as the last iterate: identical outputs are rewritten
  a.dist_out = c->dist;
  a.n = c->n_src;
  a.dbg = nullptr;
  a.count = 1;
  HIP_TRY(launch_nn(a, c->stream));
  unsigned long long h[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(h, c->counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const double n = c->n_src > 0 ? (double)c->n_src : 1.0;
  *mean_entries = (double)h[0] / n;
  *mean_points = (double)h[1] / n;
  return ICP_HIP_OK;
}

int icp_hip_target_info(icp_hip_ctx* c, int64_t* n_nodes, int64_t* n_leaves, int32_t* max_depth, int32_t* levels) {
  if (!c) return fail(ICP_HIP_EINVAL, "null ctx");
  if (c->group) return icp_hip_target_info(group_member(c, 0), n_nodes, n_leaves, max_depth, levels);
  if (n_nodes) *n_nodes = c->n_nodes;
  if (n_leaves) *n_leaves = c->n_leaves;
  if (max_depth) *max_depth = c->max_depth;
  if (levels) *levels = c->levels;
  return ICP_HIP_OK;
}

int icp_hip_timings(icp_hip_ctx* c, int k, double* nn_ms, double* it_ms) {
  if (!c || k < 0) return fail(ICP_HIP_EINVAL, "bad arguments");
  if (c->group) return group_timings(c, k, nn_ms, it_ms);
  if (k > icp_hip_ctx::kTimingRing || k > c->n_iterates) return fail(ICP_HIP_EINVAL, "fewer iterates recorded than asked");
  HIP_TRY(hipSetDevice(c->device));
  for (int j = 0; j < k; j++) {
    const int64_t slot = (c->n_iterates - k + j) % icp_hip_ctx::kTimingRing;
    hipEvent_t* ev = c->ring[slot];
    HIP_TRY(hipEventSynchronize(ev[2]));
    double a = std::nan(""), b = std::nan("");
    if (c->timed[slot]) {
      float fa = 0.f, fb = 0.f;
      HIP_TRY(hipEventElapsedTime(&fa, ev[0], ev[1]));
      HIP_TRY(hipEventElapsedTime(&fb, ev[0], ev[2]));
      a = fa;
      b = fb;
    }
    if (nn_ms) nn_ms[j] = a;
    if (it_ms) it_ms[j] = b;
  }
  return ICP_HIP_OK;
}

int icp_hip_last_timing(icp_hip_ctx* c, double* nn_ms, double* it_ms) {
  if (!c) return fail(ICP_HIP_EINVAL, "null ctx");
  if (c->group) return group_timings(c, 1, nn_ms, it_ms);
  if (c->n_iterates == 0) return fail(ICP_HIP_ENOTREADY, "no iterate has run");
  if (!c->timed[(c->n_iterates - 1) % icp_hip_ctx::kTimingRing])
    return fail(ICP_HIP_ENOTREADY, "the last iterate was not timed (config.timing_stride)");
  return icp_hip_timings(c, 1, nn_ms, it_ms);
}

int icp_hip_exchange_timings(icp_hip_ctx* c, int k, double* ms) {
  if (!c || k < 0 || (k > 0 && !ms)) return fail(ICP_HIP_EINVAL, "bad arguments");
  if (c->group) return group_exchange_timings(c, k, ms);
  if (k > icp_hip_ctx::kTimingRing || k > c->n_iterates) return fail(ICP_HIP_EINVAL, "fewer iterates recorded than asked");
  HIP_TRY(hipSetDevice(c->device));
  for (int j = 0; j < k; j++) {
    const int64_t slot = (c->n_iterates - k + j) % icp_hip_ctx::kTimingRing;
    HIP_TRY(hipEventSynchronize(c->ring[slot][2]));
    double v = std::nan("");
    if (c->xtimed[slot] == 1) {
      float f0 = 0.f, f1 = 0.f;
      HIP_TRY(hipEventElapsedTime(&f0, c->xring[slot][0], c->xring[slot][1]));
      HIP_TRY(hipEventElapsedTime(&f1, c->xring[slot][2], c->xring[slot][3]));
      v = (double)f0 + (double)f1;
    } else if (c->xtimed[slot] == 2) {
      v = c->xhost_ms[slot];
    }
    ms[j] = v;
  }
  return ICP_HIP_OK;
}

int icp_hip_comm_info(icp_hip_ctx* c, int member, int32_t* count, int32_t* rank, int32_t* device, int32_t* transport) {
  if (!c) return fail(ICP_HIP_EINVAL, "null ctx");
  if (c->group) return group_comm_info(c, member, count, rank, device, transport);
  if (member != 0) return fail(ICP_HIP_EINVAL, "a single-device context has member 0 only");
  int n = c->nranks, r = c->rank, d = c->device;
  if (c->comm) {
    // RCCL's own view of the communicator, not the arguments it was created with
    RCCL_TRY(ncclCommCount(c->comm, &n));
    RCCL_TRY(ncclCommUserRank(c->comm, &r));
    RCCL_TRY(ncclCommCuDevice(c->comm, &d));
  }
  if (count) *count = n;
  if (rank) *rank = r;
  if (device) *device = d;
  if (transport) *transport = c->comm ? ICP_XPORT_RCCL : c->xfn ? ICP_XPORT_CALLBACK : ICP_XPORT_AUTO;
  return ICP_HIP_OK;
}

int icp_hip_last_cull_path(icp_hip_ctx* c, int32_t* fused) {
  if (!c || !fused) return fail(ICP_HIP_EINVAL, "null argument");
  if (c->group) return group_cull_path(c, fused);
  if (c->last_cull_path < 0) return fail(ICP_HIP_ENOTREADY, "no host-published iterate on this source");
  *fused = c->last_cull_path;
  return ICP_HIP_OK;
}

int icp_hip_comm_abort(icp_hip_ctx* c) {
  if (!c) return fail(ICP_HIP_EINVAL, "null ctx");
  if (c->group) return fail(ICP_HIP_EINVAL, "a multi-device context aborts its communicators itself");
  icp_ctx_abort_comm(c);
  return ICP_HIP_OK;
}

int icp_hip_debug_inject_failure(icp_hip_ctx* c, int member, int where) {
  if (!c || where < 0 || where > 1) return fail(ICP_HIP_EINVAL, "bad arguments");
  if (c->group) return group_inject_failure(c, member, where);
  if (member != 0) return fail(ICP_HIP_EINVAL, "a single-device context has member 0 only");
  c->inject_failure = where;
  return ICP_HIP_OK;
}

int icp_hip_synchronize(icp_hip_ctx* c) {
  if (!c) return fail(ICP_HIP_EINVAL, "null ctx");
  if (c->group) return group_synchronize(c);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return ICP_HIP_OK;
}

const char* icp_hip_last_error(void) { return g_err.c_str(); }

}  // extern "C"
