// icp_group.cpp — a context that drives several GPUs from one process (icp_hip_create_multi).
//
// the drop-in's callers (ICPEngine::registerPointClouds, icpengine.cpp:24-60;
// the CLI's ICP(), icp_registration.cpp:443-446) are single-process, so the multi-GPU path must be
// reachable from one process. A group holds one member context per device (icp_ctx.hip: a
// replicated octree, a spatially compact shard of the source) and one driver thread per member.
// An iterate runs every member's ordinary multi-rank iterate concurrently, each on its own thread:
// the two per-iteration all-gathers are RCCL collectives over communicators from ncclCommInitAll
// (one per device), or, when devices repeat (RCCL refuses two ranks on one device) or the caller
// asks for it, an in-process host gather with the same record layout. Every member merges the
// gathered records in rank order on its device, so all members hold bitwise-identical statistics
// (the same numbers a world of N processes computes).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/icp_hip.h"
#include "icp_ctx_internal.h"
#include "group_sync.h"
#include "query_order.h"

using icp::Driver;
using icp::ExchangeSlot;
using icp::LocalExchange;
using icp::local_exchange;

struct DeviceGroup {
  std::vector<icp_hip_ctx*> members;
  std::vector<int> devices;
  int transport = ICP_XPORT_HOST;
  std::unique_ptr<LocalExchange> lx;
  std::vector<ExchangeSlot> slots;
  std::vector<std::unique_ptr<Driver>> drivers;
  std::atomic<int> abort{0};  // a member of the running job failed (peers stop waiting)
  // an iterate failed over RCCL: the communicators were aborted, only destroy is left
  bool dead = false;
  std::string dead_why;
  // the source: caller index of group slot k, and member m's slots [lo[m], lo[m + 1])
  std::vector<int32_t> order;
  std::vector<int64_t> lo;
  int64_t n_src = 0;
};

namespace {

int fail(int code, const std::string& msg) {
  icp_ctx_set_error(msg.c_str());
  return code;
}

// f(k, member) on every member's driver thread, concurrently; the first failure's code and message
// (the message is thread-local to the driver that saw it) come back to the caller. A failing member
// raises the group's abort flag, so peers waiting in an exchange or for a record give up.
int for_members(DeviceGroup* g, const std::function<int(int, icp_hip_ctx*)>& f) {
  if (g->dead)
    return fail(ICP_HIP_EDEVICE, "multi-device context unusable after a failed RCCL iterate (" + g->dead_why +
                                     "); destroy it and create a new one");
  const int n = (int)g->members.size();
  // a new job starts clean: the flag and the host exchange's count of the previous failed job
  g->abort.store(0);
  if (g->lx) g->lx->reset();
  std::vector<int> rc((size_t)n, ICP_HIP_OK);
  std::vector<std::string> msg((size_t)n);
  for (int k = 0; k < n; k++) {
    g->drivers[k]->post([g, k, &f, &rc, &msg] {
      rc[k] = f(k, g->members[k]);
      if (rc[k] != ICP_HIP_OK) {
        msg[k] = icp_hip_last_error();
        g->abort.store(1);
        if (g->lx) g->lx->wake();
      }
    });
  }
  for (int k = 0; k < n; k++) g->drivers[k]->wait();
  // report the root cause: a member's own failure before a peer's "peer failed"
  int first = -1;
  for (int k = 0; k < n; k++)
    if (rc[k] != ICP_HIP_OK && (first < 0 || (rc[first] == ICP_HIP_EEXCHANGE && rc[k] != ICP_HIP_EEXCHANGE))) first = k;
  if (first < 0) return ICP_HIP_OK;
  return fail(rc[first], "device " + std::to_string(g->devices[first]) + ": " + msg[first]);
}

void shard_ranges(int64_t n, int w, std::vector<int64_t>* lo) {
  lo->assign((size_t)w + 1, 0);
  const int64_t base = n / w, rem = n % w;
  for (int r = 0; r < w; r++) (*lo)[r + 1] = (*lo)[r] + base + (r < rem ? 1 : 0);
}

}  // namespace

extern "C" int icp_hip_create_multi(icp_hip_ctx** out, int n_devices, const int* device_ids,
                                    const icp_hip_config* cfg, int transport) {
  if (!out) return fail(ICP_HIP_EINVAL, "null out");
  *out = nullptr;
  if (n_devices < 1 || n_devices > 64 || !device_ids) return fail(ICP_HIP_EINVAL, "create_multi: bad device list");
  if (transport != ICP_XPORT_AUTO && transport != ICP_XPORT_RCCL && transport != ICP_XPORT_HOST)
    return fail(ICP_HIP_EINVAL, "create_multi: unknown transport");
  std::vector<int> devs(device_ids, device_ids + n_devices);
  std::vector<int> sorted = devs;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  if (transport == ICP_XPORT_RCCL && !distinct)
    return fail(ICP_HIP_EINVAL, "create_multi: RCCL needs distinct devices (one rank per GPU)");
  if (transport == ICP_XPORT_AUTO) {
    if (n_devices == 1) return icp_hip_create_ex(out, devs[0], cfg);  // a plain single-device context
    transport = distinct ? ICP_XPORT_RCCL : ICP_XPORT_HOST;
  }
  // the version word first, before the struct is copied (icp_hip_create_ex checks the rest)
  if (cfg && cfg->config_version != ICP_HIP_CONFIG_VERSION)
    return fail(ICP_HIP_EINVAL, "config: config_version is not ICP_HIP_CONFIG_VERSION (start from icp_hip_config_default "
                                "of this header)");
  auto* g = new DeviceGroup();
  g->devices = devs;
  g->transport = transport;
  auto* c = new icp_hip_ctx();
  c->device = devs[0];
  c->group = g;
  if (cfg) c->cfg = *cfg;
  else icp_hip_config_default(&c->cfg);
  int rc = ICP_HIP_OK;
  for (int k = 0; k < n_devices && rc == ICP_HIP_OK; k++) {
    icp_hip_ctx* m = nullptr;
    rc = icp_hip_create_ex(&m, devs[k], cfg);
    if (rc == ICP_HIP_OK) {
      m->abort = &g->abort;
      g->members.push_back(m);
    }
  }
  if (rc == ICP_HIP_OK && transport == ICP_XPORT_RCCL) {
    std::vector<ncclComm_t> comms((size_t)n_devices, nullptr);
    const ncclResult_t r = ncclCommInitAll(comms.data(), n_devices, devs.data());
    if (r != ncclSuccess) {
      rc = fail(ICP_HIP_ERCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    } else {
      for (int k = 0; k < n_devices; k++) {
        const int rk = icp_ctx_attach_comm(g->members[k], comms[k], n_devices, k);
        if (rk != ICP_HIP_OK && rc == ICP_HIP_OK) rc = rk;
        if (rk != ICP_HIP_OK) (void)ncclCommDestroy(comms[k]);
      }
    }
  } else if (rc == ICP_HIP_OK) {
    g->lx = std::make_unique<LocalExchange>();
    g->lx->n = n_devices;
    g->lx->abort = &g->abort;
    g->slots.resize((size_t)n_devices);
    for (int k = 0; k < n_devices && rc == ICP_HIP_OK; k++) {
      g->slots[k] = ExchangeSlot{g->lx.get(), k};
      rc = icp_hip_comm_init_host(g->members[k], n_devices, k, &local_exchange, &g->slots[k]);
    }
  }
  if (rc == ICP_HIP_OK)
    for (int k = 0; k < n_devices; k++) g->drivers.push_back(std::make_unique<Driver>());
  if (rc != ICP_HIP_OK) {
    const std::string why = icp_hip_last_error();
    icp_hip_destroy(c);
    return fail(rc, why);
  }
  *out = c;
  return ICP_HIP_OK;
}

void group_destroy(icp_hip_ctx* c) {
  DeviceGroup* g = c->group;
  g->drivers.clear();  // joins the driver threads
  for (icp_hip_ctx* m : g->members) icp_hip_destroy(m);
  delete g;
  c->group = nullptr;
}

icp_hip_ctx* group_member(icp_hip_ctx* c, int k) { return c->group->members[k]; }

int group_set_target(icp_hip_ctx* c, const double* xyz, int64_t n, int max_points, int max_depth, int rules) {
  // every device builds the same octree from the same cloud (a replica each)
  return for_members(c->group, [&](int, icp_hip_ctx* m) {
    return icp_hip_set_target(m, xyz, n, max_points, max_depth, rules);
  });
}

int group_target_build_info(icp_hip_ctx* c, int32_t* on_device, double* build_ms) {
  double worst = 0.0;
  int32_t od = 1;
  for (icp_hip_ctx* m : c->group->members) {
    int32_t o = 0;
    double ms = 0.0;
    const int rc = icp_hip_target_build_info(m, &o, &ms);
    if (rc != ICP_HIP_OK) return rc;
    od = od && o;
    worst = ms > worst ? ms : worst;
  }
  if (on_device) *on_device = od;
  if (build_ms) *build_ms = worst;
  return ICP_HIP_OK;
}

int group_set_source(icp_hip_ctx* c, const double* xyz, int64_t n) {
  DeviceGroup* g = c->group;
  const int w = (int)g->members.size();
  if (n < w) return fail(ICP_HIP_EINVAL, "set_source: a multi-device context needs at least one point per device");
  if (n > (int64_t)0x7fffffff) return fail(ICP_HIP_EINVAL, "set_source: 2^31 points or more (int32 query order)");
  // spatially compact shards: contiguous ranges of the kd order (icp_source_shard_order's order),
  // built on the first device (or on the host: config query_order = 1, or no device memory)
  g->order.assign((size_t)n, 0);
  bool ordered = false;
  if (c->cfg.query_order == 0) {
    icp_hip_ctx* m0 = g->members[0];
    double* d_xyz = nullptr;
    int32_t* d_perm = nullptr;
    hipError_t e = hipSetDevice(m0->device);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_xyz), 3 * sizeof(double) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&d_perm), sizeof(int32_t) * (size_t)n);
    if (e == hipSuccess) e = hipMemcpyAsync(d_xyz, xyz, 3 * sizeof(double) * (size_t)n, hipMemcpyHostToDevice, m0->stream);
    if (e == hipSuccess) e = icp::gpu_kd_query_order(d_xyz, n, 8, d_perm, m0->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(g->order.data(), d_perm, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, m0->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(m0->stream);
    if (d_xyz) (void)hipFree(d_xyz);
    if (d_perm) (void)hipFree(d_perm);
    ordered = e == hipSuccess;
    if (!ordered) (void)hipGetLastError();
  }
  if (!ordered) icp::kd_query_order(xyz, n, 8, &g->order);
  shard_ranges(n, w, &g->lo);
  g->n_src = n;
  return for_members(g, [&](int k, icp_hip_ctx* m) {
    const int64_t a = g->lo[k], b = g->lo[k + 1];
    std::vector<double> shard((size_t)(3 * (b - a)));
    for (int64_t j = a; j < b; j++) std::memcpy(&shard[3 * (j - a)], xyz + 3 * (int64_t)g->order[j], 3 * sizeof(double));
    return icp_hip_set_source(m, shard.data(), b - a);
  });
}

int group_iterate(icp_hip_ctx* c, const double* T_apply, int iter, int rules, double sigma, icp_iter_stats* out) {
  DeviceGroup* g = c->group;
  const int w = (int)g->members.size();
  if (!g->dead) {  // usage errors before any member runs leave the group usable
    for (icp_hip_ctx* m : g->members) {
      if (!m->nodes) return fail(ICP_HIP_ENOTREADY, "target not set");
      if (!m->x && m->n_src > 0) return fail(ICP_HIP_ENOTREADY, "source not set");
    }
  }
  std::vector<icp_iter_stats> st((size_t)w);
  const int rc = for_members(g, [&](int k, icp_hip_ctx* m) { return icp_hip_iterate(m, T_apply, iter, rules, sigma, &st[k]); });
  if (rc != ICP_HIP_OK) {
    if (g->transport == ICP_XPORT_RCCL && !g->dead) {
      // A member that failed before joining a collective leaves its peers' streams holding one
      // that never completes: abort every communicator (the pending collectives return, the
      // streams drain, destroy cannot block). The group cannot exchange again.
      const std::string why = icp_hip_last_error();
      for (icp_hip_ctx* m : g->members) icp_ctx_abort_comm(m);
      g->dead = true;
      g->dead_why = why;
      return fail(rc, why);
    }
    return rc;
  }
  // the statistics are merged in rank order on every device: identical on all members
  for (int k = 1; k < w; k++)
    if (st[k].valid != st[0].valid || std::memcmp(&st[k].mean, &st[0].mean, sizeof(double)) != 0 ||
        std::memcmp(st[k].H, st[0].H, sizeof(st[0].H)) != 0)
      return fail(ICP_HIP_EDEVICE, "iterate: members disagree on the merged statistics");
  *out = st[0];
  out->n_fallback = out->n_lane_search = out->n_ball_search = 0;  // per-rank counts: summed
  for (const icp_iter_stats& s : st) {
    out->n_fallback += s.n_fallback;
    out->n_lane_search += s.n_lane_search;
    out->n_ball_search += s.n_ball_search;
  }
  return ICP_HIP_OK;
}

int group_apply(icp_hip_ctx* c, const double* T) {
  return for_members(c->group, [&](int, icp_hip_ctx* m) { return icp_hip_apply(m, T); });
}

int group_get_source(icp_hip_ctx* c, double* xyz_out) {
  DeviceGroup* g = c->group;
  return for_members(g, [&](int k, icp_hip_ctx* m) {
    const int64_t a = g->lo[k], b = g->lo[k + 1];
    std::vector<double> shard((size_t)(3 * (b - a)));
    const int rc = icp_hip_get_source(m, shard.data());
    if (rc != ICP_HIP_OK) return rc;
    for (int64_t j = a; j < b; j++) std::memcpy(xyz_out + 3 * (int64_t)g->order[j], &shard[3 * (j - a)], 3 * sizeof(double));
    return ICP_HIP_OK;
  });
}

int group_get_correspondences(icp_hip_ctx* c, int32_t* idx_out, double* dist_out) {
  DeviceGroup* g = c->group;
  return for_members(g, [&](int k, icp_hip_ctx* m) {
    const int64_t a = g->lo[k], b = g->lo[k + 1];
    std::vector<int32_t> idx(idx_out ? (size_t)(b - a) : 0);
    std::vector<double> d(dist_out ? (size_t)(b - a) : 0);
    const int rc = icp_hip_get_correspondences(m, idx_out ? idx.data() : nullptr, dist_out ? d.data() : nullptr);
    if (rc != ICP_HIP_OK) return rc;
    for (int64_t j = a; j < b; j++) {
      if (idx_out) idx_out[g->order[j]] = idx[j - a];
      if (dist_out) dist_out[g->order[j]] = d[j - a];
    }
    return ICP_HIP_OK;
  });
}

int group_traversal_counts(icp_hip_ctx* c, double* mean_entries, double* mean_points) {
  DeviceGroup* g = c->group;
  const int w = (int)g->members.size();
  std::vector<double> e((size_t)w), p((size_t)w);
  const int rc = for_members(g, [&](int k, icp_hip_ctx* m) { return icp_hip_traversal_counts(m, &e[k], &p[k]); });
  if (rc != ICP_HIP_OK) return rc;
  double se = 0.0, sp = 0.0;
  for (int k = 0; k < w; k++) {
    const double nk = (double)(g->lo[k + 1] - g->lo[k]);
    se += e[k] * nk;
    sp += p[k] * nk;
  }
  const double n = g->n_src > 0 ? (double)g->n_src : 1.0;
  *mean_entries = se / n;
  *mean_points = sp / n;
  return ICP_HIP_OK;
}

int group_timings(icp_hip_ctx* c, int k, double* nn_ms, double* it_ms) {
  // per iterate, the slowest member (the iterate ends when every member's record is published)
  std::vector<double> a((size_t)k), b((size_t)k);
  bool first = true;
  for (icp_hip_ctx* m : c->group->members) {
    const int rc = icp_hip_timings(m, k, a.data(), b.data());
    if (rc != ICP_HIP_OK) return rc;
    for (int j = 0; j < k; j++) {
      if (nn_ms) nn_ms[j] = first || a[j] > nn_ms[j] ? a[j] : nn_ms[j];
      if (it_ms) it_ms[j] = first || b[j] > it_ms[j] ? b[j] : it_ms[j];
    }
    first = false;
  }
  return ICP_HIP_OK;
}

int group_exchange_timings(icp_hip_ctx* c, int k, double* ms) {
  // per iterate, the slowest member's exchange (NaN when the iterate was not timed)
  std::vector<double> a((size_t)k);
  bool first = true;
  for (icp_hip_ctx* m : c->group->members) {
    const int rc = icp_hip_exchange_timings(m, k, a.data());
    if (rc != ICP_HIP_OK) return rc;
    for (int j = 0; j < k; j++) ms[j] = first || a[j] > ms[j] ? a[j] : ms[j];
    first = false;
  }
  return ICP_HIP_OK;
}

int group_comm_info(icp_hip_ctx* c, int member, int32_t* count, int32_t* rank, int32_t* device, int32_t* transport) {
  DeviceGroup* g = c->group;
  if (member < 0 || member >= (int)g->members.size()) return fail(ICP_HIP_EINVAL, "comm_info: no such member");
  return icp_hip_comm_info(g->members[member], 0, count, rank, device, transport);
}

int group_cull_path(icp_hip_ctx* c, int32_t* fused) {
  // 1 only when every member's cull took its search's wave records
  int32_t all = 1;
  for (icp_hip_ctx* m : c->group->members) {
    int32_t f = 0;
    const int rc = icp_hip_last_cull_path(m, &f);
    if (rc != ICP_HIP_OK) return rc;
    all = all && f;
  }
  *fused = all;
  return ICP_HIP_OK;
}

int group_debug_counters(icp_hip_ctx* c, uint64_t out[ICP_DBG_SLOTS]) {
  std::memset(out, 0, ICP_DBG_SLOTS * sizeof(uint64_t));
  for (icp_hip_ctx* m : c->group->members) {
    uint64_t v[ICP_DBG_SLOTS];
    const int rc = icp_hip_debug_counters(m, v);
    if (rc != ICP_HIP_OK) return rc;
    for (int s = 0; s < ICP_DBG_SLOTS; s++) out[s] += v[s];
  }
  return ICP_HIP_OK;
}

int group_synchronize(icp_hip_ctx* c) {
  for (icp_hip_ctx* m : c->group->members) {
    const int rc = icp_hip_synchronize(m);
    if (rc != ICP_HIP_OK) return rc;
  }
  return ICP_HIP_OK;
}

int group_inject_failure(icp_hip_ctx* c, int member, int where) {
  DeviceGroup* g = c->group;
  if (member < 0 || member >= (int)g->members.size()) return fail(ICP_HIP_EINVAL, "inject_failure: no such member");
  g->members[member]->inject_failure = where;
  return ICP_HIP_OK;
}

extern "C" int icp_hip_ctx_devices(icp_hip_ctx* c, int32_t* n_devices, int32_t* device_ids, int32_t cap,
                                   int32_t* transport) {
  if (!c) return fail(ICP_HIP_EINVAL, "null context");
  if (c->group) {
    const DeviceGroup* g = c->group;
    if (n_devices) *n_devices = (int32_t)g->devices.size();
    for (int k = 0; device_ids && k < (int)g->devices.size() && k < cap; k++) device_ids[k] = g->devices[k];
    if (transport) *transport = g->transport;
    return ICP_HIP_OK;
  }
  if (n_devices) *n_devices = 1;
  if (device_ids && cap > 0) device_ids[0] = c->device;
  if (transport) *transport = c->comm ? ICP_XPORT_RCCL : c->xfn ? ICP_XPORT_CALLBACK : ICP_XPORT_AUTO;
  return ICP_HIP_OK;
}
