// reduce_kernels.hip — gfx950 reductions of one ICP iteration after the correspondence search.
//
//  k_moments        residual moments of fixed 4096-query parts (icpengine.cpp:235-245)
//  k_cull_waves     3-sigma cull (icpengine.cpp:263-278) + valid-pair centroid and cross-covariance
//                   sums (icpengine.cpp:76-90, computeBestFitTransform's H = AA * BB^T), from the
//                   wave search's per-wave records and the band pairs (wave_stats.h), or in full
//  k_tree_merge, k_merge_*_last   fixed-shape merge trees of the part sums (deterministic)
//  k_finalize_*     rank-ordered merge of the gathered per-rank records (multi-GPU)
//  publish          the last kernel of an iteration stores the finished record into pinned host
//                   memory, sequence word last: the host's only wait of the iteration
//
// fp64, -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cstddef>

#include "kernels.h"
#include "nn_device.h"
#include "wave_stats.h"

namespace icp {

namespace {

using namespace dev;

// Rank-level reductions as shifted plain sums. A part holds sums of values shifted by a constant
// of the iteration (query 0's residual, source point and match), so the sums stay at the spread
// of the data, not at its offset (LAS-sized coordinates), and the merge tree is plain additions
// in a fixed order: deterministic and cheap. The last level turns them into (count, mean, M2)
// and (count, means, co-moment) records, which ranks merge with the Chan formulas (icp_common.h).
struct MomSums {
  double n, s1, s2, dmin, dmax, nbad, pad0, pad1;  // s1 = sum (d - c), s2 = sum (d - c)^2
};
struct CovSums {
  double n, sum_d2, sa[3], sb[3], sab[9], pad[3];  // sa = sum (a - s), sb = sum (b - t), sab = sum (a - s)(b - t)^T
};
static_assert(sizeof(MomSums) == sizeof(Moments) && sizeof(CovSums) == sizeof(CovMoments), "part buffers");

__device__ __forceinline__ MomSums momsum_identity() {
  MomSums m;
  m.n = m.s1 = m.s2 = m.nbad = m.pad0 = m.pad1 = 0.0;
  m.dmin = 1.7976931348623157e308;
  m.dmax = 0.0;
  return m;
}
__device__ MomSums momsum_merge(const MomSums& a, const MomSums& b) {
  MomSums r;
  r.n = a.n + b.n;
  r.s1 = a.s1 + b.s1;
  r.s2 = a.s2 + b.s2;
  r.dmin = b.dmin < a.dmin ? b.dmin : a.dmin;
  r.dmax = b.dmax > a.dmax ? b.dmax : a.dmax;
  r.nbad = a.nbad + b.nbad;
  r.pad0 = r.pad1 = 0.0;
  return r;
}
__device__ __forceinline__ CovSums covsum_identity() {
  CovSums c;
  c.n = c.sum_d2 = 0.0;
  for (int k = 0; k < 3; k++) c.sa[k] = c.sb[k] = c.pad[k] = 0.0;
  for (int k = 0; k < 9; k++) c.sab[k] = 0.0;
  return c;
}
__device__ CovSums covsum_merge(const CovSums& a, const CovSums& b) {
  CovSums r;
  r.n = a.n + b.n;
  r.sum_d2 = a.sum_d2 + b.sum_d2;
  for (int k = 0; k < 3; k++) {
    r.sa[k] = a.sa[k] + b.sa[k];
    r.sb[k] = a.sb[k] + b.sb[k];
    r.pad[k] = 0.0;
  }
  for (int k = 0; k < 9; k++) r.sab[k] = a.sab[k] + b.sab[k];
  return r;
}

// The shifts of this iteration, from the first 64 queries (a function of this iteration's data
// only, so equal inputs give equal bits; every block and the last level compute the same values).
// Any finite shift is correct; one inside the bulk of the data keeps the sums at the scale of the
// data's spread instead of its offset (LAS-sized coordinates) or an outlier's (a far query whose
// residual is 1e10 would otherwise cancel every other pair's digits):
//   residuals: the smallest finite residual of the first 64 (outliers are large residuals);
//   pairs: the first VALID pair (d <= threshold) of the first 64, else query 0's.
// Computed by the block's first wave; `sm` (>= 6 doubles of LDS) carries them to the block.
__device__ double moment_shift_block(const double* dist, int64_t n, double* sm) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const double d = lane < n ? dist[lane] : __builtin_inf();
    const double m = wave_min_d(__builtin_isfinite(d) ? d : __builtin_inf());
    if (lane == 0) sm[0] = __builtin_isfinite(m) ? m : 0.0;
  }
  __syncthreads();
  const double c = sm[0];
  __syncthreads();
  return c;
}

// The pair-sum shift, once per iteration by the kernel that sets the threshold (its first wave),
// into it->cshift: the cull blocks and the last merge level read it from there.
__device__ void cov_shift_store(const double* x, const double* y, const double* z, const int32_t* pos,
                                const TgtPt* pts, int64_t n, double thr, IterDev* it) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double v[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    bool valid = false;
    if (lane < n) {
      const TgtPt p = pts[pos[lane]];
      v[0] = x[lane];
      v[1] = y[lane];
      v[2] = z[lane];
      v[3] = p.x;
      v[4] = p.y;
      v[5] = p.z;
      const double ex = v[3] - v[0], ey = v[4] - v[1], ez = v[5] - v[2];
      valid = __builtin_sqrt(ex * ex + ey * ey + ez * ez) <= thr;
    }
    const unsigned long long vm = __ballot(valid);
    const int src = vm ? __builtin_ctzll(vm) : 0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const double w = readlane_d(v[k], src);
      if (lane == 0) it->cshift[k] = __builtin_isfinite(w) ? w : 0.0;
    }
  }
}

// Fixed-shape merges of part sums, deterministic: the same n always gives the same merge tree.
// Inner levels: block b merges items [256 b, 256 b + 256), one per thread, pairwise in LDS. Last
// level: one block, up to 4096 items: thread t folds items t + 256 k (k < 16) in order, then the
// block's pairwise tree.
constexpr int kLastSpan = 4096;

// The pairwise tree over the block's 256 values: at step s, thread t with t % 2s == 0 merges
// t + s's value into its own. Steps 1..32 run inside each wave through shuffles, steps 64 and 128
// over the four wave results: the same merges in the same order as the tree in LDS this replaced
// (bit-identical), with 4 entries of LDS instead of 256 (so the cull blocks can run the last level
// themselves, k_cull_waves' fused tail).
template <typename T>
__device__ __forceinline__ T shfl_down_T(const T& v, int s) {
  static_assert(sizeof(T) % sizeof(double) == 0, "records of doubles");
  T r;
  const double* a = reinterpret_cast<const double*>(&v);
  double* b = reinterpret_cast<double*>(&r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / sizeof(double)); k++) b[k] = __shfl_down(a[k], s, kWave);
  return r;
}

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
__device__ __forceinline__ T block_tree(T v, T* sm) {
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
#pragma unroll
  for (int s = 1; s < kWave; s <<= 1) {
    const T o = shfl_down_T(v, s);
    if ((lane & (2 * s - 1)) == 0) v = Merge(v, o);
  }
  if (lane == 0) sm[w] = v;
  __syncthreads();
  const T r = Merge(Merge(sm[0], sm[1]), Merge(sm[2], sm[3]));
  __syncthreads();
  return r;
}

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
__device__ __forceinline__ T block_tree_last(const T* in, int64_t n, T* sm) {
  // No early exit: block_tree's barriers must be reached by every thread in uniform control flow.
  T acc = Identity();
#pragma unroll 4
  for (int k = 0; k < 16; k++) {
    const int64_t g = (int64_t)threadIdx.x + 256 * k;
    if (g < n) acc = Merge(acc, in[g]);
  }
  return block_tree<T, Merge, Identity>(acc, sm);
}

// The same last level over parts another workgroup of this launch stored with sc1 (write-through)
// stores: read with sc1 loads (L2-served, never a stale L1 line; microarch guide, hand-off row 1).
template <typename T>
__device__ __forceinline__ T load_sc1(const T* p) {
  T r;
  const double* a = reinterpret_cast<const double*>(p);
  double* b = reinterpret_cast<double*>(&r);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / sizeof(double)); k++)
    b[k] = __hip_atomic_load(a + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return r;
}
template <typename T>
__device__ __forceinline__ void store_sc1(T* p, const T& v) {
  const double* a = reinterpret_cast<const double*>(&v);
  double* b = reinterpret_cast<double*>(p);
#pragma unroll
  for (int k = 0; k < (int)(sizeof(T) / sizeof(double)); k++)
    __hip_atomic_store(b + k, a[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
__device__ __forceinline__ T block_tree_last_sc1(const T* in, int64_t n, T* sm) {
  T acc = Identity();
#pragma unroll 4
  for (int k = 0; k < 16; k++) {
    const int64_t g = (int64_t)threadIdx.x + 256 * k;
    if (g < n) acc = Merge(acc, load_sc1(in + g));
  }
  return block_tree<T, Merge, Identity>(acc, sm);
}

// "Last block done": thread 0 stores the block's part (sc1), waits for the store, then takes a
// ticket (agent-scope atomic adds, relaxed); the block whose ticket is the last one merges every
// part (sc1 loads, after the barrier that tells its other waves) and resets the counters for the
// next launch. Returns true in that block only. The hand-off needs no fence (microarch guide,
// inter-workgroup visibility, row 1): one lane per storing workgroup signals after its vmcnt
// wait, the consumer is the workgroup whose add came last. Saves the launch of the last level.
// The counter is sharded by blockIdx % 8 (one 128-B line per shard, the round-robin XCD of the
// block: speed only) with a top counter that the last arrival of each shard bumps: arrivals on
// one device-scope counter serialise at ~12 ns each (microarch guide, fanin), which cost 15 us
// for the 1221 cull blocks of a 1.25M shard with a single counter.
// Fused only for moderate grids: every block then pays a store wait and a returned atomic before
// it retires. Measured (one MI355X, interleaved, r18 with the former 1024-query cull blocks):
// 100k queries (25 moment parts, 98 cull blocks) -2 us per iteration; at 1221 cull blocks (a
// 1.25M shard) +15 us, at 2442 moment parts (10M) +5 us.
// the moments blocks: fused up to 512 parts (2M queries)
#ifndef ICP_FUSE_MOMENT_PARTS
#define ICP_FUSE_MOMENT_PARTS 512
#endif
constexpr int kFuseMaxMomentParts = ICP_FUSE_MOMENT_PARTS;
// the cull blocks (256 search waves each: 611 at 10M) up to 1024 blocks (16.7M queries)
constexpr int kFuseMaxCullBlocks = 1024;
constexpr int kTicketLine = 32;                      // uints per counter line (128 B)
constexpr int kTicketWords = 9 * kTicketLine;        // top + 8 shards
template <typename T>
__device__ __forceinline__ bool publish_part_last(T* part, const T& mine, unsigned* ticket, int* last_s) {
  if (threadIdx.x == 0) {
    store_sc1(part + blockIdx.x, mine);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned g = gridDim.x, sh = blockIdx.x & 7u;
    const unsigned in_shard = (g - sh + 7u) / 8u;  // blocks b < g with b % 8 == sh
    unsigned* sc = ticket + kTicketLine * (1 + sh);
    bool last = false;
    if (__hip_atomic_fetch_add(sc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_shard - 1u) {
      __hip_atomic_store(sc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned shards = g < 8u ? g : 8u;
      if (__hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == shards - 1u) {
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = true;
      }
    }
    *last_s = last ? 1 : 0;
  }
  __syncthreads();
  return *last_s != 0;
}

// Residual moments of the rank's queries in fixed parts of kMomPart queries, once every search
// kernel has written its residuals: deterministic whatever order the queries were settled in.
// Thread t of block p holds queries p kMomPart + t + 256 e (e < kMomPer, coalesced).
#ifndef ICP_MOM_PER
#define ICP_MOM_PER 16
#endif
constexpr int kMomPer = ICP_MOM_PER;
constexpr int kMomPart = 256 * kMomPer;

// mean = sum/row; std = sqrt(variance/row) (icpengine.cpp:235-245); threshold rule of the caller
__device__ void finalize_moments(IterDev* it, const Moments& g, const MomentsFinalize& f) {
  it->m_global = g;
  const double mean = g.mean;
  const double sd = __builtin_sqrt(g.m2 / g.n);
  it->mean = mean;
  it->sd = sd;
  it->thr = cull_threshold(mean, sd, f.k_sigma, f.iter, f.engine_rules);
}

// With the threshold known (every thread of the first wave calls it): the shift of the pair sums
// and the cull's mode. A band set by the previous iterate fixes the shift (the search summed with
// it); the wave records count when the search wrote them and the threshold lies inside the band.
__device__ void cull_params(IterDev* it, double thr, const CullLaunch& cl) {
  const bool fz = it->fz_ok != 0.0;
  if (fz) {
    if (threadIdx.x < 6) it->cshift[threadIdx.x] = it->fz_sh[threadIdx.x];
  } else {
    cov_shift_store(cl.x, cl.y, cl.z, cl.pos, cl.pts, cl.n, thr, it);
  }
  if (threadIdx.x == 0)
    it->cull_mode = (fz && cl.wstat != nullptr && it->fz_lo <= thr && thr <= it->fz_hi) ? 1.0 : 0.0;
}

// The band of the next iterate's search (thread 0, once the iterate is finished): around this
// threshold, as wide as twice its last relative change plus 5 % (at most 50 %; 25 % after a new
// source), with this iterate's pair shift.
__device__ void band_next(IterDev* it) {
  const double thr = it->thr;
  double delta = 0.25;
  if (it->fz_ok != 0.0 && it->fz_thr > 0.0) {
    const double r = thr / it->fz_thr - 1.0;
    delta = 2.0 * __builtin_fabs(r) + 0.05;
    delta = delta < 0.5 ? delta : 0.5;
  }
  bool fin = __builtin_isfinite(thr) && thr > 0.0 && delta == delta;
  for (int k = 0; k < 6; k++) {
    fin = fin && __builtin_isfinite(it->cshift[k]);
    it->fz_sh[k] = it->cshift[k];
  }
  it->fz_lo = thr * (1.0 - delta);
  it->fz_hi = thr * (1.0 + delta);
  it->fz_thr = thr;
  it->fz_ok = fin ? 1.0 : 0.0;
}

// The last level of the residual moments: the merged part sums -> (count, mean, M2) in
// it->m_local; with finalize (one rank, no communicator) also mean/std/threshold and the cull's
// pair shift. Run by k_merge_moments_last or by k_moments' last block (identical bits: the same
// tree over the same parts).
struct MomTail {
  unsigned* ticket;  // non-null: k_moments' last block runs the last level (<= kLastSpan parts)
  IterDev* it;
  MomentsFinalize fin;
  int finalize;
  CullLaunch cl;
};
__device__ void moments_last(const MomSums& r, double c, const MomTail& t) {
  __shared__ double thr_s;
  if (threadIdx.x == 0) {
    Moments m = moments_identity();
    if (r.n > 0.0) {
      m.n = r.n;
      m.mean = c + r.s1 / r.n;
      const double m2 = r.s2 - r.s1 * (r.s1 / r.n);
      m.m2 = m2 < 0.0 ? 0.0 : m2;  // rounding only; NaN propagates
      m.dmin = r.dmin;
      m.dmax = r.dmax;
    }
    m.nbad = r.nbad;
    t.it->m_local = m;
    if (t.finalize) {
      finalize_moments(t.it, m, t.fin);
      thr_s = t.it->thr;
    }
  }
  if (!t.finalize) return;
  __syncthreads();
  // the threshold, then the pair shift and the mode of the cull (the first wave)
  if (threadIdx.x < 64) cull_params(t.it, thr_s, t.cl);
}

template <bool FUSE>
__global__ void __launch_bounds__(256) k_moments(const double* __restrict__ dist, int64_t n, MomSums* part,
                                                const LoopDev* loop, MomTail tail) {
  if (loop && loop->core.done) return;  // the device loop's session finished (block-uniform)
  __shared__ double red[4 * 4];
  const double c = moment_shift_block(dist, n, red);
  const int64_t b0 = (int64_t)blockIdx.x * kMomPart + threadIdx.x;
  double v[4] = {0.0, 0.0, 0.0, 0.0};  // count, sum (d - c), sum (d - c)^2, non-finite
  double mn = 1.7976931348623157e308, mx = 0.0;
#pragma unroll
  for (int e = 0; e < kMomPer; e++) {
    const int64_t i = b0 + 256 * e;
    const bool act = i < n;
    const double d = act ? dist[i] : 0.0;
    const double dv = act ? d - c : 0.0;
    v[0] += act ? 1.0 : 0.0;
    v[1] += dv;
    v[2] += dv * dv;
    const bool fin = act && __builtin_isfinite(d);
    v[3] += (act && !fin) ? 1.0 : 0.0;
    mn = fin && d < mn ? d : mn;
    mx = fin && d > mx ? d : mx;
  }
  block_sum<4>(v, red);
  block_minmax(mn, mx, red);
  MomSums m;
  m.n = v[0];
  m.s1 = v[1];
  m.s2 = v[2];
  m.dmin = mn;
  m.dmax = mx;
  m.nbad = v[3];
  m.pad0 = m.pad1 = 0.0;
  if (!FUSE) {
    if (threadIdx.x == 0) part[blockIdx.x] = m;
    return;
  }
  __shared__ int last_s;
  if (!publish_part_last(part, m, tail.ticket, &last_s)) return;
  __shared__ MomSums sm[4];
  const MomSums r = block_tree_last_sc1<MomSums, momsum_merge, momsum_identity>(part, gridDim.x, sm);
  moments_last(r, c, tail);
}

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
__global__ void __launch_bounds__(256) k_tree_merge(const T* in, int64_t n, T* out) {
  __shared__ T sm[4];
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const T r = block_tree<T, Merge, Identity>(g < n ? in[g] : Identity(), sm);
  if (threadIdx.x == 0) out[blockIdx.x] = r;
}


// Last level of the rank's moments as its own launch (more than kLastSpan parts after the inner
// levels, or no ticket).
__global__ void __launch_bounds__(256) k_merge_moments_last(const MomSums* in, int64_t n, const double* dist,
                                                           int64_t nq, MomTail tail) {
  __shared__ MomSums sm[4];
  __shared__ double shs[1];
  const double c = moment_shift_block(dist, nq, shs);
  const MomSums r = block_tree_last<MomSums, momsum_merge, momsum_identity>(in, n, sm);
  moments_last(r, c, tail);
}

__global__ void __launch_bounds__(64) k_finalize_moments(const Moments* gathered, int nranks, IterDev* it,
                                                         MomentsFinalize fin, CullLaunch cl) {
  __shared__ double thr_s;
  if (threadIdx.x == 0) {
    Moments g = gathered[0];
    for (int r = 1; r < nranks; r++) g = moments_merge(g, gathered[r]);  // rank order: same bits everywhere
    finalize_moments(it, g, fin);
    thr_s = it->thr;
  }
  __syncthreads();
  cull_params(it, thr_s, cl);
}

// The device loop's step (one thread): the session's decisions on this iteration's finished
// record (session_step.h, the host loop's own function), then the iteration's LoopRec into pinned
// host memory (plain stores: the host reads it after synchronizing the stream).
__device__ void loop_step(LoopDev* L, const IterDev& r, LoopRec* out) {
  // fields stored one by one (a local LoopRec would live in scratch)
  out->n = r.m_global.n;
  out->mean = r.mean;
  out->sd = r.sd;
  out->thr = r.thr;
  out->valid = r.c_global.n;
  out->rmse = r.rmse;
  out->sum_d2 = r.c_global.sum_d2;
  out->dmin = r.m_global.dmin;
  out->dmax = r.m_global.dmax;
  out->nbad = r.m_global.nbad;
  for (int k = 0; k < 3; k++) {
    out->ma[k] = r.c_global.ma[k];
    out->mb[k] = r.c_global.mb[k];
    out->lists[k] = r.pad[k];
  }
  for (int k = 0; k < 9; k++) out->H[k] = r.c_global.c[k];
  SessionCore core = L->core;
  out->iter = core.iter;
  int32_t outcome = kStepNone;  // enqueued past the end of the session: nothing ran
  if (!core.done) {
    core.pending = 0;  // this iteration's search applied the pending increment
    outcome = session_core_step(core, L->p, r.rmse, (int64_t)r.c_global.n, r.c_global.ma, r.c_global.mb,
                                r.c_global.c);
    L->core = core;
  }
  out->outcome = outcome;
  out->pad[0] = (int32_t)r.n_wide;
  for (int k = 0; k < 16; k++) {
    out->T[k] = core.T[k];
    out->Tc[k] = core.Tc[k];
  }
}

// The iteration's record goes straight into the caller's pinned host buffer (no copy engine or
// blit launch on the critical path): the block copies the device record to LDS, thread 0
// completes it, the block stores it with system-scope relaxed stores, every thread waits for its
// stores to be acknowledged, then thread 0 stores the sequence word. No system-scope release
// fence: it would write back the whole L2, which the search has just dirtied with megabytes. The
// list sizes ride along (pad[0..2]) and are reset for the next search.
// LOOP = false: an instance without the device loop's step (the session decisions and the 3x3
// SVD): the cull kernel's fused tail, whose registers count for every cull block.
template <bool LOOP = true>
__device__ void finalize_cov_publish(IterDev* it, const CovMoments& g, IterPublish pub, IterDev* rec) {
  constexpr int kWords = (int)(sizeof(IterDev) / sizeof(double)) - 1;  // all but pad[3], the flag
  static_assert(offsetof(IterDev, pad) + 3 * sizeof(double) == kWords * sizeof(double), "flag is the last word");
  double* rw = reinterpret_cast<double*>(rec);
  const double* iw = reinterpret_cast<const double*>(it);
  for (int k = threadIdx.x; k < kWords + 1; k += blockDim.x) rw[k] = iw[k];  // the device record, in parallel
  __syncthreads();
  if (threadIdx.x == 0) {
    rec->c_global = g;
    rec->rmse = (g.n > 0) ? __builtin_sqrt(g.sum_d2 / g.n) : 0.0;  // icpengine.cpp:274-278
    // exact (the wave search's list + the ball search's DFS finishes), ball, per-lane
    rec->pad[0] = (double)(pub.lists[0] + pub.lists[3]);
    rec->pad[1] = (double)pub.lists[1];
    rec->pad[2] = (double)pub.lists[2];
    rec->n_wide = (double)pub.lists[6];
    for (int k = 0; k < 7; k++) pub.lists[k] = 0u;  // + the half and wide lists, overflowed waves
    it->c_global = rec->c_global;
    it->rmse = rec->rmse;
    band_next(it);
    if (LOOP && pub.loop) loop_step(pub.loop, *rec, pub.rec);
  }
  if (LOOP && pub.loop) return;  // the device loop: the host reads the batch's records after it
  __syncthreads();
  double* dst = reinterpret_cast<double*>(pub.host);
  for (int k = threadIdx.x; k < kWords; k += blockDim.x)
    __hip_atomic_store(dst + k, rw[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&pub.host->pad[3], pub.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The last level of the covariance sums: the merged part sums -> it->c_local; with finalize (one
// rank) also RMSE and the publish. Run by k_merge_cov_last or by k_cull_waves' last block.
struct CovTail {
  unsigned* ticket;  // non-null: k_cull_waves' last block runs the last level (<= kLastSpan blocks)
  IterPublish pub;
  int finalize;
};
template <bool LOOP>
__device__ void cov_last(const CovSums& r, const IterDev* shift_src, IterDev* it, const CovTail& t) {
  __shared__ IterDev rec;
  __shared__ CovMoments res;
  if (threadIdx.x == 0) {
    CovMoments m = cov_identity();
    if (r.n > 0.0) {
      m.n = r.n;
      m.sum_d2 = r.sum_d2;
      double da[3], db[3];
      for (int k = 0; k < 3; k++) {
        da[k] = r.sa[k] / r.n;
        db[k] = r.sb[k] / r.n;
        m.ma[k] = shift_src->cshift[k] + da[k];
        m.mb[k] = shift_src->cshift[3 + k] + db[k];
      }
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m.c[3 * i + j] = r.sab[3 * i + j] - r.n * (da[i] * db[j]);
    }
    it->c_local = m;
    res = m;
  }
  if (!t.finalize) return;
  __syncthreads();
  finalize_cov_publish<LOOP>(it, res, t.pub, &rec);
}

template <bool SC1>
__device__ CovSums fold_parts(const CovSums* in, int64_t n, double (*rows)[20], double* gsum);

// The last level of the cull's part sums as its own launch (the device loop; more than
// kFuseMaxCullBlocks blocks): fold_parts, the order of the fused last block.
__global__ void __launch_bounds__(256) k_merge_cov_last(const CovSums* in, int64_t n, IterDev* it, CovTail tail) {
  __shared__ __attribute__((aligned(16))) double rows[256][20];
  __shared__ double gsum[8 * 17];
  const CovSums r = fold_parts<false>(in, n, rows, gsum);
  cov_last<true>(r, it, it, tail);
}

__global__ void __launch_bounds__(64) k_finalize_cov(const CovMoments* gathered, int nranks, IterDev* it,
                                                     IterPublish pub) {
  __shared__ IterDev rec;
  CovMoments g = gathered[0];
  for (int r = 1; r < nranks; r++) g = cov_merge(g, gathered[r]);  // rank order
  finalize_cov_publish(it, g, pub, &rec);
}

// 3-sigma cull + covariance sums of up to kCullWaves search waves (64 queries each) per block:
//   1. the block's wave records (written by the search, cull_mode 1) are copied to LDS, coalesced;
//   2. the waves without one (flag 1; every wave in mode 0) are recomputed by one wave each with
//      the search's own function (wave_stats.h wave_cov_sums): against the band's lower end in
//      mode 1, against the threshold itself in mode 0 (no records, or the threshold left the band);
//   3. each wave's band pairs (mode 1) with d <= thr: added in lane order by its thread, or (many
//      band lanes) as one more canonical tree by a wave;
//   4. the block's column fold over its waves (fold_rows).
// So a wave's sums do not depend on which search settled which of its queries, nor on which
// block recomputed it. The residual is read, not recomputed: every search path stores
// d = sqrt(fl(dx^2 + dy^2 + dz^2)) (octree.cpp:139-144), and the pairs' terms use it as it is.
constexpr int kCullWaves = 256;  // search waves per block at most: one record row per thread
constexpr int kSeqBand = 8;      // band lanes a thread adds itself; more: a wave's tree

// One pair's terms added to a record row (16 sums in the record's order, then the count).
__device__ __forceinline__ void add_pair(double* row, double d, double qx, double qy, double qz, double mx, double my,
                                         double mz, const double* sh) {
  const double da[3] = {qx - sh[0], qy - sh[1], qz - sh[2]};
  const double db[3] = {mx - sh[3], my - sh[4], mz - sh[5]};
  row[0] += d * d;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    row[1 + r] += da[r];
    row[4 + r] += db[r];
  }
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) row[7 + 3 * r + c] += da[r] * db[c];
  row[16] += 1.0;
}

// Search waves per cull block for n queries: ~600 blocks up to 10M (611 at 10M; beyond, 256
// waves per block: 3052 blocks at 50M), at least 8 waves per block (a 100k cloud: 196 blocks;
// fewer, larger blocks left the small clouds' flagged waves to a handful of waves in sequence:
// +10 us per iterate at 100k).
#ifndef ICP_CULL_BLOCKS
#define ICP_CULL_BLOCKS 600
#endif
int cull_waves_per_block(int64_t n) {
  const int64_t nw = (n + 63) / 64;
  const int64_t w = (nw + ICP_CULL_BLOCKS - 1) / ICP_CULL_BLOCKS;
  return (int)(w < 8 ? 8 : w > kCullWaves ? kCullWaves : w);
}
constexpr int kRow = 20;         // doubles per row: the WaveStat layout (s[16], cnt, bm, flag, pad)
static_assert(sizeof(WaveStat) == kRow * sizeof(double), "rows are wave records");

// Column v of the 17 summed values in CovSums order (n, sum d^2, sa[3], sb[3], sab[9]) -> its
// index in a row.
__device__ __forceinline__ int row_col(int v) { return v == 0 ? 16 : v - 1; }

// The fixed-order column sums of the first `nrows` (<= 256, block-uniform) rows (LDS): thread
// 17 g + v (g < 8) adds column v of rows 32 g .. min(32 g + 31, nrows - 1) in order (0 for an
// empty group), then thread v adds the 8 group sums in order. Every thread of the (256-thread)
// block calls it; the result is the same for all. (A small cloud's cull blocks hold 8 waves:
// their fold reads those 8 rows, not 256.)
__device__ CovSums fold_rows(const double (*rows)[kRow], double* gsum, int nrows = 256) {
  const int t = threadIdx.x;
  if (t < 8 * 17) {
    const int g = t / 17, v = t % 17, c = row_col(v);
    const int r0 = 32 * g, r1 = r0 + 32 < nrows ? r0 + 32 : nrows;
    double acc = r0 < r1 ? rows[r0][c] : 0.0;
    for (int i = r0 + 1; i < r1; i++) acc += rows[i][c];
    gsum[g * 17 + v] = acc;
  }
  __syncthreads();
  __shared__ double col[17];
  if (t < 17) {
    double acc = gsum[t];
#pragma unroll
    for (int g = 1; g < 8; g++) acc += gsum[g * 17 + t];
    col[t] = acc;
  }
  __syncthreads();
  CovSums r;
  r.n = col[0];
  r.sum_d2 = col[1];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    r.sa[k] = col[2 + k];
    r.sb[k] = col[5 + k];
    r.pad[k] = 0.0;
  }
#pragma unroll
  for (int k = 0; k < 9; k++) r.sab[k] = col[8 + k];
  __syncthreads();
  return r;
}

// The last level over n <= 4096 part sums (the cull blocks'), the same in k_cull_waves' last
// block (SC1: parts other blocks of the launch stored with sc1 stores) and in k_merge_cov_last
// (the device loop's path): thread t adds parts t + 256 k in order into its row, then fold_rows.
template <bool SC1>
__device__ CovSums fold_parts(const CovSums* in, int64_t n, double (*rows)[kRow], double* gsum) {
  const int t = threadIdx.x;
  double acc[17];
#pragma unroll
  for (int v = 0; v < 17; v++) acc[v] = 0.0;
  for (int k = 0; k < 16; k++) {
    const int64_t g = (int64_t)t + 256 * k;
    if (g >= n) break;
    const CovSums c = SC1 ? load_sc1(in + g) : in[g];
    const double* cw = reinterpret_cast<const double*>(&c);
#pragma unroll
    for (int v = 0; v < 17; v++) acc[v] = k == 0 ? cw[v] : acc[v] + cw[v];
  }
#pragma unroll
  for (int v = 0; v < 17; v++) rows[t][row_col(v)] = acc[v];
  __syncthreads();
  return fold_rows(rows, gsum);
}

// FUSE: the last block runs the last merge level and (finalize) the publish; not with the device
// loop (whose step would put the SVD's registers into every cull block): that one keeps
// k_merge_cov_last.
template <bool FUSE>
__global__ void __launch_bounds__(256) k_cull_waves(CullLaunch a, CovTail tail) {
  if (a.loop && a.loop->core.done) return;  // the device loop's session finished (block-uniform)
  __shared__ __attribute__((aligned(16))) double rows[kCullWaves][kRow];
  __shared__ __attribute__((aligned(32))) double red[4][kStatLds / 8];
  __shared__ double gsum[8 * 17];
  __shared__ int list[kCullWaves];
  __shared__ int blist[kCullWaves];
  __shared__ int nlist, nblist;
  const IterDev* it = a.it;
  const double thr = it->thr;
  const bool fused = it->cull_mode != 0.0;
  const double lo = it->fz_lo, hi = it->fz_hi;
  double sh[6];
#pragma unroll
  for (int k = 0; k < 6; k++) sh[k] = it->cshift[k];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t nwaves = (a.n + 63) / 64;
  const int64_t w0 = (int64_t)blockIdx.x * a.wpb;
  const int nw = (int)(nwaves - w0 < a.wpb ? nwaves - w0 : a.wpb);  // this block's waves
  if (t == 0) nlist = 0;
  if (fused) {
    // the block's records, 16-B loads over the whole block (coalesced)
    const double2* src = reinterpret_cast<const double2*>(a.wstat + w0);
    double2* dst = reinterpret_cast<double2*>(&rows[0][0]);
    for (int k = t; k < nw * (kRow / 2); k += 256) dst[k] = src[k];
  }
  __syncthreads();
  if (t < kCullWaves) {
    const bool need = t < nw && (!fused || reinterpret_cast<const unsigned long long*>(rows[t])[18] != 0ull);
    if (t >= nw) {
#pragma unroll
      for (int k = 0; k < kRow; k++) rows[t][k] = 0.0;
    }
    if (need) list[atomicAdd(&nlist, 1)] = t;  // any order: each entry is one wave's own row
  }
  __syncthreads();
  const int nl = nlist;
  // software-pipelined: the next wave's residual, query and position are loaded while this
  // one's match is gathered and summed (one dependent round trip per wave instead of three)
  double cd = 0.0, cx = 0.0, cy = 0.0, cz = 0.0;
  int32_t cp = 0;
  auto load = [&](int e) {
    const int64_t i = (w0 + list[e]) * 64 + lane;
    const bool act = i < a.n;
    cd = act ? a.dist[i] : 0.0;
    cx = act ? a.x[i] : 0.0;
    cy = act ? a.y[i] : 0.0;
    cz = act ? a.z[i] : 0.0;
    cp = act ? a.pos[i] : 0;
  };
  if (wv < nl) load(wv);
  for (int e = wv; e < nl; e += 4) {
    const int tt = list[e];
    const int64_t i = (w0 + tt) * 64 + lane;
    const bool active = i < a.n;
    const double d = cd, qx = cx, qy = cy, qz = cz;
    const int32_t ps = cp;
    const bool in = active && (fused ? d <= lo : d <= thr);
    const bool band = fused && active && !(d <= lo) && d <= hi;
    double mx = 0.0, my = 0.0, mz = 0.0;
    if (in) {
      const TgtPt* p = a.pts + ps;
      const double2 xy = *reinterpret_cast<const double2*>(&p->x);
      mx = xy.x;
      my = xy.y;
      mz = p->z;
    }
    if (e + 4 < nl) load(e + 4);
    const double r = wave_cov_sums(in, d, qx, qy, qz, mx, my, mz, sh, red[wv], lane);
    const unsigned long long am = __ballot(in), bm = __ballot(band);
    if (lane < 16) rows[tt][lane] = r;
    if (lane == 0) {
      rows[tt][16] = (double)__popcll(am);
      reinterpret_cast<unsigned long long*>(rows[tt])[17] = bm;
    }
  }
  __syncthreads();
  // the band pairs below the threshold. A wave with at most kSeqBand band lanes: its thread adds
  // them to its row in lane order (one gather chain each, usually 0 or 1); a wave with more: one
  // more canonical tree (the same function, over its band lanes with d <= thr) added to its row
  // by one wave of the block (its band lanes in parallel). Which one is a function of the wave's
  // band mask, so the bits stay a function of the data.
  if (t == 0) nblist = 0;
  __syncthreads();
  if (fused && t < nw) {
    unsigned long long bm = reinterpret_cast<const unsigned long long*>(rows[t])[17];
    if (__popcll(bm) > kSeqBand) {
      blist[atomicAdd(&nblist, 1)] = t;
    } else if (bm) {
      double* row = rows[t];
      const int64_t base = (w0 + t) * 64;
      while (bm) {
        const int l = __builtin_ctzll(bm);
        bm &= bm - 1ull;
        const int64_t i = base + l;
        const double d = a.dist[i];
        if (d <= thr) {  // icpengine.cpp:265
          const TgtPt* p = a.pts + a.pos[i];
          add_pair(row, d, a.x[i], a.y[i], a.z[i], p->x, p->y, p->z, sh);
        }
      }
    }
  }
  __syncthreads();
  const int nb = nblist;
  for (int e = wv; e < nb; e += 4) {
    const int tt = blist[e];
    const unsigned long long bm = reinterpret_cast<const unsigned long long*>(rows[tt])[17];
    const int64_t i = (w0 + tt) * 64 + lane;
    const bool inb = (bm >> lane) & 1ull;  // band lanes are active lanes
    const double d = inb ? a.dist[i] : 0.0;
    const bool in = inb && d <= thr;  // icpengine.cpp:265
    double qx = 0.0, qy = 0.0, qz = 0.0, mx = 0.0, my = 0.0, mz = 0.0;
    if (in) {
      qx = a.x[i];
      qy = a.y[i];
      qz = a.z[i];
      const TgtPt* p = a.pts + a.pos[i];
      const double2 xy = *reinterpret_cast<const double2*>(&p->x);
      mx = xy.x;
      my = xy.y;
      mz = p->z;
    }
    const double r = wave_cov_sums(in, d, qx, qy, qz, mx, my, mz, sh, red[wv], lane);
    const int cnt = __popcll(__ballot(in));
    if (lane < 16) rows[tt][lane] = rows[tt][lane] + r;
    if (lane == 0) rows[tt][16] = rows[tt][16] + (double)cnt;
  }
  __syncthreads();
  const CovSums r = fold_rows(rows, gsum, a.wpb);
  CovSums* part = reinterpret_cast<CovSums*>(a.part);
  if (!FUSE) {
    if (t == 0) part[blockIdx.x] = r;
    return;
  }
  __shared__ int last_s;
  if (!publish_part_last(part, r, tail.ticket, &last_s)) return;
  const CovSums rr = fold_parts<true>(part, gridDim.x, rows, gsum);
  cov_last<false>(rr, a.it, const_cast<IterDev*>(a.it), tail);
}

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
const T* merge_to_last_span(const T* part, int64_t* nparts, hipStream_t s) {
  // part -> scratch levels (right behind the partials) until the last block's span is left
  const T* cur = part;
  T* next = const_cast<T*>(part) + *nparts;
  int64_t cn = *nparts;
  while (cn > kLastSpan) {
    const int64_t nb = (cn + 255) / 256;
    hipLaunchKernelGGL((k_tree_merge<T, Merge, Identity>), dim3((unsigned)nb), dim3(256), 0, s, cur, cn, next);
    cur = next;
    next += nb;
    cn = nb;
  }
  *nparts = cn;
  return cur;
}

}  // namespace

int ticket_words() { return 2 * kTicketWords; }

// Partial buffers hold the block partials followed by the merge scratch (merge_scratch_entries).
int64_t merge_scratch_entries(int64_t nparts) {
  int64_t total = 0;
  for (int64_t cn = nparts; cn > kLastSpan; cn = (cn + 255) / 256) total += (cn + 255) / 256;
  return total + 1;
}

int64_t moments_num_parts(int64_t n) { return (n + kMomPart - 1) / kMomPart; }

hipError_t launch_moments_tail(const double* dist, int64_t n, Moments* part, const LoopDev* loop, unsigned* ticket,
                               IterDev* it, const MomentsFinalize* fin, const CullLaunch& cl, hipStream_t s) {
  const int64_t nparts = moments_num_parts(n);
  MomTail tail{nullptr, it, fin ? *fin : MomentsFinalize{0.0, 0, 0}, fin ? 1 : 0, cl};
  MomSums* sums = reinterpret_cast<MomSums*>(part);
  if (ticket && nparts >= 1 && nparts <= kFuseMaxMomentParts) {  // one launch: the last block merges
    tail.ticket = ticket;
    hipLaunchKernelGGL(k_moments<true>, dim3((unsigned)nparts), dim3(256), 0, s, dist, n, sums, loop, tail);
    return hipGetLastError();
  }
  if (n > 0) hipLaunchKernelGGL(k_moments<false>, dim3((unsigned)nparts), dim3(256), 0, s, dist, n, sums, loop, tail);
  int64_t np = nparts;
  const MomSums* cur = merge_to_last_span<MomSums, momsum_merge, momsum_identity>(sums, &np, s);
  hipLaunchKernelGGL(k_merge_moments_last, dim3(1), dim3(256), 0, s, cur, np, dist, n, tail);
  return hipGetLastError();
}

hipError_t launch_finalize_moments(const Moments* gathered, int nranks, IterDev* it, MomentsFinalize fin,
                                   const CullLaunch& cl, hipStream_t s) {
  hipLaunchKernelGGL(k_finalize_moments, dim3(1), dim3(64), 0, s, gathered, nranks, it, fin, cl);
  return hipGetLastError();
}

int64_t cull_num_blocks(int64_t n) {
  const int w = cull_waves_per_block(n);
  return ((n + 63) / 64 + w - 1) / w;
}

hipError_t launch_cull_tail(const CullLaunch& a_in, unsigned* ticket, const IterPublish* pub, hipStream_t s) {
  CullLaunch a = a_in;
  a.wpb = cull_waves_per_block(a.n);
  const int64_t nb = cull_num_blocks(a.n);
  CovTail tail{nullptr, pub ? *pub : IterPublish{nullptr, nullptr, 0.0, nullptr, nullptr}, pub ? 1 : 0};
  if (ticket && nb >= 1 && nb <= kFuseMaxCullBlocks && !a.loop) {  // one launch: the last block merges and publishes
    tail.ticket = ticket;
    hipLaunchKernelGGL(k_cull_waves<true>, dim3((unsigned)nb), dim3(256), 0, s, a, tail);
    return hipGetLastError();
  }
  if (a.n > 0) hipLaunchKernelGGL(k_cull_waves<false>, dim3((unsigned)nb), dim3(256), 0, s, a, tail);
  int64_t np = nb;
  const CovSums* cur = merge_to_last_span<CovSums, covsum_merge, covsum_identity>(
      reinterpret_cast<const CovSums*>(a.part), &np, s);
  hipLaunchKernelGGL(k_merge_cov_last, dim3(1), dim3(256), 0, s, cur, np, const_cast<IterDev*>(a.it), tail);
  return hipGetLastError();
}

hipError_t launch_finalize_cov(const CovMoments* gathered, int nranks, IterDev* it, IterPublish pub,
                               hipStream_t s) {
  hipLaunchKernelGGL(k_finalize_cov, dim3(1), dim3(64), 0, s, gathered, nranks, it, pub);
  return hipGetLastError();
}

}  // namespace icp
