// kernels.hip — gfx950 (CDNA4) kernels of the ICP correspondence-and-alignment path.
//
//  k_nn        one thread per source query: (optional) rigid transform of the query in place,
//              exact depth-first octree search with a per-thread level stack in LDS, residual
//              d = |q - t|, per-block residual moments (count, mean, M2, min, max, #non-finite).
//              Reproduces Octree::searchNearest (core/octree.cpp:128-184) bit for bit: same
//              box-distance arithmetic with its sqrt, same prune test m*m >= best, children
//              visited in stable ascending-distance order, strict < in the leaf scan.
//  k_cull_cov  3-sigma cull (icpengine.cpp:263-278) + valid-pair centroids and centered
//              cross-covariance per block (icpengine.cpp:76-90), two passes over registers.
//  k_merge_*   fixed-shape tree merges of block partials (Chan et al.), deterministic.
//  k_finalize_* rank-ordered merge of the gathered per-rank partials, threshold, RMSE.
//
// Everything is fp64 and compiled with -ffp-contract=off: the reference is built without FMA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstddef>

#include "kernels.h"

namespace icp {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ double box_dist(double lx, double ly, double lz, double hx, double hy,
                                           double hz, double qx, double qy, double qz) {
  // OctreeNode::minDistanceTo (octree.cpp:32-38)
  const double dx = smax(0.0, smax(lx - qx, qx - hx));
  const double dy = smax(0.0, smax(ly - qy, qy - hy));
  const double dz = smax(0.0, smax(lz - qz, qz - hz));
  return __builtin_sqrt(dx * dx + dy * dy + dz * dz);
}

// Wave-wide reductions and scans on DPP (row shifts within 16-lane rows, then row_bcast15/31
// across rows), no LDS traffic. Must be called with every lane of the wave active.
template <int CTRL, int RM, bool ZERO>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = (int)(unsigned)b, hi = (int)(b >> 32);
  const int rlo = __builtin_amdgcn_update_dpp(ZERO ? 0 : lo, lo, CTRL, RM, 0xf, ZERO);
  const int rhi = __builtin_amdgcn_update_dpp(ZERO ? 0 : hi, hi, CTRL, RM, 0xf, ZERO);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)rhi << 32) | (unsigned)rlo));
}
__device__ __forceinline__ double lane63_d(double v) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0x111, 0xf, true>(v);
  v += dpp_d<0x112, 0xf, true>(v);
  v += dpp_d<0x114, 0xf, true>(v);
  v += dpp_d<0x118, 0xf, true>(v);
  v += dpp_d<0x142, 0xa, true>(v);
  v += dpp_d<0x143, 0xc, true>(v);
  return lane63_d(v);
}
__device__ __forceinline__ double dmin_(double a, double b) { return b < a ? b : a; }
__device__ __forceinline__ double dmax_(double a, double b) { return b > a ? b : a; }
__device__ __forceinline__ double wave_min_d(double v) {
  v = dmin_(v, dpp_d<0x111, 0xf, false>(v));
  v = dmin_(v, dpp_d<0x112, 0xf, false>(v));
  v = dmin_(v, dpp_d<0x114, 0xf, false>(v));
  v = dmin_(v, dpp_d<0x118, 0xf, false>(v));
  v = dmin_(v, dpp_d<0x142, 0xa, false>(v));
  v = dmin_(v, dpp_d<0x143, 0xc, false>(v));
  return lane63_d(v);
}
__device__ __forceinline__ double wave_max_d(double v) {
  v = dmax_(v, dpp_d<0x111, 0xf, false>(v));
  v = dmax_(v, dpp_d<0x112, 0xf, false>(v));
  v = dmax_(v, dpp_d<0x114, 0xf, false>(v));
  v = dmax_(v, dpp_d<0x118, 0xf, false>(v));
  v = dmax_(v, dpp_d<0x142, 0xa, false>(v));
  v = dmax_(v, dpp_d<0x143, 0xc, false>(v));
  return lane63_d(v);
}
// Inclusive prefix sum over the wave's lanes; *total = the wave's sum (uniform).
__device__ __forceinline__ int wave_incl_scan(int v, int* total) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  *total = __builtin_amdgcn_readlane(v, 63);
  return v;
}

template <int N>
__device__ __forceinline__ void block_sum(double (&v)[N], double* red) {
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = wave_sum_d(v[k]);
  const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave, nw = blockDim.x / kWave;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; k++) red[w * N + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++) {
    double s = red[k];
    for (int j = 1; j < nw; j++) s += red[j * N + k];
    v[k] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ void block_minmax(double& mn, double& mx, double* red) {
  mn = wave_min_d(mn);
  mx = wave_max_d(mx);
  const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave, nw = blockDim.x / kWave;
  if (lane == 0) {
    red[2 * w] = mn;
    red[2 * w + 1] = mx;
  }
  __syncthreads();
  mn = red[0];
  mx = red[1];
  for (int j = 1; j < nw; j++) {
    mn = red[2 * j] < mn ? red[2 * j] : mn;
    mx = red[2 * j + 1] > mx ? red[2 * j + 1] : mx;
  }
  __syncthreads();
}

// Stack entry: bits 0..31 first child record, bits 32..55 up to 8 pending children as 3-bit
// ranks inside the contiguous child block (next child in the low bits), bits 56..59 count.
__device__ __forceinline__ uint64_t pack_entry(int32_t first, uint32_t ranks, uint32_t cnt) {
  return ((uint64_t)(ranks | (cnt << 24)) << 32) | (uint32_t)first;
}

template <bool APPLY>
__device__ __forceinline__ void nn_load_query(const NNLaunch& a, int64_t i, bool active, double& qx, double& qy,
                                              double& qz) {
  if (!active) return;
  qx = a.x[i];
  qy = a.y[i];
  qz = a.z[i];
  if (APPLY) {
    // src = T * src, Eigen order ((T0 x + T1 y) + T2 z) + T3 (icpengine.cpp:345)
    const double nx = ((a.T[0] * qx + a.T[1] * qy) + a.T[2] * qz) + a.T[3];
    const double ny = ((a.T[4] * qx + a.T[5] * qy) + a.T[6] * qz) + a.T[7];
    const double nz = ((a.T[8] * qx + a.T[9] * qy) + a.T[10] * qz) + a.T[11];
    a.x[i] = nx;
    a.y[i] = ny;
    a.z[i] = nz;
    qx = nx;
    qy = ny;
    qz = nz;
  }
}

// Residual, outputs, per-block residual moments (and work counters in COUNT mode).
template <bool COUNT>
__device__ __forceinline__ void nn_finish(const NNLaunch& a, int64_t i, bool active, double qx, double qy,
                                          double qz, int32_t best, double best_d2, double visits, double scanned,
                                          unsigned long long* lds_stack) {
  int32_t pos = best;
  double d = 0.0;
  if (active) {
    if (best >= 0) {
      d = __builtin_sqrt(best_d2);  // == computeDistance(src, tgt) bit for bit
    } else {
      // findNearest returned its default index 0 (octree.cpp:179); distance to that point.
      pos = a.pos0;
      const TgtPt p = a.pts[pos];
      const double dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
      d = __builtin_sqrt(dx * dx + dy * dy + dz * dz);
    }
    a.pos_out[i] = pos;
    a.dist_out[i] = d;
  }

  __syncthreads();  // every traversal is done: reuse the stack LDS for the reductions
  double* red = reinterpret_cast<double*>(lds_stack);
  if (a.part) {
    double s1[2] = {active ? 1.0 : 0.0, active ? d : 0.0};
    block_sum<2>(s1, red);
    const double nb = s1[0];
    const double mean = s1[1] / nb;
    const double dev = active ? (d - mean) : 0.0;
    const bool fin = active && __builtin_isfinite(d);
    double s2[2] = {dev * dev, (active && !fin) ? 1.0 : 0.0};
    block_sum<2>(s2, red);
    double mn = fin ? d : 1.7976931348623157e308, mxv = fin ? d : 0.0;
    block_minmax(mn, mxv, red);
    if (threadIdx.x == 0) {
      Moments m;
      m.n = nb;
      m.mean = mean;
      m.m2 = s2[0];
      m.dmin = mn;
      m.dmax = mxv;
      m.nbad = s2[1];
      m.pad0 = 0.0;
      m.pad1 = 0.0;
      a.part[blockIdx.x] = m;
    }
  }
  if (COUNT) {
    double c[2] = {visits, scanned};
    block_sum<2>(c, red);
    if (threadIdx.x == 0) {
      atomicAdd(&a.counters[0], (unsigned long long)c[0]);
      atomicAdd(&a.counters[1], (unsigned long long)c[1]);
    }
  }
}

// The reference DFS (Octree::searchNearest, octree.cpp:128-173) for one query, verbatim order:
// box distance with its sqrt, prune m*m >= best, children in stable ascending-distance order,
// strict < in leaf scans. `st` is this thread's column of the LDS level stack (stride bs).
template <bool COUNT>
__device__ __forceinline__ void exact_dfs(const NNLaunch& a, double qx, double qy, double qz, unsigned long long* st,
                                          int bs, int32_t& best, double& best_d2, double& visits,
                                          double& scanned) {
  int sp = 0;
  int32_t node = 0;
  bool siblings_on_top = false;
  if (COUNT) visits += 1.0;
  while (true) {
    const NodeRec* r = a.nodes + node;
    const double2 l01 = *reinterpret_cast<const double2*>(&r->lo[0]);
    const double2 l2h0 = *reinterpret_cast<const double2*>(&r->lo[2]);
    const double2 h12 = *reinterpret_cast<const double2*>(&r->hi[1]);
    const int4 topo = *reinterpret_cast<const int4*>(&r->first);
    const double lx = l01.x, ly = l01.y, lz = l2h0.x, hx = l2h0.y, hy = h12.x, hz = h12.y;
    const double m = box_dist(lx, ly, lz, hx, hy, hz, qx, qy, qz);
    const int32_t first = topo.x;
    const uint32_t meta = (uint32_t)topo.y;
    if (m * m >= best_d2) {
      // Pruned (octree.cpp:134-135). Siblings still pending on the top level come later in
      // ascending distance, so they would all be pruned too: drop the level (exact).
      if (siblings_on_top) sp--;
    } else if (meta & kLeafBit) {
      const int32_t cnt = (int32_t)(meta & ~kLeafBit);
      if (COUNT) scanned += (double)cnt;
      for (int32_t k = 0; k < cnt; k++) {
        const TgtPt* p = a.pts + first + k;
        const double2 pxy = *reinterpret_cast<const double2*>(&p->x);
        const double pz = p->z;
        const double dx = pxy.x - qx;
        const double dy = pxy.y - qy;
        const double dz = pz - qz;
        const double d2 = dx * dx + dy * dy + dz * dz;
        if (d2 < best_d2) {  // strict <, ascending original index inside a leaf
          best_d2 = d2;
          best = first + k;
        }
      }
    } else {
      // Inner node: distances of the existing children from the parent box and its
      // midpoint (the stored child boxes are exactly these values, octree.cpp:97-120).
      const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
      const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
      const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
      const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
      const double sx[2] = {ax0 * ax0, ax1 * ax1};
      const double sy[2] = {ay0 * ay0, ay1 * ay1};
      const double sz[2] = {az0 * az0, az1 * az1};
      const uint32_t mask = meta & 0xffu;
      double cd[8];
#pragma unroll
      for (int o = 0; o < 8; o++) cd[o] = __builtin_sqrt(sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2]);
      // Stable order = sort by (distance, octant): rank = #children strictly before.
      uint32_t rk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int p = 0; p < 8; p++) {
#pragma unroll
        for (int q = p + 1; q < 8; q++) {
          const bool both = ((mask >> p) & 1u) && ((mask >> q) & 1u);
          const bool q_first = cd[q] < cd[p];
          rk[p] += (both && q_first) ? 1u : 0u;
          rk[q] += (both && !q_first) ? 1u : 0u;
        }
      }
      uint32_t ranks = 0;
#pragma unroll
      for (int o = 0; o < 8; o++) {
        if ((mask >> o) & 1u) {
          const uint32_t block_slot = (uint32_t)__builtin_popcount(mask & ((1u << o) - 1u));
          ranks |= block_slot << (3u * rk[o]);
        }
      }
      const uint32_t nch = (uint32_t)__builtin_popcount(mask);
      if (COUNT) visits += (double)nch;
      node = first + (int32_t)(ranks & 7u);
      if (nch > 1) {
        st[sp * bs] = pack_entry(first, ranks >> 3, nch - 1);
        sp++;
        siblings_on_top = true;
      } else {
        siblings_on_top = false;
      }
      continue;
    }
    if (sp == 0) break;
    const unsigned long long e = st[(sp - 1) * bs];
    const int32_t base = (int32_t)(uint32_t)e;
    const uint32_t hi = (uint32_t)(e >> 32);
    const uint32_t rem = (hi >> 24) - 1u;
    node = base + (int32_t)(hi & 7u);
    if (rem == 0) {
      sp--;
      siblings_on_top = false;
    } else {
      st[(sp - 1) * bs] = pack_entry(base, (hi & 0xffffffu) >> 3, rem);
      siblings_on_top = true;
    }
  }
}

template <bool APPLY, bool COUNT>
__global__ void __launch_bounds__(256) k_nn(NNLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const int bs = blockDim.x;
  const int64_t i = (int64_t)blockIdx.x * bs + threadIdx.x;
  const bool active = i < a.n;

  double qx = 0.0, qy = 0.0, qz = 0.0;
  nn_load_query<APPLY>(a, i, active, qx, qy, qz);

  double best_d2 = a.init_best;
  int32_t best = -1;
  double visits = 0.0, scanned = 0.0;
  // A NaN coordinate makes every leaf distance NaN, so the reference never updates best_idx
  // (octree.cpp:146): skipping the search is exact. (Its box distances stay finite: max(0,NaN)=0.)
  const bool nan_q = (qx != qx) || (qy != qy) || (qz != qz);
  if (active && !nan_q && a.n_nodes > 0)
    exact_dfs<COUNT>(a, qx, qy, qz, lds_stack + threadIdx.x, bs, best, best_d2, visits, scanned);
  nn_finish<COUNT>(a, i, active, qx, qy, qz, best, best_d2, visits, scanned, lds_stack);
}

// Exact form of the prune test m*m >= best with m = sqrt(s) (octree.cpp:134-135), without the
// sqrt in the common case: fl(fl(sqrt(s))^2) lies within a relative 3*2^-53 of s, so outside a
// 2^-48 band around best (normal range) the answer is decided by s alone; inside it, the
// reference arithmetic is evaluated literally.
__device__ __forceinline__ bool prune_test(double s, double best) {
  constexpr double kTiny = 0x1p-900;
  if (s >= kTiny) {
    if (s > best * (1.0 + 0x1p-48)) return true;
    if (best >= kTiny && s < best * (1.0 - 0x1p-48)) return false;
  }
  const double m = __builtin_sqrt(s);
  return m * m >= best;
}

// v2: same DFS as k_nn with
//  * prune_test() instead of a sqrt per node entry;
//  * children ranked by their squared box distance s (ties -> lower octant); sqrt is monotone,
//    so this equals the reference's stable sort on sqrt(s) unless two distinct s collide under
//    sqrt, which needs them within 2^-51 relative: such near-ties switch to ranking by sqrt(s);
//  * the nearest child is entered straight from registers: its box is the parent box split at
//    the midpoint (the stored child boxes are exactly these values), so only its 8-byte
//    topology word is loaded. Popped siblings load their 48-byte box.
template <bool APPLY, bool COUNT>
__global__ void __launch_bounds__(256) k_nn2(NNLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const int bs = blockDim.x;
  const int64_t i = (int64_t)blockIdx.x * bs + threadIdx.x;
  const bool active = i < a.n;

  double qx = 0.0, qy = 0.0, qz = 0.0;
  nn_load_query<APPLY>(a, i, active, qx, qy, qz);

  double best_d2 = a.init_best;
  int32_t best = -1;
  double visits = 0.0, scanned = 0.0;
  const bool nan_q = (qx != qx) || (qy != qy) || (qz != qz);  // see k_nn
  if (active && !nan_q && a.n_nodes > 0) {
    unsigned long long* st = lds_stack + threadIdx.x;
    int sp = 0;
    int32_t node = 0;
    bool siblings_on_top = false;
    bool have_box = false;  // box registers + s valid for `node`
    double lx = 0, ly = 0, lz = 0, hx = 0, hy = 0, hz = 0, s_node = 0;
    if (COUNT) visits += 1.0;
    while (true) {
      const NodeRec* r = a.nodes + node;
      if (!have_box) {
        const double2 l01 = *reinterpret_cast<const double2*>(&r->lo[0]);
        const double2 l2h0 = *reinterpret_cast<const double2*>(&r->lo[2]);
        const double2 h12 = *reinterpret_cast<const double2*>(&r->hi[1]);
        lx = l01.x; ly = l01.y; lz = l2h0.x; hx = l2h0.y; hy = h12.x; hz = h12.y;
        const double dx = smax(0.0, smax(lx - qx, qx - hx));
        const double dy = smax(0.0, smax(ly - qy, qy - hy));
        const double dz = smax(0.0, smax(lz - qz, qz - hz));
        s_node = dx * dx + dy * dy + dz * dz;
      }
      bool descend = false;
      if (prune_test(s_node, best_d2)) {
        // every pending sibling is at least as far: the reference would prune them all
        if (siblings_on_top) sp--;
      } else {
        const int2 topo = *reinterpret_cast<const int2*>(&r->first);
        const int32_t first = topo.x;
        const uint32_t meta = (uint32_t)topo.y;
        if (meta & kLeafBit) {
          const int32_t cnt = (int32_t)(meta & ~kLeafBit);
          if (COUNT) scanned += (double)cnt;
          for (int32_t k = 0; k < cnt; k++) {
            const TgtPt* p = a.pts + first + k;
            const double2 pxy = *reinterpret_cast<const double2*>(&p->x);
            const double pz = p->z;
            const double dx = pxy.x - qx;
            const double dy = pxy.y - qy;
            const double dz = pz - qz;
            const double d2 = dx * dx + dy * dy + dz * dz;
            if (d2 < best_d2) {
              best_d2 = d2;
              best = first + k;
            }
          }
        } else {
          const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
          const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
          const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
          const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
          const double sx[2] = {ax0 * ax0, ax1 * ax1};
          const double sy[2] = {ay0 * ay0, ay1 * ay1};
          const double sz[2] = {az0 * az0, az1 * az1};
          const uint32_t mask = meta & 0xffu;
          double cs[8], clo[8];
#pragma unroll
          for (int o = 0; o < 8; o++) {
            cs[o] = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
            clo[o] = cs[o] * (1.0 - 0x1p-48);
          }
          uint32_t rk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          bool hazard = false;
#pragma unroll
          for (int p = 0; p < 8; p++) {
#pragma unroll
            for (int q = p + 1; q < 8; q++) {
              const bool both = ((mask >> p) & 1u) && ((mask >> q) & 1u);
              const bool q_first = cs[q] < cs[p];
              hazard |= both && q_first && !(cs[q] < clo[p]);
              rk[p] += (both && q_first) ? 1u : 0u;
              rk[q] += (both && !q_first) ? 1u : 0u;
            }
          }
          if (hazard) {  // near-tie under sqrt: rank exactly as the reference (sqrt keys)
            double cd[8];
#pragma unroll
            for (int o = 0; o < 8; o++) cd[o] = __builtin_sqrt(cs[o]);
#pragma unroll
            for (int o = 0; o < 8; o++) rk[o] = 0;
#pragma unroll
            for (int p = 0; p < 8; p++) {
#pragma unroll
              for (int q = p + 1; q < 8; q++) {
                const bool both = ((mask >> p) & 1u) && ((mask >> q) & 1u);
                const bool q_first = cd[q] < cd[p];
                rk[p] += (both && q_first) ? 1u : 0u;
                rk[q] += (both && !q_first) ? 1u : 0u;
              }
            }
          }
          uint32_t ranks = 0, oct0 = 0;
#pragma unroll
          for (int o = 0; o < 8; o++) {
            if ((mask >> o) & 1u) {
              const uint32_t slot = (uint32_t)__builtin_popcount(mask & ((1u << o) - 1u));
              ranks |= slot << (3u * rk[o]);
              if (rk[o] == 0) oct0 = (uint32_t)o;
            }
          }
          const uint32_t nch = (uint32_t)__builtin_popcount(mask);
          if (COUNT) visits += (double)nch;
          // enter the nearest child from registers (octree.cpp:115-120 boxes)
          node = first + (int32_t)(ranks & 7u);
          s_node = cs[oct0];
          if (oct0 & 1u) lx = mx; else hx = mx;
          if (oct0 & 2u) ly = my; else hy = my;
          if (oct0 & 4u) lz = mz; else hz = mz;
          have_box = true;
          descend = true;
          if (nch > 1) {
            st[sp * bs] = pack_entry(first, ranks >> 3, nch - 1);
            sp++;
            siblings_on_top = true;
          } else {
            siblings_on_top = false;
          }
        }
      }
      if (descend) continue;
      if (sp == 0) break;
      const unsigned long long e = st[(sp - 1) * bs];
      const int32_t base = (int32_t)(uint32_t)e;
      const uint32_t hi = (uint32_t)(e >> 32);
      const uint32_t rem = (hi >> 24) - 1u;
      node = base + (int32_t)(hi & 7u);
      have_box = false;
      if (rem == 0) {
        sp--;
        siblings_on_top = false;
      } else {
        st[(sp - 1) * bs] = pack_entry(base, (hi & 0xffffffu) >> 3, rem);
        siblings_on_top = true;
      }
    }
  }
  nn_finish<COUNT>(a, i, active, qx, qy, qz, best, best_d2, visits, scanned, lds_stack);
}

// ---------------------------------------------------------------------------------------------
// v3: certified fast search + exact fallback.
//
// Claim (the basis of the fast path): let d* = fl(d2) of the nearest target point p* and assume
// no other point has fl(d2) <= d* (1 + 2^-48), d* in [2^-900, 2^900] and d* < init (1 - 2^-48)
// (or d* = 0 with no other zero). Then the reference DFS returns p*, whatever its visit order:
//  * rounding is monotone, so for a point p inside a box, fl(d2(p)) >= fl(s(box)) (same
//    operation sequence on coordinates that are at least as far), and the reference's prune
//    value fl(fl(sqrt(s))^2) <= s (1 + 3.0001 * 2^-53) <= d* (1 + 3.0001 * 2^-53);
//  * so a node holding p* can only be pruned against a best within that factor of d*, i.e. by
//    another point inside the window — there is none; p* is scanned, strict < takes it, and no
//    later point can replace it.
// The fast kernel therefore finds d*, p* and the second-smallest distance in ANY order — nearest
// child first, remaining siblings in octant order, levels dropped on a 16-bit lower-bound key —
// pruning only nodes whose s exceeds best (1 + 2^-47) (which keeps every point of the window
// visible), and certifies each query by the window test. Queries that fail it (exact or near
// ties, duplicates, far queries, tiny/huge distances) are appended to a list and re-run by the
// exact reference-order DFS (k_nn_fallback). Non-finite queries are answered directly: NaN gives
// NaN leaf distances and inf an infinite root distance, so the reference keeps index 0.

constexpr double kWindow = 0x1p-48;
constexpr double kFastPrune = 0x1p-47;

__device__ __forceinline__ double box_s(double lx, double ly, double lz, double hx, double hy, double hz,
                                        double qx, double qy, double qz) {
  const double dx = smax(0.0, smax(lx - qx, qx - hx));
  const double dy = smax(0.0, smax(ly - qy, qy - hy));
  const double dz = smax(0.0, smax(lz - qz, qz - hz));
  return dx * dx + dy * dy + dz * dz;
}

// 16-bit truncation of a non-negative double: a monotone lower bound (top 16 bits of the bits).
__device__ __forceinline__ uint32_t key16(double v) {
  return (uint32_t)((unsigned long long)__double_as_longlong(v) >> 48);
}

__device__ __forceinline__ bool certified(double best, double second, double init_best) {
  if (best == 0.0) return second > 0.0;
  return best >= 0x1p-900 && best <= 0x1p900 && second > best * (1.0 + kWindow) &&
         best < init_best * (1.0 - kWindow);
}

// Append the lanes with `want` to a list, one atomic per wave, lane order kept (the lists stay
// in Morton order wave by wave, which keeps the follow-up searches coherent). Wave-uniform call.
__device__ __forceinline__ void wave_append(bool want, int64_t i, unsigned* counter, int32_t* list) {
  const unsigned long long m = __ballot(want);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(m);
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m));
  base = (unsigned)__builtin_amdgcn_readlane((int)base, leader);
  const int off = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  if (want) list[base + off] = (int32_t)i;
}

// wave_append that also stores a per-entry payload (the guess u of the ball search).
__device__ __forceinline__ void wave_append_u(bool want, int64_t i, double u, unsigned* counter, int32_t* list,
                                              double* payload) {
  const unsigned long long m = __ballot(want);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(m);
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m));
  base = (unsigned)__builtin_amdgcn_readlane((int)base, leader);
  const int off = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
  if (want) {
    list[base + off] = (int32_t)i;
    payload[base + off] = u;
  }
}

// Per-lane certified search (the fast path of one query): nearest child first, remaining
// siblings in octant order, level drop on the 16-bit key; tracks best, second best, position.
__device__ __forceinline__ void fast_dfs(const NNLaunch& a, double qx, double qy, double qz,
                                         unsigned long long* st, int bs, double& best, double& second,
                                         int32_t& bpos, uint32_t& nvis, uint32_t& npts) {
  double thr = __builtin_inf();
  uint32_t thr_key = key16(__builtin_inf());
  int sp = 0;
  int32_t node = 0;
  const NodeRec* r0 = a.nodes;
  double lx = r0->lo[0], ly = r0->lo[1], lz = r0->lo[2], hx = r0->hi[0], hy = r0->hi[1], hz = r0->hi[2];
  double s = box_s(lx, ly, lz, hx, hy, hz, qx, qy, qz);
  while (true) {
    bool entered = false;
    if (!(s > thr)) {
      const int2 topo = *reinterpret_cast<const int2*>(&a.nodes[node].first);
      const int32_t first = topo.x;
      const uint32_t meta = (uint32_t)topo.y;
      nvis++;
      if (meta & kLeafBit) {
        const int32_t cnt = (int32_t)(meta & ~kLeafBit);
        npts += (uint32_t)cnt;
        for (int32_t k = 0; k < cnt; k++) {
          const TgtPt* p = a.pts + first + k;
          const double2 pxy = *reinterpret_cast<const double2*>(&p->x);
          const double pz = p->z;
          const double dx = pxy.x - qx;
          const double dy = pxy.y - qy;
          const double dz = pz - qz;
          const double d2 = dx * dx + dy * dy + dz * dz;
          if (d2 < best) {
            second = best;
            best = d2;
            bpos = first + k;
            thr = best * (1.0 + kFastPrune);
            thr_key = key16(thr);
          } else if (d2 < second) {
            second = d2;
          }
        }
      } else {
        const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
        const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
        const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
        const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
        const double sx[2] = {ax0 * ax0, ax1 * ax1};
        const double sy[2] = {ay0 * ay0, ay1 * ay1};
        const double sz[2] = {az0 * az0, az1 * az1};
        const uint32_t mask = meta & 0xffu;
        // nearest existing child (first minimum in octant order) and the smallest key of the rest
        double bs_ = __builtin_inf();
        uint32_t o1 = 0;
#pragma unroll
        for (int o = 0; o < 8; o++) {
          const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
          const bool take = ((mask >> o) & 1u) && c < bs_;
          bs_ = take ? c : bs_;
          o1 = take ? (uint32_t)o : o1;
        }
        const uint32_t rem = mask & ~(1u << o1);
        uint32_t kmin = 0xffffu;
#pragma unroll
        for (int o = 0; o < 8; o++) {
          const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
          const uint32_t kk = key16(c);
          kmin = ((rem >> o) & 1u) && kk < kmin ? kk : kmin;
        }
        if (rem) {
          st[sp * bs] = ((unsigned long long)kmin << 48) | ((unsigned long long)mask << 40) |
                        ((unsigned long long)rem << 32) | (uint32_t)first;
          sp++;
        }
        node = first + __builtin_popcount(mask & ((1u << o1) - 1u));
        if (o1 & 1u) lx = mx; else hx = mx;
        if (o1 & 2u) ly = my; else hy = my;
        if (o1 & 4u) lz = mz; else hz = mz;
        s = bs_;
        entered = true;
      }
    }
    if (entered) continue;
    bool found = false;
    while (sp > 0) {
      const unsigned long long e = st[(sp - 1) * bs];
      if ((uint32_t)(e >> 48) > thr_key) {  // every remaining child is beyond the threshold
        sp--;
        continue;
      }
      uint32_t rem = (uint32_t)(e >> 32) & 0xffu;
      const uint32_t pmask = (uint32_t)(e >> 40) & 0xffu;
      const int32_t first = (int32_t)(uint32_t)e;
      const uint32_t o = (uint32_t)__builtin_ctz(rem);
      rem &= rem - 1u;
      if (rem == 0) sp--;
      else st[(sp - 1) * bs] = (e & ~(0xffull << 32)) | ((unsigned long long)rem << 32);
      node = first + __builtin_popcount(pmask & ((1u << o) - 1u));
      const NodeRec* r = a.nodes + node;
      const double2 l01 = *reinterpret_cast<const double2*>(&r->lo[0]);
      const double2 l2h0 = *reinterpret_cast<const double2*>(&r->lo[2]);
      const double2 h12 = *reinterpret_cast<const double2*>(&r->hi[1]);
      lx = l01.x; ly = l01.y; lz = l2h0.x; hx = l2h0.y; hy = h12.x; hz = h12.y;
      s = box_s(lx, ly, lz, hx, hy, hz, qx, qy, qz);
      found = true;
      break;
    }
    if (!found) break;
  }
}

// Fast-path stack entry: bits 0..31 first child record, 32..39 remaining octants,
// 40..47 the parent's child mask, 48..63 key16 lower bound of the remaining children's s.
template <bool APPLY>
__global__ void __launch_bounds__(256) k_nn3(NNLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const int bs = blockDim.x;
  const int64_t i = (int64_t)blockIdx.x * bs + threadIdx.x;
  const bool active = i < a.n;

  double qx = 0.0, qy = 0.0, qz = 0.0;
  nn_load_query<APPLY>(a, i, active, qx, qy, qz);
  const bool finite_q = __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz);

  double best = __builtin_inf(), second = __builtin_inf();
  int32_t bpos = -1;
  uint32_t nvis = 0, npts = 0;
  if (active && finite_q) fast_dfs(a, qx, qy, qz, lds_stack + threadIdx.x, bs, best, second, bpos, nvis, npts);
  bool ok = true;
  int32_t pos = bpos;
  double d = 0.0;
  if (active) {
    if (!finite_q) {
      pos = a.pos0;  // findNearest keeps its default index 0 (see above)
      const TgtPt p = a.pts[pos];
      const double dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
      d = __builtin_sqrt(dx * dx + dy * dy + dz * dz);
    } else {
      ok = certified(best, second, a.init_best);
      d = __builtin_sqrt(best);
    }
    if (ok) {
      a.pos_out[i] = pos;
      a.dist_out[i] = d;
    }
  }
  wave_append(active && !ok, i, a.fb_count, a.fb_list);
  // residual moments over the certified queries of this block (launch_nn passes part = null:
  // k_moments computes them once every search kernel has written its queries)
  if (!a.part) return;
  __syncthreads();
  double* red = reinterpret_cast<double*>(lds_stack);
  const bool use = active && ok;
  double s1[2] = {use ? 1.0 : 0.0, use ? d : 0.0};
  block_sum<2>(s1, red);
  const double nb = s1[0];
  const double mean = nb > 0.0 ? s1[1] / nb : 0.0;
  const double dev = use ? (d - mean) : 0.0;
  const bool fin = use && __builtin_isfinite(d);
  double s2[2] = {dev * dev, (use && !fin) ? 1.0 : 0.0};
  block_sum<2>(s2, red);
  double mn = fin ? d : 1.7976931348623157e308, mxv = fin ? d : 0.0;
  block_minmax(mn, mxv, red);
  if (threadIdx.x == 0) {
    Moments m;
    m.n = nb;
    m.mean = mean;
    m.m2 = s2[0];
    m.dmin = mn;
    m.dmax = mxv;
    m.nbad = s2[1];
    m.pad0 = 0.0;
    m.pad1 = 0.0;
    a.part[blockIdx.x] = m;
  }
}

// Exact reference-order DFS for the queries the fast path could not certify.
__global__ void __launch_bounds__(256) k_nn_fallback(NNLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const unsigned cnt = *a.fb_count;
  for (unsigned j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt; j += gridDim.x * blockDim.x) {
    const int64_t i = a.fb_list[j];
    const double qx = a.x[i], qy = a.y[i], qz = a.z[i];
    double best_d2 = a.init_best, visits = 0.0, scanned = 0.0;
    int32_t best = -1;
    exact_dfs<false>(a, qx, qy, qz, lds_stack + threadIdx.x, blockDim.x, best, best_d2, visits, scanned);
    int32_t pos = best;
    double d;
    if (best >= 0) {
      d = __builtin_sqrt(best_d2);
    } else {
      pos = a.pos0;
      const TgtPt p = a.pts[pos];
      const double dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
      d = __builtin_sqrt(dx * dx + dy * dy + dz * dz);
    }
    a.pos_out[i] = pos;
    a.dist_out[i] = d;
  }
}

// Rank-level reductions as shifted plain sums. A part holds sums of values shifted by a constant
// of the iteration (query 0's residual, source point and match), so the sums stay at the spread
// of the data, not at its offset (LAS-sized coordinates), and the merge tree is plain additions
// in a fixed order: deterministic and cheap.
// The last level turns them into (count, mean, M2) and (count, means, co-moment) records, which
// ranks merge with the Chan formulas (icp_common.h).
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

// The shifts of this iteration: query 0's residual, its source point and its match (a function of
// this iteration's data only, so equal inputs give equal bits; every block and the last level
// compute the same values). Any finite shift is correct; one inside the data keeps the sums at
// the scale of the data's spread.
__device__ __forceinline__ double moment_shift(const double* dist, int64_t n) {
  const double d0 = n > 0 ? dist[0] : 0.0;
  return __builtin_isfinite(d0) ? d0 : 0.0;
}
__device__ __forceinline__ void cov_shift(const double* x, const double* y, const double* z, const int32_t* pos,
                                          const TgtPt* pts, int64_t n, double sh[6]) {
  for (int k = 0; k < 6; k++) sh[k] = 0.0;
  if (n <= 0) return;
  const TgtPt p = pts[pos[0]];
  const double v[6] = {x[0], y[0], z[0], p.x, p.y, p.z};
  for (int k = 0; k < 6; k++) sh[k] = __builtin_isfinite(v[k]) ? v[k] : 0.0;
}

// Residual moments of the rank's queries in fixed parts of kMomPart queries, once every search
// kernel has written its residuals: deterministic whatever order the queries were settled in.
// Thread t of block p holds queries p kMomPart + t + 256 e (e < kMomPer, coalesced).
constexpr int kMomPer = 16;
constexpr int kMomPart = 256 * kMomPer;

__global__ void __launch_bounds__(256) k_moments(const double* __restrict__ dist, int64_t n, const IterDev* it,
                                                 MomSums* part) {
  __shared__ double red[4 * 4];
  const double c = moment_shift(dist, n);
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
  if (threadIdx.x == 0) {
    MomSums m;
    m.n = v[0];
    m.s1 = v[1];
    m.s2 = v[2];
    m.dmin = mn;
    m.dmax = mx;
    m.nbad = v[3];
    m.pad0 = m.pad1 = 0.0;
    part[blockIdx.x] = m;
  }
}

// ---------------------------------------------------------------------------------------------
// v4: wave-cooperative certified search.
//
// The 64 queries of a wave are Morton neighbours. Each lane first descends (nearest child, no
// backtracking) to a leaf and scans it: u = an actual point's fl(d2), an upper bound of its
// nearest distance. Lanes whose radius r = sqrt(u)(1 + 2^-40) + |q| 2^-45 is at most 3x the
// wave's mean radius (NNLaunch::join_factor, ICP_JOIN) join one search box B = bbox of [q - r, q + r]; the wave collects every leaf
// whose box meets B by a cooperative breadth-first walk (frontier and leaf list in LDS), then
// all lanes scan those points in lockstep (wave-uniform loop, uniform addresses). Each joined
// lane's ball of radius r lies in B, so every point with fl(d2) <= best (1 + 2^-48) is among
// the scanned ones and the window certificate of k_nn3 applies unchanged. Lanes that do not
// join (outliers: far from the surface, or a wave whose candidate set overflows LDS) are queued
// for the per-lane certified search (k_nn_lists); uncertified ones for the exact DFS.

// Workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8 labels the blocks that share
// one XCD and its 4 MB L2; cdna_hip_programming.md T1). Renumbered so that each such set takes
// one contiguous range of the grid: the source is in kd-bucket order, so the blocks resident on
// one XCD cover one compact region of space and share its L2 for the node and point gathers.
// Bijective for any grid size (the first nb % 8 sets hold one block more). Speed only.
__device__ __forceinline__ int64_t xcd_block(int remap) {
  const uint32_t b = blockIdx.x;
  if (!remap) return b;
  const uint32_t nb = gridDim.x, set = b & 7u, q = nb >> 3, r = nb & 7u;
  return (int64_t)set * q + (set < r ? set : r) + (b >> 3);
}

constexpr int kWaveQueue = 256;     // node ids in the walk's circular work queue
constexpr int kMaxGroups = 8;       // lane groups of the scan (GL = 8 lanes at the finest)
// per wave: the walk's work queue (reused as the staging area once the walk is done: 64 fp32
// points or 32 fp64 points), the candidate list, the group boxes and the group index lists.
// 1 KB + 4 KB at PL = 1024: 20 KB per 4-wave block, 8 blocks (8 waves per SIMD) per CU.
__host__ __device__ constexpr int wave_lds_bytes(int gl, int pl) {
  return kWaveQueue * 4 + pl * 4 + (gl < 64 ? kMaxGroups * 64 * 2 + 64 * 32 : 0);
}
static_assert(kWaveQueue * 4 >= 64 * 16 && kWaveQueue * 4 >= 32 * 32, "staging area aliases the queue");

// Lower bound of fl64(d2) of every point whose fp32 squared distance (scan of k_nn4) is >= s32.
// Coordinates are offsets from B's centre, |offset| <= ext for points and joined queries. With
// u = 2^-24: each fp32 offset differs from the exact one by <= ext (u + 2^-53) =: ext k; the fp32
// difference dx' = (p' - q')(1 + e), |e| <= u, so |dx' - dx| <= 2 ext k + u |dx| + ..., and over three
// axes |‖d'‖ - D| <= e_abs + u D with e_abs = sqrt(3) 2 ext k (1 + u). The fp32 sum of squares
// (one mul, two fma) is ‖d'‖^2 (1 + t), |t| <= (1 + u)^3 - 1, plus <= 3 2^-126 of underflow. Hence
// D >= (sqrt((s32 - 2^-120) / (1 + 3.0001 u)) - e_abs) / (1 + u), and fl64(d2) >= D^2 (1 - 5 2^-53).
// Every step below rounds towards the bound by an explicit 2^-50 margin.
__device__ __forceinline__ double scan32_lower_bound(float s32, double ext) {
  if (!(s32 < __builtin_inff())) return __builtin_inf();
  const double u = 0x1p-24;
  const double e_abs = 1.7320509 * 2.0 * ext * (u * (1.0 + 0x1p-20)) * (1.0 + u) * (1.0 + 0x1p-40);
  double n2 = ((double)s32 - 0x1p-120) / (1.0 + 3.0001 * u);
  if (!(n2 > 0.0)) return 0.0;
  const double n = __builtin_sqrt(n2) * (1.0 - 0x1p-50);
  double d = (n - e_abs) / (1.0 + u) * (1.0 - 0x1p-50);
  if (!(d > 0.0)) return 0.0;
  return d * d * (1.0 - 0x1p-48);
}

// Bits 0..9 of v spread to bits 0, 3, 6, ... (one axis of an octant path prefix).
__device__ __forceinline__ uint32_t spread3(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }


// Start nodes of a box query from the cell tables: the cells of level L (the octree's own
// midpoint grid) that the box [bl, bh] overlaps, one lane each. Per axis, the cell index of a
// coordinate is the bit path of its comparisons with the successive midpoints (x > mid goes
// high, octree.cpp:105-108), monotone in the coordinate, so the box's cells are an index box
// [il, ih]^3, every one of them meets the box, and every target point inside the box lies in
// one of them; the table gives the node holding all points of a cell (the depth-L node or the
// leaf above it; a leaf spanning several cells is queued once, from its first cell in the box).
// L is the deepest table level at which the box spans at most 64 cells. Writes the start nodes
// to out[0 .. count) and returns count (wave-uniform). Every lane of the wave must call it.
__device__ __forceinline__ int cell_starts(const NNLaunch& a, double blx, double bly, double blz, double bhx,
                                           double bhy, double bhz, int lane, int32_t* out) {
  int L = a.cell_lmax;
  uint32_t path = 0;
  if (lane < 6) {
    const int ax = lane >> 1;
    const double v = (lane & 1) ? (ax == 0 ? bhx : ax == 1 ? bhy : bhz) : (ax == 0 ? blx : ax == 1 ? bly : blz);
    double lo = ax == 0 ? a.root_lo[0] : ax == 1 ? a.root_lo[1] : a.root_lo[2];
    double hi = ax == 0 ? a.root_hi[0] : ax == 1 ? a.root_hi[1] : a.root_hi[2];
    for (int l = 0; l < L; l++) {
      const double m = (lo + hi) / 2;
      const bool up = v > m;
      path = 2u * path + (up ? 1u : 0u);
      lo = up ? m : lo;
      hi = up ? hi : m;
    }
  }
  uint32_t ilx = (uint32_t)__builtin_amdgcn_readlane((int)path, 0), ihx = (uint32_t)__builtin_amdgcn_readlane((int)path, 1);
  uint32_t ily = (uint32_t)__builtin_amdgcn_readlane((int)path, 2), ihy = (uint32_t)__builtin_amdgcn_readlane((int)path, 3);
  uint32_t ilz = (uint32_t)__builtin_amdgcn_readlane((int)path, 4), ihz = (uint32_t)__builtin_amdgcn_readlane((int)path, 5);
  while (L > 0 && (ihx - ilx + 1) * (ihy - ily + 1) * (ihz - ilz + 1) > 64) {
    L--;
    ilx >>= 1; ihx >>= 1; ily >>= 1; ihy >>= 1; ilz >>= 1; ihz >>= 1;
  }
  const uint32_t nx = ihx - ilx + 1, ny = ihy - ily + 1, nz = ihz - ilz + 1;
  bool put = false;
  int32_t node = 0;
  if ((uint32_t)lane < nx * ny * nz) {
    const uint32_t cx = ilx + (uint32_t)lane % nx, cy = ily + ((uint32_t)lane / nx) % ny,
                   cz = ilz + (uint32_t)lane / (nx * ny);
    const uint32_t prefix = spread3(cx) | (spread3(cy) << 1) | (spread3(cz) << 2);
    const int32_t e = a.cells[(((int64_t)1 << (3 * L)) - 1) / 7 + prefix];
    if (e >= 0) {
      node = e >> 5;
      const int sh = L - (e & 31);
      const uint32_t fx = ((cx >> sh) << sh) > ilx ? ((cx >> sh) << sh) : ilx;
      const uint32_t fy = ((cy >> sh) << sh) > ily ? ((cy >> sh) << sh) : ily;
      const uint32_t fz = ((cz >> sh) << sh) > ilz ? ((cz >> sh) << sh) : ilz;
      put = cx == fx && cy == fy && cz == fz;
    }
  }
  const unsigned long long pm = __ballot(put);
  if (put) out[__builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0))] = node;
  return __popcll(pm);
}

// GL = lanes per scan group. GL = 64: the wave scans every staged point of its box B. GL < 64:
// the wave's lanes form 64/GL aligned kd sub-buckets (query order), each with its own box
// B_g (union of its joined lanes' balls, inside B); a lane scans only the staged points of its
// group's box, the groups in parallel, so the lockstep loop runs max_g |B_g ∩ chunk| times.
template <bool APPLY, int GL, int PL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) k_nn4(NNLaunch a) {
  static_assert(GL == 64 || (GL >= 8 && 64 % GL == 0), "lane group size");
  constexpr int G = 64 / GL;
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t blk = xcd_block(a.xcd_remap);
  const int64_t i = blk * blockDim.x + threadIdx.x;
  const bool active = i < a.n;
  unsigned char* wl = reinterpret_cast<unsigned char*>(lds_stack) + wv * wave_lds_bytes(GL, PL);
  int32_t* queue = reinterpret_cast<int32_t*>(wl);
  double4* stage = reinterpret_cast<double4*>(wl);                  // after the walk only
  int32_t* plist = queue + kWaveQueue;                              // candidate points
  double* gbox = reinterpret_cast<double*>(plist + PL);    // G x 8 doubles
  unsigned char* gidx = reinterpret_cast<unsigned char*>(gbox + 8 * kMaxGroups);  // G x 64
  // GL < 64: a full 64-point fp64 staging area of its own, after the group lists
  if constexpr (GL < 64) stage = reinterpret_cast<double4*>(gidx + kMaxGroups * 64);

  double qx = 0.0, qy = 0.0, qz = 0.0, ox = 0.0, oy = 0.0, oz = 0.0;
  if (active) {
    ox = a.x[i];
    oy = a.y[i];
    oz = a.z[i];
  }
  nn_load_query<APPLY>(a, i, active, qx, qy, qz);
  const bool finite_q = __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz);

  const unsigned long long t_p0 = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
  // Phase 1: a guess u of the nearest squared distance. After an iteration on the same queries:
  // (previous residual + displacement of the query)^2, by the triangle inequality (any guess is
  // safe: certification below also requires best <= u). Otherwise descend (nearest child, no
  // backtracking) to one leaf and take its smallest d2 (a true upper bound).
  double u = __builtin_inf();
  if (active && finite_q && a.have_prev) {
    const double dp = a.dist_out[i];
    const double ex = qx - ox, ey = qy - oy, ez = qz - oz;
    const double g = dp + __builtin_sqrt(ex * ex + ey * ey + ez * ez);
    u = (g * g) * (1.0 + 0x1p-30);
  } else if (active && finite_q) {
    const NodeRec* r0 = a.nodes;
    double lx = r0->lo[0], ly = r0->lo[1], lz = r0->lo[2], hx = r0->hi[0], hy = r0->hi[1], hz = r0->hi[2];
    int32_t node = 0;
    while (true) {
      const int2 topo = *reinterpret_cast<const int2*>(&a.nodes[node].first);
      const uint32_t meta = (uint32_t)topo.y;
      if (meta & kLeafBit) {
        const int32_t cnt = (int32_t)(meta & ~kLeafBit);
        for (int32_t k = 0; k < cnt; k++) {
          const TgtPt* p = a.pts + topo.x + k;
          const double dx = p->x - qx, dy = p->y - qy, dz = p->z - qz;
          const double d2 = dx * dx + dy * dy + dz * dz;
          u = d2 < u ? d2 : u;
        }
        break;
      }
      const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
      const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
      const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
      const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
      const double sx[2] = {ax0 * ax0, ax1 * ax1};
      const double sy[2] = {ay0 * ay0, ay1 * ay1};
      const double sz[2] = {az0 * az0, az1 * az1};
      const uint32_t mask = meta & 0xffu;
      double bs_ = __builtin_inf();
      uint32_t o1 = 0;
#pragma unroll
      for (int o = 0; o < 8; o++) {
        const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
        const bool take = ((mask >> o) & 1u) && c < bs_;
        bs_ = take ? c : bs_;
        o1 = take ? (uint32_t)o : o1;
      }
      node = topo.x + __builtin_popcount(mask & ((1u << o1) - 1u));
      if (o1 & 1u) lx = mx; else hx = mx;
      if (o1 & 2u) ly = my; else hy = my;
      if (o1 & 4u) lz = mz; else hz = mz;
    }
  }

  // Phase 2: the wave's search box over the lanes that join.
  const bool cand = active && finite_q && u <= 0x1p900;
  const double amax = __builtin_fmax(__builtin_fabs(qx), __builtin_fmax(__builtin_fabs(qy), __builtin_fabs(qz)));
  const double r = cand ? __builtin_sqrt(u) * (1.0 + 0x1p-40) + amax * 0x1p-45 : 0.0;
  const unsigned long long cmask = __ballot(cand);
  const double mean_r = wave_sum_d(r) / (double)(cmask ? __popcll(cmask) : 1);
  bool join = cand && r <= a.join_factor * mean_r;
  const double blx = wave_min_d(join ? qx - r : __builtin_inf());
  const double bly = wave_min_d(join ? qy - r : __builtin_inf());
  const double blz = wave_min_d(join ? qz - r : __builtin_inf());
  const double bhx = wave_max_d(join ? qx + r : -__builtin_inf());
  const double bhy = wave_max_d(join ? qy + r : -__builtin_inf());
  const double bhz = wave_max_d(join ? qz + r : -__builtin_inf());
  if constexpr (GL < 64) {
    auto gmin = [](double v) {
#pragma unroll
      for (int off = GL / 2; off >= 1; off >>= 1) {
        const double o = __shfl_xor(v, off, kWave);
        v = o < v ? o : v;
      }
      return v;
    };
    auto gmax = [](double v) {
#pragma unroll
      for (int off = GL / 2; off >= 1; off >>= 1) {
        const double o = __shfl_xor(v, off, kWave);
        v = o > v ? o : v;
      }
      return v;
    };
    const double g0 = gmin(join ? qx - r : __builtin_inf());
    const double g1 = gmin(join ? qy - r : __builtin_inf());
    const double g2 = gmin(join ? qz - r : __builtin_inf());
    const double g3 = gmax(join ? qx + r : -__builtin_inf());
    const double g4 = gmax(join ? qy + r : -__builtin_inf());
    const double g5 = gmax(join ? qz + r : -__builtin_inf());
    if ((lane & (GL - 1)) == 0) {
      double* gb = gbox + 8 * (lane / GL);
      gb[0] = g0;
      gb[1] = g1;
      gb[2] = g2;
      gb[3] = g3;
      gb[4] = g4;
      gb[5] = g5;
    }
  }

  const unsigned long long t_p2 = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
  unsigned long long t_pd = t_p2;
  // Phase 3: cooperative breadth-first collection of the leaves meeting B.
  int nleaf = 0;
  bool overflow = false;
  if (__ballot(join) != 0) {
    // Wave-uniform descent to the deepest node that holds every leaf meeting B: follow the
    // only child meeting B while there is exactly one (the top levels of the walk, where a
    // whole 64-lane round would test a single node). All values here are wave-uniform.
    int32_t start = 0;
    int tail = 1;
    if (a.cells) {
      tail = cell_starts(a, blx, bly, blz, bhx, bhy, bhz, lane, queue);
      if (a.dbg && lane == 0) atomicAdd(&a.dbg[21], (unsigned long long)tail);
    } else if (a.lca_descent) {
      while (true) {
        const NodeRec* rr = a.nodes + start;
        const int2 topo = *reinterpret_cast<const int2*>(&rr->first);
        const uint32_t meta = (uint32_t)topo.y;
        if (meta & kLeafBit) break;
        const double lx = rr->lo[0], ly = rr->lo[1], lz = rr->lo[2], hx = rr->hi[0], hy = rr->hi[1], hz = rr->hi[2];
        const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
        const bool x0 = lx <= bhx && mx >= blx, x1 = mx <= bhx && hx >= blx;
        const bool y0 = ly <= bhy && my >= bly, y1 = my <= bhy && hy >= bly;
        const bool z0 = lz <= bhz && mz >= blz, z1 = mz <= bhz && hz >= blz;
        const uint32_t mask = meta & 0xffu;
        uint32_t kids = 0;
#pragma unroll
        for (int o = 0; o < 8; o++) {
          const bool hit = ((o & 1) ? x1 : x0) && ((o & 2) ? y1 : y0) && ((o & 4) ? z1 : z0);
          kids |= (hit && ((mask >> o) & 1u)) ? (1u << o) : 0u;
        }
        kids = (uint32_t)__builtin_amdgcn_readfirstlane((int)kids);
        if (__builtin_popcount(kids) != 1) break;
        const uint32_t o = (uint32_t)__builtin_ctz(kids);
        start = __builtin_amdgcn_readfirstlane(topo.x + __builtin_popcount(mask & ((1u << o) - 1u)));
        if (a.dbg && lane == 0) atomicAdd(&a.dbg[21], 1ull);
      }
    }
    if (a.dbg) t_pd = __builtin_amdgcn_s_memtime();
    // Work stack (kWaveQueue entries): every batch pops up to 64 nodes, which already meet B
    // (tested by their parent; the start nodes by the descent or the cell box), appends the
    // points of its leaves to the candidate list and pushes its children meeting B. Popping the
    // most recent nodes first keeps the live set small (depth-first in wave-wide batches).
    if (!a.cells && lane == 0) queue[0] = start;
    wave_lds_fence();
    while (tail > 0) {
      const int batch = tail < 64 ? tail : 64;
      const bool has = lane < batch;
      bool leaf = false;
      int32_t first = 0;
      uint32_t meta = 0, kids = 0;
      if (has) {
        const NodeRec* rr = a.nodes + queue[tail - batch + lane];
        const int2 topo = *reinterpret_cast<const int2*>(&rr->first);
        first = topo.x;
        meta = (uint32_t)topo.y;
        leaf = (meta & kLeafBit) != 0;
        if (!leaf) {
          const double2 l01 = *reinterpret_cast<const double2*>(&rr->lo[0]);
          const double2 l2h0 = *reinterpret_cast<const double2*>(&rr->lo[2]);
          const double2 h12 = *reinterpret_cast<const double2*>(&rr->hi[1]);
          const double lx = l01.x, ly = l01.y, lz = l2h0.x, hx = l2h0.y, hy = h12.x, hz = h12.y;
          const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
          // child o spans [lo or mid, mid or hi] per axis (octree.cpp:115-120)
          const bool x0 = lx <= bhx && mx >= blx, x1 = mx <= bhx && hx >= blx;
          const bool y0 = ly <= bhy && my >= bly, y1 = my <= bhy && hy >= bly;
          const bool z0 = lz <= bhz && mz >= blz, z1 = mz <= bhz && hz >= blz;
          const uint32_t mask = meta & 0xffu;
#pragma unroll
          for (int o = 0; o < 8; o++) {
            const bool hit = ((o & 1) ? x1 : x0) && ((o & 2) ? y1 : y0) && ((o & 4) ? z1 : z0);
            kids |= (hit && ((mask >> o) & 1u)) ? (1u << o) : 0u;
          }
        }
      }
      // a leaf contributes its points (contiguous in leaf order) to the candidate list
      const int lcnt = (has && leaf) ? (int)(meta & ~kLeafBit) : 0;
      int ltot;
      const int lincl = wave_incl_scan(lcnt, &ltot);
      const int lpos = nleaf + lincl - lcnt;
      if (lcnt > 0 && lpos + lcnt <= PL)
        for (int c = 0; c < lcnt; c++) plist[lpos + c] = first + c;
      nleaf += ltot;
      const int nch = __builtin_popcount(kids);
      int tot;
      const int incl = wave_incl_scan(nch, &tot);
      tail -= batch;  // the popped entries are in registers; children overwrite them
      if (nleaf > PL || tail + tot > kWaveQueue) {
        overflow = true;
        break;
      }
      int off = tail + incl - nch;
      const uint32_t mask = meta & 0xffu;
      uint32_t kk = kids;
      while (kk) {
        const uint32_t o = (uint32_t)__builtin_ctz(kk);
        kk &= kk - 1u;
        queue[off++] = first + __builtin_popcount(mask & ((1u << o) - 1u));
      }
      tail += tot;
      if (a.dbg && lane == 0) atomicAdd(&a.dbg[5], 1ull);
      wave_lds_fence();
    }
  }
  if (overflow) join = false;
  if (a.dbg && lane == 0) {
    atomicAdd(&a.dbg[0], 1ull);
    if (overflow) atomicAdd(&a.dbg[1], 1ull);
  }

  const unsigned long long t_p3 = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
  // Phase 4: every joined lane scans the candidate points in lockstep: 64 points per chunk are
  // gathered by one load per lane (the next chunk's gather is in flight while the current one is
  // scanned from LDS by broadcast reads).
  double best = __builtin_inf(), second = __builtin_inf();
  int32_t bpos = -1;
  const int npts = nleaf;
  int scanned_pts = 0;
  // fp32 filter scan (GL = 64): the staged points and the joined queries lie in B, so relative
  // to B's centre o every coordinate is at most A in magnitude and an fp32 offset carries an
  // absolute error of at most ~A 2^-24. The wave tracks, per lane, the two smallest fp32 squared
  // distances s1 <= s2 and the position of s1's point; that point's fp64 distance (the
  // reference arithmetic) is recomputed and the certificate uses a rigorous lower bound of every
  // other point's fp64 distance derived from s2 (error analysis at scan32_lower_bound). A wave
  // where any joined lane cannot be certified this way redoes the scan in fp64 below.
  bool need64 = GL == 64 && __ballot(join) != 0 && npts > 0;
  if (GL == 64 && a.scan32 && need64) {
    const double ocx = (blx + bhx) * 0.5, ocy = (bly + bhy) * 0.5, ocz = (blz + bhz) * 0.5;
    const double ext = dmax_(dmax_(dmax_(bhx - ocx, ocx - blx), dmax_(bhy - ocy, ocy - bly)),
                             dmax_(bhz - ocz, ocz - blz)) * (1.0 + 0x1p-40);
    if (ext >= 0x1p-40 && ext <= 0x1p60) {
      const float qx32 = (float)(qx - ocx), qy32 = (float)(qy - ocy), qz32 = (float)(qz - ocz);
      // staging area: points in pairs, [x0 x1 y0 y1 z0 z1 w0 w1] (32 B), so that one packed fp32
      // instruction (v_pk_add/mul/fma_f32) evaluates an axis of two points
      float* stage32 = reinterpret_cast<float*>(wl);
      float s1 = __builtin_inff(), s2 = __builtin_inff();
      int32_t p1 = -1;
      wave_lds_fence();
      double4 nxtp = make_double4(0.0, 0.0, 0.0, 0.0);
      if (lane < npts) {
        const int32_t g = plist[lane];
        const TgtPt* p = a.pts + g;
        const double2 xy = *reinterpret_cast<const double2*>(&p->x);
        nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
      }
      for (int base = 0; base < npts; base += 64) {
        const bool nin = base + lane < npts && nxtp.x >= blx && nxtp.x <= bhx && nxtp.y >= bly && nxtp.y <= bhy &&
                         nxtp.z >= blz && nxtp.z <= bhz;
        const unsigned long long im = __ballot(nin);
        const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0));
        const float vx = (float)(nxtp.x - ocx), vy = (float)(nxtp.y - ocy), vz = (float)(nxtp.z - ocz);
        const float vw = __int_as_float((int)__double_as_longlong(nxtp.w));
        const int m = __popcll(im);
        wave_lds_fence();  // previous chunk's reads are done before overwriting the staging slots
        if (nin) {
          float* sp = stage32 + 8 * (slot >> 1) + (slot & 1);
          sp[0] = vx;
          sp[2] = vy;
          sp[4] = vz;
          sp[6] = vw;
        }
        if ((m & 1) && lane == 63) {
          // odd count: the last pair's second point at +inf (its sq = +inf never replaces s1 and
          // leaves s2 unchanged; no NaN can arise from inf - finite)
          float* sp = stage32 + 8 * (m >> 1) + 1;
          sp[0] = __builtin_inff();
          sp[2] = __builtin_inff();
          sp[4] = __builtin_inff();
        }
        wave_lds_fence();
        const int nb = base + 64;
        if (nb + lane < npts) {
          const int32_t g = plist[nb + lane];
          const TgtPt* p = a.pts + g;
          const double2 xy = *reinterpret_cast<const double2*>(&p->x);
          nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
        }
        scanned_pts += m;
        // lockstep over the staged pairs (16-B broadcast reads). Point 2k is selected before point
        // 2k + 1: the same sequence of updates as a one-point-at-a-time scan.
        typedef float f2 __attribute__((ext_vector_type(2)));
        typedef int v4i __attribute__((ext_vector_type(4)));
        const f2 qx2 = {qx32, qx32}, qy2 = {qy32, qy32}, qz2 = {qz32, qz32};
        auto sel = [&](float sq, int w) {
          const bool lt = sq < s1;
          s2 = __builtin_amdgcn_fmed3f(s1, s2, sq);
          s1 = lt ? sq : s1;
          p1 = lt ? w : p1;
        };
        auto eval2 = [&](const v4i xy, const v4i zw) {
          const f2 X = {__int_as_float(xy.x), __int_as_float(xy.y)};
          const f2 Y = {__int_as_float(xy.z), __int_as_float(xy.w)};
          const f2 Z = {__int_as_float(zw.x), __int_as_float(zw.y)};
          const f2 dx = X - qx2, dy = Y - qy2, dz = Z - qz2;
          const f2 sq = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
          sel(sq.x, zw.z);
          sel(sq.y, zw.w);
        };
        const v4i* st4 = reinterpret_cast<const v4i*>(stage32);
        const int mp = (m + 1) >> 1;
        int k = 0;
        for (; k + 2 <= mp; k += 2) {
          const v4i a0 = st4[2 * k], b0 = st4[2 * k + 1], a1 = st4[2 * k + 2], b1 = st4[2 * k + 3];
          eval2(a0, b0);
          eval2(a1, b1);
        }
        if (k < mp) eval2(st4[2 * k], st4[2 * k + 1]);
      }
      // fp64 distance of the fp32 winner, exactly as the leaf scan computes it (octree.cpp:139-144)
      double b64 = __builtin_inf();
      if (join && p1 >= 0) {
        const TgtPt* p = a.pts + p1;
        const double dx = p->x - qx, dy = p->y - qy, dz = p->z - qz;
        b64 = dx * dx + dy * dy + dz * dz;
      }
      const double lb2 = scan32_lower_bound(s2, ext);
      // a lane whose fp32 winner is not within its guess goes to the per-lane search either way
      const bool ok = !join || p1 < 0 || !(b64 <= u) || certified(b64, lb2, a.init_best);
      if (__ballot(!ok) == 0) {
        best = b64;
        second = lb2;
        bpos = p1;
        need64 = false;
      }
    }
  }
  if (GL == 64 && need64) {
    // Points outside B are farther than r from every joined lane (each ball lies in B), so
    // they can neither be a joined lane's nearest point nor sit in its certificate window.
    wave_lds_fence();
    double4 nxtp = make_double4(0.0, 0.0, 0.0, 0.0);
    bool nin = false;
    if (lane < npts) {
      const int32_t g = plist[lane];
      const TgtPt* p = a.pts + g;
      const double2 xy = *reinterpret_cast<const double2*>(&p->x);
      nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
    }
    for (int base = 0; base < npts; base += 64) {
      nin = base + lane < npts && nxtp.x >= blx && nxtp.x <= bhx && nxtp.y >= bly && nxtp.y <= bhy &&
            nxtp.z >= blz && nxtp.z <= bhz;
      const unsigned long long im = __ballot(nin);
      const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0));
      const double4 cur = nxtp;
      const int nb = base + 64;
      if (nb + lane < npts) {
        const int32_t g = plist[nb + lane];
        const TgtPt* p = a.pts + g;
        const double2 xy = *reinterpret_cast<const double2*>(&p->x);
        nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
      }
      const int m = __popcll(im);
      scanned_pts += m;
      // the staging area holds 32 fp64 points: the chunk's in-B points in two halves
      for (int h = 0; h < m; h += 32) {
        wave_lds_fence();  // the previous half's reads are done before its slots are rewritten
        if (nin && slot >= h && slot < h + 32) stage[slot - h] = cur;
        wave_lds_fence();
        const int mh = m - h < 32 ? m - h : 32;
        for (int k = 0; k < mh; k++) {
          const double4 pt = stage[k];
          const double dx = pt.x - qx, dy = pt.y - qy, dz = pt.z - qz;
          const double d2 = dx * dx + dy * dy + dz * dz;
          if (d2 < best) {
            second = best;
            best = d2;
            bpos = (int32_t)__double_as_longlong(pt.w);
          } else if (d2 < second) {
            second = d2;
          }
        }
      }
    }
    if (a.dbg && lane == 0) atomicAdd(&a.dbg[4], (unsigned long long)scanned_pts);
  }
  if (GL < 64 && __ballot(join) != 0 && npts > 0) {
    // Each joined lane's ball lies in its group's box B_g (inside B), so the points of B_g
    // hold every point the lane's certificate needs. Lane l stages chunk point l (unfiltered),
    // tests it against every B_g and appends its slot to the group lists; then each lane walks
    // its own group's list, branch-free.
    const int mg = lane / GL;
    wave_lds_fence();
    double4 nxtp = make_double4(0.0, 0.0, 0.0, 0.0);
    if (lane < npts) {
      const int32_t g = plist[lane];
      const TgtPt* p = a.pts + g;
      const double2 xy = *reinterpret_cast<const double2*>(&p->x);
      nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
    }
    for (int base = 0; base < npts; base += 64) {
      const bool have = base + lane < npts;
      wave_lds_fence();  // the previous chunk's reads are done before the slots are rewritten
      stage[lane] = nxtp;
      int mycnt = 0, maxcnt = 0;
#pragma unroll
      for (int g = 0; g < G; g++) {
        const double* gb = gbox + 8 * g;
        const bool in = have && nxtp.x >= gb[0] && nxtp.x <= gb[3] && nxtp.y >= gb[1] && nxtp.y <= gb[4] &&
                        nxtp.z >= gb[2] && nxtp.z <= gb[5];
        const unsigned long long m = __ballot(in);
        const int slot = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        if (in) gidx[64 * g + slot] = (unsigned char)lane;
        const int c = __popcll(m);
        mycnt = (g == mg) ? c : mycnt;
        maxcnt = c > maxcnt ? c : maxcnt;
      }
      wave_lds_fence();
      const int nb = base + 64;
      if (nb + lane < npts) {
        const int32_t g = plist[nb + lane];
        const TgtPt* p = a.pts + g;
        const double2 xy = *reinterpret_cast<const double2*>(&p->x);
        nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
      }
      scanned_pts += maxcnt;
      const unsigned char* my = gidx + 64 * mg;
      for (int k = 0; k < maxcnt; k++) {
        const bool valid = k < mycnt;
        const double4 pt = stage[my[k] & 63];
        const double dx = pt.x - qx, dy = pt.y - qy, dz = pt.z - qz;
        const double d2 = dx * dx + dy * dy + dz * dz;
        const bool lt = valid && d2 < best;
        const bool ls = valid && d2 < second;
        second = lt ? best : (ls ? d2 : second);
        best = lt ? d2 : best;
        bpos = lt ? (int32_t)__double_as_longlong(pt.w) : bpos;
      }
    }
    if (a.dbg && lane == 0) atomicAdd(&a.dbg[4], (unsigned long long)scanned_pts);
  }
  if (a.dbg) {
    const unsigned long long ex = __ballot(cand && !join && !overflow);
    const unsigned long long cov = __ballot(join && !(best <= u));
    const unsigned long long nc = __ballot(active && finite_q && !cand);
    if (lane == 0) {
      atomicAdd(&a.dbg[2], (unsigned long long)__popcll(ex));
      atomicAdd(&a.dbg[3], (unsigned long long)__popcll(cov));
      atomicAdd(&a.dbg[6], (unsigned long long)__popcll(nc));
      atomicAdd(&a.dbg[7], (unsigned long long)nleaf);
    }
  }

  const unsigned long long t_p4 = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
  // Phase 5: certify, write, or queue.
  bool written = false, to_exact = false, to_lane = false;
  double d = 0.0;
  int32_t pos = bpos;
  if (active) {
    if (!finite_q) {
      pos = a.pos0;
      const TgtPt p = a.pts[pos];
      const double dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
      d = __builtin_sqrt(dx * dx + dy * dy + dz * dz);
      written = true;
    } else if (join && !(best <= u)) {
      to_lane = true;  // the guess did not cover the nearest point: search this one per lane
    } else if (join) {
      written = certified(best, second, a.init_best);
      to_exact = !written;
      d = __builtin_sqrt(best);
    } else {
      to_lane = true;
    }
    if (written) {
      a.pos_out[i] = pos;
      a.dist_out[i] = d;
    }
  }
  wave_append(to_exact, i, a.fb_count, a.fb_list);
  const bool covered = !(join && !(best <= u));
  wave_append_u(to_lane, i, covered ? u : __builtin_inf(), a.fb_count + 1, a.fb_list2, a.fb_u2);
  if (a.dbg && lane == 0) {
    const unsigned long long t_p5 = __builtin_amdgcn_s_memtime();
    atomicAdd(&a.dbg[16], t_p2 - t_p0);
    atomicAdd(&a.dbg[17], t_p3 - t_pd);
    atomicAdd(&a.dbg[20], t_pd - t_p2);
    atomicAdd(&a.dbg[18], t_p4 - t_p3);
    atomicAdd(&a.dbg[19], t_p5 - t_p4);
  }
  // residual moments: k_moments, once every search kernel has written its queries
}

// One wave per query for the queries a k_nn4 wave did not take (outliers far from the surface,
// waves whose candidate set overflowed). The guess u bounds the query's nearest distance: the
// wave collects, breadth-first, every leaf whose box distance s <= u (1 + 2^-47) — a sphere test,
// tighter than k_nn4's box — and scans their points one per lane. Certification as in k_nn4
// (best <= u and the window test). Leaves of boxes with s > u (1 + 2^-47) only hold points with
// fl(d2) > best (1 + 2^-48) (monotone rounding, see k_nn3), so nothing in the window is missed.
// No usable guess or an overflowing candidate set -> per-lane search (k_nn_lists).
constexpr int kBallStack = 512;
constexpr int kBallPoints = 1024;
constexpr int kBallLdsBytes = kBallStack * 4 + kBallPoints * 4;

__global__ void __launch_bounds__(64) k_nn_ball(NNLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  int32_t* stack = reinterpret_cast<int32_t*>(lds_stack);
  int32_t* plist = stack + kBallStack;
  const int lane = threadIdx.x;
  const unsigned cnt = a.fb_count[1];
  for (unsigned j = blockIdx.x; j < cnt; j += gridDim.x) {
    const int64_t i = a.fb_list2[j];
    const double u = a.fb_u2[j];
    const double qx = a.x[i], qy = a.y[i], qz = a.z[i];
    if (!(u <= 0x1p900)) {
      if (lane == 0) a.fb_list3[atomicAdd(a.fb_count + 2, 1u)] = (int32_t)i;
      continue;
    }
    const double thr = u * (1.0 + kFastPrune);
    int tail = 1, npts = 0;
    bool overflow = false;
    wave_lds_fence();
    if (a.cells) {
      // every point with fl(d2) <= thr lies in the box q +- r (see k_nn4's radius)
      const double amax = __builtin_fmax(__builtin_fabs(qx), __builtin_fmax(__builtin_fabs(qy), __builtin_fabs(qz)));
      const double r = __builtin_sqrt(thr) * (1.0 + 0x1p-40) + amax * 0x1p-45;
      tail = cell_starts(a, qx - r, qy - r, qz - r, qx + r, qy + r, qz + r, lane, stack);
    } else if (lane == 0) {
      stack[0] = 0;
    }
    wave_lds_fence();
    // LIFO batches of up to 64 nodes, sphere test s <= thr on the children
    while (tail > 0) {
      const int batch = tail < 64 ? tail : 64;
      const bool has = lane < batch;
      bool leaf = false;
      int32_t first = 0;
      uint32_t meta = 0, kids = 0;
      if (has) {
        const NodeRec* rr = a.nodes + stack[tail - batch + lane];
        const int2 topo = *reinterpret_cast<const int2*>(&rr->first);
        first = topo.x;
        meta = (uint32_t)topo.y;
        leaf = (meta & kLeafBit) != 0;
        if (!leaf) {
          const double2 l01 = *reinterpret_cast<const double2*>(&rr->lo[0]);
          const double2 l2h0 = *reinterpret_cast<const double2*>(&rr->lo[2]);
          const double2 h12 = *reinterpret_cast<const double2*>(&rr->hi[1]);
          const double lx = l01.x, ly = l01.y, lz = l2h0.x, hx = l2h0.y, hy = h12.x, hz = h12.y;
          const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
          const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
          const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
          const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
          const double sx[2] = {ax0 * ax0, ax1 * ax1};
          const double sy[2] = {ay0 * ay0, ay1 * ay1};
          const double sz[2] = {az0 * az0, az1 * az1};
          const uint32_t mask = meta & 0xffu;
#pragma unroll
          for (int o = 0; o < 8; o++) {
            const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
            kids |= (((mask >> o) & 1u) && !(c > thr)) ? (1u << o) : 0u;
          }
        }
      }
      const int lcnt = (has && leaf) ? (int)(meta & ~kLeafBit) : 0;
      int ltot;
      const int lincl = wave_incl_scan(lcnt, &ltot);
      const int lpos = npts + lincl - lcnt;
      if (lcnt > 0 && lpos + lcnt <= kBallPoints)
        for (int c = 0; c < lcnt; c++) plist[lpos + c] = first + c;
      npts += ltot;
      const int nch = __builtin_popcount(kids);
      int tot;
      const int incl = wave_incl_scan(nch, &tot);
      tail -= batch;
      if (npts > kBallPoints || tail + tot > kBallStack) {
        overflow = true;
        break;
      }
      int off = tail + incl - nch;
      const uint32_t mask = meta & 0xffu;
      uint32_t kk = kids;
      while (kk) {
        const uint32_t o = (uint32_t)__builtin_ctz(kk);
        kk &= kk - 1u;
        stack[off++] = first + __builtin_popcount(mask & ((1u << o) - 1u));
      }
      tail += tot;
      wave_lds_fence();
    }
    if (a.dbg && lane == 0) {
      atomicAdd(&a.dbg[14], overflow ? 1ull : 0ull);
      atomicAdd(&a.dbg[15], (unsigned long long)npts);
    }
    if (overflow) {
      if (lane == 0) a.fb_list3[atomicAdd(a.fb_count + 2, 1u)] = (int32_t)i;
      wave_lds_fence();
      continue;
    }
    wave_lds_fence();
    double best = __builtin_inf(), second = __builtin_inf();
    int32_t bpos = 0x7fffffff;
    for (int k = lane; k < npts; k += 64) {
      const int32_t g = plist[k];
      const TgtPt* p = a.pts + g;
      const double2 xy = *reinterpret_cast<const double2*>(&p->x);
      const double dx = xy.x - qx, dy = xy.y - qy, dz = p->z - qz;
      const double d2 = dx * dx + dy * dy + dz * dz;
      if (d2 < best) {
        second = best;
        best = d2;
        bpos = g;
      } else if (d2 < second) {
        second = d2;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double ob = __shfl_xor(best, o, kWave);
      const double os = __shfl_xor(second, o, kWave);
      const int32_t op = __shfl_xor(bpos, o, kWave);
      const double lo_ = ob < best ? ob : best;
      const double hi_ = ob < best ? best : ob;
      const double ss = os < second ? os : second;
      second = hi_ < ss ? hi_ : ss;
      bpos = (ob < best || (ob == best && op < bpos)) ? op : bpos;
      best = lo_;
    }
    if (lane == 0) {
      if (!(best <= u)) {
        a.fb_list3[atomicAdd(a.fb_count + 2, 1u)] = (int32_t)i;
      } else if (certified(best, second, a.init_best)) {
        a.pos_out[i] = bpos;
        a.dist_out[i] = __builtin_sqrt(best);
      } else {
        a.fb_list[atomicAdd(a.fb_count, 1u)] = (int32_t)i;
      }
    }
    wave_lds_fence();
  }
}

// The ball search with four queries per wave, one 16-lane group (a DPP row) each: the list's
// queries are latency-bound walks of a few dependent rounds, so four in flight per wave hide four
// times the latency of one. Same walk, sphere test and certificate as k_nn_ball per group; the
// group's candidate list holds 256 points (more: the query goes to the per-lane search).
constexpr int kBallGroups = 4;
constexpr int kBallGL = 64 / kBallGroups;         // lanes per query
constexpr int kBallGStack = kBallStack / kBallGroups;
constexpr int kBallGPoints = kBallPoints / kBallGroups;

// Inclusive prefix sum within each 16-lane row (row_shr 1, 2, 4, 8); *total = the row's sum.
__device__ __forceinline__ int row_incl_scan(int v, int row_base, int* total) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  *total = __shfl(v, row_base + 15, kWave);
  return v;
}

// cell_starts for one 16-lane group: at most 16 cells (one per lane), paths from the group's
// first 6 lanes. Writes the start nodes to out[0 .. count) and returns count (group-uniform).
__device__ __forceinline__ int cell_starts_g(const NNLaunch& a, double blx, double bly, double blz, double bhx,
                                             double bhy, double bhz, int gl, int gbase, int32_t* out) {
  int L = a.cell_lmax;
  uint32_t path = 0;
  if (gl < 6) {
    const int ax = gl >> 1;
    const double v = (gl & 1) ? (ax == 0 ? bhx : ax == 1 ? bhy : bhz) : (ax == 0 ? blx : ax == 1 ? bly : blz);
    double lo = ax == 0 ? a.root_lo[0] : ax == 1 ? a.root_lo[1] : a.root_lo[2];
    double hi = ax == 0 ? a.root_hi[0] : ax == 1 ? a.root_hi[1] : a.root_hi[2];
    for (int l = 0; l < L; l++) {
      const double m = (lo + hi) / 2;
      const bool up = v > m;
      path = 2u * path + (up ? 1u : 0u);
      lo = up ? m : lo;
      hi = up ? hi : m;
    }
  }
  uint32_t ilx = (uint32_t)__shfl((int)path, gbase + 0, kWave), ihx = (uint32_t)__shfl((int)path, gbase + 1, kWave);
  uint32_t ily = (uint32_t)__shfl((int)path, gbase + 2, kWave), ihy = (uint32_t)__shfl((int)path, gbase + 3, kWave);
  uint32_t ilz = (uint32_t)__shfl((int)path, gbase + 4, kWave), ihz = (uint32_t)__shfl((int)path, gbase + 5, kWave);
  while (L > 0 && (ihx - ilx + 1) * (ihy - ily + 1) * (ihz - ilz + 1) > (uint32_t)kBallGL) {
    L--;
    ilx >>= 1; ihx >>= 1; ily >>= 1; ihy >>= 1; ilz >>= 1; ihz >>= 1;
  }
  const uint32_t nx = ihx - ilx + 1, ny = ihy - ily + 1, nz = ihz - ilz + 1;
  bool put = false;
  int32_t node = 0;
  if ((uint32_t)gl < nx * ny * nz) {
    const uint32_t cx = ilx + (uint32_t)gl % nx, cy = ily + ((uint32_t)gl / nx) % ny, cz = ilz + (uint32_t)gl / (nx * ny);
    const uint32_t prefix = spread3(cx) | (spread3(cy) << 1) | (spread3(cz) << 2);
    const int32_t e = a.cells[(((int64_t)1 << (3 * L)) - 1) / 7 + prefix];
    if (e >= 0) {
      node = e >> 5;
      const int sh = L - (e & 31);
      const uint32_t fx = ((cx >> sh) << sh) > ilx ? ((cx >> sh) << sh) : ilx;
      const uint32_t fy = ((cy >> sh) << sh) > ily ? ((cy >> sh) << sh) : ily;
      const uint32_t fz = ((cz >> sh) << sh) > ilz ? ((cz >> sh) << sh) : ilz;
      put = cx == fx && cy == fy && cz == fz;
    }
  }
  const uint32_t pm = (uint32_t)((__ballot(put) >> gbase) & 0xffffull);
  if (put) out[__builtin_popcount(pm & ((1u << gl) - 1u))] = node;
  return __builtin_popcount(pm);
}

__global__ void __launch_bounds__(64) k_nn_ball4(NNLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const int lane = threadIdx.x, g = lane / kBallGL, gl = lane % kBallGL, gbase = g * kBallGL;
  int32_t* stack = reinterpret_cast<int32_t*>(lds_stack) + g * kBallGStack;
  int32_t* plist = reinterpret_cast<int32_t*>(lds_stack) + kBallStack + g * kBallGPoints;
  const unsigned cnt = a.fb_count[1];
  for (unsigned j0 = blockIdx.x * kBallGroups; j0 < cnt; j0 += gridDim.x * kBallGroups) {
    const unsigned j = j0 + g;
    bool live = j < cnt;  // group-uniform
    int64_t i = 0;
    double u = 0.0, qx = 0.0, qy = 0.0, qz = 0.0;
    if (live) {
      i = a.fb_list2[j];
      u = a.fb_u2[j];
      qx = a.x[i];
      qy = a.y[i];
      qz = a.z[i];
      if (!(u <= 0x1p900)) {
        if (gl == 0) a.fb_list3[atomicAdd(a.fb_count + 2, 1u)] = (int32_t)i;
        live = false;
      }
    }
    const double thr = u * (1.0 + kFastPrune);
    int tail = 0, npts = 0;
    bool overflow = false;
    wave_lds_fence();
    {
      // every point with fl(d2) <= thr lies in the box q +- r (see k_nn4's radius)
      const double amax = __builtin_fmax(__builtin_fabs(qx), __builtin_fmax(__builtin_fabs(qy), __builtin_fabs(qz)));
      const double r = live ? __builtin_sqrt(thr) * (1.0 + 0x1p-40) + amax * 0x1p-45 : 0.0;
      const int t = cell_starts_g(a, qx - r, qy - r, qz - r, qx + r, qy + r, qz + r, gl, gbase, stack);
      tail = live ? t : 0;
    }
    wave_lds_fence();
    // LIFO batches of up to 16 nodes per group, sphere test s <= thr on the children
    while (__ballot(tail > 0) != 0) {
      const int batch = tail < kBallGL ? tail : kBallGL;
      const bool has = gl < batch;
      bool leaf = false;
      int32_t first = 0;
      uint32_t meta = 0, kids = 0;
      if (has) {
        const NodeRec* rr = a.nodes + stack[tail - batch + gl];
        const int2 topo = *reinterpret_cast<const int2*>(&rr->first);
        first = topo.x;
        meta = (uint32_t)topo.y;
        leaf = (meta & kLeafBit) != 0;
        if (!leaf) {
          const double2 l01 = *reinterpret_cast<const double2*>(&rr->lo[0]);
          const double2 l2h0 = *reinterpret_cast<const double2*>(&rr->lo[2]);
          const double2 h12 = *reinterpret_cast<const double2*>(&rr->hi[1]);
          const double lx = l01.x, ly = l01.y, lz = l2h0.x, hx = l2h0.y, hy = h12.x, hz = h12.y;
          const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
          const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
          const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
          const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
          const double sx[2] = {ax0 * ax0, ax1 * ax1};
          const double sy[2] = {ay0 * ay0, ay1 * ay1};
          const double sz[2] = {az0 * az0, az1 * az1};
          const uint32_t mask = meta & 0xffu;
#pragma unroll
          for (int o = 0; o < 8; o++) {
            const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
            kids |= (((mask >> o) & 1u) && !(c > thr)) ? (1u << o) : 0u;
          }
        }
      }
      const int lcnt = (has && leaf) ? (int)(meta & ~kLeafBit) : 0;
      int ltot;
      const int lincl = row_incl_scan(lcnt, gbase, &ltot);
      const int lpos = npts + lincl - lcnt;
      if (lcnt > 0 && lpos + lcnt <= kBallGPoints)
        for (int c = 0; c < lcnt; c++) plist[lpos + c] = first + c;
      const int nch = __builtin_popcount(kids);
      int tot;
      const int incl = row_incl_scan(nch, gbase, &tot);
      if (tail > 0) {
        npts += ltot;
        tail -= batch;
        if (npts > kBallGPoints || tail + tot > kBallGStack) {
          overflow = true;
          tail = 0;
        } else {
          int off = tail + incl - nch;
          const uint32_t mask = meta & 0xffu;
          uint32_t kk = kids;
          while (kk) {
            const uint32_t o = (uint32_t)__builtin_ctz(kk);
            kk &= kk - 1u;
            stack[off++] = first + __builtin_popcount(mask & ((1u << o) - 1u));
          }
          tail += tot;
        }
      }
      wave_lds_fence();
    }
    if (live && overflow && gl == 0) a.fb_list3[atomicAdd(a.fb_count + 2, 1u)] = (int32_t)i;
    if (overflow) live = false;
    wave_lds_fence();
    double best = __builtin_inf(), second = __builtin_inf();
    int32_t bpos = 0x7fffffff;
    if (live) {
      for (int k = gl; k < npts; k += kBallGL) {
        const int32_t pg = plist[k];
        const TgtPt* p = a.pts + pg;
        const double2 xy = *reinterpret_cast<const double2*>(&p->x);
        const double dx = xy.x - qx, dy = xy.y - qy, dz = p->z - qz;
        const double d2 = dx * dx + dy * dy + dz * dz;
        if (d2 < best) {
          second = best;
          best = d2;
          bpos = pg;
        } else if (d2 < second) {
          second = d2;
        }
      }
    }
#pragma unroll
    for (int o = kBallGL / 2; o >= 1; o >>= 1) {
      const double ob = __shfl_xor(best, o, kWave);
      const double os = __shfl_xor(second, o, kWave);
      const int32_t op = __shfl_xor(bpos, o, kWave);
      const double lo_ = ob < best ? ob : best;
      const double hi_ = ob < best ? best : ob;
      const double ss = os < second ? os : second;
      second = hi_ < ss ? hi_ : ss;
      bpos = (ob < best || (ob == best && op < bpos)) ? op : bpos;
      best = lo_;
    }
    if (live && gl == 0) {
      if (!(best <= u)) {
        a.fb_list3[atomicAdd(a.fb_count + 2, 1u)] = (int32_t)i;
      } else if (certified(best, second, a.init_best)) {
        a.pos_out[i] = bpos;
        a.dist_out[i] = __builtin_sqrt(best);
      } else {
        a.fb_list[atomicAdd(a.fb_count, 1u)] = (int32_t)i;
      }
    }
    wave_lds_fence();
  }
}


// The two short lists the ball search leaves, in one launch: thread j < n3 takes lane-list entry
// j (per-lane certified search; a query it cannot certify gets the reference-order DFS right
// away, in the same thread), the rest take the exact list (queries k_nn4 or the ball search could
// not certify). Both lists are complete when this kernel starts; it appends nothing.
__global__ void __launch_bounds__(64) k_nn_lists(NNLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const unsigned n3 = a.fb_count[2], n0 = a.fb_count[0];
  for (unsigned j = blockIdx.x * blockDim.x + threadIdx.x; j < n3 + n0; j += gridDim.x * blockDim.x) {
    const bool lane_list = j < n3;
    const int64_t i = lane_list ? a.fb_list3[j] : a.fb_list[j - n3];
    const double qx = a.x[i], qy = a.y[i], qz = a.z[i];
    if (lane_list) {
      double best = __builtin_inf(), second = __builtin_inf();
      int32_t bpos = -1;
      uint32_t nvis = 0, npts = 0;
      fast_dfs(a, qx, qy, qz, lds_stack + threadIdx.x, blockDim.x, best, second, bpos, nvis, npts);
      if (certified(best, second, a.init_best)) {
        a.pos_out[i] = bpos;
        a.dist_out[i] = __builtin_sqrt(best);
        continue;
      }
    }
    double best_d2 = a.init_best, visits = 0.0, scanned = 0.0;
    int32_t best = -1;
    exact_dfs<false>(a, qx, qy, qz, lds_stack + threadIdx.x, blockDim.x, best, best_d2, visits, scanned);
    int32_t pos = best;
    double d;
    if (best >= 0) {
      d = __builtin_sqrt(best_d2);
    } else {
      pos = a.pos0;
      const TgtPt p = a.pts[pos];
      const double dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
      d = __builtin_sqrt(dx * dx + dy * dy + dz * dz);
    }
    a.pos_out[i] = pos;
    a.dist_out[i] = d;
  }
}

// Fixed-shape merges of block partials (plain sums; Moments/CovMoments keep the Chan formulas for
// the rank merge), deterministic: the same
// n always gives the same merge tree. Inner levels: block b merges items [256 b, 256 b + 256),
// one per thread, pairwise in LDS. Last level: one block, up to 4096 items: thread t folds items
// t + 256 k (k < 16) in order, then the block's pairwise tree.
constexpr int kLastSpan = 4096;

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
__device__ __forceinline__ T block_tree(T v, T* sm) {
  const int t = threadIdx.x;
  sm[t] = v;
  __syncthreads();
  for (int s = 1; s < 256; s <<= 1) {
    if ((t & (2 * s - 1)) == 0) sm[t] = Merge(sm[t], sm[t + s]);
    __syncthreads();
  }
  return sm[0];
}

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
__device__ __forceinline__ T block_tree_last(const T* in, int64_t n, T* sm) {
  // thread t folds items t, t + 256, ..., t + 15 * 256 in that order (coalesced across the block;
  // the merges of the partial sums are additions, cheap in a chain), then the block's tree.
  // No early exit: block_tree's barriers must be reached by every thread in uniform control flow.
  T acc = Identity();
#pragma unroll 4
  for (int k = 0; k < 16; k++) {
    const int64_t g = (int64_t)threadIdx.x + 256 * k;
    if (g < n) acc = Merge(acc, in[g]);
  }
  return block_tree<T, Merge, Identity>(acc, sm);
}

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
__global__ void __launch_bounds__(256) k_tree_merge(const T* in, int64_t n, T* out) {
  __shared__ T sm[256];
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const T r = block_tree<T, Merge, Identity>(g < n ? in[g] : Identity(), sm);
  if (threadIdx.x == 0) out[blockIdx.x] = r;
}


// mean = sum/row; std = sqrt(variance/row) (icpengine.cpp:235-245); threshold rule of the caller
__device__ void finalize_moments(IterDev* it, const Moments& g, const MomentsFinalize& f) {
  it->m_global = g;
  const double mean = g.mean;
  const double sd = __builtin_sqrt(g.m2 / g.n);
  it->mean = mean;
  it->sd = sd;
  it->thr = cull_threshold(mean, sd, f.k_sigma, f.iter, f.engine_rules);
}

// Last level of the rank's moments: the summed part -> (count, mean, M2) in it->m_local; with fin
// (one rank) also the statistics.
__global__ void __launch_bounds__(256) k_merge_moments_last(const MomSums* in, int64_t n, const double* dist,
                                                           int64_t nq, IterDev* it, MomentsFinalize fin, int finalize) {
  __shared__ MomSums sm[256];
  const MomSums r = block_tree_last<MomSums, momsum_merge, momsum_identity>(in, n, sm);
  if (threadIdx.x == 0) {
    const double c = moment_shift(dist, nq);
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
    it->m_local = m;
    if (finalize) finalize_moments(it, m, fin);
  }
}

__global__ void k_finalize_moments(const Moments* gathered, int nranks, IterDev* it, MomentsFinalize fin) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Moments g = gathered[0];
  for (int r = 1; r < nranks; r++) g = moments_merge(g, gathered[r]);  // rank order: same bits everywhere
  finalize_moments(it, g, fin);
}

// The iteration's record goes straight into the caller's pinned host buffer (no copy engine or
// blit launch on the critical path): thread 0 completes it in LDS, the block stores it, and the
// stream synchronisation that follows makes it visible. The list sizes ride along (pad[0..2])
// and are reset for the next search.
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
    for (int k = 0; k < 3; k++) {
      rec->pad[k] = (double)pub.lists[k];
      pub.lists[k] = 0u;
    }
    it->c_global = rec->c_global;
    it->rmse = rec->rmse;
  }
  __syncthreads();
  // System-scope stores straight to the host page (no L2 write-back of the whole cache, which a
  // system-scope release fence would do: the search just dirtied megabytes of it); each thread
  // waits for its stores to be acknowledged before the block's sequence word goes out.
  double* dst = reinterpret_cast<double*>(pub.host);
  for (int k = threadIdx.x; k < kWords; k += blockDim.x)
    __hip_atomic_store(dst + k, rw[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(&pub.host->pad[3], pub.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(256) k_merge_cov_last(const CovSums* in, int64_t n, CullLaunch cl, IterDev* it,
                                                       IterPublish pub, int finalize) {
  __shared__ CovSums sm[256];
  __shared__ IterDev rec;
  const CovSums r = block_tree_last<CovSums, covsum_merge, covsum_identity>(in, n, sm);
  __shared__ CovMoments res;
  if (threadIdx.x == 0) {
    double sh[6];
    cov_shift(cl.x, cl.y, cl.z, cl.pos, cl.pts, cl.n, sh);
    CovMoments m = cov_identity();
    if (r.n > 0.0) {
      m.n = r.n;
      m.sum_d2 = r.sum_d2;
      double da[3], db[3];
      for (int k = 0; k < 3; k++) {
        da[k] = r.sa[k] / r.n;
        db[k] = r.sb[k] / r.n;
        m.ma[k] = sh[k] + da[k];
        m.mb[k] = sh[3 + k] + db[k];
      }
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m.c[3 * i + j] = r.sab[3 * i + j] - r.n * (da[i] * db[j]);
    }
    it->c_local = m;
    res = m;
  }
  if (!finalize) return;
  __syncthreads();
  finalize_cov_publish(it, res, pub, &rec);
}

__global__ void __launch_bounds__(64) k_finalize_cov(const CovMoments* gathered, int nranks, IterDev* it,
                                                     IterPublish pub) {
  __shared__ IterDev rec;
  CovMoments g = gathered[0];
  for (int r = 1; r < nranks; r++) g = cov_merge(g, gathered[r]);  // rank order
  finalize_cov_publish(it, g, pub, &rec);
}

constexpr int kCullPer = 4;  // queries per thread of k_cull_cov

__global__ void __launch_bounds__(256) k_cull_cov(CullLaunch a) {
  __shared__ double red[4 * 17];
  const double thr = a.it->thr;
  double sh[6];
  cov_shift(a.x, a.y, a.z, a.pos, a.pts, a.n, sh);
  const int64_t blk = xcd_block(a.xcd_remap);
  const int64_t base = blk * (256 * kCullPer) + threadIdx.x;
  // count, sum d^2, sum (a - s), sum (b - t), sum (a - s)(b - t)^T over the valid pairs
  double v[17];
#pragma unroll
  for (int k = 0; k < 17; k++) v[k] = 0.0;
  // All streamed loads first, then all match gathers (a culled or missing query gathers point 0,
  // always valid): two dependent memory round trips per thread instead of three.
  double dq[kCullPer], qx[kCullPer], qy[kCullPer], qz[kCullPer];
  int32_t pq[kCullPer];
#pragma unroll
  for (int e = 0; e < kCullPer; e++) {
    const int64_t i = base + e * 256;
    const bool in = i < a.n;
    dq[e] = in ? a.dist[i] : __builtin_nan("");  // NaN <= thr is false: not a valid pair
    pq[e] = in ? a.pos[i] : 0;
    qx[e] = in ? a.x[i] : 0.0;
    qy[e] = in ? a.y[i] : 0.0;
    qz[e] = in ? a.z[i] : 0.0;
  }
  double mx[kCullPer], my[kCullPer], mz[kCullPer];
#pragma unroll
  for (int e = 0; e < kCullPer; e++) {
    const TgtPt* p = a.pts + (dq[e] <= thr ? pq[e] : 0);
    const double2 pxy = *reinterpret_cast<const double2*>(&p->x);
    mx[e] = pxy.x;
    my[e] = pxy.y;
    mz[e] = p->z;
  }
#pragma unroll
  for (int e = 0; e < kCullPer; e++) {
    {
      const double d = dq[e];
      if (d <= thr) {  // icpengine.cpp:265
        const double da[3] = {qx[e] - sh[0], qy[e] - sh[1], qz[e] - sh[2]};
        const double db[3] = {mx[e] - sh[3], my[e] - sh[4], mz[e] - sh[5]};
        v[0] += 1.0;
        v[1] += d * d;
#pragma unroll
        for (int r = 0; r < 3; r++) {
          v[2 + r] += da[r];
          v[5 + r] += db[r];
#pragma unroll
          for (int c = 0; c < 3; c++) v[8 + 3 * r + c] += da[r] * db[c];
        }
      }
    }
  }
  block_sum<17>(v, red);
  if (threadIdx.x == 0) {
    CovSums m;
    m.n = v[0];
    m.sum_d2 = v[1];
    for (int k = 0; k < 3; k++) {
      m.sa[k] = v[2 + k];
      m.sb[k] = v[5 + k];
      m.pad[k] = 0.0;
    }
    for (int k = 0; k < 9; k++) m.sab[k] = v[8 + k];
    reinterpret_cast<CovSums*>(a.part)[blk] = m;
  }
}

__global__ void k_apply(const double* __restrict__ Tm, double* x, double* y, double* z, int64_t n) {
  // T passed through a tiny device buffer to keep kernel args small
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double qx = x[i], qy = y[i], qz = z[i];
  x[i] = ((Tm[0] * qx + Tm[1] * qy) + Tm[2] * qz) + Tm[3];
  y[i] = ((Tm[4] * qx + Tm[5] * qy) + Tm[6] * qz) + Tm[7];
  z[i] = ((Tm[8] * qx + Tm[9] * qy) + Tm[10] * qz) + Tm[11];
}

struct T12 {
  double v[12];
};

__global__ void k_apply_arg(T12 T, double* x, double* y, double* z, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double qx = x[i], qy = y[i], qz = z[i];
  x[i] = ((T.v[0] * qx + T.v[1] * qy) + T.v[2] * qz) + T.v[3];
  y[i] = ((T.v[4] * qx + T.v[5] * qy) + T.v[6] * qz) + T.v[7];
  z[i] = ((T.v[8] * qx + T.v[9] * qy) + T.v[10] * qz) + T.v[11];
}

__device__ __forceinline__ uint64_t spread3(uint64_t v) {
  v &= 0x1fffff;
  v = (v | (v << 32)) & 0x1f00000000ffffull;
  v = (v | (v << 16)) & 0x1f0000ff0000ffull;
  v = (v | (v << 8)) & 0x100f00f00f00f00full;
  v = (v | (v << 4)) & 0x10c30c30c30c30c3ull;
  v = (v | (v << 2)) & 0x1249249249249249ull;
  return v;
}

__device__ __forceinline__ uint64_t quant21(double v, double lo, double inv) {
  double f = (v - lo) * inv;
  if (!(f > 0.0)) f = 0.0;  // also maps NaN to cell 0
  if (f > 1.0) f = 1.0;
  return (uint64_t)(f * 2097151.0);
}

struct Box {
  double lo[3], inv[3];
};

__global__ void k_morton(const double* aos, int64_t n, Box b, double* x, double* y, double* z,
                         uint64_t* keys, int32_t* iota) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double px = aos[3 * i], py = aos[3 * i + 1], pz = aos[3 * i + 2];
  x[i] = px;
  y[i] = py;
  z[i] = pz;
  keys[i] = spread3(quant21(px, b.lo[0], b.inv[0])) | (spread3(quant21(py, b.lo[1], b.inv[1])) << 1) |
            (spread3(quant21(pz, b.lo[2], b.inv[2])) << 2);
  iota[i] = (int32_t)i;
}

__global__ void k_gather_soa(const int32_t* perm, const double* xi, const double* yi, const double* zi,
                             double* xo, double* yo, double* zo, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t j = perm[i];
  xo[i] = xi[j];
  yo[i] = yi[j];
  zo[i] = zi[j];
}

__global__ void k_scatter_aos(const int32_t* perm, const double* x, const double* y, const double* z,
                              double* aos, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t j = perm ? perm[i] : i;
  aos[3 * j] = x[i];
  aos[3 * j + 1] = y[i];
  aos[3 * j + 2] = z[i];
}

__global__ void k_scatter_corr(const int32_t* perm, const int32_t* pos, const TgtPt* pts, int32_t* idx_out,
                               const double* dist_in, double* dist_out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t j = perm ? perm[i] : i;
  if (idx_out) idx_out[j] = pts[pos[i]].orig;
  if (dist_out) dist_out[j] = dist_in[i];
}

__global__ void k_deinterleave(const double* aos, double* x, double* y, double* z, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  x[i] = aos[3 * i];
  y[i] = aos[3 * i + 1];
  z[i] = aos[3 * i + 2];
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

int nn_block_threads(int levels) {
  // LDS stack: levels x threads x 8 B. Keep <= 64 KiB per block.
  if (levels <= 32) return 256;
  if (levels <= 64) return 128;
  return 64;
}

int64_t nn_num_blocks(int64_t n, int levels) {
  const int bs = nn_block_threads(levels);
  return (n + bs - 1) / bs;
}

// The search kernels only settle queries (pos, residual); the caller computes the residual
// moments afterwards (launch_moments), so a.part is ignored here.
hipError_t launch_nn(const NNLaunch& a_in, hipStream_t s) {
  if (a_in.n <= 0) return hipSuccess;
  NNLaunch a = a_in;
  a.part = nullptr;
  const int levels = a.levels < 1 ? 1 : a.levels;
  const int bs = nn_block_threads(levels);
  size_t shmem = (size_t)levels * bs * sizeof(unsigned long long);
  if (shmem < 1024) shmem = 1024;  // also hosts the block reductions
  const unsigned grid = grid_for(a.n, bs);
  if (a.variant == 4 && !a.count) {
    // wave-cooperative search -> ball search -> per-lane search -> exact fallback
    const int gl = (a.scan_group == 8 || a.scan_group == 16 || a.scan_group == 32) ? a.scan_group : 64;
    const int pl = (gl == 64 && (a.wave_points == 512 || a.wave_points == 768)) ? a.wave_points : 1024;
    const size_t shm4 = (size_t)(bs / kWave) * wave_lds_bytes(gl, pl);
#define ICP_NN4(GL, PL)                                                                         \
  do {                                                                                         \
    if (a.apply) hipLaunchKernelGGL((k_nn4<true, GL, PL>), dim3(grid), dim3(bs), shm4, s, a);  \
    else hipLaunchKernelGGL((k_nn4<false, GL, PL>), dim3(grid), dim3(bs), shm4, s, a);         \
  } while (0)
    if (gl == 8) ICP_NN4(8, 1024);
    else if (gl == 16) ICP_NN4(16, 1024);
    else if (gl == 32) ICP_NN4(32, 1024);
    else if (pl == 512) ICP_NN4(64, 512);
    else if (pl == 768) ICP_NN4(64, 768);
    else ICP_NN4(64, 1024);
#undef ICP_NN4
    if (a.ev_fast_done) (void)hipEventRecord(a.ev_fast_done, s);
    // the lists are short (usually empty after the first iteration): small grids of 64-thread
    // blocks, grid-stride over the list
    const unsigned lgrid = (unsigned)((a.n + 63) / 64 < 1024 ? (a.n + 63) / 64 : 1024);
    const size_t lshm = (size_t)levels * 64 * sizeof(unsigned long long) < 1024 ? 1024
                        : (size_t)levels * 64 * sizeof(unsigned long long);
    const unsigned bgrid = (unsigned)((a.n < 16384) ? a.n : 16384);
    if (a.cells && a.ball_groups != 1)
      hipLaunchKernelGGL(k_nn_ball4, dim3((unsigned)((a.n + kBallGroups - 1) / kBallGroups < 8192
                                                     ? (a.n + kBallGroups - 1) / kBallGroups : 8192)),
                         dim3(64), kBallLdsBytes, s, a);
    else
      hipLaunchKernelGGL(k_nn_ball, dim3(bgrid), dim3(64), kBallLdsBytes, s, a);
    hipLaunchKernelGGL(k_nn_lists, dim3(lgrid), dim3(64), lshm, s, a);
    return hipGetLastError();
  }
  if (a.variant == 3 && !a.count) {
    // certified fast path -> exact fallback for the uncertified rest
    if (a.apply) hipLaunchKernelGGL((k_nn3<true>), dim3(grid), dim3(bs), shmem, s, a);
    else hipLaunchKernelGGL((k_nn3<false>), dim3(grid), dim3(bs), shmem, s, a);
    if (a.ev_fast_done) (void)hipEventRecord(a.ev_fast_done, s);
    const unsigned fb_grid = grid < 1024u ? grid : 1024u;
    hipLaunchKernelGGL(k_nn_fallback, dim3(fb_grid), dim3(bs), shmem, s, a);
    return hipGetLastError();
  }
  if (a.variant == 1 || a.count) {
    if (a.apply) {
      if (a.count) hipLaunchKernelGGL((k_nn<true, true>), dim3(grid), dim3(bs), shmem, s, a);
      else hipLaunchKernelGGL((k_nn<true, false>), dim3(grid), dim3(bs), shmem, s, a);
    } else {
      if (a.count) hipLaunchKernelGGL((k_nn<false, true>), dim3(grid), dim3(bs), shmem, s, a);
      else hipLaunchKernelGGL((k_nn<false, false>), dim3(grid), dim3(bs), shmem, s, a);
    }
  } else {
    if (a.apply) {
      if (a.count) hipLaunchKernelGGL((k_nn2<true, true>), dim3(grid), dim3(bs), shmem, s, a);
      else hipLaunchKernelGGL((k_nn2<true, false>), dim3(grid), dim3(bs), shmem, s, a);
    } else {
      if (a.count) hipLaunchKernelGGL((k_nn2<false, true>), dim3(grid), dim3(bs), shmem, s, a);
      else hipLaunchKernelGGL((k_nn2<false, false>), dim3(grid), dim3(bs), shmem, s, a);
    }
  }
  return hipGetLastError();
}

// Partial buffers hold the block partials followed by the merge scratch (merge_scratch_entries).
int64_t merge_scratch_entries(int64_t nparts) {
  int64_t total = 0;
  for (int64_t cn = nparts; cn > kLastSpan; cn = (cn + 255) / 256) total += (cn + 255) / 256;
  return total + 1;
}

template <typename T, T (*Merge)(const T&, const T&), T (*Identity)()>
static const T* merge_to_last_span(const T* part, int64_t* nparts, hipStream_t s) {
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

hipError_t launch_merge_moments(const Moments* part, int64_t nparts, const double* dist, int64_t nq, IterDev* it,
                                const MomentsFinalize* fin, hipStream_t s) {
  const MomSums* cur = merge_to_last_span<MomSums, momsum_merge, momsum_identity>(
      reinterpret_cast<const MomSums*>(part), &nparts, s);
  hipLaunchKernelGGL(k_merge_moments_last, dim3(1), dim3(256), 0, s, cur, nparts, dist, nq, it,
                     fin ? *fin : MomentsFinalize{0.0, 0, 0}, fin ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_merge_cov(const CovMoments* part, int64_t nparts, const CullLaunch& cl, IterDev* it,
                            const IterPublish* pub, hipStream_t s) {
  const CovSums* cur = merge_to_last_span<CovSums, covsum_merge, covsum_identity>(
      reinterpret_cast<const CovSums*>(part), &nparts, s);
  hipLaunchKernelGGL(k_merge_cov_last, dim3(1), dim3(256), 0, s, cur, nparts, cl, it,
                     pub ? *pub : IterPublish{nullptr, nullptr, 0.0}, pub ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_finalize_moments(const Moments* gathered, int nranks, IterDev* it, MomentsFinalize fin,
                                   hipStream_t s) {
  hipLaunchKernelGGL(k_finalize_moments, dim3(1), dim3(64), 0, s, gathered, nranks, it, fin);
  return hipGetLastError();
}

int64_t moments_num_parts(int64_t n) { return (n + kMomPart - 1) / kMomPart; }

hipError_t launch_moments(const double* dist, int64_t n, const IterDev* it, Moments* part, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_moments, dim3((unsigned)moments_num_parts(n)), dim3(256), 0, s, dist, n, it,
                     reinterpret_cast<MomSums*>(part));
  return hipGetLastError();
}

int64_t cull_num_blocks(int64_t n) { return (n + 256 * kCullPer - 1) / (256 * kCullPer); }

hipError_t launch_cull_cov(const CullLaunch& a, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_cull_cov, dim3((unsigned)cull_num_blocks(a.n)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_finalize_cov(const CovMoments* gathered, int nranks, IterDev* it, IterPublish pub,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_finalize_cov, dim3(1), dim3(64), 0, s, gathered, nranks, it, pub);
  return hipGetLastError();
}

hipError_t launch_apply(const double T[12], double* x, double* y, double* z, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  T12 t;
  for (int k = 0; k < 12; k++) t.v[k] = T[k];
  hipLaunchKernelGGL(k_apply_arg, dim3(grid_for(n, 256)), dim3(256), 0, s, t, x, y, z, n);
  return hipGetLastError();
}

hipError_t launch_morton(const double* aos, int64_t n, const double lo[3], const double inv_ext[3], double* x,
                         double* y, double* z, uint64_t* keys, int32_t* iota, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  Box b;
  for (int k = 0; k < 3; k++) {
    b.lo[k] = lo[k];
    b.inv[k] = inv_ext[k];
  }
  hipLaunchKernelGGL(k_morton, dim3(grid_for(n, 256)), dim3(256), 0, s, aos, n, b, x, y, z, keys, iota);
  return hipGetLastError();
}

hipError_t launch_gather_soa(const int32_t* perm, const double* xi, const double* yi, const double* zi, double* xo,
                             double* yo, double* zo, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_soa, dim3(grid_for(n, 256)), dim3(256), 0, s, perm, xi, yi, zi, xo, yo, zo, n);
  return hipGetLastError();
}

hipError_t launch_scatter_aos(const int32_t* perm, const double* x, const double* y, const double* z, double* aos,
                              int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_aos, dim3(grid_for(n, 256)), dim3(256), 0, s, perm, x, y, z, aos, n);
  return hipGetLastError();
}

hipError_t launch_scatter_corr(const int32_t* perm, const int32_t* pos, const TgtPt* pts, int32_t* idx_out,
                               double* dist_in, double* dist_out, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_corr, dim3(grid_for(n, 256)), dim3(256), 0, s, perm, pos, pts, idx_out, dist_in,
                     dist_out, n);
  return hipGetLastError();
}

hipError_t launch_deinterleave(const double* aos, double* x, double* y, double* z, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_deinterleave, dim3(grid_for(n, 256)), dim3(256), 0, s, aos, x, y, z, n);
  return hipGetLastError();
}

hipError_t sort_pairs(void* temp, size_t* temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                      const int32_t* vals_in, int32_t* vals_out, int64_t n, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0, 63,
                                            s);
}

}  // namespace icp
