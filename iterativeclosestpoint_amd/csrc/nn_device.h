// nn_device.h — device helpers of the octree search kernels (nn_kernels.hip): wave-wide DPP
// reductions and scans, the reference's box distance, the literal reference-order DFS, the
// per-lane certified search, the window certificate and the cell-table start nodes.
//
// Reference arithmetic (fp64, no contraction; build with -ffp-contract=off):
//   OctreeNode::minDistanceTo   PointCloudRegistration/core/octree.cpp:32-38
//   Octree::searchNearest       octree.cpp:128-173
//   Octree::findNearest         octree.cpp:175-184
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "icp_common.h"
#include "kernels.h"

namespace icp {
namespace dev {

constexpr int kWave = 64;

__device__ __forceinline__ double box_dist(double lx, double ly, double lz, double hx, double hy, double hz,
                                           double qx, double qy, double qz) {
  // OctreeNode::minDistanceTo (octree.cpp:32-38)
  const double dx = smax(0.0, smax(lx - qx, qx - hx));
  const double dy = smax(0.0, smax(ly - qy, qy - hy));
  const double dz = smax(0.0, smax(lz - qz, qz - hz));
  return __builtin_sqrt(dx * dx + dy * dy + dz * dz);
}

// The same without the sqrt: the squared box distance s (monotone in the reference's value).
__device__ __forceinline__ double box_s(double lx, double ly, double lz, double hx, double hy, double hz,
                                        double qx, double qy, double qz) {
  const double dx = smax(0.0, smax(lx - qx, qx - hx));
  const double dy = smax(0.0, smax(ly - qy, qy - hy));
  const double dz = smax(0.0, smax(lz - qz, qz - hz));
  return dx * dx + dy * dy + dz * dz;
}

// ---- wave-wide reductions and scans on DPP (row shifts within 16-lane rows, then
// row_bcast15/31 across rows), no LDS traffic. Every lane of the wave must be active.
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
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// A wave-uniform double moved to scalar registers (fp64 arithmetic is vector-only, so uniform
// results otherwise occupy two vector registers each).
__device__ __forceinline__ double uniform_d(double v) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(b >> 32));
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
// 32-bit wave reductions: row shifts then row broadcasts, each step one DPP-combined VALU
// instruction (the old operand is the operation's identity, so the compiler folds the move).
__device__ __forceinline__ int wave_min_i(int v) {
  constexpr int I = 0x7fffffff;
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x111, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x112, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x114, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x118, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x142, 0xa, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_max_i(int v) {
  constexpr int I = (int)0x80000000;
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x114, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x118, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x143, 0xc, 0xf, false));
  return __builtin_amdgcn_readlane(v, 63);
}
// Steps of the same reductions, exposed so that the row (16-lane) and half (32-lane) partial
// results can be read on the way: after rows_* lane 16 r + 15 holds row r's result, after
// halves_* lanes 31 and 63 hold the halves', after wave_* lane 63 the wave's.
__device__ __forceinline__ int rows_min_i(int v) {
  constexpr int I = 0x7fffffff;
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x111, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x112, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(I, v, 0x114, 0xf, 0xf, false));
  return min(v, __builtin_amdgcn_update_dpp(I, v, 0x118, 0xf, 0xf, false));
}
__device__ __forceinline__ int rows_max_i(int v) {
  constexpr int I = (int)0x80000000;
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(I, v, 0x114, 0xf, 0xf, false));
  return max(v, __builtin_amdgcn_update_dpp(I, v, 0x118, 0xf, 0xf, false));
}
__device__ __forceinline__ int halves_min_i(int v) {
  return min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x142, 0xa, 0xf, false));
}
__device__ __forceinline__ int halves_max_i(int v) {
  return max(v, __builtin_amdgcn_update_dpp((int)0x80000000, v, 0x142, 0xa, 0xf, false));
}
__device__ __forceinline__ int wave_min_from_halves(int v) {
  return min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x143, 0xc, 0xf, false));
}
__device__ __forceinline__ int wave_max_from_halves(int v) {
  return max(v, __builtin_amdgcn_update_dpp((int)0x80000000, v, 0x143, 0xc, 0xf, false));
}
__device__ __forceinline__ float wave_sum_f(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xf, 0xf, true));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false));
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// Order-preserving map of non-NaN floats to int32 (and back: the map is an involution), so that
// float min/max reductions run as integer DPP min/max.
__device__ __forceinline__ int fkey(float f) {
  const int b = __float_as_int(f);
  return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float funkey(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }

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
// Inclusive prefix sum within each 16-lane row (row_shr 1, 2, 4, 8); *total = the row's sum.
__device__ __forceinline__ int row_incl_scan(int v, int row_base, int* total) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  *total = __shfl(v, row_base + 15, kWave);
  return v;
}
// The wave's ballot of a condition, taken on the condition itself: HIP's wballot(int) first
// materialises the bool in a vector register (v_cndmask) and compares it again (v_cmp), two VALU
// instructions per ballot that the compare's own lane mask makes unnecessary.
__device__ __forceinline__ unsigned long long wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
// Position of this lane among the set lanes of a ballot mask.
__device__ __forceinline__ int mask_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// The wave's LDS accesses are complete (a wave reading what its own lanes wrote: no barrier).
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

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

// ---- queries

// Element i of a per-query array addressed by a 32-bit byte offset from the array's (scalar) base:
// global loads/stores in the saddr + 32-bit voffset form, no 64-bit address per lane (the wave
// search's 64-bit query index was spilled to scratch). Shards hold < 2^29 queries (set_source).
template <class T>
__device__ __forceinline__ T& qat(T* base, int32_t i) {
  return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (uint32_t)i * (uint32_t)sizeof(T));
}

// Load query i; with APPLY also src = T * src in place, Eigen's order ((T0 x + T1 y) + T2 z) + T3
// (icpengine.cpp:345; Matrix4d * MatrixXd without FMA on baseline x86-64).
template <bool APPLY>
__device__ __forceinline__ void load_query(const NNLaunch& a, int64_t i, bool active, double& qx, double& qy,
                                           double& qz) {
  if (!active) return;
  qx = a.x[i];
  qy = a.y[i];
  qz = a.z[i];
  if (APPLY) {
    const double* T = a.loop ? a.loop->core.T : a.T;  // the device loop's pending increment
    const double nx = ((T[0] * qx + T[1] * qy) + T[2] * qz) + T[3];
    const double ny = ((T[4] * qx + T[5] * qy) + T[6] * qz) + T[7];
    const double nz = ((T[8] * qx + T[9] * qy) + T[10] * qz) + T[11];
    a.x[i] = nx;
    a.y[i] = ny;
    a.z[i] = nz;
    qx = nx;
    qy = ny;
    qz = nz;
  }
}

// The iterate's transform (the device loop's pending increment, or the launch's), read with scalar
// loads into scalar registers: one pointer select between the kernel argument and global memory
// made it a generic pointer, loaded by flat loads into 24 vector registers (spills in the wave
// search). The device loop's T was written by an earlier kernel of the stream: the scalar cache
// holds nothing of it (it is invalidated at every dispatch) and nothing writes it meanwhile.
typedef const __attribute__((address_space(4))) double* const_dptr;
__device__ __forceinline__ void load_T(const NNLaunch& a, double (&T)[12]) {
  if (a.loop) {
    const_dptr p = (const_dptr)(a.loop->core.T);
#pragma unroll
    for (int k = 0; k < 12; k++) T[k] = p[k];
  } else {
#pragma unroll
    for (int k = 0; k < 12; k++) T[k] = a.T[k];
  }
}

// load_query for a 32-bit index (qat addressing; the wave search), WITHOUT the store of the moved
// query: the wave search stores it with its results (store_query32), so that no store is pending
// while its first loads are waited for.
template <bool APPLY>
__device__ __forceinline__ void load_query32(const NNLaunch& a, int32_t i, bool active, double& qx, double& qy,
                                             double& qz) {
  if (!active) return;
  qx = qat(a.x, i);
  qy = qat(a.y, i);
  qz = qat(a.z, i);
  if (APPLY) {
    double T[12];
    load_T(a, T);
    const double nx = ((T[0] * qx + T[1] * qy) + T[2] * qz) + T[3];
    const double ny = ((T[4] * qx + T[5] * qy) + T[6] * qz) + T[7];
    const double nz = ((T[8] * qx + T[9] * qy) + T[10] * qz) + T[11];
    qx = nx;
    qy = ny;
    qz = nz;
  }
}
template <bool APPLY>
__device__ __forceinline__ void store_query32(const NNLaunch& a, int32_t i, bool active, double qx, double qy,
                                              double qz) {
  if (APPLY && active) {
    qat(a.x, i) = qx;
    qat(a.y, i) = qy;
    qat(a.z, i) = qz;
  }
}

// findNearest's answer when no leaf point ever beat the initial best (octree.cpp:179-183: the
// default index 0), with the residual to that point (icpengine.cpp:193-206).
__device__ __forceinline__ double residual_to(const TgtPt* pts, int32_t pos, double qx, double qy, double qz) {
  const TgtPt p = pts[pos];
  const double dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
  return __builtin_sqrt(dx * dx + dy * dy + dz * dz);
}

// ---- the reference DFS, verbatim order

// Stack entry: bits 0..31 first child record, bits 32..55 up to 8 pending children as 3-bit
// ranks inside the contiguous child block (next child in the low bits), bits 56..59 count.
__device__ __forceinline__ uint64_t pack_entry(int32_t first, uint32_t ranks, uint32_t cnt) {
  return ((uint64_t)(ranks | (cnt << 24)) << 32) | (uint32_t)first;
}

// Octree::searchNearest (octree.cpp:128-173) for one query: box distance with its sqrt, prune
// m*m >= best, children in stable ascending-distance order, strict < in leaf scans. `st` is this
// thread's column of the LDS level stack (stride bs). COUNT also counts node entries and leaf
// points compared (the work of the reference DFS).
template <bool COUNT>
__device__ __forceinline__ void exact_dfs(const NNLaunch& a, double qx, double qy, double qz, unsigned long long* st,
                                          int bs, int32_t& best, double& best_d2, double& visits, double& scanned) {
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

// ---- the certificate
//
// Claim: let d* = fl(d2) of the nearest target point p* and assume no other point has
// fl(d2) <= d* (1 + 2^-48), d* in [2^-900, 2^900] and d* < init (1 - 2^-48) (or d* = 0 with no
// other zero). Then the reference DFS returns p*, whatever its visit order:
//  * rounding is monotone, so for a point p inside a box, fl(d2(p)) >= fl(s(box)) (same
//    operation sequence on coordinates that are at least as far), and the reference's prune
//    value fl(fl(sqrt(s))^2) <= s (1 + 3.0001 * 2^-53) <= d* (1 + 3.0001 * 2^-53);
//  * so a node holding p* can only be pruned against a best within that factor of d*, i.e. by
//    another point inside the window — there is none; p* is scanned, strict < takes it, and no
//    later point can replace it.
// Any search that finds d*, p* and a lower bound of every other point's fl(d2) — in any order —
// can therefore certify a query. Queries that fail (exact or near ties, duplicates, far queries,
// tiny or huge distances) run the reference-order DFS.
constexpr double kWindow = 0x1p-48;
constexpr double kFastPrune = 0x1p-47;

__device__ __forceinline__ bool certified(double best, double second, double init_best) {
  if (best == 0.0) return second > 0.0;
  return best >= 0x1p-900 && best <= 0x1p900 && second > best * (1.0 + kWindow) &&
         best < init_best * (1.0 - kWindow);
}

// 16-bit truncation of a non-negative double: a monotone lower bound (top 16 bits of the bits).
__device__ __forceinline__ uint32_t key16(double v) {
  return (uint32_t)((unsigned long long)__double_as_longlong(v) >> 48);
}

// Per-lane certified search of one query: nearest child first, remaining siblings in octant
// order, levels dropped on a 16-bit lower-bound key; prunes only nodes whose s exceeds
// best (1 + 2^-47), so every point of the certificate window stays visible. Tracks the best,
// the second best and the position of the best.
// Stack entry: bits 0..31 first child record, 32..39 remaining octants, 40..47 the parent's
// child mask, 48..63 key16 lower bound of the remaining children's s.
// budget > 0: give up after that many node visits (returns false: the results are incomplete).
// thr0: the initial prune bound, u (1 + 2^-47) for an upper bound u of the nearest fl(d2) (inf: none).
__device__ __forceinline__ bool fast_dfs(const NNLaunch& a, double qx, double qy, double qz, unsigned long long* st,
                                         int bs, double& best, double& second, int32_t& bpos, int budget = 0,
                                         double thr0 = __builtin_inf()) {
  int visits = 0;
  double thr = thr0;
  uint32_t thr_key = key16(thr0);
  int sp = 0;
  int32_t node = 0;
  const NodeRec* r0 = a.nodes;
  double lx = r0->lo[0], ly = r0->lo[1], lz = r0->lo[2], hx = r0->hi[0], hy = r0->hi[1], hz = r0->hi[2];
  double s = box_s(lx, ly, lz, hx, hy, hz, qx, qy, qz);
  while (true) {
    bool entered = false;
    if (budget > 0 && ++visits > budget) return false;
    if (!(s > thr)) {
      const int2 topo = *reinterpret_cast<const int2*>(&a.nodes[node].first);
      const int32_t first = topo.x;
      const uint32_t meta = (uint32_t)topo.y;
      if (meta & kLeafBit) {
        const int32_t cnt = (int32_t)(meta & ~kLeafBit);
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
  return true;
}

// Append the lanes with `want` to a list, one atomic per wave, lane order kept (the lists stay
// in query order wave by wave, which keeps the follow-up searches coherent). Wave-uniform call.
__device__ __forceinline__ void wave_append(bool want, int64_t i, unsigned* counter, int32_t* list) {
  const unsigned long long m = wballot(want);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(m);
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m));
  base = (unsigned)__builtin_amdgcn_readlane((int)base, leader);
  if (want) list[base + mask_rank(m)] = (int32_t)i;
}

// wave_append that also stores a per-entry payload (the guess u of the ball search).
__device__ __forceinline__ void wave_append_u(bool want, int64_t i, double u, unsigned* counter, int32_t* list,
                                              double* payload) {
  const unsigned long long m = wballot(want);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int leader = __builtin_ctzll(m);
  unsigned base = 0;
  if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m));
  base = (unsigned)__builtin_amdgcn_readlane((int)base, leader);
  if (want) {
    const int off = mask_rank(m);
    list[base + off] = (int32_t)i;
    payload[base + off] = u;
  }
}

// ---- start nodes from the cell tables

// Bits 0..9 of v spread to bits 0, 3, 6, ... (one axis of an octant path prefix).
__device__ __forceinline__ uint32_t spread3(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// Level-L path (cell index along one axis) of coordinate v: the bit path of its comparisons
// with the successive midpoints (x > mid goes high, octree.cpp:105-108), monotone in v.
__device__ __forceinline__ uint32_t axis_path(double v, double lo, double hi, int L) {
  uint32_t path = 0;
  for (int l = 0; l < L; l++) {
    const double m = (lo + hi) / 2;
    const bool up = v > m;
    path = 2u * path + (up ? 1u : 0u);
    lo = up ? m : lo;
    hi = up ? hi : m;
  }
  return path;
}

// Start nodes of a box query from the cell tables: the cells of level L (the octree's own
// midpoint grid) that the box [bl, bh] overlaps, K per lane. The box's cells are an index box
// [il, ih]^3, every one of them meets the box, and every target point inside the box lies in one
// of them; the table gives the node holding all points of a cell (the depth-L node or the leaf
// above it; a leaf spanning several cells is taken once, from its first cell in the box). L is
// the deepest table level at which the box spans at most K G cells (G = lanes of the group).
// Lanes gl < 6 of the group compute the six axis paths. Writes the start nodes to out[0..count)
// and returns count (group-uniform). Every lane of the group must call it.
template <int G, int K>
__device__ __forceinline__ int cell_starts(const NNLaunch& a, double blx, double bly, double blz, double bhx,
                                           double bhy, double bhz, int gl, int gbase, int32_t* out) {
  int L = a.cell_lmax;
  uint32_t path = 0;
  if (gl < 6) {
    const int ax = gl >> 1;
    const double v = (gl & 1) ? (ax == 0 ? bhx : ax == 1 ? bhy : bhz) : (ax == 0 ? blx : ax == 1 ? bly : blz);
    path = axis_path(v, a.root_lo[ax], a.root_hi[ax], L);
  }
  uint32_t ilx, ihx, ily, ihy, ilz, ihz;
  if (G == 64) {
    ilx = (uint32_t)__builtin_amdgcn_readlane((int)path, 0);
    ihx = (uint32_t)__builtin_amdgcn_readlane((int)path, 1);
    ily = (uint32_t)__builtin_amdgcn_readlane((int)path, 2);
    ihy = (uint32_t)__builtin_amdgcn_readlane((int)path, 3);
    ilz = (uint32_t)__builtin_amdgcn_readlane((int)path, 4);
    ihz = (uint32_t)__builtin_amdgcn_readlane((int)path, 5);
  } else {
    ilx = (uint32_t)__shfl((int)path, gbase + 0, kWave);
    ihx = (uint32_t)__shfl((int)path, gbase + 1, kWave);
    ily = (uint32_t)__shfl((int)path, gbase + 2, kWave);
    ihy = (uint32_t)__shfl((int)path, gbase + 3, kWave);
    ilz = (uint32_t)__shfl((int)path, gbase + 4, kWave);
    ihz = (uint32_t)__shfl((int)path, gbase + 5, kWave);
  }
  while (L > 0 && (ihx - ilx + 1) * (ihy - ily + 1) * (ihz - ilz + 1) > (uint32_t)(K * G)) {
    L--;
    ilx >>= 1; ihx >>= 1; ily >>= 1; ihy >>= 1; ilz >>= 1; ihz >>= 1;
  }
  const uint32_t nx = ihx - ilx + 1, ny = ihy - ily + 1, nz = ihz - ilz + 1, ncell = nx * ny * nz;
  const int64_t base = (((int64_t)1 << (3 * L)) - 1) / 7;
  // all K table reads in flight before any is used
  uint32_t cx[K], cy[K], cz[K];
  int32_t e[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t c = (uint32_t)gl + (uint32_t)(k * G);
    e[k] = -1;
    cx[k] = ilx + c % nx;
    cy[k] = ily + (c / nx) % ny;
    cz[k] = ilz + c / (nx * ny);
    if (c < ncell) e[k] = a.cells[base + (spread3(cx[k]) | (spread3(cy[k]) << 1) | (spread3(cz[k]) << 2))];
  }
  int count = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    bool put = false;
    int32_t node = 0;
    if (e[k] >= 0) {
      node = e[k] >> 5;
      const int sh = L - (e[k] & 31);
      const uint32_t fx = ((cx[k] >> sh) << sh) > ilx ? ((cx[k] >> sh) << sh) : ilx;
      const uint32_t fy = ((cy[k] >> sh) << sh) > ily ? ((cy[k] >> sh) << sh) : ily;
      const uint32_t fz = ((cz[k] >> sh) << sh) > ilz ? ((cz[k] >> sh) << sh) : ilz;
      put = cx[k] == fx && cy[k] == fy && cz[k] == fz;
    }
    if (G == 64) {
      const unsigned long long pm = wballot(put);
      if (put) out[count + mask_rank(pm)] = node;
      count += __popcll(pm);
    } else {
      const uint32_t pm = (uint32_t)((wballot(put) >> gbase) & ((1ull << G) - 1ull));
      if (put) out[count + __builtin_popcount(pm & ((1u << gl) - 1u))] = node;
      count += __builtin_popcount(pm);
    }
  }
  return count;
}

// A node record loaded whole: four 16-B loads of one 64-B line, all in flight together.
struct NodeLoad {
  double2 l01, l2h0, h12;
  int4 topo;  // first, meta, depth, pad
};
__device__ __forceinline__ NodeLoad load_node(const NodeRec* rr) {
  NodeLoad n;
  n.l01 = *reinterpret_cast<const double2*>(&rr->lo[0]);
  n.l2h0 = *reinterpret_cast<const double2*>(&rr->lo[2]);
  n.h12 = *reinterpret_cast<const double2*>(&rr->hi[1]);
  n.topo = *reinterpret_cast<const int4*>(&rr->first);
  return n;
}

// Children of an inner node that meet the closed box [bl, bh] (child o spans [lo or mid,
// mid or hi] per axis, octree.cpp:115-120), as a bit mask over octants.
__device__ __forceinline__ uint32_t children_in_box(const NodeLoad& n, uint32_t mask, double blx, double bly,
                                                    double blz, double bhx, double bhy, double bhz) {
  const double lx = n.l01.x, ly = n.l01.y, lz = n.l2h0.x, hx = n.l2h0.y, hy = n.h12.x, hz = n.h12.y;
  const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
  const bool x0 = lx <= bhx && mx >= blx, x1 = mx <= bhx && hx >= blx;
  const bool y0 = ly <= bhy && my >= bly, y1 = my <= bhy && hy >= bly;
  const bool z0 = lz <= bhz && mz >= blz, z1 = mz <= bhz && hz >= blz;
  uint32_t kids = 0;
#pragma unroll
  for (int o = 0; o < 8; o++) {
    const bool hit = ((o & 1) ? x1 : x0) && ((o & 2) ? y1 : y0) && ((o & 4) ? z1 : z0);
    kids |= (hit && ((mask >> o) & 1u)) ? (1u << o) : 0u;
  }
  return kids;
}

// Children of an inner node whose squared box distance to q is <= thr (sphere test).
__device__ __forceinline__ uint32_t children_in_ball(const NodeRec* rr, uint32_t mask, double qx, double qy,
                                                     double qz, double thr) {
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
  uint32_t kids = 0;
#pragma unroll
  for (int o = 0; o < 8; o++) {
    const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
    kids |= (((mask >> o) & 1u) && !(c > thr)) ? (1u << o) : 0u;
  }
  return kids;
}

}  // namespace dev
}  // namespace icp
