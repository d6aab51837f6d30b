// icp_common.h — data layout in HBM and the exact-arithmetic helpers shared by the host
// builder/merger and the gfx950 kernels.
//
// Reference arithmetic being reproduced (all fp64, no contraction: build with -ffp-contract=off):
//   OctreeNode::minDistanceTo      PointCloudRegistration/core/octree.cpp:32-38
//   leaf distance                  octree.cpp:139-144
//   child box from parent + mid    octree.cpp:97-99, :115-120
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define ICP_HD __host__ __device__ __forceinline__
#else
#define ICP_HD inline
#endif

namespace icp {

// One octree node = one 64-byte record (a single cache line, 4 x dwordx4 loads).
// Children of an inner node are stored contiguously, ascending octant, starting at `first`;
// child with octant o sits at first + popcount(mask & ((1 << o) - 1)).
// Leaves point at `count` consecutive entries of the leaf-ordered target array.
struct alignas(64) NodeRec {
  double lo[3];   // min_x, min_y, min_z   (octree.h:12)
  double hi[3];   // max_x, max_y, max_z
  int32_t first;  // inner: first child record; leaf: first leaf-ordered point
  uint32_t meta;  // bit31 = leaf; leaf: bits 0..30 = point count; inner: bits 0..7 = child mask
  int32_t depth;  // depth of this node (root 0)
  int32_t pad;
};
static_assert(sizeof(NodeRec) == 64, "NodeRec must be one 64-byte line");

constexpr uint32_t kLeafBit = 0x80000000u;

// The tight box of a node: the bounding box of the target points below it, fp32 rounded outwards
// (k_tight_boxes). The certified searches prune with it where the reference's own order does not
// matter (a node's points all lie inside, so its squared box distance bounds every point's fl(d2)
// from below, as the cell box does); cells are cubes, the points of a surface a thin slab: a far
// query's ball dips into far fewer tight boxes than cells. One per NodeRec, 32 B.
struct alignas(32) TBox {
  float lo[3];
  float hi[3];
  float pad[2];
};
static_assert(sizeof(TBox) == 32, "TBox is 32 bytes");

// Target point in leaf order (leaves in preorder, points in ascending original index —
// the order the reference scans point_indices, octree.cpp:139).
struct alignas(32) TgtPt {
  double x, y, z;
  int32_t orig;  // original index into the caller's target array
  float sep;     // lower bound of the exact distance from this point to every other target point
                 // (0 = none known; computed on the device after either build, k_target_sep);
                 // its sign bit: this point is a copy of an earlier one (k_mark_copies)
};
// Points a target point is compared with, looking back in leaf order, for its copy flag: a leaf
// holds at most max_points (default 10) points unless it sits at the maximum depth.
constexpr int kCopyWindow = 32;
// The copy flag from the 64-bit word (orig, sep) of a point: sep's sign bit is the word's.
ICP_HD bool tgt_copy_word(double w) {
  long long b;
  __builtin_memcpy(&b, &w, 8);
  return b < 0;
}
static_assert(sizeof(TgtPt) == 32, "TgtPt must be 32 bytes");

// Residual moments of one block / rank: count, mean, centered M2 (Chan et al. merge),
// plus finite min/max and the count of non-finite distances (icpengine.cpp:192-228).
struct Moments {
  double n, mean, m2, dmin, dmax, nbad, pad0, pad1;
};
static_assert(sizeof(Moments) == 64, "Moments is 8 doubles");

// Valid-pair moments: count, sum of d^2 (RMSE, icpengine.cpp:274-278), centroids of the
// source (a) and matched target (b) points, centered cross-covariance
// C = sum (a - mean_a)(b - mean_b)^T (row-major), i.e. H of icpengine.cpp:86-90.
struct CovMoments {
  double n, sum_d2;
  double ma[3], mb[3];
  double c[9];
  double pad[3];
};
static_assert(sizeof(CovMoments) == 160, "CovMoments is 20 doubles");

// std::max(a, b) == (a < b) ? b : a, NaN behaviour included.
ICP_HD double smax(double a, double b) { return (a < b) ? b : a; }

ICP_HD Moments moments_identity() {
  Moments m;
  m.n = 0; m.mean = 0; m.m2 = 0;
  m.dmin = 1.7976931348623157e308; m.dmax = 0; m.nbad = 0; m.pad0 = 0; m.pad1 = 0;
  return m;
}

// Chan/Golub/LeVeque pairwise merge; deterministic for a fixed merge tree.
ICP_HD Moments moments_merge(const Moments& a, const Moments& b) {
  if (b.n == 0) {
    Moments r = a;
    r.nbad = a.nbad + b.nbad;
    return r;
  }
  if (a.n == 0) {
    Moments r = b;
    r.nbad = a.nbad + b.nbad;
    return r;
  }
  Moments r;
  r.n = a.n + b.n;
  double delta = b.mean - a.mean;
  r.mean = a.mean + delta * (b.n / r.n);
  r.m2 = (a.m2 + b.m2) + (delta * delta) * ((a.n * b.n) / r.n);
  r.dmin = a.dmin < b.dmin ? a.dmin : b.dmin;
  r.dmax = a.dmax > b.dmax ? a.dmax : b.dmax;
  r.nbad = a.nbad + b.nbad;
  r.pad0 = 0; r.pad1 = 0;
  return r;
}

ICP_HD CovMoments cov_identity() {
  CovMoments c;
  c.n = 0; c.sum_d2 = 0;
  for (int k = 0; k < 3; k++) { c.ma[k] = 0; c.mb[k] = 0; }
  for (int k = 0; k < 9; k++) c.c[k] = 0;
  c.pad[0] = 0; c.pad[1] = 0; c.pad[2] = 0;
  return c;
}

ICP_HD CovMoments cov_merge(const CovMoments& a, const CovMoments& b) {
  if (b.n == 0) return a;
  if (a.n == 0) return b;
  CovMoments r;
  r.n = a.n + b.n;
  r.sum_d2 = a.sum_d2 + b.sum_d2;
  const double wb = b.n / r.n;
  const double f = (a.n * b.n) / r.n;
  double da[3], db[3];
  for (int k = 0; k < 3; k++) {
    da[k] = b.ma[k] - a.ma[k];
    db[k] = b.mb[k] - a.mb[k];
    r.ma[k] = a.ma[k] + da[k] * wb;
    r.mb[k] = a.mb[k] + db[k] * wb;
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r.c[3 * i + j] = (a.c[3 * i + j] + b.c[3 * i + j]) + (da[i] * db[j]) * f;
  r.pad[0] = 0; r.pad[1] = 0; r.pad[2] = 0;
  return r;
}

// Threshold rule. Engine (icpengine.cpp:249-255): iteration 0 uses
// mean + max(k*std, 0.5*mean), later mean + k*std. CLI (icp_registration.cpp:523): mean + 3*std.
ICP_HD double cull_threshold(double mean, double sd, double k_sigma, int iter, int engine_rules) {
  if (engine_rules && iter == 0) return mean + smax(k_sigma * sd, mean * 0.5);
  return mean + k_sigma * sd;
}

}  // namespace icp
