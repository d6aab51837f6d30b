// util_kernels.hip — layout kernels around the search: the standalone transform
// (icpengine.cpp:345-346, src = T * src in Eigen's order) and the AoS <-> SoA conversions at the
// boundary (caller's AoS xyz, pointcloud.h:12-23 / the kd-ordered SoA source in HBM).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace icp {

namespace {

struct T12 {
  double v[12];
};

__global__ void k_apply(T12 T, double* x, double* y, double* z, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double qx = x[i], qy = y[i], qz = z[i];
  x[i] = ((T.v[0] * qx + T.v[1] * qy) + T.v[2] * qz) + T.v[3];
  y[i] = ((T.v[4] * qx + T.v[5] * qy) + T.v[6] * qz) + T.v[7];
  z[i] = ((T.v[8] * qx + T.v[9] * qy) + T.v[10] * qz) + T.v[11];
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

// x[k] = aos[perm[k]] (the kd-ordered SoA source from the caller's AoS cloud)
__global__ void k_gather_deinterleave(const double* aos, const int32_t* perm, double* x, double* y, double* z,
                                      int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t j = perm[i];
  x[i] = aos[3 * j];
  y[i] = aos[3 * j + 1];
  z[i] = aos[3 * j + 2];
}

// The copy flag of the leaf-ordered target (TgtPt::sep's sign bit, kCopyWindow): a point whose
// coordinates equal an earlier point's among the kCopyWindow points before it. Identical points
// share a leaf (the same octant at every split), so the earlier one comes first in the leaf's
// order, and the reference's strict < keeps it: a flagged copy is never the answer, and its
// distance is its earlier twin's. A copy further back stays unflagged (only a search's shortcut
// is lost; a max-depth leaf of many points).
__global__ void k_mark_copies(TgtPt* pts, int64_t n) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const double x = pts[j].x, y = pts[j].y, z = pts[j].z;
  bool copy = false;
  for (int m = 1; m <= kCopyWindow && j - m >= 0 && !copy; m++) {
    const TgtPt& p = pts[j - m];
    copy = p.x == x && p.y == y && p.z == z;
  }
  if (copy) pts[j].sep = -0.0f;  // a copy's separation is 0 (certify_prev): the sign is the flag
}

// v rounded down / up to fp32 (finite v; the conversion rounds to nearest, then one ulp outwards
// when it went the wrong way)
__device__ __forceinline__ float f32_step(float f, bool up) {
  if (f == 0.f) return up ? 0x1p-149f : -0x1p-149f;
  const int b = __float_as_int(f);
  return __int_as_float((f > 0.f) == up ? b + 1 : b - 1);
}
__device__ __forceinline__ float f32_down(double v) {
  const float f = (float)v;
  return (double)f > v ? f32_step(f, false) : f;
}
__device__ __forceinline__ float f32_up(double v) {
  const float f = (float)v;
  return (double)f < v ? f32_step(f, true) : f;
}

// Tight boxes of the nodes at one depth (deepest first): a leaf's from its points, an inner node's
// the union of its children's (one level deeper, done by the previous launch).
__global__ void k_tight_boxes(const NodeRec* nodes, const TgtPt* pts, TBox* tb, int64_t n_nodes, int depth) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_nodes) return;
  const NodeRec& nd = nodes[j];
  if (nd.depth != depth) return;
  TBox b;
  if (nd.meta & kLeafBit) {
    double lo[3] = {__builtin_inf(), __builtin_inf(), __builtin_inf()};
    double hi[3] = {-__builtin_inf(), -__builtin_inf(), -__builtin_inf()};
    const int32_t cnt = (int32_t)(nd.meta & ~kLeafBit);
    for (int32_t k = 0; k < cnt; k++) {
      const TgtPt& p = pts[nd.first + k];
      lo[0] = p.x < lo[0] ? p.x : lo[0];
      lo[1] = p.y < lo[1] ? p.y : lo[1];
      lo[2] = p.z < lo[2] ? p.z : lo[2];
      hi[0] = p.x > hi[0] ? p.x : hi[0];
      hi[1] = p.y > hi[1] ? p.y : hi[1];
      hi[2] = p.z > hi[2] ? p.z : hi[2];
    }
    for (int k = 0; k < 3; k++) {
      b.lo[k] = cnt > 0 ? f32_down(lo[k]) : __builtin_inff();  // an empty leaf: an empty box
      b.hi[k] = cnt > 0 ? f32_up(hi[k]) : -__builtin_inff();
    }
  } else {
    for (int k = 0; k < 3; k++) {
      b.lo[k] = __builtin_inff();
      b.hi[k] = -__builtin_inff();
    }
    const int nk = __builtin_popcount(nd.meta & 0xffu);
    for (int c = 0; c < nk; c++) {
      const TBox& cb = tb[nd.first + c];
      for (int k = 0; k < 3; k++) {
        b.lo[k] = cb.lo[k] < b.lo[k] ? cb.lo[k] : b.lo[k];
        b.hi[k] = cb.hi[k] > b.hi[k] ? cb.hi[k] : b.hi[k];
      }
    }
  }
  b.pad[0] = b.pad[1] = 0.f;
  tb[j] = b;
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

hipError_t launch_tight_boxes(const NodeRec* nodes, const TgtPt* pts, TBox* tb, int64_t n_nodes, int max_depth,
                              hipStream_t s) {
  if (n_nodes <= 0) return hipSuccess;
  for (int d = max_depth; d >= 0; d--)
    hipLaunchKernelGGL(k_tight_boxes, dim3(grid_for(n_nodes, 256)), dim3(256), 0, s, nodes, pts, tb, n_nodes, d);
  return hipGetLastError();
}

hipError_t launch_mark_copies(TgtPt* pts, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mark_copies, dim3(grid_for(n, 256)), dim3(256), 0, s, pts, n);
  return hipGetLastError();
}

hipError_t launch_gather_deinterleave(const double* aos, const int32_t* perm, double* x, double* y, double* z,
                                      int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_deinterleave, dim3(grid_for(n, 256)), dim3(256), 0, s, aos, perm, x, y, z, n);
  return hipGetLastError();
}

hipError_t launch_apply(const double T[12], double* x, double* y, double* z, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  T12 t;
  for (int k = 0; k < 12; k++) t.v[k] = T[k];
  hipLaunchKernelGGL(k_apply, dim3(grid_for(n, 256)), dim3(256), 0, s, t, x, y, z, n);
  return hipGetLastError();
}

hipError_t launch_scatter_aos(const int32_t* perm, const double* x, const double* y, const double* z, double* aos,
                              int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_aos, dim3(grid_for(n, 256)), dim3(256), 0, s, perm, x, y, z, aos, n);
  return hipGetLastError();
}

hipError_t launch_scatter_corr(const int32_t* perm, const int32_t* pos, const TgtPt* pts, int32_t* idx_out,
                               const double* dist_in, double* dist_out, int64_t n, hipStream_t s) {
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

}  // namespace icp
