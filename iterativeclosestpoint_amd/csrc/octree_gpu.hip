// octree_gpu.hip — device build of the linear octree (§8 row f2): the same arrays, bit for bit,
// as the host builder (octree_build.cpp), which follows Octree::Octree + buildTree
// (PointCloudRegistration/core/octree.cpp:41-126). No recursion and no per-node work lists:
//
//  1. root box: min/max of the target +- 0.001 (octree.cpp:47-66), non-finite count.
//  2. path key of every point: descending from the root box, level l's octant (x > mid -> 1,
//     y > mid -> 2, z > mid -> 4, octree.cpp:105-108) goes into bits 3 (max_d - l) .. +2, the box
//     halves exactly as the child boxes are derived (octree.cpp:97-99, :115-120). Points sharing a
//     node at depth d share the key's top d levels, so sorting by key puts every node's points in
//     one run, nodes in preorder (ascending octant = the reference's child order).
//  3. leaf depth of every point without building anything: with m = max_pts, the node at depth d
//     holding point i has more than m points iff some m+1 consecutive sorted points containing i
//     share their top d levels. So D_i = min(max_d, 1 + max over windows [j, j+m] containing i of
//     lcp(key_j, key_{j+m})) (the leaf rule |idx| <= m || depth >= max_d, octree.cpp:88).
//  4. truncate each key to its leaf depth and sort again, stably from the ORIGINAL order: leaves
//     in preorder, points inside a leaf in ascending original index (the reference's
//     point_indices order, octree.cpp:139) — the leaf-ordered target array.
//  5. nodes: point j starts the nodes at depths c_j+1 .. D_j, c_j = deepest node shared with
//     point j-1; an exclusive scan gives every node its preorder rank. The parent of a node is the
//     last node of depth d-1 before it in preorder (binary search in the per-depth list).
//  6. record numbering of the host builder: a parent's children form one block, blocks allocated
//     when the parent is expanded, i.e. in preorder of the inner nodes — first child id =
//     1 + exclusive scan of child counts over the preorder; a child's id = that + its rank among
//     its siblings.
// Depths up to 21 (63 key bits); deeper trees use the host builder.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <string>
#include <vector>

#include "octree_gpu.h"

namespace icp {

namespace {

constexpr int kTB = 256;

inline unsigned grid_for(int64_t n, int tb) {
  int64_t g = (n + tb - 1) / tb;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Common top levels of two max_d-level keys (max_d when equal).
__device__ __forceinline__ int lcp_levels(uint64_t a, uint64_t b, int max_d) {
  const uint64_t x = a ^ b;
  if (x == 0) return max_d;
  const int hb = 63 - __clzll((long long)x);  // highest differing bit
  return max_d - hb / 3 - 1;
}

__global__ void __launch_bounds__(kTB) k_bbox_partial(const double* __restrict__ xyz, int64_t n,
                                                      double* __restrict__ part, unsigned int* nbad) {
  __shared__ double red[6][kTB];
  double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  unsigned bad = 0;
  for (int64_t i = blockIdx.x * (int64_t)kTB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kTB) {
    for (int a = 0; a < 3; a++) {
      const double v = xyz[3 * i + a];
      if (!isfinite(v)) {
        bad++;
        continue;
      }
      lo[a] = v < lo[a] ? v : lo[a];
      hi[a] = v > hi[a] ? v : hi[a];
    }
  }
  if (bad) atomicAdd(nbad, bad);
  for (int a = 0; a < 3; a++) {
    red[a][threadIdx.x] = lo[a];
    red[3 + a][threadIdx.x] = hi[a];
  }
  __syncthreads();
  for (int w = kTB / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      for (int a = 0; a < 3; a++) {
        const double l2 = red[a][threadIdx.x + w], h2 = red[3 + a][threadIdx.x + w];
        if (l2 < red[a][threadIdx.x]) red[a][threadIdx.x] = l2;
        if (h2 > red[3 + a][threadIdx.x]) red[3 + a][threadIdx.x] = h2;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[6 * (int64_t)blockIdx.x + threadIdx.x] = red[threadIdx.x][0];
}

// Root box = extreme coordinates -+ eps (octree.cpp:47-66; eps = 0.001, :63-66). min/max of
// finite doubles does not depend on the order (a signed-zero pick is absorbed by the -+ eps).
__global__ void k_bbox_final(const double* __restrict__ part, int nparts, double* __restrict__ box) {
  if (threadIdx.x >= 6) return;
  const int a = threadIdx.x;
  double v = part[a];
  for (int p = 1; p < nparts; p++) {
    const double w = part[6 * (int64_t)p + a];
    if (a < 3) v = w < v ? w : v;
    else v = w > v ? w : v;
  }
  const double eps = 0.001;
  box[a] = a < 3 ? v - eps : v + eps;
}

__global__ void __launch_bounds__(kTB) k_path_keys(const double* __restrict__ xyz, int64_t n,
                                                   const double* __restrict__ box, int max_d,
                                                   uint64_t* __restrict__ keys, int32_t* __restrict__ iota) {
  const int64_t i = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (i >= n) return;
  const double px = xyz[3 * i], py = xyz[3 * i + 1], pz = xyz[3 * i + 2];
  double lx = box[0], ly = box[1], lz = box[2], hx = box[3], hy = box[4], hz = box[5];
  uint64_t key = 0;
  for (int l = 1; l <= max_d; l++) {
    const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;  // octree.cpp:97-99
    uint64_t o = 0;
    if (px > mx) { o |= 1; lx = mx; } else { hx = mx; }
    if (py > my) { o |= 2; ly = my; } else { hy = my; }
    if (pz > mz) { o |= 4; lz = mz; } else { hz = mz; }
    key |= o << (3 * (max_d - l));
  }
  keys[i] = key;
  iota[i] = (int32_t)i;
}

// L[j] = lcp(key_j, key_{j+m}) for j in [0, n - m).
__global__ void __launch_bounds__(kTB) k_window_lcp(const uint64_t* __restrict__ K, int64_t nL, int64_t m,
                                                    int max_d, uint8_t* __restrict__ L) {
  const int64_t j = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (j >= nL) return;
  L[j] = (uint8_t)lcp_levels(K[j], K[j + m], max_d);
}

// Doubling step of the range max: out[j] = max(in[j], in[min(j + h, nL - 1)]).
__global__ void __launch_bounds__(kTB) k_range_max_step(const uint8_t* __restrict__ in, int64_t nL, int64_t h,
                                                        uint8_t* __restrict__ out) {
  const int64_t j = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (j >= nL) return;
  const int64_t k = j + h < nL ? j + h : nL - 1;
  const uint8_t a = in[j], b = in[k];
  out[j] = a > b ? a : b;
}

// Leaf depth D_i of sorted point i and its truncated key, scattered to the original order.
// L = per-window lcp; W = its range max over spans of length span (W == L, span == 1 when the
// doubling was skipped).
__global__ void __launch_bounds__(kTB) k_leaf_depth(const uint64_t* __restrict__ K, const int32_t* __restrict__ idx,
                                                    int64_t n, int64_t m, int max_d, const uint8_t* __restrict__ L,
                                                    const uint8_t* __restrict__ W, int64_t span,
                                                    uint64_t* __restrict__ tk_orig, uint8_t* __restrict__ d_orig) {
  const int64_t i = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (i >= n) return;
  int D = 0;
  if (max_d > 0 && n > m) {
    const int64_t nL = n - m;
    const int64_t a = i - m > 0 ? i - m : 0;
    const int64_t b = i < nL - 1 ? i : nL - 1;  // windows [j, j+m] containing i: j in [a, b]
    int best = 0;
    if (b - a + 1 >= span) {
      const uint8_t u = W[a], v = W[b - span + 1];
      best = u > v ? u : v;
    } else {
      for (int64_t j = a; j <= b; j++) best = L[j] > best ? L[j] : best;
    }
    D = best + 1 < max_d ? best + 1 : max_d;
  }
  const int sh = 3 * (max_d - D);
  const uint64_t k = K[i];
  const uint64_t tk = sh >= 64 ? 0 : (k >> sh) << sh;
  const int32_t o = idx[i];
  tk_orig[o] = tk;
  d_orig[o] = (uint8_t)D;
}

// Per leaf-ordered point j: D_j, c_j (deepest node shared with point j-1, -1 for j = 0), the
// number of nodes starting at j (D_j - c_j) and whether a leaf starts at j.
__global__ void __launch_bounds__(kTB) k_node_starts(const uint64_t* __restrict__ TK, const int32_t* __restrict__ idx2,
                                                     const uint8_t* __restrict__ d_orig, int64_t n, int max_d,
                                                     uint8_t* __restrict__ D2, int8_t* __restrict__ c_out,
                                                     int64_t* __restrict__ nstart, int64_t* __restrict__ leaf_flag,
                                                     int32_t* __restrict__ pos0, unsigned int* __restrict__ maxdep) {
  const int64_t j = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (j >= n) return;
  const int32_t o = idx2[j];
  const int D = d_orig[o];
  int c = -1;
  if (j > 0) {
    const int Dp = d_orig[idx2[j - 1]];
    c = lcp_levels(TK[j], TK[j - 1], max_d);
    c = c < D ? c : D;
    c = c < Dp ? c : Dp;
  }
  D2[j] = (uint8_t)D;
  c_out[j] = (int8_t)c;
  nstart[j] = D - c;
  leaf_flag[j] = D - c > 0 ? 1 : 0;
  if (o == 0) *pos0 = (int32_t)j;
  if (D - c > 0) atomicMax(maxdep, (unsigned)D);
}

__global__ void __launch_bounds__(kTB) k_emit_nodes(const uint8_t* __restrict__ D2, const int8_t* __restrict__ c_in,
                                                    const int64_t* __restrict__ base, const int64_t* __restrict__ leaf_ix,
                                                    int64_t n, int32_t* __restrict__ ns, uint8_t* __restrict__ nd,
                                                    int32_t* __restrict__ leaf_start) {
  const int64_t j = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (j >= n) return;
  const int D = D2[j], c = c_in[j];
  if (D - c <= 0) return;
  int64_t r = base[j];
  for (int d = c + 1; d <= D; d++, r++) {
    ns[r] = (int32_t)j;
    nd[r] = (uint8_t)d;
  }
  leaf_start[leaf_ix[j]] = (int32_t)j;
}

__global__ void __launch_bounds__(kTB) k_iota(int32_t* __restrict__ v, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}

// Per-depth spans of the depth-sorted node list and each node's position inside its span.
__global__ void __launch_bounds__(kTB) k_level_spans(const uint8_t* __restrict__ dk, const int32_t* __restrict__ lv,
                                                     int64_t nn, int32_t* __restrict__ lstart, int32_t* __restrict__ lend) {
  const int64_t k = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (k >= nn) return;
  const uint8_t d = dk[k];
  if (k == 0 || dk[k - 1] != d) lstart[d] = (int32_t)k;
  if (k == nn - 1 || dk[k + 1] != d) lend[d] = (int32_t)(k + 1);
}

__global__ void __launch_bounds__(kTB) k_level_pos(const uint8_t* __restrict__ dk, const int32_t* __restrict__ lv,
                                                   int64_t nn, const int32_t* __restrict__ lstart,
                                                   int32_t* __restrict__ lpos) {
  const int64_t k = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (k >= nn) return;
  lpos[lv[k]] = (int32_t)(k - lstart[dk[k]]);
}

// Parent of node r = last node of depth d-1 before r in preorder; child count and octant mask
// of the parent (children only exist when non-empty, octree.cpp:113).
__global__ void __launch_bounds__(kTB) k_parents(const int32_t* __restrict__ ns, const uint8_t* __restrict__ nd,
                                                 const uint64_t* __restrict__ TK, int64_t nn, int max_d,
                                                 const int32_t* __restrict__ lv, const int32_t* __restrict__ lstart,
                                                 const int32_t* __restrict__ lend, int32_t* __restrict__ parent,
                                                 int32_t* __restrict__ nch, uint32_t* __restrict__ mask) {
  const int64_t r = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (r >= nn) return;
  if (r == 0) {
    parent[0] = -1;
    return;
  }
  const int d = nd[r];
  int32_t p;
  if (nd[r - 1] == d - 1) {
    p = (int32_t)(r - 1);  // first child: right after its parent in preorder
  } else {
    // lv[lo .. hi) ascending preorder ranks of depth d-1; find the last one < r
    int32_t lo = lstart[d - 1], hi = lend[d - 1];
    while (hi - lo > 1) {
      const int32_t mid = lo + (hi - lo) / 2;
      if (lv[mid] < r) lo = mid;
      else hi = mid;
    }
    p = lv[lo];
  }
  parent[r] = p;
  const uint32_t oct = (uint32_t)(TK[ns[r]] >> (3 * (max_d - d))) & 7u;
  atomicAdd(&nch[p], 1);
  atomicOr(&mask[p], 1u << oct);
}

// Node records in the host builder's numbering (children blocks allocated in preorder of the
// inner nodes) and the leaf-ordered target points.
__global__ void __launch_bounds__(kTB) k_write_nodes(const int32_t* __restrict__ ns, const uint8_t* __restrict__ nd,
                                                     const uint64_t* __restrict__ TK, const uint8_t* __restrict__ D2,
                                                     const int64_t* __restrict__ leaf_ix,
                                                     const int32_t* __restrict__ leaf_start, int64_t n_leaves,
                                                     int64_t n, int64_t nn, int max_d, const double* __restrict__ box,
                                                     const int32_t* __restrict__ parent, const int32_t* __restrict__ lpos,
                                                     const int32_t* __restrict__ fcx, const uint32_t* __restrict__ mask,
                                                     NodeRec* __restrict__ out) {
  const int64_t r = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (r >= nn) return;
  const int32_t j = ns[r];
  const int d = nd[r];
  int64_t id = 0;
  if (r > 0) {
    const int32_t p = parent[r];
    id = 1 + (int64_t)fcx[p] + (lpos[r] - lpos[p + 1]);
  }
  const uint64_t key = TK[j];
  double lx = box[0], ly = box[1], lz = box[2], hx = box[3], hy = box[4], hz = box[5];
  for (int l = 1; l <= d; l++) {
    const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
    const uint32_t o = (uint32_t)(key >> (3 * (max_d - l))) & 7u;
    if (o & 1) lx = mx; else hx = mx;  // child box, octree.cpp:115-120
    if (o & 2) ly = my; else hy = my;
    if (o & 4) lz = mz; else hz = mz;
  }
  NodeRec rec;
  rec.lo[0] = lx; rec.lo[1] = ly; rec.lo[2] = lz;
  rec.hi[0] = hx; rec.hi[1] = hy; rec.hi[2] = hz;
  if (d == D2[j]) {
    const int64_t li = leaf_ix[j];
    const int64_t end = li + 1 < n_leaves ? leaf_start[li + 1] : n;
    rec.first = j;
    rec.meta = kLeafBit | (uint32_t)(end - j);
  } else {
    rec.first = 1 + fcx[r];
    rec.meta = mask[r];
  }
  rec.depth = d;
  rec.pad = 0;
  out[id] = rec;
}

__global__ void __launch_bounds__(kTB) k_write_points(const double* __restrict__ xyz, const int32_t* __restrict__ idx2,
                                                      int64_t n, TgtPt* __restrict__ pts) {
  const int64_t j = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (j >= n) return;
  const int32_t o = idx2[j];
  TgtPt p;
  p.x = xyz[3 * (int64_t)o];
  p.y = xyz[3 * (int64_t)o + 1];
  p.z = xyz[3 * (int64_t)o + 2];
  p.orig = o;
  p.sep = 0.f;
  pts[j] = p;
}

__global__ void k_total(const int64_t* __restrict__ excl, const int64_t* __restrict__ last_in, int64_t n,
                        int64_t* __restrict__ out) {
  *out = excl[n - 1] + last_in[n - 1];
}

// Scratch arrays, freed on every exit path.
struct Scratch {
  std::vector<void*> ptrs;
  ~Scratch() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  hipError_t alloc(T** p, size_t count) {
    *p = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), (count ? count : 1) * sizeof(T));
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
};

// Cell table of level L: entry e (an L-level path prefix, level 1 in the top 3 bits) = the
// node holding every target point of that cell: the node at depth L, or the leaf above it, as
// (node id << 5) | node depth; -1 when the cell holds no point (a child on the path is absent).
__global__ void __launch_bounds__(kTB) k_cell_table(const NodeRec* __restrict__ nodes, int L, int64_t nent,
                                                    int32_t* __restrict__ table) {
  const int64_t e = blockIdx.x * (int64_t)kTB + threadIdx.x;
  if (e >= nent) return;
  int32_t node = 0;
  int d = 0;
  for (; d < L; d++) {
    const int2 topo = *reinterpret_cast<const int2*>(&nodes[node].first);
    const uint32_t meta = (uint32_t)topo.y;
    if (meta & kLeafBit) break;
    const uint32_t o = (uint32_t)(e >> (3 * (L - 1 - d))) & 7u;
    if (!((meta >> o) & 1u)) {
      node = -1;
      break;
    }
    node = topo.x + __builtin_popcount(meta & 0xffu & ((1u << o) - 1u));
  }
  table[e] = node < 0 ? -1 : (int32_t)(((uint32_t)node << 5) | (uint32_t)d);
}

}  // namespace

int64_t cell_table_entries(int lmax) {
  int64_t tot = 0, w = 1;
  for (int l = 0; l <= lmax; l++, w *= 8) tot += w;
  return tot;
}

int64_t cell_table_offset(int l) { return l == 0 ? 0 : cell_table_entries(l - 1); }

int cell_table_depth(int64_t n_leaves, int max_inner_depth) {
  // about eight cells per leaf at the deepest table level (a wave's box then spans mostly
  // leaves there), at most 9 levels (153M entries, 0.6 GB)
  int l = 1;
  while (l < 9 && ((int64_t)1 << (3 * l)) < 8 * n_leaves) l++;
  if (l > max_inner_depth + 1) l = max_inner_depth + 1;
  return l < 0 ? 0 : l;
}

hipError_t build_cell_tables(const NodeRec* nodes, int lmax, int32_t* tables, hipStream_t s) {
  for (int l = 0; l <= lmax; l++) {
    const int64_t nent = (int64_t)1 << (3 * l);
    hipLaunchKernelGGL(k_cell_table, dim3(grid_for(nent, kTB)), dim3(kTB), 0, s, nodes, l, nent,
                       tables + cell_table_offset(l));
  }
  return hipGetLastError();
}

namespace {

}  // namespace

#define OCT_TRY(expr)                                      \
  do {                                                     \
    hipError_t e_ = (expr);                                \
    if (e_ != hipSuccess) {                                \
      *why = std::string(#expr) + ": " + hipGetErrorString(e_); \
      return e_ == hipErrorOutOfMemory ? -2 : -3;          \
    }                                                      \
  } while (0)

int gpu_build_octree(const double* xyz, int64_t n, int max_pts, int max_d, hipStream_t s, GpuOctree* out,
                     std::string* why) {
  *out = GpuOctree();
  if (n <= 0 || n > (int64_t)0x7fffffff) {
    *why = "target size out of range (int32 indices, as the reference)";
    return 1;
  }
  if (max_d < 0 || max_d > kGpuBuildMaxDepth) {
    *why = "max_depth beyond the device build's 21 levels";
    return 1;
  }
  const int64_t m = max_pts > 0 ? max_pts : 0;  // count <= max_pts with max_pts < 0 never holds
  Scratch S;

  // 1. root box
  const int nbb = (int)std::min<int64_t>(1024, grid_for(n, kTB));
  double *part = nullptr, *box = nullptr;
  unsigned int* u32 = nullptr;  // [0] non-finite count, [1] max leaf depth
  int32_t* pos0 = nullptr;
  int64_t* total = nullptr;     // [0] nodes, [1] leaves
  OCT_TRY(S.alloc(&part, 6 * (size_t)nbb));
  OCT_TRY(S.alloc(&box, 6));
  OCT_TRY(S.alloc(&u32, 2));
  OCT_TRY(S.alloc(&pos0, 1));
  OCT_TRY(S.alloc(&total, 2));
  OCT_TRY(hipMemsetAsync(u32, 0, 2 * sizeof(unsigned int), s));
  hipLaunchKernelGGL(k_bbox_partial, dim3(nbb), dim3(kTB), 0, s, xyz, n, part, u32);
  hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(64), 0, s, part, nbb, box);
  OCT_TRY(hipGetLastError());
  unsigned int nbad = 0;
  OCT_TRY(hipMemcpyAsync(&nbad, u32, sizeof(nbad), hipMemcpyDeviceToHost, s));
  OCT_TRY(hipStreamSynchronize(s));
  if (nbad) {
    *why = "target contains non-finite coordinates";
    return 1;
  }

  // 2. path keys, first sort
  uint64_t *keys = nullptr, *K = nullptr;
  int32_t *iota = nullptr, *idx = nullptr;
  OCT_TRY(S.alloc(&keys, n));
  OCT_TRY(S.alloc(&K, n));
  OCT_TRY(S.alloc(&iota, n));
  OCT_TRY(S.alloc(&idx, n));
  hipLaunchKernelGGL(k_path_keys, dim3(grid_for(n, kTB)), dim3(kTB), 0, s, xyz, n, box, max_d, keys, iota);
  OCT_TRY(hipGetLastError());
  const int end_bit = max_d > 0 ? 3 * max_d : 1;
  size_t tb_sort = 0;
  OCT_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, keys, K, iota, idx, (int)n, 0, end_bit, s));
  void* tmp = nullptr;
  size_t tb_scan = 0;
  int64_t* dummy64 = nullptr;
  OCT_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb_scan, dummy64, dummy64, (int)n, s));
  size_t tb = std::max(tb_sort, tb_scan);
  OCT_TRY(S.alloc(reinterpret_cast<uint8_t**>(&tmp), tb));
  OCT_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb_sort, keys, K, iota, idx, (int)n, 0, end_bit, s));

  // 3. leaf depth per point (window lcp + range max), truncated keys in the original order
  uint8_t *L = nullptr, *W = nullptr, *W2 = nullptr, *d_orig = nullptr;
  uint64_t* tk_orig = keys;  // reuse
  OCT_TRY(S.alloc(&d_orig, n));
  int64_t span = 1;
  const uint8_t* Wfinal = nullptr;
  if (max_d > 0 && n > m) {
    const int64_t nL = n - m;
    OCT_TRY(S.alloc(&L, nL));
    hipLaunchKernelGGL(k_window_lcp, dim3(grid_for(nL, kTB)), dim3(kTB), 0, s, K, nL, m, max_d, L);
    OCT_TRY(hipGetLastError());
    Wfinal = L;
    if (m >= 32) {  // range max over spans 2^k <= m + 1 by doubling
      OCT_TRY(S.alloc(&W, nL));
      OCT_TRY(S.alloc(&W2, nL));
      const uint8_t* in = L;
      uint8_t* o = W;
      while (2 * span <= m + 1) {
        hipLaunchKernelGGL(k_range_max_step, dim3(grid_for(nL, kTB)), dim3(kTB), 0, s, in, nL, span, o);
        OCT_TRY(hipGetLastError());
        span *= 2;
        in = o;
        o = (o == W) ? W2 : W;
      }
      Wfinal = in;
    } else {
      span = m + 2;  // never satisfied: direct loop over the <= m + 1 windows
    }
  }
  hipLaunchKernelGGL(k_leaf_depth, dim3(grid_for(n, kTB)), dim3(kTB), 0, s, K, idx, n, m, max_d, L, Wfinal, span,
                     tk_orig, d_orig);
  OCT_TRY(hipGetLastError());

  // 4. leaf order: stable sort of the truncated keys from the original order
  uint64_t* TK = K;  // reuse
  int32_t* idx2 = idx;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n, kTB)), dim3(kTB), 0, s, iota, n);
  OCT_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb_sort, tk_orig, TK, iota, idx2, (int)n, 0, end_bit, s));

  // 5. node starts, preorder ranks, leaf starts
  uint8_t* D2 = nullptr;
  int8_t* cj = nullptr;
  int64_t *nstart = nullptr, *base = nullptr, *lflag = nullptr, *lix = nullptr;
  OCT_TRY(S.alloc(&D2, n));
  OCT_TRY(S.alloc(&cj, n));
  OCT_TRY(S.alloc(&nstart, n));
  OCT_TRY(S.alloc(&base, n));
  OCT_TRY(S.alloc(&lflag, n));
  OCT_TRY(S.alloc(&lix, n));
  hipLaunchKernelGGL(k_node_starts, dim3(grid_for(n, kTB)), dim3(kTB), 0, s, TK, idx2, d_orig, n, max_d, D2, cj,
                     nstart, lflag, pos0, u32 + 1);
  OCT_TRY(hipGetLastError());
  OCT_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb_scan, nstart, base, (int)n, s));
  OCT_TRY(hipcub::DeviceScan::ExclusiveSum(tmp, tb_scan, lflag, lix, (int)n, s));
  hipLaunchKernelGGL(k_total, dim3(1), dim3(1), 0, s, base, nstart, n, total);
  hipLaunchKernelGGL(k_total, dim3(1), dim3(1), 0, s, lix, lflag, n, total + 1);
  OCT_TRY(hipGetLastError());
  int64_t tot[2] = {0, 0};
  unsigned int maxdep = 0;
  int32_t p0 = 0;
  OCT_TRY(hipMemcpyAsync(tot, total, sizeof(tot), hipMemcpyDeviceToHost, s));
  OCT_TRY(hipMemcpyAsync(&maxdep, u32 + 1, sizeof(maxdep), hipMemcpyDeviceToHost, s));
  OCT_TRY(hipMemcpyAsync(&p0, pos0, sizeof(p0), hipMemcpyDeviceToHost, s));
  OCT_TRY(hipStreamSynchronize(s));
  const int64_t nn = tot[0], nleaves = tot[1];
  if (nn > (int64_t)0x7ffffffe) {
    *why = "octree has more than INT32_MAX nodes";
    return 1;
  }

  int32_t *ns = nullptr, *leaf_start = nullptr, *riota = nullptr, *lv = nullptr, *lpos = nullptr, *parent = nullptr,
          *nch = nullptr, *fcx = nullptr, *lspan = nullptr;
  uint8_t *nd = nullptr, *dk = nullptr;
  uint32_t* mask = nullptr;
  OCT_TRY(S.alloc(&ns, nn));
  OCT_TRY(S.alloc(&nd, nn));
  OCT_TRY(S.alloc(&leaf_start, nleaves));
  hipLaunchKernelGGL(k_emit_nodes, dim3(grid_for(n, kTB)), dim3(kTB), 0, s, D2, cj, base, lix, n, ns, nd, leaf_start);
  OCT_TRY(hipGetLastError());

  // per-depth lists (stable sort of the preorder ranks by depth)
  OCT_TRY(S.alloc(&riota, nn));
  OCT_TRY(S.alloc(&lv, nn));
  OCT_TRY(S.alloc(&dk, nn));
  OCT_TRY(S.alloc(&lpos, nn));
  OCT_TRY(S.alloc(&lspan, 2 * 64));
  hipLaunchKernelGGL(k_iota, dim3(grid_for(nn, kTB)), dim3(kTB), 0, s, riota, nn);
  size_t tb_sort2 = 0;
  OCT_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort2, nd, dk, riota, lv, (int)nn, 0, 5, s));
  void* tmp2 = tmp;
  if (tb_sort2 > tb) OCT_TRY(S.alloc(reinterpret_cast<uint8_t**>(&tmp2), tb_sort2));
  OCT_TRY(hipcub::DeviceRadixSort::SortPairs(tmp2, tb_sort2, nd, dk, riota, lv, (int)nn, 0, 5, s));
  hipLaunchKernelGGL(k_level_spans, dim3(grid_for(nn, kTB)), dim3(kTB), 0, s, dk, lv, nn, lspan, lspan + 64);
  hipLaunchKernelGGL(k_level_pos, dim3(grid_for(nn, kTB)), dim3(kTB), 0, s, dk, lv, nn, lspan, lpos);
  OCT_TRY(hipGetLastError());

  // 6. parents, child counts/masks, child-block numbering
  OCT_TRY(S.alloc(&parent, nn));
  OCT_TRY(S.alloc(&nch, nn));
  OCT_TRY(S.alloc(&fcx, nn));
  OCT_TRY(S.alloc(&mask, nn));
  OCT_TRY(hipMemsetAsync(nch, 0, nn * sizeof(int32_t), s));
  OCT_TRY(hipMemsetAsync(mask, 0, nn * sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_parents, dim3(grid_for(nn, kTB)), dim3(kTB), 0, s, ns, nd, TK, nn, max_d, lv, lspan,
                     lspan + 64, parent, nch, mask);
  OCT_TRY(hipGetLastError());
  size_t tb_scan2 = 0;
  OCT_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tb_scan2, nch, fcx, (int)nn, s));
  void* tmp3 = tmp2;
  if (tb_scan2 > std::max(tb, tb_sort2)) OCT_TRY(S.alloc(reinterpret_cast<uint8_t**>(&tmp3), tb_scan2));
  OCT_TRY(hipcub::DeviceScan::ExclusiveSum(tmp3, tb_scan2, nch, fcx, (int)nn, s));

  NodeRec* nodes = nullptr;
  TgtPt* pts = nullptr;
  OCT_TRY(hipMalloc(reinterpret_cast<void**>(&nodes), nn * sizeof(NodeRec)));
  if (hipMalloc(reinterpret_cast<void**>(&pts), n * sizeof(TgtPt)) != hipSuccess) {
    (void)hipFree(nodes);
    *why = "allocating the leaf-ordered target failed";
    return -2;
  }
  hipLaunchKernelGGL(k_write_nodes, dim3(grid_for(nn, kTB)), dim3(kTB), 0, s, ns, nd, TK, D2, lix, leaf_start, nleaves,
                     n, nn, max_d, box, parent, lpos, fcx, mask, nodes);
  hipLaunchKernelGGL(k_write_points, dim3(grid_for(n, kTB)), dim3(kTB), 0, s, xyz, idx2, n, pts);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    (void)hipFree(nodes);
    (void)hipFree(pts);
    *why = std::string("octree build kernels: ") + hipGetErrorString(e);
    return -3;
  }
  out->nodes = nodes;
  out->pts = pts;
  out->n_nodes = nn;
  out->n_leaves = nleaves;
  out->max_depth = (int32_t)maxdep;
  out->max_inner_depth = (int32_t)maxdep - 1;  // the deepest leaf's parent (-1: the root is a leaf)
  out->pos_of_orig0 = p0;
  return 0;
}

}  // namespace icp
