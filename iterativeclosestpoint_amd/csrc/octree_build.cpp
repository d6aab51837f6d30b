// octree_build.cpp — host build of the flattened octree (see octree_build.h).
//
// The recursion mirrors Octree::buildTree (octree.cpp:86-126) but partitions one shared index
// array in place (stable counting sort by octant) instead of allocating per-node vectors, and
// emits 64-byte node records with each node's children in one contiguous block.
#include "octree_build.h"

#include <cmath>
#include <cstring>

namespace icp {

namespace {

struct Builder {
  const double* xyz;
  int max_pts, max_d;
  FlatOctree* out;
  std::vector<int32_t> idx, tmp;
  std::vector<uint8_t> oct;

  void leaf(int32_t node, int64_t begin, int64_t count) {
    NodeRec& r = out->nodes[node];
    r.first = (int32_t)out->pts.size();
    r.meta = kLeafBit | (uint32_t)count;
    for (int64_t k = 0; k < count; k++) {
      int32_t id = idx[begin + k];
      TgtPt p;
      p.x = xyz[3 * (int64_t)id];
      p.y = xyz[3 * (int64_t)id + 1];
      p.z = xyz[3 * (int64_t)id + 2];
      p.orig = id;
      p.sep = 0.f;
      if (id == 0) out->pos_of_orig0 = (int32_t)out->pts.size();
      out->pts.push_back(p);
    }
    out->n_leaves++;
  }

  void expand(int32_t node, int64_t begin, int64_t count, int depth) {
    if (depth > out->max_depth) out->max_depth = depth;
    // leaf rule: octree.cpp:88 (indices.size() <= max_points_per_node || depth >= max_depth)
    if (count <= (int64_t)max_pts || depth >= max_d) {
      leaf(node, begin, count);
      return;
    }
    if (depth > out->max_inner_depth) out->max_inner_depth = depth;
    double lo[3], hi[3];
    for (int k = 0; k < 3; k++) {
      lo[k] = out->nodes[node].lo[k];
      hi[k] = out->nodes[node].hi[k];
    }
    // midpoint split: octree.cpp:97-99
    const double mid_x = (lo[0] + hi[0]) / 2;
    const double mid_y = (lo[1] + hi[1]) / 2;
    const double mid_z = (lo[2] + hi[2]) / 2;
    int64_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t k = 0; k < count; k++) {
      const double* p = xyz + 3 * (int64_t)idx[begin + k];
      int o = 0;  // octree.cpp:105-108: strictly greater goes high
      if (p[0] > mid_x) o |= 1;
      if (p[1] > mid_y) o |= 2;
      if (p[2] > mid_z) o |= 4;
      oct[begin + k] = (uint8_t)o;
      cnt[o]++;
    }
    int64_t off[8];
    int64_t run = 0;
    uint32_t mask = 0;
    for (int o = 0; o < 8; o++) {
      off[o] = run;
      run += cnt[o];
      if (cnt[o]) mask |= 1u << o;
    }
    for (int64_t k = 0; k < count; k++) tmp[begin + off[oct[begin + k]]++] = idx[begin + k];
    std::memcpy(&idx[begin], &tmp[begin], sizeof(int32_t) * count);

    const int32_t first = (int32_t)out->nodes.size();
    out->nodes[node].first = first;
    out->nodes[node].meta = mask;
    // children boxes: octree.cpp:115-120, created only when non-empty (:113)
    for (int o = 0; o < 8; o++) {
      if (!cnt[o]) continue;
      NodeRec c;
      c.lo[0] = (o & 1) ? mid_x : lo[0];
      c.hi[0] = (o & 1) ? hi[0] : mid_x;
      c.lo[1] = (o & 2) ? mid_y : lo[1];
      c.hi[1] = (o & 2) ? hi[1] : mid_y;
      c.lo[2] = (o & 4) ? mid_z : lo[2];
      c.hi[2] = (o & 4) ? hi[2] : mid_z;
      c.first = 0;
      c.meta = 0;
      c.depth = depth + 1;
      c.pad = 0;
      out->nodes.push_back(c);
    }
    int32_t child = first;
    int64_t sub = begin;
    for (int o = 0; o < 8; o++) {
      if (!cnt[o]) continue;
      expand(child, sub, cnt[o], depth + 1);
      child++;
      sub += cnt[o];
    }
  }
};

}  // namespace

bool build_flat_octree(const double* xyz, int64_t n, int max_pts, int max_d, FlatOctree* out,
                       const char** why) {
  *out = FlatOctree();
  out->max_pts = max_pts;
  out->max_d = max_d;
  if (n < 0 || n > (int64_t)0x7fffffff) {
    if (why) *why = "target size out of range (int32 indices, as the reference)";
    return false;
  }
  for (int64_t i = 0; i < 3 * n; i++) {
    if (!std::isfinite(xyz[i])) {
      if (why) *why = "target contains non-finite coordinates";
      return false;
    }
  }
  if (n == 0) return true;
  // root box: octree.cpp:47-66
  double min_x = xyz[0], max_x = xyz[0], min_y = xyz[1], max_y = xyz[1], min_z = xyz[2], max_z = xyz[2];
  for (int64_t i = 0; i < n; i++) {
    const double* p = xyz + 3 * i;
    if (p[0] < min_x) min_x = p[0];
    if (p[0] > max_x) max_x = p[0];
    if (p[1] < min_y) min_y = p[1];
    if (p[1] > max_y) max_y = p[1];
    if (p[2] < min_z) min_z = p[2];
    if (p[2] > max_z) max_z = p[2];
  }
  const double eps = 0.001;
  min_x -= eps; max_x += eps;
  min_y -= eps; max_y += eps;
  min_z -= eps; max_z += eps;
  NodeRec root;
  root.lo[0] = min_x; root.hi[0] = max_x;
  root.lo[1] = min_y; root.hi[1] = max_y;
  root.lo[2] = min_z; root.hi[2] = max_z;
  root.first = 0;
  root.meta = 0;
  root.depth = 0;
  root.pad = 0;
  out->nodes.reserve((size_t)(n / 2 + 16));
  out->pts.reserve((size_t)n);
  out->nodes.push_back(root);
  Builder b;
  b.xyz = xyz;
  b.max_pts = max_pts;
  b.max_d = max_d;
  b.out = out;
  b.idx.resize(n);
  b.tmp.resize(n);
  b.oct.resize(n);
  for (int64_t i = 0; i < n; i++) b.idx[i] = (int32_t)i;
  b.expand(0, 0, n, 0);
  out->nodes.shrink_to_fit();
  return true;
}

}  // namespace icp
