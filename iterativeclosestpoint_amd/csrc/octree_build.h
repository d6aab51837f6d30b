// octree_build.h — host construction of the linear (flattened) octree that the gfx950
// traversal kernel walks. Same tree as the reference's pointer octree
// (PointCloudRegistration/core/octree.cpp:41-126): same root box and eps, same midpoint split,
// same "p > mid goes high" octant rule, same leaf rule (|idx| <= max_pts or depth >= max_d),
// non-empty children only, ascending octant order, leaf points in ascending original index.
#pragma once

#include <cstdint>
#include <vector>

#include "icp_common.h"

namespace icp {

struct FlatOctree {
  std::vector<NodeRec> nodes;  // nodes[0] = root (empty when the target is empty)
  std::vector<TgtPt> pts;      // target in leaf order
  int64_t n_leaves = 0;
  int32_t max_depth = -1;        // deepest node
  int32_t max_inner_depth = -1;  // deepest inner node (stack levels needed = this + 1)
  int32_t pos_of_orig0 = 0;      // leaf position of original index 0 (findNearest's default)
  int32_t max_pts = 10;
  int32_t max_d = 20;
};

// Returns false on invalid input (non-finite target coordinates or n > INT32_MAX).
bool build_flat_octree(const double* xyz, int64_t n, int max_pts, int max_d, FlatOctree* out,
                       const char** why);

}  // namespace icp
