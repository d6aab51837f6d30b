// octree_gpu.h — device build of the linear octree (octree_gpu.hip). Produces exactly the arrays
// of the host builder (octree_build.h) directly in HBM: same node records in the same numbering,
// same leaf-ordered points. Reference: Octree::Octree + buildTree, core/octree.cpp:41-126.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "icp_common.h"

namespace icp {

constexpr int kGpuBuildMaxDepth = 21;  // 3 key bits per level in a 64-bit sort key

struct GpuOctree {
  NodeRec* nodes = nullptr;  // device, n_nodes records (caller frees with hipFree)
  TgtPt* pts = nullptr;      // device, leaf order (caller frees with hipFree)
  int64_t n_nodes = 0, n_leaves = 0;
  int32_t max_depth = -1, max_inner_depth = -1, pos_of_orig0 = 0;
};

// xyz: device AoS target (n points). Runs on stream s and synchronizes it before returning.
// Returns 0 on success, 1 on invalid input (non-finite coordinates, n out of range, max_d > 21),
// -2 out of device memory, -3 other device errors; *why says what.
int gpu_build_octree(const double* xyz, int64_t n, int max_pts, int max_d, hipStream_t s, GpuOctree* out,
                     std::string* why);

// Per-level cell tables (SURVEY.md §8 a5 acceleration, search side only): for every level
// l <= lmax, 8^l int32 entries indexed by an l-level path prefix (the octant bits of the
// octree's own midpoint splits, level 1 most significant), each = (node << 5) | depth of the
// node holding all points of the cell (the depth-l node, or the leaf above it), -1 if empty.
// Levels are stored back to back (offset of level l = (8^l - 1) / 7).
int64_t cell_table_entries(int lmax);
int64_t cell_table_offset(int l);
int cell_table_depth(int64_t n_leaves, int max_inner_depth);
hipError_t build_cell_tables(const NodeRec* nodes, int lmax, int32_t* tables, hipStream_t s);

}  // namespace icp
