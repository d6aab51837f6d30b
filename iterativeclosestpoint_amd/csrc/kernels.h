// kernels.h — launch wrappers of the gfx950 kernels (kernels.hip). Internal C++ API used by
// the C-ABI context (icp_ctx.hip); no torch types anywhere.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "icp_common.h"

namespace icp {

// Per-iteration record. Device-resident copy written by the merge/finalize kernels (the cull
// kernel reads the threshold from it); the last kernel of the iteration stores the finished
// record into pinned host memory (IterPublish), the one host read of the iteration.
struct IterDev {
  Moments m_local;      // this rank's residual moments
  Moments m_global;     // merged over ranks (rank order)
  CovMoments c_local;   // this rank's valid-pair moments
  CovMoments c_global;  // merged over ranks
  double mean, sd, thr, rmse;
  double pad[4];
};

struct NNLaunch {
  const NodeRec* nodes;
  const TgtPt* pts;
  double* x;
  double* y;
  double* z;
  int32_t* pos_out;
  double* dist_out;
  Moments* part;                   // one per block, may be null
  unsigned long long* counters;    // [node entries, leaf points] (count mode only)
  int64_t n;
  int32_t n_nodes;
  int32_t pos0;
  int32_t levels;
  double init_best;
  double T[12];                    // row-major 3x4, used when apply != 0
  int apply;
  int count;
  int variant;  // 1 = k_nn (reference order), 2 = k_nn2, 3 = certified per-lane, 4 = wave-cooperative
  int32_t* fb_list;        // variants 3/4: queries sent to the exact fallback
  int32_t* fb_list2;       // variant 4: queries a wave did not take -> one-wave ball search
  double* fb_u2;           // variant 4: the distance guess u of each fb_list2 entry
  int32_t* fb_list3;       // variant 4: queries left to the per-lane certified search
  unsigned int* fb_count;  // [0] exact, [1] ball, [2] per-lane list sizes; zero at the launch
  hipEvent_t ev_fast_done; // optional: recorded right after the fast kernel
  int have_prev;           // variant 4: dist_out holds the previous residuals of these queries
  int scan_group;          // variant 4: lanes per scan group (8, 16, 32 or 64 = whole wave)
  int wave_points;         // variant 4: candidate-list capacity per wave (512, 768 or 1024)
  int scan32;              // variant 4: fp32 filter scan with fp64 certification (0: fp64 scan)
  int lca_descent;         // variant 4: wave-uniform descent to the deepest node covering B first
  const int32_t* cells;    // variant 4: per-level cell tables (octree_gpu.h), null = not used
  int cell_lmax;           // deepest table level
  double root_lo[3], root_hi[3];  // root box (the octree's midpoint recursion starts here)
  unsigned long long* dbg; // optional diagnostics of the wave-cooperative search (ICP_NN_DEBUG)
  int xcd_remap;           // variant 4: each XCD takes one contiguous range of query blocks
  int ball_groups;         // variant 4: queries per wave of the ball search (4; 1 = one per wave)
  double join_factor;      // variant 4: a lane joins the wave box if its radius <= this x the mean radius
};

// Threads per block of the NN kernel for a given stack depth.
int nn_block_threads(int levels);
int64_t nn_num_blocks(int64_t n, int levels);
hipError_t launch_nn(const NNLaunch& a, hipStream_t s);

// Residual moments of the settled queries in fixed parts (deterministic), then the merges.
int64_t moments_num_parts(int64_t n);
hipError_t launch_moments(const double* dist, int64_t n, const IterDev* it, Moments* part, hipStream_t s);
// Partial buffers need merge_scratch_entries(nparts) entries of fold scratch behind the partials.
int64_t merge_scratch_entries(int64_t nparts);

struct MomentsFinalize {
  double k_sigma;
  int iter;
  int engine_rules;
};
// Merge the rank's partials into it->m_local; with fin (single rank) also mean/std/threshold.
hipError_t launch_merge_moments(const Moments* part, int64_t nparts, const double* dist, int64_t nq, IterDev* it,
                                const MomentsFinalize* fin, hipStream_t s);
// Merge `nranks` gathered moments in rank order and compute mean/std/threshold.
hipError_t launch_finalize_moments(const Moments* gathered, int nranks, IterDev* it, MomentsFinalize fin,
                                   hipStream_t s);

// Where the finished record goes: a device-visible pinned host IterDev (list sizes in pad[0..2]);
// the three list counters are reset for the next search.
struct IterPublish {
  IterDev* host;
  unsigned int* lists;
  double seq;  // stored last into host->pad[3]: the record is complete
};

struct CullLaunch {
  const double* x;
  const double* y;
  const double* z;
  const int32_t* pos;
  const double* dist;
  const TgtPt* pts;
  const IterDev* it;
  CovMoments* part;
  int64_t n;
  int xcd_remap;  // each XCD takes one contiguous range of blocks (target gathers share its L2)
};
int64_t cull_num_blocks(int64_t n);
hipError_t launch_cull_cov(const CullLaunch& a, hipStream_t s);
// Merge the rank's partials into it->c_local; with pub (single rank) also RMSE + publish.
struct CullLaunch;
hipError_t launch_merge_cov(const CovMoments* part, int64_t nparts, const CullLaunch& cl, IterDev* it,
                            const IterPublish* pub, hipStream_t s);
// Merge `nranks` gathered covariance moments in rank order, RMSE, publish.
hipError_t launch_finalize_cov(const CovMoments* gathered, int nranks, IterDev* it, IterPublish pub, hipStream_t s);

hipError_t launch_apply(const double T[12], double* x, double* y, double* z, int64_t n, hipStream_t s);

// Setup helpers: AoS -> SoA + 63-bit Morton keys over [lo, lo + ext] (21 bits per axis).
hipError_t launch_morton(const double* aos, int64_t n, const double lo[3], const double inv_ext[3],
                         double* x, double* y, double* z, uint64_t* keys, int32_t* iota, hipStream_t s);
hipError_t launch_gather_soa(const int32_t* perm, const double* xi, const double* yi, const double* zi,
                             double* xo, double* yo, double* zo, int64_t n, hipStream_t s);
hipError_t launch_scatter_aos(const int32_t* perm, const double* x, const double* y, const double* z,
                              double* aos, int64_t n, hipStream_t s);
hipError_t launch_scatter_corr(const int32_t* perm, const int32_t* pos, const TgtPt* pts,
                               int32_t* idx_out, double* dist_in, double* dist_out, int64_t n,
                               hipStream_t s);
hipError_t launch_deinterleave(const double* aos, double* x, double* y, double* z, int64_t n, hipStream_t s);

// Radix sort of (key, value) pairs via hipCUB; temp storage managed by the caller.
hipError_t sort_pairs(void* temp, size_t* temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                      const int32_t* vals_in, int32_t* vals_out, int64_t n, hipStream_t s);

}  // namespace icp
