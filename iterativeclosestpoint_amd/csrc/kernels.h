// kernels.h — launch wrappers of the gfx950 kernels (nn_kernels.hip, reduce_kernels.hip,
// util_kernels.hip). Internal C++ API used by the C-ABI context (icp_ctx.hip); no torch types.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/icp_hip.h"
#include "icp_common.h"
#include "session_step.h"

namespace icp {

// The device-resident loop's state (device memory): the session (engine.cpp's decisions,
// session_step.h) stepped by each iteration's last kernel; every kernel of a later iteration
// reads `done` and returns at once after the session finished, and the search applies core.T.
struct LoopDev {
  SessionCore core;
  SessionParams p;
};

// Per-iteration record. Device-resident copy written by the merge/finalize kernels (the cull
// kernel reads the threshold from it); the last kernel of the iteration stores the finished
// record into pinned host memory (IterPublish), the one host read of the iteration.
struct IterDev {
  Moments m_local;      // this rank's residual moments
  Moments m_global;     // merged over ranks (rank order)
  CovMoments c_local;   // this rank's valid-pair moments
  CovMoments c_global;  // merged over ranks
  double mean, sd, thr, rmse;
  double cshift[6];  // this iteration's shift of the pair sums (set with the threshold)
  // The band of the fused covariance sums (wave_stats.h), set at the end of every iterate for the
  // next one's search: it sums the pairs with d <= fz_lo with the shift fz_sh and marks those in
  // (fz_lo, fz_hi]. fz_ok = 0: no band (a new source, a non-finite threshold): full cull pass.
  double fz_lo, fz_hi, fz_thr, fz_ok;
  double fz_sh[6];
  double cull_mode;  // this iterate: 1 = the search's wave records + the band pairs, 0 = full cull
  double n_wide;     // this iterate: waves of the wave search whose candidate set overflowed
  double pad[4];
};

// One wave's covariance record, written by the wave search's epilogue when the band is set
// (wave_stats.h): the canonical sums of its pairs with d <= fz_lo (s: d^2, a - s, b - t, the 9
// products), their count, the mask of its band lanes; flag = 1: the wave did not settle every
// query itself (ball / exact / per-lane searches finish them): the cull kernel recomputes it.
struct WaveStat {
  double s[16];
  double cnt;
  unsigned long long bm;
  unsigned long long flag;
  double pad;
};
static_assert(sizeof(WaveStat) == 160, "WaveStat is 20 doubles");

// The wave search's candidate cache (one record per wave of 64 queries): the box B+ whose leaves'
// points were collected, their count and the generation (target / source upload) it belongs to.
// The entries are the points inside B+ as fp32 offsets from B+'s centre (the scan's own staging
// values) with the point's id in the fourth word: a reusing wave streams them, no gathers.
constexpr int kWaveCandCap = 1008;  // candidate points per wave (the walk's list in LDS; the cache)
// One wave's candidate-cache record: its stored box B+ (the scan frame is B+'s centre), the count
// of entries, the generation, and vmin = vol(B+) / candidate_loose (the loose test: reused only
// while vol(B) >= vmin). One 64-B line, loaded by lanes 0..7 of the wave with its query.
struct WaveBox {
  double lo[3];
  double hi[3];
  int32_t count;
  uint32_t gen;
  float vmin;
  uint32_t pad;
};
static_assert(sizeof(WaveBox) == 64, "one line, eight words");

struct NNLaunch {
  const LoopDev* loop;      // device loop (null: the host drives the iterate); T from loop->core.T
  const NodeRec* nodes;
  const TBox* tbox;         // tight boxes of the nodes (prune tests of the certified searches)
  const TgtPt* pts;
  double* x;
  double* y;
  double* z;
  int32_t* pos_out;
  double* dist_out;
  unsigned long long* counters;  // [node entries, leaf points] (count mode only)
  int64_t n;
  int32_t n_nodes;
  int32_t pos0;
  int32_t levels;
  double init_best;
  double T[12];             // row-major 3x4, used when apply != 0
  int apply;
  int count;                // reference-order kernel counting the reference DFS's work
  int search;               // ICP_SEARCH_CERTIFIED (wave search) / ICP_SEARCH_REFERENCE
  int32_t* fb_list;         // queries sent to the exact reference-order DFS
  int32_t* fb_list2;        // queries a wave did not take -> ball search
  double* fb_u2;            // the distance guess u of each fb_list2 entry
  unsigned int* fb_count;   // [0] exact list, [1] ball list sizes; [2] per-lane searches, [3] DFS
                            // finishes of the ball search (counts); [4] half list size; [5] wide
                            // list size; [6] overflowed waves of the wave search; zero at the launch
  int32_t* fb_list3;        // 32-query halves of overflowed waves, (half id, lane mask) pairs
                            // (null: no half pass)
  int32_t* fb_list4;        // the wide pass (k_nn_wide): overflowed waves / halves as (first query,
                            // lane mask low, high) triples; null: overflowed lanes take the ball search
  hipEvent_t ev_start;      // optional: the main search kernel's start and end, recorded by its
  hipEvent_t ev_fast_done;  // own dispatch (hipExtLaunchKernel: no marker packets between kernels)
  int have_prev;            // dist_out holds the previous residuals of these queries
  int scan32;               // fp32 filter scan with fp64 certification (0: fp64 scan)
  const int32_t* cells;     // per-level cell tables (octree_gpu.h), null = root descent
  int cell_lmax;            // deepest table level
  double root_lo[3], root_hi[3];  // root box (the octree's midpoint recursion starts here)
  unsigned long long* dbg;  // optional diagnostics of the wave search (ICP_DBG_* slots)
  double join_factor;       // a lane joins the wave box if its radius <= this x the mean radius
  int xcd_blocks;           // renumber the wave search's blocks XCD-contiguously
  int scan_groups;          // lane groups of the fp32 filter scan (1, 2, 4)
  WaveBox* wc_box;          // candidate cache (iterate only; null: every wave walks)
  float4* wc_ents;          // kWaveCandCap entries per wave: (x, y, z) - centre of B+ in fp32, id
  uint32_t wc_gen;          // records of this generation are valid
  double wc_margin;         // a walk collects the leaves of B enlarged by this x B's half-extent
  double wc_loose;          // a record is reused only while vol(B+) <= this x vol(B)
  double wc_lead;           // a stored B+ leads the wave's motion by this many iterates' displacement
  int certify_prev;         // previous-match certificate mode (icp_hip_config.certify_prev)
  WaveStat* wstat;          // per-wave covariance records (null: none; the cull pass does it all)
  const IterDev* fz;        // the band of this iterate (IterDev::fz_*)
  int32_t ball_queue_off;   // k_nn_ball: byte offset of its follow-up queue in LDS
  int32_t ball_mode;        // icp_hip_config.ball_mode (k_nn_ball's direct mode)
};

// Threads per block of the per-thread search kernels for a given stack depth.
int nn_block_threads(int levels);
hipError_t launch_nn(const NNLaunch& a, hipStream_t s);
// TgtPt::sep of every target point (lower bound of its distance to every other point).
hipError_t launch_target_sep(const NodeRec* nodes, TgtPt* pts, int64_t n, int levels, hipStream_t s);
hipError_t launch_mark_copies(TgtPt* pts, int64_t n, hipStream_t s);
// TBox of every node (icp_common.h), deepest level first; max_depth: the deepest node's depth.
hipError_t launch_tight_boxes(const NodeRec* nodes, const TgtPt* pts, TBox* tb, int64_t n_nodes, int max_depth,
                              hipStream_t s);

struct CullLaunch {
  const LoopDev* loop;  // device loop: nothing to do once the session is done
  const double* x;
  const double* y;
  const double* z;
  const int32_t* pos;
  const TgtPt* pts;
  const IterDev* it;
  CovMoments* part;
  int64_t n;
  const double* dist;       // the residuals (the band's and the recomputed waves' pairs)
  const WaveStat* wstat;    // the search's wave records (null: it wrote none this iterate)
  int wpb;                  // search waves per cull block (set by launch_cull_tail)
};

// Residual moments of the settled queries in fixed parts (deterministic), then the merges.
int64_t moments_num_parts(int64_t n);
// Partial buffers need merge_scratch_entries(nparts) entries of fold scratch behind the partials.
int64_t merge_scratch_entries(int64_t nparts);

struct MomentsFinalize {
  double k_sigma;
  int iter;
  int engine_rules;
};
// Residual moments of the rank's queries (part sums) and their last merge level into it->m_local;
// with fin (no communicator) also mean/std/threshold and the cull's pair shift (it->cshift, from
// cl's first 64 queries). With a ticket counter (zero between launches) and at most 4096 parts
// the last block of the moments launch runs the last level itself (one launch instead of two).
// uints of the two "last block done" counters (moments, cull), zero-initialised once
int ticket_words();
hipError_t launch_moments_tail(const double* dist, int64_t n, Moments* part, const LoopDev* loop, unsigned* ticket,
                               IterDev* it, const MomentsFinalize* fin, const CullLaunch& cl, hipStream_t s);
// Merge `nranks` gathered moments in rank order and compute mean/std/threshold.
hipError_t launch_finalize_moments(const Moments* gathered, int nranks, IterDev* it, MomentsFinalize fin,
                                   const CullLaunch& cl, hipStream_t s);

// Where the finished record goes: a device-visible pinned host IterDev (list sizes in pad[0..2]);
// the three list counters are reset for the next search.
struct IterPublish {
  IterDev* host;
  unsigned int* lists;
  double seq;  // stored last into host->pad[3]: the record is complete
  // device loop (host null): the session steps on the device and the iteration's LoopRec goes
  // to `rec` (pinned host memory, read after the batch)
  LoopDev* loop;
  LoopRec* rec;
};


int64_t cull_num_blocks(int64_t n);
// 3-sigma cull + covariance part sums (from the search's wave records and the band pairs, or a
// full pass; wave_stats.h) and their last merge level into it->c_local; with pub (no
// communicator) also RMSE + publish. With a ticket counter and a small grid the last block runs
// the last level and the publish itself (one launch instead of two).
hipError_t launch_cull_tail(const CullLaunch& a, unsigned* ticket, const IterPublish* pub, hipStream_t s);
// Merge `nranks` gathered covariance moments in rank order, RMSE, publish.
hipError_t launch_finalize_cov(const CovMoments* gathered, int nranks, IterDev* it, IterPublish pub, hipStream_t s);

hipError_t launch_apply(const double T[12], double* x, double* y, double* z, int64_t n, hipStream_t s);
hipError_t launch_scatter_aos(const int32_t* perm, const double* x, const double* y, const double* z,
                              double* aos, int64_t n, hipStream_t s);
hipError_t launch_scatter_corr(const int32_t* perm, const int32_t* pos, const TgtPt* pts,
                               int32_t* idx_out, const double* dist_in, double* dist_out, int64_t n,
                               hipStream_t s);
hipError_t launch_deinterleave(const double* aos, double* x, double* y, double* z, int64_t n, hipStream_t s);
hipError_t launch_gather_deinterleave(const double* aos, const int32_t* perm, double* x, double* y, double* z,
                                      int64_t n, hipStream_t s);

}  // namespace icp
