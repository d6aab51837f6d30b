/*
 * icp_host.h — host-side helpers exported by libicp_hip.so (no GPU needed):
 *   - the linear-octree builder the device path uploads (inspection / tests);
 *     same tree as Octree::Octree + buildTree, core/octree.cpp:41-126
 *   - the rank-merge of per-rank partial statistics (the exchange step of the multi-GPU path)
 *   - a deterministic synthetic cloud-pair generator (the test_icp.cpp:165-229 recipe with a
 *     fixed, counter-based RNG instead of rand()/time())
 */
#ifndef ICP_HOST_H
#define ICP_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct icp_octree icp_octree;

typedef struct icp_octree_info {
  int64_t n_nodes;
  int64_t n_leaves;
  int64_t n_points;
  int32_t max_depth;
  int32_t max_inner_depth;
  int32_t pos_of_orig0;
} icp_octree_info;

/* Build; returns null (and sets icp_hip_last_error) on invalid input. */
icp_octree* icp_octree_build(const double* xyz, int64_t n, int max_points, int max_depth);
void icp_octree_free(icp_octree* t);
void icp_octree_get_info(const icp_octree* t, icp_octree_info* info);
/* Node records: lo[3], hi[3] (6 doubles per node), first, meta (leaf bit 31 | count or
 * child mask), depth. Leaf-ordered points: xyz (3 doubles) and original index. */
void icp_octree_copy_nodes(const icp_octree* t, double* box6, int32_t* first, uint32_t* meta, int32_t* depth);
void icp_octree_copy_points(const icp_octree* t, double* xyz, int32_t* orig);

/* Partial statistics: Moments = 8 doubles {n, mean, M2, min, max, n_bad, 0, 0};
 * CovMoments = 20 doubles {n, sum_d2, ma[3], mb[3], C[9], 0, 0, 0}. Merged left to right. */
void icp_moments_from_values(const double* d, int64_t n, double out8[8]);
void icp_moments_merge(const double* parts8, int32_t nparts, double out8[8]);
void icp_cov_from_pairs(const double* a_xyz, const double* b_xyz, const double* d, int64_t n, double threshold,
                        double out20[20]);
void icp_cov_merge(const double* parts20, int32_t nparts, double out20[20]);
double icp_cull_threshold(double mean, double sd, double k_sigma, int iter, int engine_rules);

/* Spatial sharding of the source for the multi-GPU path: order[] = a permutation of 0..n-1 in
 * which every contiguous range is spatially compact (kd buckets, the query order of the search
 * kernel). Rank r of W takes the points order[lo_r .. hi_r) of the balanced contiguous split, so
 * its queries keep the full density of the cloud (a strided or shuffled split would thin them W
 * times and every search box would hold W times more target points). Returns 0, or -1 on bad
 * arguments. No reference counterpart: the reference has one CPU thread and no sharding. */
int icp_source_shard_order(const double* xyz, int64_t n, int32_t* order);

typedef struct icp_synth_spec {
  double sigma[3];        /* target ~ N(0, diag(sigma^2)), default (5, 5, 1) m           */
  double yaw_deg, pitch_deg, roll_deg; /* R = Rz(yaw) Ry(pitch) Rx(roll), test_icp.cpp:165-189 */
  double t[3];            /* translation, default (0.5, -0.3, 0.1) m                     */
  double noise_sigma;     /* source jitter, default 1e-3 m                               */
  double outlier_fraction;/* replaced by uniform points in the target bbox, default 0.01 */
  uint64_t seed_target;   /* default 42 */
  uint64_t seed_source;   /* default 43 (noise, outliers, shuffle) */
} icp_synth_spec;

void icp_synth_default(icp_synth_spec* s);
/* target (n_tgt points) and source (n_src points): source_i = R^T (target_{pi(i)} - t) + noise,
 * pi a seeded shuffle of the first n_src target points (n_src <= n_tgt), 1 % outliers.
 * T_true (row-major 4x4) maps source onto target. */
int icp_synth_pair(const icp_synth_spec* s, int64_t n_tgt, int64_t n_src, double* tgt_xyz, double* src_xyz,
                   double T_true[16]);

/* A LiDAR-like scene pair (2.5-D surfaces, the data the reference's LAS flow feeds it,
 * lasio.cpp:7-125 / icp_registration.cpp:248-378): a terrestrial scanner at scanner_height above
 * an undulating ground (amplitude terrain_amp) with n_walls vertical walls (facades) standing
 * within site_radius; rays uniform in azimuth and in elevation [elev_min, elev_max] (so the point
 * density falls with range as the scanner's does), the nearest hit within 1.5 site_radius,
 * jittered along the beam by range_noise and rounded to `quantum` (LAS 1.2's int32 x 0.001 grid).
 * The target is one scan in the world frame; the source an independent scan from the scanner
 * moved by t, expressed in its own frame: source = R^T (world - t), R = Rz(yaw) Ry(pitch)
 * Rx(roll), rounded to the grid there; outlier_fraction of its points are uniform in its bbox.
 * T_true maps source onto target. Deterministic (counter-based streams). Returns 0 or -1. */
typedef struct icp_scene_spec {
  double site_radius;      /* m, default 40                                      */
  double scanner_height;   /* m, default 1.8                                     */
  int32_t n_walls;         /* default 8                                          */
  double wall_height;      /* m, default 6                                       */
  double terrain_amp;      /* m, default 0.3                                     */
  double elev_min_deg, elev_max_deg; /* default -45, 35                          */
  double range_noise;      /* m, default 2e-3                                    */
  double quantum;          /* m, default 1e-3 (0: no rounding)                   */
  double yaw_deg, pitch_deg, roll_deg; /* default 2, 0.5, -0.5                   */
  double t[3];             /* m, default (0.3, -0.2, 0.05)                       */
  double outlier_fraction; /* default 0.002                                      */
  uint64_t seed_target;    /* default 7                                          */
  uint64_t seed_source;    /* default 8                                          */
} icp_scene_spec;

void icp_scene_default(icp_scene_spec* s);
int icp_synth_scene(const icp_scene_spec* s, int64_t n_tgt, int64_t n_src, double* tgt_xyz, double* src_xyz,
                    double T_true[16]);

#ifdef __cplusplus
}
#endif
#endif
