/*
 * icp_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker, never the product).
 *
 * A plain-C restatement of the reference ICP hot path of B1AnKAlpha/IterativeClosestPoint:
 *   - Octree build            PointCloudRegistration/core/octree.cpp:41-126
 *                             (CLI copy: icp_registration.cpp:59-190)
 *   - Octree NN search        core/octree.cpp:128-184 (CLI: icp_registration.cpp:107-205)
 *   - ICP loop, engine rules  core/icpengine.cpp:117-394
 *   - ICP loop, CLI rules     icp_registration.cpp:443-622
 *   - best-fit transform      core/icpengine.cpp:76-115, icp_registration.cpp:389-440
 *   - 3x3 JacobiSVD           Eigen 3.3.4 (vendored in the reference):
 *                             Eigen/src/SVD/JacobiSVD.h:663-786, misc/RealSvd2x2.h:19-50,
 *                             Jacobi/Jacobi.h:85-110, :300-420
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * Parity is pinned against fixtures produced by the compiled reference CLI
 * (oracle/_ref, see oracle/Makefile and tests/golden/gen_golden.py).
 */
#ifndef ICP_ORACLE_H
#define ICP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_tree orc_tree;

#define ORC_SEM_ENGINE 0 /* core/icpengine.cpp semantics */
#define ORC_SEM_CLI 1    /* icp_registration.cpp semantics */

/* Build the reference octree over AoS xyz (n points). The points are copied. */
orc_tree* orc_octree_build(const double* xyz, int64_t n, int max_pts, int max_depth);
void orc_octree_free(orc_tree* t);

/* Number of nodes, leaves, and deepest node depth. */
void orc_octree_shape(const orc_tree* t, int64_t* n_nodes, int64_t* n_leaves, int32_t* max_depth);

/* Preorder dump (node, then existing children in ascending octant order).
 * Per node: depth, octant (root: -1), box[6] = min_x,max_x,min_y,max_y,min_z,max_z,
 * is_leaf, npts (leaf point count, 0 for inner). Leaf point indices (original order)
 * are written back to back in preorder into leaf_idx. Returns the node count. */
int64_t orc_octree_dump(const orc_tree* t, int32_t* depth, int32_t* octant, double* box6,
                        int32_t* is_leaf, int32_t* npts, int32_t* leaf_idx);

/* findNearest (octree.cpp:175-184). init_best = DBL_MAX (engine) or 1e20 (CLI).
 * visits/scanned (optional) accumulate node entries / leaf points compared. */
int32_t orc_find_nearest(const orc_tree* t, const double q[3], double init_best,
                         int64_t* visits, int64_t* scanned);

/* NN + residual loop (icpengine.cpp:172-206): idx[i] and d[i] = |q_i - tgt[idx_i]|. */
void orc_nn_batch(const orc_tree* t, const double* q, int64_t n, double init_best,
                  int32_t* idx_out, double* d_out, int64_t* visits, int64_t* scanned);

/* OpenMP threads of the NN loop (results do not depend on it). 0/negative: unchanged. */
void orc_set_threads(int n);
int orc_get_threads(void);

/* Eigen-style JacobiSVD of a 3x3 (row-major in/out): H = U diag(S) V^T. */
void orc_jacobi_svd3(const double H[9], double U[9], double S[3], double V[9]);

/* computeBestFitTransform / best_fit_transform for 3xN pairs given as AoS. T row-major. */
void orc_best_fit(const double* a_xyz, const double* b_xyz, int64_t n, double T[16]);

/* x' = T * x in the reference's Eigen evaluation order, AoS in place. */
void orc_transform(const double T[16], double* xyz, int64_t n);

typedef struct orc_params {
  int32_t max_iterations;
  double tolerance;
  double sigma_multiplier;
  int32_t octree_max_points;
  int32_t octree_max_depth;
  int32_t semantics; /* ORC_SEM_ENGINE / ORC_SEM_CLI */
} orc_params;

typedef struct orc_iter {
  int32_t iteration;
  double rmse;
  int32_t valid;
  int32_t outliers;
  double mean, std, threshold;
  double T_inc[16];
  double T_cum[16];
  double rotation_deg;
  double translation;
  int32_t has_transform; /* 0 for the engine's convergence record (icpengine.cpp:293-301) */
} orc_iter;

typedef struct orc_result {
  int32_t success;
  int32_t status; /* 0 max-iter, 1 converged, 2 diverged, 3 too few valid */
  int32_t total_iterations;
  double final_rmse;
  double final_R[9];
  double final_t[3];
  int32_t n_history;
} orc_result;

/* Full ICP. src is updated in place (engine: only on success, as the reference). */
int orc_icp(const orc_params* p, double* src_xyz, int64_t n_src, const double* tgt_xyz,
            int64_t n_tgt, orc_result* res, orc_iter* hist, int32_t hist_cap);

#ifdef __cplusplus
}
#endif
#endif
