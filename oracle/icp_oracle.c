/*
 * icp_oracle.c — TEST INFRASTRUCTURE ONLY. See icp_oracle.h for scope and citations.
 *
 * Written as a plain-C restatement of the reference algorithm: pointer octree built
 * by the same split rule, recursive DFS with the same arithmetic and visit order,
 * sequential double sums exactly where the reference sums sequentially.
 * Build flags matter: -O2 -ffp-contract=off, never -march=native (the reference is
 * built for baseline x86-64 without FMA; CMakeLists.txt:7-12).
 */
#include "icp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct orc_node {
  double min_x, max_x, min_y, max_y, min_z, max_z; /* octree.h:12 */
  int32_t* idx;                                    /* leaf point_indices, ascending */
  int64_t n;
  struct orc_node* child[8];
  int is_leaf;
} orc_node;

struct orc_tree {
  orc_node* root;
  double* pts; /* AoS copy of the target */
  int64_t n;
  int max_pts, max_d;
};

/* std::max(a, b) == (a < b) ? b : a — the exact NaN behaviour matters (octree.cpp:34-36). */
static double smax(double a, double b) { return (a < b) ? b : a; }

/* OctreeNode::minDistanceTo (octree.cpp:32-38). */
static double min_dist(const orc_node* nd, const double* q) {
  double dx = smax(0.0, smax(nd->min_x - q[0], q[0] - nd->max_x));
  double dy = smax(0.0, smax(nd->min_y - q[1], q[1] - nd->max_y));
  double dz = smax(0.0, smax(nd->min_z - q[2], q[2] - nd->max_z));
  return sqrt(dx * dx + dy * dy + dz * dz);
}

static orc_node* new_node(double a, double b, double c, double d, double e, double f) {
  orc_node* nd = (orc_node*)calloc(1, sizeof(orc_node));
  nd->min_x = a; nd->max_x = b; nd->min_y = c; nd->max_y = d; nd->min_z = e; nd->max_z = f;
  nd->is_leaf = 1;
  return nd;
}

/* Octree::buildTree (octree.cpp:86-126). */
static void build(orc_tree* t, orc_node* node, const int32_t* idx, int64_t n, int depth) {
  if (n <= (int64_t)t->max_pts || depth >= t->max_d) {
    node->idx = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    memcpy(node->idx, idx, sizeof(int32_t) * n);
    node->n = n;
    node->is_leaf = 1;
    return;
  }
  node->is_leaf = 0;
  double mid_x = (node->min_x + node->max_x) / 2;
  double mid_y = (node->min_y + node->max_y) / 2;
  double mid_z = (node->min_z + node->max_z) / 2;
  int64_t cnt[8] = {0};
  unsigned char* oct = (unsigned char*)malloc(n > 0 ? n : 1);
  for (int64_t k = 0; k < n; k++) {
    const double* p = t->pts + 3 * (int64_t)idx[k];
    int o = 0;
    if (p[0] > mid_x) o |= 1;
    if (p[1] > mid_y) o |= 2;
    if (p[2] > mid_z) o |= 4;
    oct[k] = (unsigned char)o;
    cnt[o]++;
  }
  for (int i = 0; i < 8; i++) {
    if (cnt[i] == 0) continue;
    int32_t* sub = (int32_t*)malloc(sizeof(int32_t) * cnt[i]);
    int64_t m = 0;
    for (int64_t k = 0; k < n; k++)
      if (oct[k] == i) sub[m++] = idx[k];
    double minx = (i & 1) ? mid_x : node->min_x;
    double maxx = (i & 1) ? node->max_x : mid_x;
    double miny = (i & 2) ? mid_y : node->min_y;
    double maxy = (i & 2) ? node->max_y : mid_y;
    double minz = (i & 4) ? mid_z : node->min_z;
    double maxz = (i & 4) ? node->max_z : mid_z;
    node->child[i] = new_node(minx, maxx, miny, maxy, minz, maxz);
    build(t, node->child[i], sub, cnt[i], depth + 1);
    free(sub);
  }
  free(oct);
}

/* Octree::Octree (octree.cpp:41-77): bbox of the target, eps 0.001, build from 0..n-1. */
orc_tree* orc_octree_build(const double* xyz, int64_t n, int max_pts, int max_depth) {
  orc_tree* t = (orc_tree*)calloc(1, sizeof(orc_tree));
  t->n = n;
  t->max_pts = max_pts;
  t->max_d = max_depth;
  t->pts = (double*)malloc(sizeof(double) * 3 * (n > 0 ? n : 1));
  if (n > 0) memcpy(t->pts, xyz, sizeof(double) * 3 * n);
  if (n <= 0) return t;
  double min_x = xyz[0], max_x = xyz[0], min_y = xyz[1], max_y = xyz[1], min_z = xyz[2],
         max_z = xyz[2];
  for (int64_t i = 0; i < n; i++) {
    const double* p = xyz + 3 * i;
    if (p[0] < min_x) min_x = p[0];
    if (p[0] > max_x) max_x = p[0];
    if (p[1] < min_y) min_y = p[1];
    if (p[1] > max_y) max_y = p[1];
    if (p[2] < min_z) min_z = p[2];
    if (p[2] > max_z) max_z = p[2];
  }
  double eps = 0.001;
  min_x -= eps; max_x += eps;
  min_y -= eps; max_y += eps;
  min_z -= eps; max_z += eps;
  t->root = new_node(min_x, max_x, min_y, max_y, min_z, max_z);
  int32_t* all = (int32_t*)malloc(sizeof(int32_t) * n);
  for (int64_t i = 0; i < n; i++) all[i] = (int32_t)i;
  build(t, t->root, all, n, 0);
  free(all);
  return t;
}

static void free_node(orc_node* nd) {
  if (!nd) return;
  for (int i = 0; i < 8; i++) free_node(nd->child[i]);
  free(nd->idx);
  free(nd);
}

void orc_octree_free(orc_tree* t) {
  if (!t) return;
  free_node(t->root);
  free(t->pts);
  free(t);
}

static void shape_rec(const orc_node* nd, int d, int64_t* nn, int64_t* nl, int32_t* md) {
  (*nn)++;
  if (d > *md) *md = d;
  if (nd->is_leaf) { (*nl)++; return; }
  for (int i = 0; i < 8; i++)
    if (nd->child[i]) shape_rec(nd->child[i], d + 1, nn, nl, md);
}

void orc_octree_shape(const orc_tree* t, int64_t* n_nodes, int64_t* n_leaves, int32_t* max_depth) {
  *n_nodes = 0; *n_leaves = 0; *max_depth = -1;
  if (t->root) shape_rec(t->root, 0, n_nodes, n_leaves, max_depth);
}

typedef struct dump_ctx {
  int32_t *depth, *octant, *is_leaf, *npts, *leaf_idx;
  double* box6;
  int64_t k, li;
} dump_ctx;

static void dump_rec(const orc_node* nd, int d, int oct, dump_ctx* c) {
  int64_t k = c->k++;
  c->depth[k] = d;
  c->octant[k] = oct;
  double* b = c->box6 + 6 * k;
  b[0] = nd->min_x; b[1] = nd->max_x; b[2] = nd->min_y;
  b[3] = nd->max_y; b[4] = nd->min_z; b[5] = nd->max_z;
  c->is_leaf[k] = nd->is_leaf;
  c->npts[k] = nd->is_leaf ? (int32_t)nd->n : 0;
  if (nd->is_leaf) {
    for (int64_t j = 0; j < nd->n; j++) c->leaf_idx[c->li++] = nd->idx[j];
    return;
  }
  for (int i = 0; i < 8; i++)
    if (nd->child[i]) dump_rec(nd->child[i], d + 1, i, c);
}

int64_t orc_octree_dump(const orc_tree* t, int32_t* depth, int32_t* octant, double* box6,
                        int32_t* is_leaf, int32_t* npts, int32_t* leaf_idx) {
  dump_ctx c = {depth, octant, is_leaf, npts, leaf_idx, box6, 0, 0};
  if (t->root) dump_rec(t->root, 0, -1, &c);
  return c.k;
}

typedef struct child_dist { int index; double dist; } child_dist;

/* libstdc++ std::sort on <= 16 elements is __insertion_sort (stable for strict <). */
static void insertion_sort(child_dist* a, int n) {
  for (int i = 1; i < n; i++) {
    child_dist val = a[i];
    if (val.dist < a[0].dist) {
      for (int j = i; j > 0; j--) a[j] = a[j - 1];
      a[0] = val;
    } else {
      int j = i;
      while (val.dist < a[j - 1].dist) { a[j] = a[j - 1]; j--; }
      a[j] = val;
    }
  }
}

typedef struct search_state {
  const orc_tree* t;
  const double* q;
  int32_t best_idx;
  double best;
  int64_t visits, scanned;
} search_state;

/* Octree::searchNearest (octree.cpp:128-173). */
static void search(search_state* s, const orc_node* node) {
  if (!node) return;
  s->visits++;
  double md = min_dist(node, s->q);
  if (md * md >= s->best) return;
  if (node->is_leaf) {
    for (int64_t j = 0; j < node->n; j++) {
      int32_t id = node->idx[j];
      const double* p = s->t->pts + 3 * (int64_t)id;
      double dx = p[0] - s->q[0];
      double dy = p[1] - s->q[1];
      double dz = p[2] - s->q[2];
      double d2 = dx * dx + dy * dy + dz * dz;
      s->scanned++;
      if (d2 < s->best) { s->best = d2; s->best_idx = id; }
    }
    return;
  }
  child_dist cd[8];
  int nc = 0;
  for (int i = 0; i < 8; i++) {
    if (node->child[i]) { cd[nc].index = i; cd[nc].dist = min_dist(node->child[i], s->q); nc++; }
  }
  insertion_sort(cd, nc);
  for (int k = 0; k < nc; k++) search(s, node->child[cd[k].index]);
}

int32_t orc_find_nearest(const orc_tree* t, const double q[3], double init_best, int64_t* visits,
                         int64_t* scanned) {
  if (!t->root || t->n == 0) return 0;
  search_state s = {t, q, 0, init_best, 0, 0};
  search(&s, t->root);
  if (visits) *visits += s.visits;
  if (scanned) *scanned += s.scanned;
  return s.best_idx;
}

/* ICPEngine::computeDistance (icpengine.cpp:68-74). */
static double point_dist(const double* a, const double* b) {
  double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
  return sqrt(dx * dx + dy * dy + dz * dz);
}

/* The queries are independent (icpengine.cpp:169-184 runs them one after another); OpenMP splits
 * them over threads, which changes no query's result. The work counters are summed per thread. */
void orc_nn_batch(const orc_tree* t, const double* q, int64_t n, double init_best, int32_t* idx_out,
                  double* d_out, int64_t* visits, int64_t* scanned) {
  int64_t v = 0, sc = 0;
#pragma omp parallel for schedule(dynamic, 1024) reduction(+ : v, sc)
  for (int64_t i = 0; i < n; i++) {
    int32_t id = orc_find_nearest(t, q + 3 * i, init_best, &v, &sc);
    if (idx_out) idx_out[i] = id;
    if (d_out) d_out[i] = (t->n > 0) ? point_dist(q + 3 * i, t->pts + 3 * (int64_t)id) : 0.0;
  }
  if (visits) *visits += v;
  if (scanned) *scanned += sc;
}

void orc_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

int orc_get_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ---------------- Eigen JacobiSVD<Matrix3d> restatement ---------------- */

typedef struct rot { double c, s; } rot;

/* rows p,q (left) : x = c*x + s*y ; y = -s*x + c*y  (Jacobi.h:300-420, scalar path) */
static void rot_rows(double M[3][3], int p, int q, rot j) {
  if (j.c == 1.0 && j.s == 0.0) return;
  for (int i = 0; i < 3; i++) {
    double xi = M[p][i], yi = M[q][i];
    M[p][i] = j.c * xi + j.s * yi;
    M[q][i] = -j.s * xi + j.c * yi;
  }
}

/* columns p,q with rotation j applied as in apply_rotation_in_the_plane(col p, col q, j) */
static void rot_cols_raw(double M[3][3], int p, int q, rot j) {
  if (j.c == 1.0 && j.s == 0.0) return;
  for (int i = 0; i < 3; i++) {
    double xi = M[i][p], yi = M[i][q];
    M[i][p] = j.c * xi + j.s * yi;
    M[i][q] = -j.s * xi + j.c * yi;
  }
}

static rot rot_transpose(rot j) { rot r = {j.c, -j.s}; return r; }

/* MatrixBase::applyOnTheRight(p,q,j) == apply_rotation_in_the_plane(col p, col q, j^T) */
static void apply_right(double M[3][3], int p, int q, rot j) { rot_cols_raw(M, p, q, rot_transpose(j)); }

/* JacobiRotation::makeJacobi(x, y, z) (Jacobi.h:85-110). */
static rot make_jacobi(double x, double y, double z) {
  rot r;
  double deno = 2.0 * fabs(y);
  if (deno < DBL_MIN) { r.c = 1.0; r.s = 0.0; return r; }
  double tau = (x - z) / deno;
  double w = sqrt(tau * tau + 1.0);
  double t;
  if (tau > 0.0) t = 1.0 / (tau + w);
  else t = 1.0 / (tau - w);
  double sign_t = t > 0.0 ? 1.0 : -1.0;
  double n = 1.0 / sqrt(t * t + 1.0);
  r.s = -sign_t * (y / fabs(y)) * fabs(t) * n;
  r.c = n;
  return r;
}

/* internal::real_2x2_jacobi_svd (misc/RealSvd2x2.h:19-50). */
static void real_2x2(double W[3][3], int p, int q, rot* jl, rot* jr) {
  double m[2][2] = {{W[p][p], W[p][q]}, {W[q][p], W[q][q]}};
  rot rot1;
  double t = m[0][0] + m[1][1];
  double d = m[1][0] - m[0][1];
  if (fabs(d) < DBL_MIN) {
    rot1.s = 0.0; rot1.c = 1.0;
  } else {
    double u = t / d;
    double tmp = sqrt(1.0 + u * u);
    rot1.s = 1.0 / tmp;
    rot1.c = u / tmp;
  }
  if (!(rot1.c == 1.0 && rot1.s == 0.0)) {
    for (int i = 0; i < 2; i++) {
      double xi = m[0][i], yi = m[1][i];
      m[0][i] = rot1.c * xi + rot1.s * yi;
      m[1][i] = -rot1.s * xi + rot1.c * yi;
    }
  }
  *jr = make_jacobi(m[0][0], m[0][1], m[1][1]);
  rot o = rot_transpose(*jr);
  jl->c = rot1.c * o.c - rot1.s * o.s;
  jl->s = rot1.c * o.s + rot1.s * o.c;
}

void orc_jacobi_svd3(const double H[9], double U9[9], double S[3], double V9[9]) {
  const double precision = 2.0 * DBL_EPSILON;
  const double consider_zero = DBL_MIN;
  double scale = fabs(H[0]);
  for (int i = 1; i < 9; i++) if (fabs(H[i]) > scale) scale = fabs(H[i]);
  if (scale == 0.0) scale = 1.0;
  double W[3][3], U[3][3], V[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      W[i][j] = H[3 * i + j] / scale;
      U[i][j] = (i == j) ? 1.0 : 0.0;
      V[i][j] = (i == j) ? 1.0 : 0.0;
    }
  double max_diag = fabs(W[0][0]);
  for (int i = 1; i < 3; i++) if (fabs(W[i][i]) > max_diag) max_diag = fabs(W[i][i]);
  int finished = 0;
  while (!finished) {
    finished = 1;
    for (int p = 1; p < 3; p++) {
      for (int q = 0; q < p; q++) {
        double thr = smax(consider_zero, precision * max_diag);
        if (fabs(W[p][q]) > thr || fabs(W[q][p]) > thr) {
          finished = 0;
          rot jl, jr;
          real_2x2(W, p, q, &jl, &jr);
          rot_rows(W, p, q, jl);
          apply_right(U, p, q, rot_transpose(jl));
          apply_right(W, p, q, jr);
          apply_right(V, p, q, jr);
          max_diag = smax(max_diag, smax(fabs(W[p][p]), fabs(W[q][q])));
        }
      }
    }
  }
  for (int i = 0; i < 3; i++) {
    double a = W[i][i];
    S[i] = fabs(a);
    if (a < 0.0)
      for (int r = 0; r < 3; r++) U[r][i] = -U[r][i];
  }
  for (int i = 0; i < 3; i++) S[i] *= scale;
  for (int i = 0; i < 3; i++) {
    int pos = i;
    double mx = S[i];
    for (int k = i + 1; k < 3; k++) if (S[k] > mx) { mx = S[k]; pos = k; }
    if (mx == 0.0) break;
    if (pos != i) {
      double tmp = S[i]; S[i] = S[pos]; S[pos] = tmp;
      for (int r = 0; r < 3; r++) {
        tmp = U[r][i]; U[r][i] = U[r][pos]; U[r][pos] = tmp;
        tmp = V[r][i]; V[r][i] = V[r][pos]; V[r][pos] = tmp;
      }
    }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) { U9[3 * i + j] = U[i][j]; V9[3 * i + j] = V[i][j]; }
}

static double det3(const double M[9]) {
  /* Eigen bruteforce_det3_helper order */
  double a = M[0] * (M[4] * M[8] - M[5] * M[7]);
  double b = M[1] * (M[3] * M[8] - M[5] * M[6]);
  double c = M[2] * (M[3] * M[7] - M[4] * M[6]);
  return a - b + c;
}

/* computeBestFitTransform (icpengine.cpp:76-115) / best_fit_transform (icp_registration.cpp:389-440). */
void orc_best_fit(const double* A, const double* B, int64_t n, double T[16]) {
  double ca[3] = {0, 0, 0}, cb[3] = {0, 0, 0};
  for (int64_t i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) { ca[k] += A[3 * i + k]; cb[k] += B[3 * i + k]; }
  for (int k = 0; k < 3; k++) { ca[k] /= (double)n; cb[k] /= (double)n; }
  double H[9] = {0};
  for (int64_t i = 0; i < n; i++) {
    double a[3], b[3];
    for (int k = 0; k < 3; k++) { a[k] = A[3 * i + k] - ca[k]; b[k] = B[3 * i + k] - cb[k]; }
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) H[3 * r + c] += a[r] * b[c];
  }
  double U[9], S[3], V[9], R[9];
  orc_jacobi_svd3(H, U, S, V);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      R[3 * r + c] = V[3 * r + 0] * U[3 * c + 0] + V[3 * r + 1] * U[3 * c + 1] + V[3 * r + 2] * U[3 * c + 2];
  if (det3(R) < 0) {
    for (int r = 0; r < 3; r++) V[3 * r + 2] *= -1;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++)
        R[3 * r + c] = V[3 * r + 0] * U[3 * c + 0] + V[3 * r + 1] * U[3 * c + 1] + V[3 * r + 2] * U[3 * c + 2];
  }
  double t[3];
  for (int r = 0; r < 3; r++) t[r] = cb[r] - (R[3 * r] * ca[0] + R[3 * r + 1] * ca[1] + R[3 * r + 2] * ca[2]);
  for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.0 : 0.0;
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) T[4 * r + c] = R[3 * r + c];
    T[4 * r + 3] = t[r];
  }
}

/* src = T * src with Eigen's order ((T0 x + T1 y) + T2 z) + T3 (icpengine.cpp:345). */
void orc_transform(const double T[16], double* xyz, int64_t n) {
  for (int64_t i = 0; i < n; i++) {
    double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    for (int r = 0; r < 3; r++)
      xyz[3 * i + r] = ((T[4 * r] * x + T[4 * r + 1] * y) + T[4 * r + 2] * z) + T[4 * r + 3];
  }
}

static void mat4_mul(const double A[16], const double B[16], double C[16]) {
  double R[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      R[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
  memcpy(C, R, sizeof(R));
}

/* ICPEngine::runICP (icpengine.cpp:117-394) and ICP() (icp_registration.cpp:443-622). */
int orc_icp(const orc_params* p, double* src, int64_t n, const double* tgt, int64_t m,
            orc_result* res, orc_iter* hist, int32_t cap) {
  memset(res, 0, sizeof(*res));
  const int cli = p->semantics == ORC_SEM_CLI;
  if (n <= 0 || m <= 0) return -1;
  const int max_pts = cli ? 10 : p->octree_max_points;   /* CLI hard-codes 10/20 (:454) */
  const int max_d = cli ? 20 : p->octree_max_depth;
  const double init_best = cli ? 1e20 : DBL_MAX;         /* :201 vs octree.cpp:180 */
  const double k_sigma = cli ? 3.0 : p->sigma_multiplier;
  orc_tree* tree = orc_octree_build(tgt, m, max_pts, max_d);
  double* cur = (double*)malloc(sizeof(double) * 3 * n);
  memcpy(cur, src, sizeof(double) * 3 * n);
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * n);
  double* d = (double*)malloc(sizeof(double) * n);
  double* va = (double*)malloc(sizeof(double) * 3 * n);
  double* vb = (double*)malloc(sizeof(double) * 3 * n);
  double T[16], Tc[16];
  for (int i = 0; i < 16; i++) T[i] = Tc[i] = (i % 5 == 0) ? 1.0 : 0.0;
  double prev = 1e10;
  int no_imp = 0, nh = 0, fail = 0, status = 0;
  double last_rec_rmse = 0.0;
  for (int iter = 0; iter < p->max_iterations; iter++) {
    orc_nn_batch(tree, cur, n, init_best, idx, d, NULL, NULL);
    double mean = 0;
    for (int64_t i = 0; i < n; i++) mean += d[i];
    mean /= (double)n;
    double var = 0;
    for (int64_t i = 0; i < n; i++) var += (d[i] - mean) * (d[i] - mean);
    double sd = sqrt(var / (double)n);
    double thr;
    if (!cli && iter == 0) thr = mean + smax(k_sigma * sd, mean * 0.5);
    else thr = mean + k_sigma * sd;
    int64_t V = 0;
    double sum_sq = 0;
    for (int64_t i = 0; i < n; i++) {
      if (d[i] <= thr) {
        memcpy(va + 3 * V, cur + 3 * i, sizeof(double) * 3);
        memcpy(vb + 3 * V, tgt + 3 * (int64_t)idx[i], sizeof(double) * 3);
        V++;
      }
    }
    /* sum over valid in index order (icpengine.cpp:274-277) */
    for (int64_t i = 0; i < n; i++) if (d[i] <= thr) sum_sq += d[i] * d[i];
    double rmse = (V > 0) ? sqrt(sum_sq / (double)V) : 0;
    double improvement = prev - rmse;
    if (fabs(improvement) < p->tolerance) {
      no_imp++;
      if (no_imp >= 3) {
        status = 1;
        if (!cli && hist && nh < cap) {
          orc_iter* h = &hist[nh];
          memset(h, 0, sizeof(*h));
          h->iteration = iter + 1; h->rmse = rmse; h->valid = (int32_t)V;
          h->outliers = (int32_t)(n - V); h->mean = mean; h->std = sd; h->threshold = thr;
          memcpy(h->T_cum, Tc, sizeof(Tc));
          h->has_transform = 0;
        }
        if (!cli) { nh++; last_rec_rmse = rmse; }
        break;
      }
    } else {
      no_imp = 0;
    }
    if (rmse > prev * 1.1) { status = 2; break; }
    prev = rmse;
    if (V < 3) {
      status = 3;
      if (!cli) fail = 1;
      break;
    }
    orc_best_fit(va, vb, V, T);
    mat4_mul(T, Tc, Tc);
    orc_transform(T, cur, n);
    if (hist && nh < cap) {
      orc_iter* h = &hist[nh];
      h->iteration = iter + 1; h->rmse = rmse; h->valid = (int32_t)V;
      h->outliers = (int32_t)(n - V); h->mean = mean; h->std = sd; h->threshold = thr;
      memcpy(h->T_inc, T, sizeof(T));
      memcpy(h->T_cum, Tc, sizeof(Tc));
      double tr = Tc[0] + Tc[5] + Tc[10];
      h->rotation_deg = acos((tr - 1.0) / 2.0) * 180.0 / M_PI;
      h->translation = sqrt(Tc[3] * Tc[3] + Tc[7] * Tc[7] + Tc[11] * Tc[11]);
      h->has_transform = 1;
    }
    nh++;
    last_rec_rmse = rmse;
  }
  res->status = status;
  res->n_history = nh < cap ? nh : cap;
  if (!fail) {
    memcpy(src, cur, sizeof(double) * 3 * n);
    /* engine: final = T_cumulative (icpengine.cpp:378-383); CLI: last incremental T (:616-621) */
    const double* F = cli ? T : Tc;
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) res->final_R[3 * r + c] = F[4 * r + c];
      res->final_t[r] = F[4 * r + 3];
    }
    res->success = 1;
    res->total_iterations = nh;
    if (cli) res->final_rmse = prev;                       /* cout "最终RMSE" prints prev_error */
    else res->final_rmse = nh > 0 ? last_rec_rmse : 0.0;     /* icpengine.cpp:387 */
  }
  free(cur); free(idx); free(d); free(va); free(vb);
  orc_octree_free(tree);
  return fail ? -3 : 0;
}
