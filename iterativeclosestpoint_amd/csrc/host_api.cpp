// host_api.cpp — host-side exports of libicp_hip.so (include/icp_host.h).
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/icp_host.h"
#include "icp_common.h"
#include "icp_ctx_internal.h"
#include "octree_build.h"
#include "query_order.h"

struct icp_octree {
  icp::FlatOctree t;
};

namespace {

// splitmix64: the k-th output of a stream seeded with `seed` is mix(seed + (k + 1) * gamma),
// so any element is addressable (parallel-safe, bit-reproducible on every host).
inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
constexpr uint64_t kGamma = 0x9e3779b97f4a7c15ull;
inline uint64_t rng_at(uint64_t seed, uint64_t k) { return mix64(seed + (k + 1) * kGamma); }
// uniform in (0, 1]
inline double u01(uint64_t r) { return ((double)(r >> 11) + 1.0) * (1.0 / 9007199254740992.0); }

inline void normal_pair(uint64_t seed, uint64_t k, double* z0, double* z1) {
  const double u1 = u01(rng_at(seed, 2 * k)), u2 = u01(rng_at(seed, 2 * k + 1));
  const double r = std::sqrt(-2.0 * std::log(u1));
  const double th = 6.283185307179586 * u2;
  *z0 = r * std::cos(th);
  *z1 = r * std::sin(th);
}

inline double normal_at(uint64_t seed, uint64_t k) {
  double a, b;
  normal_pair(seed, k >> 1, &a, &b);
  return (k & 1) ? b : a;
}

}  // namespace

extern "C" {

icp_octree* icp_octree_build(const double* xyz, int64_t n, int max_points, int max_depth) {
  icp_octree* o = new icp_octree();
  const char* why = nullptr;
  if (!icp::build_flat_octree(xyz, n, max_points, max_depth, &o->t, &why)) {
    icp_ctx_set_error(why ? why : "invalid target");
    delete o;
    return nullptr;
  }
  return o;
}

void icp_octree_free(icp_octree* t) { delete t; }

void icp_octree_get_info(const icp_octree* o, icp_octree_info* info) {
  info->n_nodes = (int64_t)o->t.nodes.size();
  info->n_leaves = o->t.n_leaves;
  info->n_points = (int64_t)o->t.pts.size();
  info->max_depth = o->t.max_depth;
  info->max_inner_depth = o->t.max_inner_depth;
  info->pos_of_orig0 = o->t.pos_of_orig0;
}

void icp_octree_copy_nodes(const icp_octree* o, double* box6, int32_t* first, uint32_t* meta, int32_t* depth) {
  for (size_t k = 0; k < o->t.nodes.size(); k++) {
    const icp::NodeRec& r = o->t.nodes[k];
    if (box6)
      for (int a = 0; a < 3; a++) {
        box6[6 * k + a] = r.lo[a];
        box6[6 * k + 3 + a] = r.hi[a];
      }
    if (first) first[k] = r.first;
    if (meta) meta[k] = r.meta;
    if (depth) depth[k] = r.depth;
  }
}

void icp_octree_copy_points(const icp_octree* o, double* xyz, int32_t* orig) {
  for (size_t k = 0; k < o->t.pts.size(); k++) {
    const icp::TgtPt& p = o->t.pts[k];
    if (xyz) {
      xyz[3 * k] = p.x;
      xyz[3 * k + 1] = p.y;
      xyz[3 * k + 2] = p.z;
    }
    if (orig) orig[k] = p.orig;
  }
}

void icp_moments_from_values(const double* d, int64_t n, double out8[8]) {
  icp::Moments m = icp::moments_identity();
  if (n > 0) {
    double s = 0.0, nb = 0.0;
    double mn = 1.7976931348623157e308, mx = 0.0;
    for (int64_t i = 0; i < n; i++) {
      s += d[i];
      if (std::isfinite(d[i])) {
        mn = d[i] < mn ? d[i] : mn;
        mx = d[i] > mx ? d[i] : mx;
      } else {
        nb += 1.0;
      }
    }
    m.n = (double)n;
    m.mean = s / (double)n;
    double m2 = 0.0;
    for (int64_t i = 0; i < n; i++) m2 += (d[i] - m.mean) * (d[i] - m.mean);
    m.m2 = m2;
    m.dmin = mn;
    m.dmax = mx;
    m.nbad = nb;
  }
  std::memcpy(out8, &m, sizeof(m));
}

void icp_moments_merge(const double* parts8, int32_t nparts, double out8[8]) {
  icp::Moments acc = icp::moments_identity();
  for (int32_t r = 0; r < nparts; r++) {
    icp::Moments p;
    std::memcpy(&p, parts8 + 8 * r, sizeof(p));
    acc = r == 0 ? p : icp::moments_merge(acc, p);
  }
  std::memcpy(out8, &acc, sizeof(acc));
}

void icp_cov_from_pairs(const double* a, const double* b, const double* d, int64_t n, double thr, double out20[20]) {
  icp::CovMoments c = icp::cov_identity();
  double cnt = 0.0, sd2 = 0.0, sa[3] = {0, 0, 0}, sb[3] = {0, 0, 0};
  for (int64_t i = 0; i < n; i++) {
    if (!(d[i] <= thr)) continue;
    cnt += 1.0;
    sd2 += d[i] * d[i];
    for (int k = 0; k < 3; k++) {
      sa[k] += a[3 * i + k];
      sb[k] += b[3 * i + k];
    }
  }
  if (cnt > 0) {
    c.n = cnt;
    c.sum_d2 = sd2;
    for (int k = 0; k < 3; k++) {
      c.ma[k] = sa[k] / cnt;
      c.mb[k] = sb[k] / cnt;
    }
    for (int64_t i = 0; i < n; i++) {
      if (!(d[i] <= thr)) continue;
      for (int r = 0; r < 3; r++)
        for (int q = 0; q < 3; q++) c.c[3 * r + q] += (a[3 * i + r] - c.ma[r]) * (b[3 * i + q] - c.mb[q]);
    }
  }
  std::memcpy(out20, &c, sizeof(c));
}

void icp_cov_merge(const double* parts20, int32_t nparts, double out20[20]) {
  icp::CovMoments acc = icp::cov_identity();
  for (int32_t r = 0; r < nparts; r++) {
    icp::CovMoments p;
    std::memcpy(&p, parts20 + 20 * r, sizeof(p));
    acc = r == 0 ? p : icp::cov_merge(acc, p);
  }
  std::memcpy(out20, &acc, sizeof(acc));
}

double icp_cull_threshold(double mean, double sd, double k_sigma, int iter, int engine_rules) {
  return icp::cull_threshold(mean, sd, k_sigma, iter, engine_rules);
}

void icp_synth_default(icp_synth_spec* s) {
  s->sigma[0] = 5.0;
  s->sigma[1] = 5.0;
  s->sigma[2] = 1.0;
  s->yaw_deg = 5.0;
  s->pitch_deg = 2.5;
  s->roll_deg = -2.5;
  s->t[0] = 0.5;
  s->t[1] = -0.3;
  s->t[2] = 0.1;
  s->noise_sigma = 1e-3;
  s->outlier_fraction = 0.01;
  s->seed_target = 42;
  s->seed_source = 43;
}

int icp_source_shard_order(const double* xyz, int64_t n, int32_t* order) {
  if (n < 0 || (n > 0 && (!xyz || !order)) || n > (int64_t)0x7fffffff) {
    icp_ctx_set_error("icp_source_shard_order: bad arguments");
    return -1;
  }
  std::vector<int32_t> perm;
  icp::kd_query_order(xyz, n, 8, &perm);
  std::memcpy(order, perm.data(), sizeof(int32_t) * (size_t)n);
  return 0;
}

int icp_synth_pair(const icp_synth_spec* s, int64_t n_tgt, int64_t n_src, double* tgt, double* src, double T_true[16]) {
  if (!s || n_tgt < 0 || n_src < 0 || n_src > n_tgt || (n_tgt > 0 && !tgt) || (n_src > 0 && !src) ||
      !(s->outlier_fraction >= 0.0 && s->outlier_fraction <= 1.0)) {
    icp_ctx_set_error("icp_synth_pair: bad arguments (need 0 <= n_src <= n_tgt, outlier_fraction in [0, 1])");
    return -1;
  }
  // R = Rz(yaw) Ry(pitch) Rx(roll) as test_icp.cpp:165-189
  const double d2r = M_PI / 180.0;
  const double cy = std::cos(s->yaw_deg * d2r), sy = std::sin(s->yaw_deg * d2r);
  const double cp = std::cos(s->pitch_deg * d2r), sp = std::sin(s->pitch_deg * d2r);
  const double cr = std::cos(s->roll_deg * d2r), sr = std::sin(s->roll_deg * d2r);
  const double Rz[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1};
  const double Ry[9] = {cp, 0, sp, 0, 1, 0, -sp, 0, cp};
  const double Rx[9] = {1, 0, 0, 0, cr, -sr, 0, sr, cr};
  double Rzy[9], R[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      Rzy[3 * i + j] = (Rz[3 * i] * Ry[j] + Rz[3 * i + 1] * Ry[3 + j]) + Rz[3 * i + 2] * Ry[6 + j];
    }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[3 * i + j] = (Rzy[3 * i] * Rx[j] + Rzy[3 * i + 1] * Rx[3 + j]) + Rzy[3 * i + 2] * Rx[6 + j];
  if (T_true) {
    for (int k = 0; k < 16; k++) T_true[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) T_true[4 * i + j] = R[3 * i + j];
      T_true[4 * i + 3] = s->t[i];
    }
  }
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n_tgt; i++)
    for (int k = 0; k < 3; k++) tgt[3 * i + k] = s->sigma[k] * normal_at(s->seed_target, (uint64_t)(3 * i + k));
  for (int64_t i = 0; i < n_tgt; i++)
    for (int k = 0; k < 3; k++) {
      const double v = tgt[3 * i + k];
      if (i == 0 || v < lo[k]) lo[k] = v;
      if (i == 0 || v > hi[k]) hi[k] = v;
    }
  if (n_src == 0) return 0;
  // seeded Fisher-Yates over the target indices; the first n_src become the source
  std::vector<int64_t> perm((size_t)n_tgt);
  for (int64_t i = 0; i < n_tgt; i++) perm[i] = i;
  const uint64_t shuffle_seed = s->seed_source ^ 0x5bd1e995ull;
  for (int64_t i = n_tgt - 1; i > 0; i--) {
    const uint64_t r = rng_at(shuffle_seed, (uint64_t)i);
    const int64_t j = (int64_t)(r % (uint64_t)(i + 1));
    const int64_t t = perm[i];
    perm[i] = perm[j];
    perm[j] = t;
  }
  const uint64_t noise_seed = s->seed_source;
  const uint64_t outlier_seed = s->seed_source ^ 0x27d4eb2f165667c5ull;
  // f in [0, 1); f = 1: every point (the cast of 2^64 would be undefined)
  const bool all = s->outlier_fraction >= 1.0;
  const uint64_t thresh = all ? 0 : (uint64_t)(s->outlier_fraction * 18446744073709551616.0);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n_src; i++) {
    double* o = src + 3 * i;
    const uint64_t pick = rng_at(outlier_seed, (uint64_t)(4 * i));
    if (s->outlier_fraction > 0 && (all || pick < thresh)) {
      for (int k = 0; k < 3; k++) o[k] = lo[k] + (hi[k] - lo[k]) * u01(rng_at(outlier_seed, (uint64_t)(4 * i + 1 + k)));
      continue;
    }
    const double* p = tgt + 3 * perm[i];
    const double q[3] = {p[0] - s->t[0], p[1] - s->t[1], p[2] - s->t[2]};
    for (int k = 0; k < 3; k++) {
      // R^T q
      const double v = (R[k] * q[0] + R[3 + k] * q[1]) + R[6 + k] * q[2];
      o[k] = v + s->noise_sigma * normal_at(noise_seed, (uint64_t)(3 * i + k));
    }
  }
  return 0;
}

void icp_scene_default(icp_scene_spec* s) {
  s->site_radius = 40.0;
  s->scanner_height = 1.8;
  s->n_walls = 8;
  s->wall_height = 6.0;
  s->terrain_amp = 0.3;
  s->elev_min_deg = -45.0;
  s->elev_max_deg = 35.0;
  s->range_noise = 2e-3;
  s->quantum = 1e-3;
  s->yaw_deg = 2.0;
  s->pitch_deg = 0.5;
  s->roll_deg = -0.5;
  s->t[0] = 0.3;
  s->t[1] = -0.2;
  s->t[2] = 0.05;
  s->outlier_fraction = 0.002;
  s->seed_target = 7;
  s->seed_source = 8;
}

}  // extern "C"

namespace {

// The scene of icp_synth_scene: a height field and vertical wall rectangles (base segment on the
// ground, height wall_height); fixed by the spec (the walls from a stream of their own).
struct Scene {
  double h, amp, H, rmax;
  std::vector<double> wx0, wy0, wx1, wy1;
  explicit Scene(const icp_scene_spec& s) : h(s.scanner_height), amp(s.terrain_amp), H(s.wall_height) {
    rmax = 1.5 * s.site_radius;
    const uint64_t seed = 0x6a09e667f3bcc909ull;  // the same walls for every scan of a spec
    for (int w = 0; w < s.n_walls; w++) {
      const double ang = 6.283185307179586 * u01(rng_at(seed, 4 * w));
      const double dist = s.site_radius * (0.25 + 0.75 * u01(rng_at(seed, 4 * w + 1)));
      const double len = s.site_radius * (0.2 + 0.4 * u01(rng_at(seed, 4 * w + 2)));
      const double turn = 1.5707963267948966 * (u01(rng_at(seed, 4 * w + 3)) - 0.5);  // facade orientation
      const double cx = dist * std::cos(ang), cy = dist * std::sin(ang);
      const double ux = -std::sin(ang + turn), uy = std::cos(ang + turn);
      wx0.push_back(cx - 0.5 * len * ux);
      wy0.push_back(cy - 0.5 * len * uy);
      wx1.push_back(cx + 0.5 * len * ux);
      wy1.push_back(cy + 0.5 * len * uy);
    }
  }
  double ground(double x, double y) const {
    return amp * (std::sin(x / 11.0) * std::cos(y / 7.0) + 0.5 * std::sin((x + y) / 5.0));
  }
  // Range of the nearest surface along the unit ray d from the scanner at (ox, oy, h + oz); <= 0: none
  double hit(double ox, double oy, double oz, const double d[3]) const {
    double best = -1.0;
    const double z0 = h + oz;
    if (d[2] < -1e-9) {  // the ground, as the plane z = 0 (the height field displaces z afterwards)
      const double t = -z0 / d[2];
      if (t <= rmax) best = t;
    }
    for (size_t w = 0; w < wx0.size(); w++) {
      // ray (ox + dx t, oy + dy t) against the segment P0 + u (P1 - P0), u in [0, 1]
      const double ex = wx1[w] - wx0[w], ey = wy1[w] - wy0[w];
      const double den = d[0] * ey - d[1] * ex;
      if (std::fabs(den) < 1e-12) continue;
      const double px = wx0[w] - ox, py = wy0[w] - oy;
      const double t = (px * ey - py * ex) / den;
      const double u = (px * d[1] - py * d[0]) / den;
      const double z = z0 + d[2] * t;
      if (t > 0.5 && t <= rmax && u >= 0.0 && u <= 1.0 && z >= 0.0 && z <= H && (best < 0.0 || t < best)) best = t;
    }
    return best;
  }
  // One return of the scanner at (ox, oy, oz) (world; oz above scanner height), ray stream `seed`,
  // point k: up to 64 rays until one hits.
  void scan_point(const icp_scene_spec& s, double ox, double oy, double oz, uint64_t seed, uint64_t k,
                  double out[3]) const {
    const double d2r = 3.141592653589793 / 180.0;
    for (uint64_t tr = 0; tr < 64; tr++) {
      const uint64_t q = 64 * k + tr;
      const double az = 6.283185307179586 * u01(rng_at(seed, 3 * q));
      const double el = d2r * (s.elev_min_deg + (s.elev_max_deg - s.elev_min_deg) * u01(rng_at(seed, 3 * q + 1)));
      const double d[3] = {std::cos(el) * std::cos(az), std::cos(el) * std::sin(az), std::sin(el)};
      double t = hit(ox, oy, oz, d);
      if (t <= 0.0) continue;
      t += s.range_noise * normal_at(seed ^ 0x243f6a8885a308d3ull, q);
      out[0] = ox + d[0] * t;
      out[1] = oy + d[1] * t;
      out[2] = h + oz + d[2] * t;
      // a ground return follows the height field (walls stand on z = 0 of their own)
      if (out[2] < 0.01 + 4.0 * s.range_noise && d[2] < 0.0) out[2] += ground(out[0], out[1]);
      return;
    }
    out[0] = ox;  // no return in 64 rays (a scan of the sky): the ground below the scanner
    out[1] = oy;
    out[2] = ground(ox, oy);
  }
};

inline double quantize(double v, double q) { return q > 0.0 ? std::nearbyint(v / q) * q : v; }

}  // namespace

extern "C" {

int icp_synth_scene(const icp_scene_spec* s, int64_t n_tgt, int64_t n_src, double* tgt, double* src,
                    double T_true[16]) {
  if (!s || n_tgt < 0 || n_src < 0 || (n_tgt > 0 && !tgt) || (n_src > 0 && !src) || !(s->site_radius > 0.0) ||
      s->n_walls < 0 || s->n_walls > 4096 || !(s->elev_max_deg > s->elev_min_deg) || !(s->quantum >= 0.0) ||
      !(s->outlier_fraction >= 0.0 && s->outlier_fraction <= 1.0)) {
    icp_ctx_set_error("icp_synth_scene: bad arguments");
    return -1;
  }
  const Scene sc(*s);
  const double d2r = M_PI / 180.0;
  const double cy = std::cos(s->yaw_deg * d2r), sy = std::sin(s->yaw_deg * d2r);
  const double cp = std::cos(s->pitch_deg * d2r), sp = std::sin(s->pitch_deg * d2r);
  const double cr = std::cos(s->roll_deg * d2r), sr = std::sin(s->roll_deg * d2r);
  const double Rz[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1};
  const double Ry[9] = {cp, 0, sp, 0, 1, 0, -sp, 0, cp};
  const double Rx[9] = {1, 0, 0, 0, cr, -sr, 0, sr, cr};
  double Rzy[9], R[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Rzy[3 * i + j] = (Rz[3 * i] * Ry[j] + Rz[3 * i + 1] * Ry[3 + j]) + Rz[3 * i + 2] * Ry[6 + j];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[3 * i + j] = (Rzy[3 * i] * Rx[j] + Rzy[3 * i + 1] * Rx[3 + j]) + Rzy[3 * i + 2] * Rx[6 + j];
  if (T_true) {
    for (int k = 0; k < 16; k++) T_true[k] = (k % 5 == 0) ? 1.0 : 0.0;
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) T_true[4 * i + j] = R[3 * i + j];
      T_true[4 * i + 3] = s->t[i];
    }
  }
  for (int64_t i = 0; i < n_tgt; i++) {
    double p[3];
    sc.scan_point(*s, 0.0, 0.0, 0.0, s->seed_target, (uint64_t)i, p);
    for (int k = 0; k < 3; k++) tgt[3 * i + k] = quantize(p[k], s->quantum);
  }
  if (n_src == 0) return 0;
  double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  for (int64_t i = 0; i < n_src; i++) {
    double p[3];
    sc.scan_point(*s, s->t[0], s->t[1], s->t[2], s->seed_source, (uint64_t)i, p);
    const double q[3] = {p[0] - s->t[0], p[1] - s->t[1], p[2] - s->t[2]};
    for (int k = 0; k < 3; k++) {
      const double v = quantize((R[k] * q[0] + R[3 + k] * q[1]) + R[6 + k] * q[2], s->quantum);  // R^T q
      src[3 * i + k] = v;
      if (i == 0 || v < lo[k]) lo[k] = v;
      if (i == 0 || v > hi[k]) hi[k] = v;
    }
  }
  const uint64_t oseed = s->seed_source ^ 0x13198a2e03707344ull;
  // f in [0, 1); f = 1: every point (the cast of 2^64 would be undefined)
  const bool all = s->outlier_fraction >= 1.0;
  const uint64_t thresh = all ? 0 : (uint64_t)(s->outlier_fraction * 18446744073709551616.0);
  if (s->outlier_fraction > 0)
    for (int64_t i = 0; i < n_src; i++)
      if (all || rng_at(oseed, (uint64_t)(4 * i)) < thresh)
        for (int k = 0; k < 3; k++)
          src[3 * i + k] = quantize(lo[k] + (hi[k] - lo[k]) * u01(rng_at(oseed, (uint64_t)(4 * i + 1 + k))), s->quantum);
  return 0;
}

}  // extern "C"
