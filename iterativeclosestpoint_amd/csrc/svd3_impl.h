// svd3_impl.h — the 3x3 two-sided Jacobi SVD (the algorithm of Eigen 3.3.4's JacobiSVD that the
// reference calls at icpengine.cpp:93 / icp_registration.cpp:418), the rigid best fit built on it
// (icpengine.cpp:76-115, icp_registration.cpp:389-440) and the 4x4 product, as host + device
// functions: the host engine (engine.cpp) and the device-resident loop
// (reduce_kernels.hip, the publishing kernel) run the same operations in the same order, so with
// IEEE fp64 (+, -, *, /, sqrt correctly rounded on both; no contraction: -ffp-contract=off) they
// give the same bits (tests/test_gpu_parity.py::test_device_loop_*).
// Two-sided Jacobi sweeps over the (p, q) = (1,0), (2,0), (2,1) pairs of the scaled matrix,
// each pair diagonalised by a left rotation composed from a symmetrising rotation and a
// symmetric Jacobi rotation, until every off-diagonal entry is below 2*eps*max|diag|; then the
// diagonal is made non-negative (negating U columns) and sorted descending.
// (Algorithm: Eigen/src/SVD/JacobiSVD.h:663-786, misc/RealSvd2x2.h:19-50, Jacobi/Jacobi.h:85-110.)
#pragma once

#include "icp_common.h"

namespace icp {
namespace svd {

constexpr double kDblMin = 2.2250738585072014e-308;
constexpr double kDblEps = 2.220446049250313e-16;

struct Givens {
  double c, s;
};
ICP_HD Givens transposed(Givens g) { return Givens{g.c, -g.s}; }
ICP_HD bool is_identity(Givens g) { return g.c == 1.0 && g.s == 0.0; }

struct M3 {
  double a[3][3];
};

// rows p, q  <-  G applied from the left: [x; y] -> [c x + s y; -s x + c y]
ICP_HD void left(M3& m, int p, int q, Givens g) {
  if (is_identity(g)) return;
  for (int k = 0; k < 3; k++) {
    const double x = m.a[p][k], y = m.a[q][k];
    m.a[p][k] = g.c * x + g.s * y;
    m.a[q][k] = -g.s * x + g.c * y;
  }
}

// columns p, q  <-  M * G  (Eigen applyOnTheRight(p, q, G) rotates the columns with G^T)
ICP_HD void right(M3& m, int p, int q, Givens g) {
  const Givens h = transposed(g);
  if (is_identity(h)) return;
  for (int k = 0; k < 3; k++) {
    const double x = m.a[k][p], y = m.a[k][q];
    m.a[k][p] = h.c * x + h.s * y;
    m.a[k][q] = -h.s * x + h.c * y;
  }
}

// symmetric 2x2 Jacobi rotation for [[x, y], [y, z]]
ICP_HD Givens sym_jacobi(double x, double y, double z) {
  const double deno = 2.0 * __builtin_fabs(y);
  if (deno < kDblMin) return Givens{1.0, 0.0};
  const double tau = (x - z) / deno;
  const double w = __builtin_sqrt(tau * tau + 1.0);
  const double t = (tau > 0.0) ? 1.0 / (tau + w) : 1.0 / (tau - w);
  const double sign_t = t > 0.0 ? 1.0 : -1.0;
  const double n = 1.0 / __builtin_sqrt(t * t + 1.0);
  return Givens{n, -sign_t * (y / __builtin_fabs(y)) * __builtin_fabs(t) * n};
}

ICP_HD void svd_2x2(const M3& w, int p, int q, Givens* gl, Givens* gr) {
  double b00 = w.a[p][p], b01 = w.a[p][q], b10 = w.a[q][p], b11 = w.a[q][q];
  Givens sym{1.0, 0.0};
  const double t = b00 + b11;
  const double d = b10 - b01;
  if (!(__builtin_fabs(d) < kDblMin)) {
    const double u = t / d;
    const double r = __builtin_sqrt(1.0 + u * u);
    sym = Givens{u / r, 1.0 / r};
  }
  if (!is_identity(sym)) {
    const double n00 = sym.c * b00 + sym.s * b10, n01 = sym.c * b01 + sym.s * b11;
    const double n10 = -sym.s * b00 + sym.c * b10, n11 = -sym.s * b01 + sym.c * b11;
    b00 = n00; b01 = n01; b10 = n10; b11 = n11;
  }
  *gr = sym_jacobi(b00, b01, b11);
  const Givens o = transposed(*gr);
  gl->c = sym.c * o.c - sym.s * o.s;
  gl->s = sym.c * o.s + sym.s * o.c;
}

// H = U * diag(S) * V^T, all row-major; singular values descending.
ICP_HD void jacobi_svd3(const double H[9], double U9[9], double S[3], double V9[9]) {
  const double precision = 2.0 * kDblEps;
  double scale = 0.0;
  for (int k = 0; k < 9; k++) {
    const double v = __builtin_fabs(H[k]);
    if (k == 0 || v > scale) scale = v;
  }
  if (scale == 0.0) scale = 1.0;
  M3 w, u, v;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      w.a[i][j] = H[3 * i + j] / scale;
      u.a[i][j] = v.a[i][j] = (i == j) ? 1.0 : 0.0;
    }
  double max_diag = __builtin_fabs(w.a[0][0]);
  for (int i = 1; i < 3; i++) max_diag = smax(max_diag, __builtin_fabs(w.a[i][i]));
  // first index of a maximum, as Eigen's maxCoeff visitor (strict >)
  for (bool done = false; !done;) {
    done = true;
    // (p, q) = (1, 0), (2, 0), (2, 1), unrolled: constant indices keep the matrices in registers
    // on the device (a dynamic index puts them in scratch)
#pragma unroll
    for (int p = 1; p < 3; p++) {
#pragma unroll
      for (int q = 0; q < p; q++) {
        const double thr = smax(kDblMin, precision * max_diag);
        if (__builtin_fabs(w.a[p][q]) > thr || __builtin_fabs(w.a[q][p]) > thr) {
          done = false;
          Givens gl, gr;
          svd_2x2(w, p, q, &gl, &gr);
          left(w, p, q, gl);
          right(u, p, q, transposed(gl));
          right(w, p, q, gr);
          right(v, p, q, gr);
          max_diag = smax(max_diag, smax(__builtin_fabs(w.a[p][p]), __builtin_fabs(w.a[q][q])));
        }
      }
    }
  }
  for (int i = 0; i < 3; i++) {
    const double a = w.a[i][i];
    S[i] = __builtin_fabs(a);
    if (a < 0.0)
      for (int r = 0; r < 3; r++) u.a[r][i] = -u.a[r][i];
  }
  for (int i = 0; i < 3; i++) S[i] *= scale;
  // selection sort, descending: at step i the first index of the maximum of S[i..2] (strict >)
  // is swapped in; a zero maximum ends it (Eigen's JacobiSVD). Written with constant indices
  // (each swap candidate tested in turn) so that nothing is indexed dynamically.
  bool sorted_end = false;
#pragma unroll
  for (int i = 0; i < 2; i++) {
    if (sorted_end) break;
    int pos = i;
    double best = S[i];
#pragma unroll
    for (int k = i + 1; k < 3; k++)
      if (S[k] > best) {
        pos = k;
        best = S[k];
      }
    if (best == 0.0) {
      sorted_end = true;
      break;
    }
#pragma unroll
    for (int k = i + 1; k < 3; k++)
      if (pos == k) {
        double t = S[i]; S[i] = S[k]; S[k] = t;
#pragma unroll
        for (int r = 0; r < 3; r++) {
          t = u.a[r][i]; u.a[r][i] = u.a[r][k]; u.a[r][k] = t;
          t = v.a[r][i]; v.a[r][i] = v.a[r][k]; v.a[r][k] = t;
        }
      }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      U9[3 * i + j] = u.a[i][j];
      V9[3 * i + j] = v.a[i][j];
    }
}

ICP_HD void vut(const double V[9], const double U[9], double R[9]) {
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      R[3 * r + c] = (V[3 * r] * U[3 * c] + V[3 * r + 1] * U[3 * c + 1]) + V[3 * r + 2] * U[3 * c + 2];
}

// Rigid transform (row-major 4x4): R = V U^T (reflection fixed by negating V's third column,
// icpengine.cpp:98-104), t = mb - R ma (:107).
ICP_HD void best_fit_from_moments(const double ma[3], const double mb[3], const double C[9], double T[16]) {
  double U[9], S[3], V[9], R[9];
  jacobi_svd3(C, U, S, V);
  vut(V, U, R);
  // det via the 3x3 cofactor expansion along row 0 (Eigen bruteforce_det3_helper order)
  const double det = (R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6])) +
                     R[2] * (R[3] * R[7] - R[4] * R[6]);
  if (det < 0) {
    for (int r = 0; r < 3; r++) V[3 * r + 2] = -V[3 * r + 2];
    vut(V, U, R);
  }
  for (int k = 0; k < 16; k++) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  for (int r = 0; r < 3; r++) {
    const double Ra = (R[3 * r] * ma[0] + R[3 * r + 1] * ma[1]) + R[3 * r + 2] * ma[2];
    for (int c = 0; c < 3; c++) T[4 * r + c] = R[3 * r + c];
    T[4 * r + 3] = mb[r] - Ra;
  }
}

// 4x4 row-major C = A * B with the reference's summation order (C may alias A or B).
ICP_HD void mat4_mul(const double A[16], const double B[16], double C[16]) {
  double R[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      R[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
  for (int k = 0; k < 16; k++) C[k] = R[k];
}

}  // namespace svd
}  // namespace icp
