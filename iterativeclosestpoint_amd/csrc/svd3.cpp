// svd3.cpp — see svd3.h.
//
// Two-sided Jacobi sweeps over the (p, q) = (1,0), (2,0), (2,1) pairs of the scaled matrix,
// each pair diagonalised by a left rotation composed from a symmetrising rotation and a
// symmetric Jacobi rotation, until every off-diagonal entry is below 2*eps*max|diag|; then the
// diagonal is made non-negative (negating U columns) and sorted descending.
// (Algorithm: Eigen/src/SVD/JacobiSVD.h:663-786, misc/RealSvd2x2.h:19-50, Jacobi/Jacobi.h:85-110.)
#include "svd3.h"

#include <cfloat>
#include <cmath>
#include <cstring>

namespace icp {

namespace {

struct Givens {
  double c, s;
  Givens T() const { return Givens{c, -s}; }
  bool identity() const { return c == 1.0 && s == 0.0; }
};

struct M3 {
  double a[3][3];
};

// rows p, q  <-  G applied from the left: [x; y] -> [c x + s y; -s x + c y]
void left(M3& m, int p, int q, Givens g) {
  if (g.identity()) return;
  for (int k = 0; k < 3; k++) {
    const double x = m.a[p][k], y = m.a[q][k];
    m.a[p][k] = g.c * x + g.s * y;
    m.a[q][k] = -g.s * x + g.c * y;
  }
}

// columns p, q  <-  M * G  (Eigen applyOnTheRight(p, q, G) rotates the columns with G^T)
void right(M3& m, int p, int q, Givens g) {
  const Givens h = g.T();
  if (h.identity()) return;
  for (int k = 0; k < 3; k++) {
    const double x = m.a[k][p], y = m.a[k][q];
    m.a[k][p] = h.c * x + h.s * y;
    m.a[k][q] = -h.s * x + h.c * y;
  }
}

// symmetric 2x2 Jacobi rotation for [[x, y], [y, z]]
Givens sym_jacobi(double x, double y, double z) {
  const double deno = 2.0 * std::fabs(y);
  if (deno < DBL_MIN) return Givens{1.0, 0.0};
  const double tau = (x - z) / deno;
  const double w = std::sqrt(tau * tau + 1.0);
  const double t = (tau > 0.0) ? 1.0 / (tau + w) : 1.0 / (tau - w);
  const double sign_t = t > 0.0 ? 1.0 : -1.0;
  const double n = 1.0 / std::sqrt(t * t + 1.0);
  return Givens{n, -sign_t * (y / std::fabs(y)) * std::fabs(t) * n};
}

void svd_2x2(const M3& w, int p, int q, Givens* gl, Givens* gr) {
  double b00 = w.a[p][p], b01 = w.a[p][q], b10 = w.a[q][p], b11 = w.a[q][q];
  Givens sym{1.0, 0.0};
  const double t = b00 + b11;
  const double d = b10 - b01;
  if (!(std::fabs(d) < DBL_MIN)) {
    const double u = t / d;
    const double r = std::sqrt(1.0 + u * u);
    sym = Givens{u / r, 1.0 / r};
  }
  if (!sym.identity()) {
    const double n00 = sym.c * b00 + sym.s * b10, n01 = sym.c * b01 + sym.s * b11;
    const double n10 = -sym.s * b00 + sym.c * b10, n11 = -sym.s * b01 + sym.c * b11;
    b00 = n00; b01 = n01; b10 = n10; b11 = n11;
  }
  *gr = sym_jacobi(b00, b01, b11);
  const Givens o = gr->T();
  gl->c = sym.c * o.c - sym.s * o.s;
  gl->s = sym.c * o.s + sym.s * o.c;
}

}  // namespace

void jacobi_svd3(const double H[9], double U9[9], double S[3], double V9[9]) {
  const double precision = 2.0 * DBL_EPSILON;
  double scale = 0.0;
  for (int k = 0; k < 9; k++) {
    const double v = std::fabs(H[k]);
    if (k == 0 || v > scale) scale = v;
  }
  if (scale == 0.0) scale = 1.0;
  M3 w, u, v;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      w.a[i][j] = H[3 * i + j] / scale;
      u.a[i][j] = v.a[i][j] = (i == j) ? 1.0 : 0.0;
    }
  double max_diag = std::fabs(w.a[0][0]);
  for (int i = 1; i < 3; i++) max_diag = smax(max_diag, std::fabs(w.a[i][i]));
  // first index of a maximum, as Eigen's maxCoeff visitor (strict >)
  for (bool done = false; !done;) {
    done = true;
    for (int p = 1; p < 3; p++) {
      for (int q = 0; q < p; q++) {
        const double thr = smax(DBL_MIN, precision * max_diag);
        if (std::fabs(w.a[p][q]) > thr || std::fabs(w.a[q][p]) > thr) {
          done = false;
          Givens gl, gr;
          svd_2x2(w, p, q, &gl, &gr);
          left(w, p, q, gl);
          right(u, p, q, gl.T());
          right(w, p, q, gr);
          right(v, p, q, gr);
          max_diag = smax(max_diag, smax(std::fabs(w.a[p][p]), std::fabs(w.a[q][q])));
        }
      }
    }
  }
  for (int i = 0; i < 3; i++) {
    const double a = w.a[i][i];
    S[i] = std::fabs(a);
    if (a < 0.0)
      for (int r = 0; r < 3; r++) u.a[r][i] = -u.a[r][i];
  }
  for (int i = 0; i < 3; i++) S[i] *= scale;
  for (int i = 0; i < 3; i++) {
    int pos = i;
    for (int k = i + 1; k < 3; k++)
      if (S[k] > S[pos]) pos = k;
    if (S[pos] == 0.0) break;
    if (pos != i) {
      double t = S[i]; S[i] = S[pos]; S[pos] = t;
      for (int r = 0; r < 3; r++) {
        t = u.a[r][i]; u.a[r][i] = u.a[r][pos]; u.a[r][pos] = t;
        t = v.a[r][i]; v.a[r][i] = v.a[r][pos]; v.a[r][pos] = t;
      }
    }
  }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      U9[3 * i + j] = u.a[i][j];
      V9[3 * i + j] = v.a[i][j];
    }
}

static void vut(const double V[9], const double U[9], double R[9]) {
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++)
      R[3 * r + c] = (V[3 * r] * U[3 * c] + V[3 * r + 1] * U[3 * c + 1]) + V[3 * r + 2] * U[3 * c + 2];
}

void best_fit_from_moments(const double ma[3], const double mb[3], const double C[9], double T[16]) {
  double U[9], S[3], V[9], R[9];
  jacobi_svd3(C, U, S, V);
  vut(V, U, R);
  // det via the 3x3 cofactor expansion along row 0 (Eigen bruteforce_det3_helper order)
  const double det = (R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6])) +
                     R[2] * (R[3] * R[7] - R[4] * R[6]);
  if (det < 0) {  // icpengine.cpp:101-104
    for (int r = 0; r < 3; r++) V[3 * r + 2] = -V[3 * r + 2];
    vut(V, U, R);
  }
  for (int k = 0; k < 16; k++) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  for (int r = 0; r < 3; r++) {
    const double Ra = (R[3 * r] * ma[0] + R[3 * r + 1] * ma[1]) + R[3 * r + 2] * ma[2];
    for (int c = 0; c < 3; c++) T[4 * r + c] = R[3 * r + c];
    T[4 * r + 3] = mb[r] - Ra;  // icpengine.cpp:107
  }
}

void mat4_mul(const double A[16], const double B[16], double C[16]) {
  double R[16];
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++)
      R[4 * r + c] = ((A[4 * r] * B[c] + A[4 * r + 1] * B[4 + c]) + A[4 * r + 2] * B[8 + c]) + A[4 * r + 3] * B[12 + c];
  std::memcpy(C, R, sizeof(R));
}

}  // namespace icp
