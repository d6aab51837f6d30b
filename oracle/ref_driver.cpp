// ref_driver.cpp — TEST INFRASTRUCTURE ONLY.
//
// Builds the REFERENCE itself (icp_registration.cpp + its vendored Eigen 3.3.4, compiled where
// they lie under /root/reference; nothing is copied) into oracle/_ref/libicp_ref.so and exposes
// a few C entry points used to generate golden fixtures (tests/golden/gen_golden.py) and to time
// the reference CPU path (oracle/_ref/ref_bench, bench.py cpu_baseline leg).
//
// Recipe: oracle/Makefile. Flags: -O2 -ffp-contract=off, no -march (CMakeLists.txt:7-12 builds
// with plain -std=c++17, i.e. baseline x86-64 without FMA).
#include <cstdint>
#include <cstring>

#define main icp_reference_cli_main
#include "icp_registration.cpp"
#undef main

namespace {
struct RefTree {
  std::vector<Point3D> pts;
  Octree* tree = nullptr;
};
}  // namespace

extern "C" {

// Octree(target.points, max_pts, max_d) (icp_registration.cpp:154-190).
void* ref_octree_build(const double* xyz, int64_t n, int max_pts, int max_d) {
  RefTree* r = new RefTree;
  r->pts.resize(n);
  for (int64_t i = 0; i < n; i++) r->pts[i] = Point3D(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
  r->tree = new Octree(r->pts, max_pts, max_d);
  return r;
}

void ref_octree_free(void* h) {
  RefTree* r = static_cast<RefTree*>(h);
  delete r->tree;
  delete r;
}

// Octree::findNearest (icp_registration.cpp:197-205), best initialised to 1e20.
void ref_nn_batch(void* h, const double* q, int64_t n, int32_t* idx_out) {
  RefTree* r = static_cast<RefTree*>(h);
  for (int64_t i = 0; i < n; i++) idx_out[i] = r->tree->findNearest(Point3D(q[3 * i], q[3 * i + 1], q[3 * i + 2]));
}

// distance() (icp_registration.cpp:381-386).
double ref_distance(const double a[3], const double b[3]) {
  return distance(Point3D(a[0], a[1], a[2]), Point3D(b[0], b[1], b[2]));
}

// ICP() (icp_registration.cpp:443-622). T_cum list: cap x 16 row-major.
void ref_icp_cli(double* src, int64_t n, const double* tgt, int64_t m, int max_iters, double tol,
                 double R_out[9], double t_out[3], double* tcums, int cap, int* n_tcums) {
  PointCloud s, t;
  for (int64_t i = 0; i < n; i++) s.addPoint(Point3D(src[3 * i], src[3 * i + 1], src[3 * i + 2]));
  for (int64_t i = 0; i < m; i++) t.addPoint(Point3D(tgt[3 * i], tgt[3 * i + 1], tgt[3 * i + 2]));
  double R[3][3], tt[3];
  std::vector<Eigen::Matrix4d> hist;
  ICP(s, t, max_iters, tol, R, tt, &hist);
  for (int64_t i = 0; i < n; i++) {
    src[3 * i] = s.points[i].x;
    src[3 * i + 1] = s.points[i].y;
    src[3 * i + 2] = s.points[i].z;
  }
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) R_out[3 * r + c] = R[r][c];
    t_out[r] = tt[r];
  }
  int k = 0;
  for (; k < (int)hist.size() && k < cap; k++)
    for (int r = 0; r < 4; r++)
      for (int c = 0; c < 4; c++) tcums[16 * k + 4 * r + c] = hist[k](r, c);
  *n_tcums = (int)hist.size();
}

// best_fit_transform (icp_registration.cpp:389-440) on N x 3 inputs given as AoS.
void ref_best_fit_transform(const double* a, const double* b, int64_t n, double T_out[16]) {
  Eigen::MatrixXd A(n, 3), B(n, 3);
  for (int64_t i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) {
      A(i, k) = a[3 * i + k];
      B(i, k) = b[3 * i + k];
    }
  Eigen::Matrix4d T = best_fit_transform(A, B);
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) T_out[4 * r + c] = T(r, c);
}

// Eigen::JacobiSVD on a 3x3, fixed (Matrix3d, icpengine.cpp:93) or dynamic (MatrixXd, :418).
void ref_jacobi_svd3(const double H9[9], int dynamic, double U9[9], double S3[3], double V9[9]) {
  Eigen::Matrix3d U, V;
  Eigen::Vector3d S;
  if (dynamic) {
    Eigen::MatrixXd H(3, 3);
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) H(r, c) = H9[3 * r + c];
    Eigen::JacobiSVD<Eigen::MatrixXd> svd(H, Eigen::ComputeFullU | Eigen::ComputeFullV);
    U = svd.matrixU();
    V = svd.matrixV();
    S = svd.singularValues();
  } else {
    Eigen::Matrix3d H;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) H(r, c) = H9[3 * r + c];
    Eigen::JacobiSVD<Eigen::Matrix3d> svd(H, Eigen::ComputeFullU | Eigen::ComputeFullV);
    U = svd.matrixU();
    V = svd.matrixV();
    S = svd.singularValues();
  }
  for (int r = 0; r < 3; r++) {
    S3[r] = S(r);
    for (int c = 0; c < 3; c++) {
      U9[3 * r + c] = U(r, c);
      V9[3 * r + c] = V(r, c);
    }
  }
}

// src = T * src with Eigen's Matrix4d * MatrixXd(4 x N) (icpengine.cpp:345, CLI :598).
void ref_transform(const double T16[16], double* xyz, int64_t n) {
  Eigen::Matrix4d T;
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) T(r, c) = T16[4 * r + c];
  Eigen::MatrixXd src = Eigen::MatrixXd::Ones(4, n);
  for (int64_t i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) src(k, i) = xyz[3 * i + k];
  src = T * src;
  for (int64_t i = 0; i < n; i++)
    for (int k = 0; k < 3; k++) xyz[3 * i + k] = src(k, i);
}

// T_cumulative = T * T_cumulative (Matrix4d * Matrix4d, icpengine.cpp:342).
void ref_mat4_mul(const double A16[16], const double B16[16], double C16[16]) {
  Eigen::Matrix4d A, B;
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) {
      A(r, c) = A16[4 * r + c];
      B(r, c) = B16[4 * r + c];
    }
  Eigen::Matrix4d C = A * B;
  for (int r = 0; r < 4; r++)
    for (int c = 0; c < 4; c++) C16[4 * r + c] = C(r, c);
}

}  // extern "C"

extern "C" {

// readLASFile (icp_registration.cpp:248-378). Returns the number of points (<= cap copied),
// -1 on failure; scale/offset of the file in so[6].
int64_t ref_read_las(const char* path, double* xyz, int64_t cap, double so[6]) {
  PointCloud c;
  std::streambuf* old = std::cout.rdbuf();
  std::ofstream devnull("/dev/null");
  std::cout.rdbuf(devnull.rdbuf());
  bool ok = readLASFile(path, c);
  std::cout.rdbuf(old);
  if (!ok) return -1;
  for (int64_t i = 0; i < (int64_t)c.points.size() && i < cap; i++) {
    xyz[3 * i] = c.points[i].x;
    xyz[3 * i + 1] = c.points[i].y;
    xyz[3 * i + 2] = c.points[i].z;
  }
  so[0] = c.x_scale; so[1] = c.y_scale; so[2] = c.z_scale;
  so[3] = c.x_offset; so[4] = c.y_offset; so[5] = c.z_offset;
  return (int64_t)c.points.size();
}

// saveResultAsLAS (icp_registration.cpp:698-815) with the given scale/offset.
void ref_save_las(const char* path, const double* xyz, int64_t n, const double scale[3], const double offset[3]) {
  PointCloud c;
  c.x_scale = scale[0]; c.y_scale = scale[1]; c.z_scale = scale[2];
  c.x_offset = offset[0]; c.y_offset = offset[1]; c.z_offset = offset[2];
  for (int64_t i = 0; i < n; i++) c.addPoint(Point3D(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]));
  std::streambuf* old = std::cout.rdbuf();
  std::ofstream devnull("/dev/null");
  std::cout.rdbuf(devnull.rdbuf());
  saveResultAsLAS(c, path);
  std::cout.rdbuf(old);
}

// saveTransformation (icp_registration.cpp:625-695).
void ref_save_transformation(const char* path, const double R9[9], const double t3[3], const double* T16, int n) {
  double R[3][3], t[3];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) R[i][j] = R9[3 * i + j];
    t[i] = t3[i];
  }
  std::vector<Eigen::Matrix4d> hist;
  for (int k = 0; k < n; k++) {
    Eigen::Matrix4d M;
    for (int r = 0; r < 4; r++)
      for (int c = 0; c < 4; c++) M(r, c) = T16[16 * k + 4 * r + c];
    hist.push_back(M);
  }
  std::streambuf* old = std::cout.rdbuf();
  std::ofstream devnull("/dev/null");
  std::cout.rdbuf(devnull.rdbuf());
  saveTransformation(R, t, path, n > 0 ? &hist : nullptr);
  std::cout.rdbuf(old);
}

}  // extern "C"
