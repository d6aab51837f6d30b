// svd3.h — host 3x3 two-sided Jacobi SVD (the algorithm of Eigen 3.3.4's JacobiSVD that the
// reference calls at icpengine.cpp:93 / icp_registration.cpp:418) and the rigid best fit built
// on it (icpengine.cpp:76-115, icp_registration.cpp:389-440). Eigen is not installed on the
// target systems, so the product carries this from-scratch implementation; it is pinned to
// Eigen outputs by tests/golden (tolerance 1e-13, see tests/test_host_svd.py).
#pragma once

#include "icp_common.h"

namespace icp {

// H = U * diag(S) * V^T, all row-major; singular values descending, U/V orthogonal.
void jacobi_svd3(const double H[9], double U[9], double S[3], double V[9]);

// Rigid transform (row-major 4x4) mapping the source centroid frame onto the target:
// R = V U^T (reflection fixed by negating V's third column), t = mb - R ma.
void best_fit_from_moments(const double ma[3], const double mb[3], const double C[9], double T[16]);

// 4x4 row-major product C = A * B with the reference's summation order.
void mat4_mul(const double A[16], const double B[16], double C[16]);

}  // namespace icp
