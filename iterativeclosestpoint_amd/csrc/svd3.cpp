// svd3.cpp — see svd3.h; the arithmetic lives in svd3_impl.h (shared with the device loop).
#include "svd3.h"

#include "svd3_impl.h"

namespace icp {

void jacobi_svd3(const double H[9], double U9[9], double S[3], double V9[9]) { svd::jacobi_svd3(H, U9, S, V9); }

void best_fit_from_moments(const double ma[3], const double mb[3], const double C[9], double T[16]) {
  svd::best_fit_from_moments(ma, mb, C, T);
}

void mat4_mul(const double A[16], const double B[16], double C[16]) { svd::mat4_mul(A, B, C); }

}  // namespace icp
