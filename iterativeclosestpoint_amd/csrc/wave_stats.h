// wave_stats.h — the covariance sums of one wave's queries (64 consecutive queries of the kd
// order), computed by the wave search itself (nn_kernels.hip, its epilogue) and, for the waves it
// could not settle alone, by the cull kernel (reduce_kernels.hip k_cull_waves). Both call the one
// function below, so a wave's sums have the same bits whoever computes them (and therefore
// whichever search path settled which of its queries).
//
// The 3-sigma threshold (icpengine.cpp:263-278) is not known while the search runs. The search
// sums the pairs below a band [lo, hi] around the previous iterate's threshold (the band is
// set at the end of every iterate, kernels.h IterDev::fz_*): every pair with d <= lo is valid
// when lo <= thr. Pairs inside the band (lo < d <= hi) are marked in the record and settled once
// the threshold is known; pairs above hi are invalid when thr <= hi. A threshold outside the
// band (the first iterates of a registration, a new source, another rule) makes the cull kernel
// recompute every wave against the threshold itself: the band only decides how much work the
// cull pass has left, never which pairs are valid.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"
#include "nn_device.h"

namespace icp {
namespace dev {

// doubles per lane row of the transposed reduction (9, not 8: the 8 lane groups' rows then fall
// on two bank windows instead of one)
constexpr int kStatStride = 9;
constexpr int kStatLds = 64 * kStatStride * 8;  // bytes of LDS per wave (4.5 KB)

// v ^ lane X within 32-lane groups (ds_swizzle bitmask mode: and 0x1f, xor X): LDS crossbar, no
// vector ALU issue
template <int X>
__device__ __forceinline__ double swz_xor_d(double v) {
  constexpr int kPat = 0x1f | (X << 10);
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)(unsigned)b, kPat);
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), kPat);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Sum over the wave of 8 values per lane, in a fixed order: every lane writes its row, lane
// 8 k + p adds value k of rows 8 p .. 8 p + 7 in row order, then the 8 partial sums of value k
// (lanes 8 k .. 8 k + 7) are added pairwise (p ^ 1, p ^ 2, p ^ 4; fp addition commutes, so every
// lane of the group ends with the same bits). Returns value (lane >> 3)'s sum.
__device__ __forceinline__ double wave_sum8(const double (&v)[8], double* lds, int lane) {
  double* row = lds + lane * kStatStride;
#pragma unroll
  for (int k = 0; k < 8; k++) row[k] = v[k];
  wave_lds_fence();
  const double* col = lds + (8 * (lane & 7)) * kStatStride + (lane >> 3);
  double acc = col[0];
#pragma unroll
  for (int j = 1; j < 8; j++) acc += col[j * kStatStride];
  acc += swz_xor_d<1>(acc);
  acc += swz_xor_d<2>(acc);
  acc += swz_xor_d<4>(acc);
  wave_lds_fence();  // every read of the rows is done before they are rewritten
  return acc;
}

// The canonical sums of the lanes with `in` (every lane of the wave calls it): 16 values,
//   0 sum d^2, 1..3 sum (a - s), 4..6 sum (b - t), 7..15 sum (a - s)_r (b - t)_c (r-major)
// (a = query, b = its match, (s, t) = the iterate's shift sh[0..5]; icpengine.cpp:76-90's H).
// Lane 8 k + p returns value k in r1 and value 8 + k in r2. Lanes without `in` add +0.0.
__device__ __forceinline__ void wave_cov_sums(bool in, double d, double qx, double qy, double qz, double mx,
                                              double my, double mz, const double* sh, double* lds, int lane,
                                              double& r1, double& r2) {
  const double da0 = in ? qx - sh[0] : 0.0, da1 = in ? qy - sh[1] : 0.0, da2 = in ? qz - sh[2] : 0.0;
  const double db0 = in ? mx - sh[3] : 0.0, db1 = in ? my - sh[4] : 0.0, db2 = in ? mz - sh[5] : 0.0;
  {
    const double v[8] = {in ? d * d : 0.0, da0, da1, da2, db0, db1, db2, da0 * db0};
    r1 = wave_sum8(v, lds, lane);
  }
  const double v[8] = {da0 * db1, da0 * db2, da1 * db0, da1 * db1, da1 * db2, da2 * db0, da2 * db1, da2 * db2};
  r2 = wave_sum8(v, lds, lane);
}

// One pair's terms added to a record's sums, in a fixed order (the cull kernel's band pairs).
__device__ __forceinline__ void add_pair(double* s, double& cnt, double d, double qx, double qy, double qz, double mx,
                                         double my, double mz, const double* sh) {
  const double da[3] = {qx - sh[0], qy - sh[1], qz - sh[2]};
  const double db[3] = {mx - sh[3], my - sh[4], mz - sh[5]};
  cnt += 1.0;
  s[0] += d * d;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    s[1 + r] += da[r];
    s[4 + r] += db[r];
  }
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) s[7 + 3 * r + c] += da[r] * db[c];
}

}  // namespace dev
}  // namespace icp
