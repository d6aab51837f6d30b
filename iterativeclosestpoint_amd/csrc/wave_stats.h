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

constexpr int kStatLds = 64 * 4 * 8;  // bytes of LDS per wave (2 KB)

// gfx950 v_permlane32_swap / v_permlane16_swap on a double: (x, y) -> (x', y') with
//   32: x' = [x lanes 0-31, y lanes 0-31], y' = [x lanes 32-63, y lanes 32-63]
//   16: x' = rows [x0, y0, x2, y2], y' = rows [x1, y1, x3, y3] (rows of 16 lanes)
// Vector ALU instructions, one per dword: no LDS traffic.
template <bool W32>
__device__ __forceinline__ void swap_d(double& x, double& y) {
  const long long bx = __double_as_longlong(x), by = __double_as_longlong(y);
  const unsigned xl = (unsigned)bx, xh = (unsigned)(bx >> 32), yl = (unsigned)by, yh = (unsigned)(by >> 32);
  unsigned nxl, nyl, nxh, nyh;
  if (W32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    nxl = lo[0], nyl = lo[1], nxh = hi[0], nyh = hi[1];
  } else {
    const auto lo = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
    nxl = lo[0], nyl = lo[1], nxh = hi[0], nyh = hi[1];
  }
  x = __longlong_as_double((long long)(((unsigned long long)nxh << 32) | nxl));
  y = __longlong_as_double((long long)(((unsigned long long)nyh << 32) | nyl));
}

// Sum over the wave of 16 values per lane, in a fixed order; returns value (lane & 15)'s sum (the
// four lanes holding a value hold the same bits). Reduce-scatter: value k and k + 8 swap halves
// (lanes l, l + 32 added), then k and k + 4 swap rows (l, l + 16 added): row r of lanes then holds
// values 4r .. 4r + 3, each summed over 4 lanes; the 16 partial sums of a value go through LDS
// (2 KB per wave; lane l adds partials 4 (l >> 4) .. +3 of value l & 15 in order), and the four
// quarters are added by a half swap and a row swap (commutative adds: equal bits everywhere).
__device__ __forceinline__ double wave_sum16(double (&c)[16], double* lds, int lane) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    swap_d<true>(c[k], c[k + 8]);
    c[k] = c[k] + c[k + 8];
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    swap_d<false>(c[k], c[k + 4]);
    c[k] = c[k] + c[k + 4];
  }
  // value-major blocks of 64, lane l's entry of register j at l ^ (4 j + (l >> 4)): the writes of
  // a register are one contiguous 512 B, and the 64 reads of one step fall on 16 different 8-B
  // bank pairs (4 lanes each, the minimum for 512 B) instead of 4
#pragma unroll
  for (int j = 0; j < 4; j++) lds[64 * j + (lane ^ (4 * j + (lane >> 4)))] = c[j];
  wave_lds_fence();
  const int v = lane & 15, q = lane >> 4, vr = v >> 2, vj = v & 3, key = 4 * vj + vr;
  const double* blk = lds + 64 * vj;
  const int s0 = 16 * vr + 4 * q;
  double g = blk[s0 ^ key];
#pragma unroll
  for (int i = 1; i < 4; i++) g += blk[(s0 + i) ^ key];
  wave_lds_fence();  // every read is done before the area is rewritten
  double h = g;
  swap_d<true>(g, h);
  g = g + h;
  h = g;
  swap_d<false>(g, h);
  return g + h;
}

// The canonical sums of the lanes with `in` (every lane of the wave calls it): 16 values,
//   0 sum d^2, 1..3 sum (a - s), 4..6 sum (b - t), 7..15 sum (a - s)_r (b - t)_c (r-major)
// (a = query, b = its match, (s, t) = the iterate's shift sh[0..5]; icpengine.cpp:76-90's H).
// Returns value (lane & 15). Lanes without `in` add +0.0.
__device__ __forceinline__ double wave_cov_sums(bool in, double d, double qx, double qy, double qz, double mx,
                                                double my, double mz, const double* sh, double* lds, int lane) {
  double da0 = qx - sh[0], da1 = qy - sh[1], da2 = qz - sh[2];
  double db0 = mx - sh[3], db1 = my - sh[4], db2 = mz - sh[5];
  double dd = d * d;
  if (wballot(in) != ~0ull) {  // some lane does not count: zero its terms (most waves skip this)
    da0 = in ? da0 : 0.0, da1 = in ? da1 : 0.0, da2 = in ? da2 : 0.0;
    db0 = in ? db0 : 0.0, db1 = in ? db1 : 0.0, db2 = in ? db2 : 0.0;
    dd = in ? dd : 0.0;
  }
  double c[16] = {dd, da0, da1, da2, db0, db1, db2, da0 * db0,
                  da0 * db1, da0 * db2, da1 * db0, da1 * db1, da1 * db2, da2 * db0, da2 * db1, da2 * db2};
  return wave_sum16(c, lds, lane);
}

}  // namespace dev
}  // namespace icp
