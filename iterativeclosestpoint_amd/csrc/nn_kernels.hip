// nn_kernels.hip — gfx950 octree nearest-neighbour search of the ICP correspondence step.
//
// Replaces the reference's per-source-point loop over Octree::findNearest
// (core/icpengine.cpp:169-184 -> octree.cpp:128-184; CLI icp_registration.cpp:481-496).
// Every kernel returns, for each query, exactly the index and residual the reference DFS returns.
//
//  k_nn_ref    one thread per query, the literal reference-order DFS (the parity kernel, and the
//              work counter of the roofline's "reference work" figure).
//  k_nn_wave   the product search: 64 spatially coherent queries per wave share one search box,
//              one cooperative walk of the octree, one lockstep fp32 filter scan, and a rigorous
//              per-query certificate (nn_device.h) that the reference returns the same point.
//  k_nn_ball   the queries a wave did not take, four per wave (16-lane groups), sphere walks; what
//              those cannot decide, and the wave search's exact list: per-lane certified search,
//              else the reference-order DFS.
//
// Everything is fp64 except the scan's filter, whose result is re-evaluated in fp64; built with
// -ffp-contract=off (the reference is built without FMA).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <type_traits>

#include "kernels.h"
#include "nn_device.h"
#include "wave_stats.h"

// Diagnostic build only (-DICP_PHASE_CLOCKS=1): per-phase s_memtime deltas of the wave search
// summed into the debug slots 16..21 (the product build has no clock reads).
#ifndef ICP_PHASE_CLOCKS
#define ICP_PHASE_CLOCKS 0
#endif
constexpr bool kDbgCounts = !ICP_PHASE_CLOCKS;  // the clock build counts nothing (no atomics)
#if ICP_PHASE_CLOCKS
#define PCLK(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define PCLK(v)
#endif
// Diagnostic build only (-DICP_PHASE_STOP=1): the wave search returns after the phase set by
// icp_hip_debug_phase_stop (1: the first round trip, 2: the guess, 3: the box, 4: the walk, 5: the
// scan and the winner's fp64 distance, 6: certify, write and queue; 0: none), so SQ counters of one
// launch per setting give the instructions of each phase (tools/phase_insts.py). The results of
// such a launch are not the search's: it is for counting only.
#ifndef ICP_PHASE_STOP
#define ICP_PHASE_STOP 0
#endif
#if ICP_PHASE_STOP
namespace icp {
__device__ int g_phase_stop;
}
#define PSTOP(k) \
  if (__builtin_amdgcn_readfirstlane(icp::g_phase_stop) == (k)) return
#else
#define PSTOP(k)
#endif
namespace icp {

namespace {

using namespace dev;

// ---------------------------------------------------------------------------------------------
// The reference-order kernel.
template <bool APPLY, bool COUNT>
__global__ void __launch_bounds__(256) k_nn_ref(NNLaunch a) {
  if (a.loop && a.loop->core.done) return;  // the device loop's session finished
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_stack[];
  const int bs = blockDim.x;
  const int64_t i = (int64_t)blockIdx.x * bs + threadIdx.x;
  const bool active = i < a.n;

  double qx = 0.0, qy = 0.0, qz = 0.0;
  load_query<APPLY>(a, i, active, qx, qy, qz);

  double best_d2 = a.init_best;
  int32_t best = -1;
  double visits = 0.0, scanned = 0.0;
  // A NaN coordinate makes every leaf distance NaN, so the reference never updates best_idx
  // (octree.cpp:146): skipping the search is exact. (Its box distances stay finite: max(0,NaN)=0.)
  const bool nan_q = (qx != qx) || (qy != qy) || (qz != qz);
  if (active && !nan_q && a.n_nodes > 0)
    exact_dfs<COUNT>(a, qx, qy, qz, lds_stack + threadIdx.x, bs, best, best_d2, visits, scanned);
  if (active) {
    const int32_t pos = best >= 0 ? best : a.pos0;
    a.pos_out[i] = pos;
    a.dist_out[i] = best >= 0 ? __builtin_sqrt(best_d2)  // == computeDistance bit for bit
                              : residual_to(a.pts, a.pos0, qx, qy, qz);
  }
  if (COUNT) {
    __syncthreads();  // every traversal is done: reuse the stack LDS for the reduction
    double c[2] = {visits, scanned};
    block_sum<2>(c, reinterpret_cast<double*>(lds_stack));
    if (threadIdx.x == 0) {
      atomicAdd(&a.counters[0], (unsigned long long)c[0]);
      atomicAdd(&a.counters[1], (unsigned long long)c[1]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// The wave search.
//
// The 64 queries of a wave are one kd bucket of the source: spatially compact.
//  1. Guess u >= each query's nearest squared distance: after an iteration on the same queries,
//     (previous residual + displacement)^2 (triangle inequality); otherwise one nearest-child
//     descent to a leaf and its smallest d2.
//  2. Lanes with radius r = sqrt(u)(1 + 2^-40) + |q| 2^-45 <= join x the wave's mean radius
//     join one search box B = the bbox of their balls (DPP reductions).
//  3. The leaves meeting B are collected by a cooperative walk (LIFO stack in LDS, up to 64 nodes
//     per batch), started from the cell tables (or a wave-uniform descent without them).
//  4. The points of those leaves that lie in B are staged 64 at a time as fp32 offsets from B's
//     centre, in pairs, and every joined lane scans them in lockstep (packed fp32), keeping its
//     two smallest values and the position of the smallest.
//  5. The winner's fp64 distance is recomputed with the reference arithmetic; every other point's
//     fl(d2) is bounded below from the second-smallest fp32 value (scan32_lower_bound). A wave
//     with a lane this cannot certify re-scans in fp64.
// Each joined lane's ball lies in B, so every point within best (1 + 2^-48) of it was scanned:
// the certificate of nn_device.h applies. Non-joined lanes go to the ball list, uncertified ones
// to the exact list.
constexpr int kOpenToBall = 4;   // certify_prev 3: open queries a wave hands to the ball search
constexpr int kMaxTableLevels = 9;  // cell tables are built for levels 0..9 at most (octree_gpu.hip)
#ifndef ICP_TABLE_DESCENT
#define ICP_TABLE_DESCENT 1  // a source's first-iterate descent starts from the cell tables
#endif
constexpr int kWaveQueue = 256;  // node ids of the walk's LIFO stack (staging area after the walk)
constexpr int kWaveStartK = 2;   // start cells per lane (up to 128 start nodes per wave)
constexpr int kWavePoints = 1024;  // candidate list area (up to kWaveCandCap ids)
static_assert(kWaveCandCap <= kWavePoints, "candidate list");
constexpr int kWaveLds = kWaveQueue * 4 + kWavePoints * 4;  // 5 KB per wave
constexpr int kWideQueue = 512;  // the wide pass's node stack (after its staging area)
#ifndef ICP_WIDE_SEGS
#define ICP_WIDE_SEGS 2
#endif
#ifndef ICP_WIDE_SEGS0
#define ICP_WIDE_SEGS0 6
#endif
// segments a wide walk scans before it gives up: after a search (the bounds are the previous
// matches' distances, tight), and in a source's first iterate (descent guesses, which the first
// segments tighten)
constexpr int kWideSegs = ICP_WIDE_SEGS, kWideSegs0 = ICP_WIDE_SEGS0;
static_assert(kWaveQueue * 4 >= 64 * 16 && kWaveQueue * 4 >= 32 * 32, "staging area aliases the stack");
static_assert(kWaveQueue * 4 + kWavePoints * 4 >= 128 * 16, "a reusing wave stages 128 points (stack + list area)");

// fp32 radius r >= sqrt(u) (1 + 2^-40) + amax 2^-45 (the ball of the wave search's certificate):
// the fp32 square root rounded up ((float) rounds by <= 2^-24, v_sqrt_f32 is within 1 ulp, each
// fp32 product by <= 2^-24), the amax term doubled, 2^-49 absolute for u
// below the fp32 normal range (a flushed denormal input gives 0), and the sum's rounding covered
// by the 2^-21 factors. The bare v_sqrt_f32 (__builtin_amdgcn_sqrtf), not the correctly rounded
// sequence __builtin_sqrtf compiles to (~13 more instructions per wave).
__device__ __forceinline__ float ball_radius32(double u, double amax) {
  const float s = __builtin_amdgcn_sqrtf((float)u * (1.0f + 0x1p-21f)) * (1.0f + 0x1p-21f);
  return s + ((float)(amax * 0x1p-44) + 0x1p-49f);
}

// fp64 box bound o + f rounded down / up (the addition rounds by <= 2^-53 of the result).
__device__ __forceinline__ double box_lo(double o, float f) {
  const double b = o + (double)f;
  return b - (__builtin_fabs(b) * 0x1p-52 + 0x1p-1000);
}
__device__ __forceinline__ double box_hi(double o, float f) {
  const double b = o + (double)f;
  return b + (__builtin_fabs(b) * 0x1p-52 + 0x1p-1000);
}

// Lower bound of fl64(d2) of every point whose fp32 squared distance (the scan) is >= s32.
// Coordinates are offsets from B's centre, |offset| <= ext for points and joined queries. With
// u = 2^-24: each fp32 offset differs from the exact one by <= ext (u + 2^-53) =: ext k; the fp32
// difference dx' = (p' - q')(1 + e), |e| <= u, so |dx' - dx| <= 2 ext k + u |dx| + ..., and over
// three axes |‖d'‖ - D| <= e_abs + u D with e_abs = sqrt(3) 2 ext k (1 + u). The fp32 sum of
// squares (one mul, two fma) is ‖d'‖^2 (1 + t), |t| <= (1 + u)^3 - 1, plus <= 3 2^-126 of
// underflow. Hence D >= (sqrt((s32 - 2^-120) / (1 + 3.0001 u)) - e_abs) / (1 + u), and
// fl64(d2) >= D^2 (1 - 5 2^-53). Every step rounds towards the bound by an explicit 2^-50 margin.
__device__ __forceinline__ double scan32_lower_bound(float s32, double ext) {
  if (!(s32 < __builtin_inff())) return __builtin_inf();
  const double u = 0x1p-24;
  const double e_abs = 1.7320509 * 2.0 * ext * (u * (1.0 + 0x1p-20)) * (1.0 + u) * (1.0 + 0x1p-40);
  // x / (1 + a) >= x (1 - a) for x >= 0: products instead of divisions
  const double n2 = ((double)s32 - 0x1p-120) * (1.0 - 3.0001 * u);
  if (!(n2 > 0.0)) return 0.0;
  // sqrt(n2) from below: (float) rounds by <= 2^-24 (scaled down first), v_sqrt_f32 is within
  // 1 ulp, the fp64 factor covers both (a flushed denormal gives 0, still a lower bound)
  const double n = (double)__builtin_amdgcn_sqrtf((float)(n2 * (1.0 - 0x1p-22))) * (1.0 - 0x1p-21);
  const double d = (n - e_abs) * (1.0 - u) * (1.0 - 0x1p-50);
  if (!(d > 0.0)) return 0.0;
  return d * d * (1.0 - 0x1p-48);
}

// The certificate of the previous match p* (fl(d2) = u from the moved query, p*'s separation S):
// every other point p has D(q', p) >= S - D* with D* <= sqrt(u) (1 + 2^-50), and
// fl(d2(q', p)) >= D^2 (1 - 5 2^-53); so the window test of nn_device.h's certificate applies
// with the lower bound (S - D*)^2 (1 - 2^-50) (its rounding covered by the 2^-52 / 2^-50 factors).
__device__ __forceinline__ bool prev_certified(double u, float sep, double init_best) {
  const double dstar = __builtin_sqrt(u) * (1.0 + 0x1p-50);
  const double g = ((double)sep - dstar) * (1.0 - 0x1p-52);
  if (!(g > 0.0)) return false;
  return certified(u, g * g * (1.0 - 0x1p-50), init_best);
}

// A candidate point for the scans: x, y, z and its id (-1: a copy of an earlier point, whose twin
// is the reference's answer whenever it would be; TgtPt::sep's sign, k_mark_copies). One 16-B load
// of (x, y) and one of (z, orig | sep): the flag rides with z.
__device__ __forceinline__ double4 load_cand(const TgtPt* pts, int32_t g) {
  const TgtPt* p = pts + g;
  const double2 xy = *reinterpret_cast<const double2*>(&p->x);
  const double2 zw = *reinterpret_cast<const double2*>(&p->z);
  return make_double4(xy.x, xy.y, zw.x, __longlong_as_double(tgt_copy_word(zw.y) ? -1ll : (long long)g));
}

// Workgroups are dispatched round-robin over the 8 XCDs (block b runs on XCD b % 8), each with
// its own 4 MB L2. Renumbered, XCD x takes runs of C consecutive logical blocks (C = chunk), the
// runs dealt round-robin over the XCDs: the waves an XCD runs at a time are neighbours in the kd
// order (their candidate points and nodes shared in its L2), and the XCDs still share the cloud
// evenly. Blocks past the last whole round of 8 C keep their number.
__device__ __forceinline__ unsigned xcd_block(unsigned chunk) {
  const unsigned b = blockIdx.x, nb = gridDim.x;
  if (chunk == 0) return b;
  const unsigned round = 8u * chunk, full = nb / round * round;
  if (b >= full) return b;
  const unsigned x = b & 7u, k = b >> 3;
  return ((k / chunk) * 8u + x) * chunk + k % chunk;
}

// The wave's covariance record (wave_stats.h), once the wave has settled its queries: the
// canonical sums of its pairs below the band, its band lanes, or flag = 1 when some of its queries
// are left to the other searches (the cull kernel then recomputes the whole wave, so the sums are
// the same whichever path settled which query). Every lane calls it (wave-uniform exits).
template <bool DBG>
__device__ __forceinline__ void wave_record(const NNLaunch& a, uint32_t wid, int lane, bool active, bool settled,
                                            double d, int32_t pos, double qx, double qy, double qz,
                                            unsigned char* wl) {
  if (a.wstat == nullptr || !(a.fz->fz_ok != 0.0)) return;
  WaveStat* rec = a.wstat + wid;
  if (wballot(active && !settled) != 0) {
    if (lane == 0) {
      rec->flag = 1ull;
      if (DBG && kDbgCounts && a.dbg) atomicAdd(&a.dbg[30], 1ull);
    }
    return;
  }
  const double lo = a.fz->fz_lo, hi = a.fz->fz_hi;
  const bool in = active && d <= lo;
  const bool band = active && !(d <= lo) && d <= hi;
  double mx = 0.0, my = 0.0, mz = 0.0;
  if (in) {
    const TgtPt* p = a.pts + pos;
    const double2 xy = *reinterpret_cast<const double2*>(&p->x);
    mx = xy.x;
    my = xy.y;
    mz = p->z;
  }
  double sh[6];
#pragma unroll
  for (int k = 0; k < 6; k++) sh[k] = a.fz->fz_sh[k];
  wave_lds_fence();  // the scan's reads of the staging area are done
  const double r = wave_cov_sums(in, d, qx, qy, qz, mx, my, mz, sh, reinterpret_cast<double*>(wl), lane);
  const unsigned long long am = wballot(in), bm = wballot(band);
  if (lane < 16) rec->s[lane] = r;
  if (lane == 0) {
    rec->cnt = (double)__popcll(am);
    rec->bm = bm;
    rec->flag = 0ull;
    if (DBG && kDbgCounts && a.dbg) atomicAdd(&a.dbg[31], (unsigned long long)__popcll(bm));
  }
}
static_assert(kStatLds <= kWaveLds, "the record's reduction fits the wave's LDS area");

// The search of one wave's queries (query i per lane; i >= n: an idle lane). HALF: the second
// pass over the 32-query halves of the waves whose box overflowed (k_nn_half: queries already
// moved, no candidate cache; lanes 32..63 idle).
// DBG: the instance of a context with debug counters (ICP_DBG_* slots); the product instances
// carry none of their code.
#ifndef ICP_GUESS_LANES
#define ICP_GUESS_LANES 64  // lanes sharing their first-iterate guess points (16, 32, 64)
#endif
// CM, the candidate-cache instance: 1 (WC) an iterate with the cache and previous residuals (every
// wave that joins either reuses its record or walks and stores one): a walking wave stores its
// entries before the scan and then streams them back as a reusing wave does, so the instance
// carries one scan path (ICP_WALK_STREAM); 2 (NC) a first iterate without a transform (no record
// is reused or stored: the instance carries no cache code); 0 either.
template <bool APPLY, int NG, bool CERT, bool HALF, bool DBG, int CM = 0, bool WIDE = false>
__device__ __forceinline__ void wave_search(const NNLaunch& a, const int32_t i, const int lane, unsigned char* wl) {
  // previous residuals: known to the WC (yes) and NC (no) instances
  const bool have_prev = CM == 1 ? true : CM == 2 ? false : a.have_prev != 0;
  constexpr bool kDbg = DBG && kDbgCounts;
  // a second pass (the half pass, the wide pass): queries already moved, no cache, no wave record
  constexpr bool kSecond = HALF || WIDE;
  static_assert(NG == 1 || NG == 2 || NG == 4, "scan groups: 1, 2 or 4");
  static_assert(!(kSecond && (APPLY || CERT)), "the second passes search moved queries");
  static_assert(!(HALF && WIDE), "one second pass per instance");
  const bool active = i < a.n;
  int32_t* queue = reinterpret_cast<int32_t*>(wl);
  double4* stage = reinterpret_cast<double4*>(wl);  // after the walk only
  int32_t* plist = queue + kWaveQueue;               // candidate points

  // The first round trip: the query, its previous match (leaf order), the wave's cache record (8
  // words on lanes 0..7) and its first 64 entries, all issued before any of them is used (a
  // reusing wave has its first chunk before the box is known; unused otherwise).
  const int32_t i0 = __builtin_amdgcn_readfirstlane(i);
  const uint32_t wid = (uint32_t)i0 >> 6;
  const bool use_wc = !kSecond && CM != 2 && a.wc_box != nullptr && i0 < a.n;
  // the previous match, whose fl(d2) is u (read unconditionally: an unused load costs no wait,
  // while a conditional one is waited for inside its branch)
  const int32_t prev_pos = qat(a.pos_out, active ? i : 0);
  double hdr = 0.0;
  float4 ent0 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (use_wc) {
    if (lane < 8) hdr = reinterpret_cast<const double*>(a.wc_box + wid)[lane];
    ent0 = a.wc_ents[(size_t)wid * kWaveCandCap + lane];
  }
  double qx = 0.0, qy = 0.0, qz = 0.0;
  load_query32<APPLY>(a, i, active, qx, qy, qz);
  // every load of the first round trip has landed (a real s_waitcnt, which the compiler's wait
  // bookkeeping sees, on every path: otherwise it waits again inside each branch below)
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  const bool finite_q = __builtin_isfinite(qx) && __builtin_isfinite(qy) && __builtin_isfinite(qz);

  PCLK(t_p0);
  PSTOP(1);
  // Phase 1: the guess (any value is safe: certification also requires best <= u).
  double u = __builtin_inf();
  int32_t gpos = -1;  // (first iterate) the target point whose distance is u
  bool safe = false;  // the previous match certified from its separation: no search
  if (active && finite_q && have_prev) {
    // the previous match is a candidate: its fl(d2) from the moved query bounds the nearest
    // point's (usually well below (previous residual + displacement)^2)
    const TgtPt* pp = a.pts + prev_pos;
    const double2 pxy = *reinterpret_cast<const double2*>(&pp->x);
    const double dx = pxy.x - qx, dy = pxy.y - qy, dz = pp->z - qz;
    u = dx * dx + dy * dy + dz * dz;
    if (CERT) safe = prev_certified(u, pp->sep, a.init_best);
  } else if (active && finite_q) {
    int32_t node = 0;
    if (ICP_TABLE_DESCENT && a.cells && a.cell_lmax > 0) {
      // The descent's first levels from the cell tables: the query's cell path at the deepest
      // table level (the octree's own midpoint comparisons), then the deepest level whose cell
      // holds points (every level's entry read at once). Any start gives a valid guess; this one
      // is the node the descent from the root would pass through when the query's cells exist.
      const int L = a.cell_lmax;
      const uint32_t px = axis_path(qx, a.root_lo[0], a.root_hi[0], L);
      const uint32_t py = axis_path(qy, a.root_lo[1], a.root_hi[1], L);
      const uint32_t pz = axis_path(qz, a.root_lo[2], a.root_hi[2], L);
      const uint32_t key = spread3(px) | (spread3(py) << 1) | (spread3(pz) << 2);
      int32_t e[kMaxTableLevels];
#pragma unroll
      for (int l = 1; l <= kMaxTableLevels; l++)
        e[l - 1] = l <= L ? a.cells[((((int64_t)1 << (3 * l)) - 1) / 7) + (key >> (3 * (L - l)))] : -1;
#pragma unroll
      for (int l = 1; l <= kMaxTableLevels; l++) node = e[l - 1] >= 0 ? (e[l - 1] >> 5) : node;
    }
    const NodeRec* r0 = a.nodes + node;
    double lx = r0->lo[0], ly = r0->lo[1], lz = r0->lo[2], hx = r0->hi[0], hy = r0->hi[1], hz = r0->hi[2];
    int32_t pfirst = -1;  // the current node's parent: its first child record, child mask, the
    uint32_t pmask = 0, po = 0;  // octant taken and its children's squared axis distances
    double psx[2] = {0.0, 0.0}, psy[2] = {0.0, 0.0}, psz[2] = {0.0, 0.0};
    auto scan_leaf = [&](int2 topo) {
      const int32_t cnt = (int32_t)((uint32_t)topo.y & ~kLeafBit);
      for (int32_t k = 0; k < cnt; k++) {
        const TgtPt* p = a.pts + topo.x + k;
        const double dx = p->x - qx, dy = p->y - qy, dz = p->z - qz;
        const double d2 = dx * dx + dy * dy + dz * dz;
        const bool t = d2 < u;
        u = t ? d2 : u;
        if (!APPLY) gpos = t ? topo.x + k : gpos;
      }
    };
    while (true) {
      const int2 topo = *reinterpret_cast<const int2*>(&a.nodes[node].first);
      const uint32_t meta = (uint32_t)topo.y;
      if (meta & kLeafBit) {
        scan_leaf(topo);
        // (in the instances without a transform: a session's first iterate; the steady-state
        // instances keep their registers for the scan)
        if (!APPLY && pfirst >= 0) {
          // then the points of the parent's other leaf children whose box is nearer than the
          // best so far (~3 points per leaf: the reached leaf alone bounds the nearest distance
          // loosely, and the first iterate's boxes, overflows and ball searches grow with it)
#pragma unroll
          for (int o = 0; o < 8; o++) {
            const double c = psx[o & 1] + psy[(o >> 1) & 1] + psz[o >> 2];
            if (((pmask >> o) & 1u) && (uint32_t)o != po && c < u) {
              const int2 t =
                  *reinterpret_cast<const int2*>(&a.nodes[pfirst + __builtin_popcount(pmask & ((1u << o) - 1u))].first);
              if ((uint32_t)t.y & kLeafBit) scan_leaf(t);
            }
          }
        }
        break;
      }
      const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
      const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
      const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
      const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
      const double sx[2] = {ax0 * ax0, ax1 * ax1};
      const double sy[2] = {ay0 * ay0, ay1 * ay1};
      const double sz[2] = {az0 * az0, az1 * az1};
      const uint32_t mask = meta & 0xffu;
      double bs_ = __builtin_inf();
      uint32_t o1 = 0;
#pragma unroll
      for (int o = 0; o < 8; o++) {
        const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
        const bool take = ((mask >> o) & 1u) && c < bs_;
        bs_ = take ? c : bs_;
        o1 = take ? (uint32_t)o : o1;
      }
      node = topo.x + __builtin_popcount(mask & ((1u << o1) - 1u));
      pfirst = topo.x;
      pmask = mask;
      po = o1;
#pragma unroll
      for (int k = 0; k < 2; k++) {
        psx[k] = sx[k];
        psy[k] = sy[k];
        psz[k] = sz[k];
      }
      if (o1 & 1u) lx = mx; else hx = mx;
      if (o1 & 2u) ly = my; else hy = my;
      if (o1 & 4u) lz = mz; else hz = mz;
    }
  }

  // Phase 1a (first iterate): the 64 lanes hold one kd bucket of queries, near each other: every
  // lane also tries the other lanes' guess points (fp32 offsets from a wave-uniform query; the
  // nearest one's exact fl(d2) becomes u when smaller). A lane whose own leaf guessed poorly (a
  // query near its leaf's boundary) gets its neighbours' points: smaller boxes, fewer overflows
  // and follow-up searches in the iterate with the loosest guesses. Measured at 10M (one MI355X,
  // profiles/r21/ab_first_iterate_guess.txt): lanes not joining their wave's box 14651 -> 1214,
  // overflowing waves 3546 -> 1075, first iterate 2.78 -> 2.52 ms (16 lanes: 2.61, 32: 2.58).
  if (!APPLY && !have_prev) {
    constexpr int kGL = ICP_GUESS_LANES;
    const double rx = __shfl(qx, lane & (64 - kGL), kWave), ry = __shfl(qy, lane & (64 - kGL), kWave),
                 rz = __shfl(qz, lane & (64 - kGL), kWave);
    float gx = 3.0e38f, gy = 3.0e38f, gz = 3.0e38f;
    if (gpos >= 0) {
      const TgtPt* p = a.pts + gpos;
      gx = (float)(p->x - rx);
      gy = (float)(p->y - ry);
      gz = (float)(p->z - rz);
    }
    const float fx = (float)(qx - rx), fy = (float)(qy - ry), fz = (float)(qz - rz);
    float bd = 3.0e38f;
    int bm = 0;
#pragma unroll
    for (int m = 1; m < kGL; m++) {
      const float ox = __shfl_xor(gx, m, kWave) - fx, oy = __shfl_xor(gy, m, kWave) - fy,
                  oz = __shfl_xor(gz, m, kWave) - fz;
      const float d = __builtin_fmaf(oz, oz, __builtin_fmaf(oy, oy, ox * ox));
      bm = d < bd ? m : bm;
      bd = d < bd ? d : bd;
    }
    const int32_t op = __shfl(gpos, lane ^ bm, kWave);
    if (active && finite_q && bm != 0 && op >= 0) {
      const TgtPt* p = a.pts + op;
      const double dx = p->x - qx, dy = p->y - qy, dz = p->z - qz;
      const double d2 = dx * dx + dy * dy + dz * dz;
      u = d2 < u ? d2 : u;
    }
  }

  // Phase 1b (icp_hip_config.certify_prev): lanes whose previous match is certified are settled
  // (their match position stays; the residual is sqrt(u), computeDistance bit for bit).
  //   1: a wave whose active lanes are all certified ends here; other waves search every lane
  //   2: certified lanes settle, the others search (join) as usual
  //   3: certified lanes settle; a wave left with at most kOpenToBall open queries sends them to
  //      the ball search (with u as their guess) and ends here, otherwise it searches them (2)
  if (CERT && have_prev) {
    const unsigned long long open = wballot(active && !safe);
    if (kDbg && a.dbg) {
      const unsigned long long settled = wballot(safe);  // every lane takes part in the ballot
      if (lane == 0) {
        atomicAdd(&a.dbg[19], (unsigned long long)__popcll(settled));
        if (open == 0) atomicAdd(&a.dbg[18], 1ull);
      }
    }
    if (open == 0 || (a.certify_prev == 3 && __popcll(open) <= kOpenToBall)) {
      store_query32<APPLY>(a, i, active, qx, qy, qz);
      double d = 0.0;
      int32_t pos = prev_pos;
      if (safe) {
        d = __builtin_sqrt(u);
        qat(a.dist_out, i) = d;
      }
      if (open != 0) {
        if (active && !finite_q) {
          pos = a.pos0;
          d = residual_to(a.pts, a.pos0, qx, qy, qz);
          qat(a.pos_out, i) = pos;
          qat(a.dist_out, i) = d;
        }
        wave_append_u(active && finite_q && !safe, i, u, a.fb_count + 1, a.fb_list2, a.fb_u2);
      }
      if (!kSecond) wave_record<DBG>(a, wid, lane, active, safe || !finite_q, d, pos, qx, qy, qz, wl);
      return;
    }
    if (a.certify_prev == 1) safe = false;  // the whole wave searches
  }

  PCLK(t_p1);
  PSTOP(2);
  // Phase 2: the wave's search box over the lanes that join. Every point with fl(d2) <= u (1 +
  // 2^-47) lies within r of the query, r >= sqrt(u) (1 + 2^-40) + |q|_max 2^-45 (ball_radius32).
  const double amax = __builtin_fmax(__builtin_fabs(qx), __builtin_fmax(__builtin_fabs(qy), __builtin_fabs(qz)));
  // |q| <= 2^100 keeps every fp32 offset of the wave finite
  const bool cand = active && finite_q && !safe && u <= 0x1p900 && amax <= 0x1p100;
  float r = cand ? ball_radius32(u, amax) : 0.f;  // (the wide pass shrinks it as its bounds tighten)
  const unsigned long long cmask = wballot(cand);
  // the join rule is a heuristic (any subset may join): fp32 mean
  const float mean_r = wave_sum_f(r) * __builtin_amdgcn_rcpf((float)(cmask ? __popcll(cmask) : 1));
  bool join = cand && r <= (float)a.join_factor * mean_r;
  const unsigned long long jm = wballot(join);

  // The frame of the box reductions: fp32 offsets from an origin o. A wave whose cache record is of
  // this generation takes o = the centre of its stored B+, the frame its entries were stored in: a
  // reusing wave then gets its search box (for the reuse test), its scan groups' boxes and its
  // queries' scan offsets out of one reduction, in the frame it scans in, with no fp64 box and no
  // conversion of the group boxes (which cost ~290 VALU instructions per wave, most of them on
  // wave-uniform values). Any other wave takes o = its first joined query and, once its frame is
  // known (after its walk), reduces again in that frame.
  const bool have_rec =
      use_wc && jm != 0 &&
      (uint32_t)__builtin_amdgcn_readlane((int)((unsigned long long)__double_as_longlong(hdr) >> 32), 6) == a.wc_gen;
  double ox_ = 0.0, oy_ = 0.0, oz_ = 0.0;
  int pkl[3] = {0, 0, 0}, pkh[3] = {0, 0, 0};  // B+ - o rounded inwards (fp32 keys; have_rec)
  float pext = 0.f;                            // max |B+ - o| (1 + 2^-22) >= that of every point in B+
  if (have_rec) {
    // lanes 0..5 hold B+'s bounds (lo x, y, z, hi x, y, z): lanes j and j + 3 form axis j's centre,
    // the same operation as the store's (lo + hi) * 0.5 (the sum commutes exactly)
    const double part = __shfl(hdr, lane < 3 ? lane + 3 : (lane < 6 ? lane - 3 : lane), kWave);
    const double c = (hdr + part) * 0.5;
    ox_ = readlane_d(c, 0);
    oy_ = readlane_d(c, 1);
    oz_ = readlane_d(c, 2);
    // the bounds relative to o, in fp32 rounded inwards (the conversion rounds by <= 2^-24
    // relative, the fma moves the bound inwards by |f| 2^-22): containment in them is containment
    // in B+
    const float f = (float)(hdr - c);
    const int key = fkey(__builtin_fmaf(__builtin_fabsf(f), lane < 3 ? 0x1p-22f : -0x1p-22f, f));
#pragma unroll
    for (int k = 0; k < 3; k++) {
      pkl[k] = __builtin_amdgcn_readlane(key, k);
      pkh[k] = __builtin_amdgcn_readlane(key, k + 3);
    }
    // max over lanes 0..5 of |f| (row_shr 1, 2, 4: lane 5 sees lanes 0..5)
    int e = lane < 6 ? __float_as_int(__builtin_fabsf(f)) : 0;
    e = max(e, __builtin_amdgcn_update_dpp(0, e, 0x111, 0xf, 0xf, false));
    e = max(e, __builtin_amdgcn_update_dpp(0, e, 0x112, 0xf, 0xf, false));
    e = max(e, __builtin_amdgcn_update_dpp(0, e, 0x114, 0xf, 0xf, false));
    pext = __int_as_float(__builtin_amdgcn_readlane(e, 5)) * (1.0f + 0x1p-21f);
  } else if (jm != 0) {
    const int ol = __builtin_ctzll(jm);
    ox_ = readlane_d(qx, ol);
    oy_ = readlane_d(qy, ol);
    oz_ = readlane_d(qz, ol);
  }
  // The reductions: per axis, the joined balls' bounds in fp32 offsets from o, rounded outwards
  // (m covers the conversion of q - o and the roundings of the two sums), reduced with integer
  // DPP min/max on order-preserving keys: the scan groups' boxes (NG kd sub-buckets of 64 / NG
  // lanes) at their rows' / halves' last lanes, the wave's box (B) as scalar keys.
  int gkl[3], gkh[3];  // group-level keys: lane 16 g + 15 (NG 4), 32 g + 31 (NG 2), 63 (NG 1)
  int wkl[3], wkh[3];  // the wave's box B - o (scalar)
  auto reduce = [&](float d0, float d1, float d2) {
    const float dd[3] = {d0, d1, d2};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float d = dd[k];
      const float m = (__builtin_fabsf(d) + r) * 0x1p-21f + 0x1p-126f;
      int kl = fkey(join ? (d - r) - m : __builtin_inff());
      int kh = fkey(join ? (d + r) + m : -__builtin_inff());
      kl = rows_min_i(kl);
      kh = rows_max_i(kh);
      if (NG == 4) {
        gkl[k] = kl;
        gkh[k] = kh;
      }
      kl = halves_min_i(kl);
      kh = halves_max_i(kh);
      if (NG == 2) {
        gkl[k] = kl;
        gkh[k] = kh;
      }
      kl = wave_min_from_halves(kl);
      kh = wave_max_from_halves(kh);
      if (NG == 1) {
        gkl[k] = kl;
        gkh[k] = kh;
      }
      wkl[k] = __builtin_amdgcn_readlane(kl, 63);
      wkh[k] = __builtin_amdgcn_readlane(kh, 63);
    }
  };
  // Group boxes in the scan frame, widened by mg >= ext 2^-20: a point of a joined lane's ball is
  // staged for the lane's group whatever the fp32 rounding of its offset (<= ext 2^-24). Widened on
  // the group lanes, then read into scalar registers (an empty group: +inf / -inf).
  float gl[NG][3], gh[NG][3];
  auto group_bounds = [&](float mg) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const float lo = funkey(gkl[k]) - mg, hi = funkey(gkh[k]) + mg;
#pragma unroll
      for (int g = 0; g < NG; g++) {
        gl[g][k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lo), (64 / NG) * g + 64 / NG - 1));
        gh[g][k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(hi), (64 / NG) * g + 64 / NG - 1));
      }
    }
  };
  if (jm != 0) reduce((float)(qx - ox_), (float)(qy - oy_), (float)(qz - oz_));
  // a wave with a record takes its group boxes in the record's frame right away (the reduction's
  // vector registers die here; a wave that then walks reduces again in its new frame)
  if (have_rec) group_bounds(pext * 0x1p-20f);

  PCLK(t_p2);
  PSTOP(3);
  // Phase 3: the leaves meeting B. With the candidate cache (iterate only), a walk collects the
  // leaves meeting B+ = B enlarged by wc_margin x its largest half-extent per side and stores the
  // points inside B+ (as the scan stages them: fp32 offsets from B+'s centre, and the id); the
  // next iterate's wave streams them back without walking or gathering while its own B lies
  // inside B+ (every point inside B is then in the list). The scan frame is B+'s centre whenever
  // the cache is on, so stored and freshly staged offsets are the same values.
  int nleaf = 0;
  bool overflow = false;
  // the cooperative walk over the leaves meeting the box [wl, wh] (wave-uniform)
  auto walk = [&](double wlx, double wly, double wlz, double whx, double why, double whz) {
    nleaf = 0;
    overflow = false;
      int tail = 1;
      if (a.cells) {
        tail = cell_starts<64, kWaveStartK>(a, wlx, wly, wlz, whx, why, whz, lane, 0, queue);
        if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[21], (unsigned long long)tail);
      } else {
        // Wave-uniform descent to the deepest node that holds every leaf meeting B: follow the
        // only child meeting B while there is exactly one.
        int32_t start = 0;
        while (true) {
          const NodeLoad nd = load_node(a.nodes + start);
          const int2 topo = make_int2(nd.topo.x, nd.topo.y);
          const uint32_t meta = (uint32_t)topo.y;
          if (meta & kLeafBit) break;
          uint32_t kids = children_in_box(nd, meta & 0xffu, wlx, wly, wlz, whx, why, whz);
          kids = (uint32_t)__builtin_amdgcn_readfirstlane((int)kids);
          if (__builtin_popcount(kids) != 1) break;
          const uint32_t o = (uint32_t)__builtin_ctz(kids);
          start = __builtin_amdgcn_readfirstlane(topo.x + __builtin_popcount((meta & 0xffu) & ((1u << o) - 1u)));
          if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[21], 1ull);
        }
        if (lane == 0) queue[0] = start;
      }
      // Every batch pops up to 64 nodes (one per lane), which already meet B (tested by their
      // parent; the start nodes by the cell box or the descent), appends the points of its leaves
      // to the candidate list and pushes its children meeting B. Most recent first: the live set
      // stays small. (Two nodes per lane, both loads in flight, cost the kernel 16 more live
      // vector registers through this rare path, ~3 % of the waves per iterate: spills on the
      // common path.)
      wave_lds_fence();
      while (tail > 0) {
        const int batch = tail < 64 ? tail : 64;
        const bool has = lane < batch;
        // the record's box and topology in one round trip; lanes without a node read the root
        // (in bounds, ignored)
        const NodeRec* nr = a.nodes + (has ? queue[tail - batch + lane] : 0);
        NodeLoad nd;
        nd.l01 = *reinterpret_cast<const double2*>(&nr->lo[0]);
        nd.l2h0 = *reinterpret_cast<const double2*>(&nr->lo[2]);
        nd.h12 = *reinterpret_cast<const double2*>(&nr->hi[1]);
        const int2 topo = *reinterpret_cast<const int2*>(&nr->first);
        const int32_t first = has ? topo.x : 0;
        const uint32_t meta = has ? (uint32_t)topo.y : 0u;
        const uint32_t kids = (has && !(meta & kLeafBit)) ? children_in_box(nd, meta & 0xffu, wlx, wly, wlz, whx, why, whz) : 0u;
        // a leaf contributes its points (contiguous in leaf order) to the candidate list
        const int lcnt = (has && (meta & kLeafBit)) ? (int)(meta & ~kLeafBit) : 0;
        int ltot;
        const int lincl = wave_incl_scan(lcnt, &ltot);
        const int lpos = nleaf + lincl - lcnt;
        if (lcnt > 0 && lpos + lcnt <= kWaveCandCap)
          for (int c = 0; c < lcnt; c++) plist[lpos + c] = first + c;
        nleaf += ltot;
        const int nch = __builtin_popcount(kids);
        int tot;
        const int incl = wave_incl_scan(nch, &tot);
        tail -= batch;  // the popped entries are in registers; children overwrite them
        if (nleaf > kWaveCandCap || tail + tot > kWaveQueue) {
          overflow = true;
          return;
        }
        int off = tail + incl - nch;
        uint32_t kk = kids;
        while (kk) {
          const uint32_t o = (uint32_t)__builtin_ctz(kk);
          kk &= kk - 1u;
          queue[off++] = first + __builtin_popcount(meta & 0xffu & ((1u << o) - 1u));
        }
        tail += tot;
        if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[5], 1ull);
        wave_lds_fence();
      }
  };
  // The wide pass (WIDE): the same walk over a box of any size, in segments. A batch whose leaves
  // would overflow the candidate list appends the ones that fit (a prefix of its leaf lanes: the
  // inclusive sums grow with the lane) and pushes the others back on the stack (LIFO: they start
  // the next segment); the full list is scanned by seg(count), then refilled. Every leaf meeting
  // the box is listed in exactly one segment. Returns false when the stack overflows or one leaf
  // holds more points than the list (nothing is then decided here: the ball search takes it).
  // The wide pass's group spheres: per scan group (its NG kd sub-buckets of lanes), a ball around
  // the centre of the group's box holding every joined lane's ball (|q - c| + r, rounded up). A
  // node whose box is farther than every sphere from its centre holds no point of any ball. Far
  // queries near a surface make boxes much larger than their balls (the box's corners cut the
  // surface, the balls only touch it): the spheres keep the walk to what the balls reach.
  double sph_c[NG][3], sph_r2[NG];
  // The box is read at every batch: seg() may shrink it (a node pushed against an older, larger
  // box is tested again when popped).
  auto walk_seg = [&](const double& wlx, const double& wly, const double& wlz, const double& whx, const double& why,
                      const double& whz, auto&& seg) -> bool {
    nleaf = 0;
    int tail = 1;
    int32_t* wq = reinterpret_cast<int32_t*>(wl + kWaveLds + 1024);  // the wide pass's own stack
    if (a.cells) {
      tail = cell_starts<64, kWaveStartK>(a, wlx, wly, wlz, whx, why, whz, lane, 0, wq);
    } else if (lane == 0) {
      wq[0] = 0;
    }
    wave_lds_fence();
    int segs = 0, listed = 0;
    while (tail > 0) {
      // a popped node pushes at most 8 entries (its children, or itself back): batches shrink
      // while the stack is nearly full, so it never overflows (depth-first: the deepest entries
      // are popped first and the stack drains)
      int batch = (kWideQueue - tail) / 7;
      batch = batch < 1 ? 1 : batch > 64 ? 64 : batch;
      batch = tail < batch ? tail : batch;
      const bool has = lane < batch;
      const int32_t nid = has ? wq[tail - batch + lane] : 0;
      const NodeRec* nr = a.nodes + nid;
      NodeLoad nd;
      nd.l01 = *reinterpret_cast<const double2*>(&nr->lo[0]);
      nd.l2h0 = *reinterpret_cast<const double2*>(&nr->lo[2]);
      nd.h12 = *reinterpret_cast<const double2*>(&nr->hi[1]);
      const int2 topo = *reinterpret_cast<const int2*>(&nr->first);
      const int32_t first = has ? topo.x : 0;
      // the node's tight box (its points' bounding box; it was pushed by its cell) against the
      // current box (it met the box it was pushed against) and the group spheres: its squared box
      // distance from a sphere's centre (rounding up to a few ulps, covered by the spheres'
      // margin) at most the radius squared
      const float4 tb0 = *reinterpret_cast<const float4*>(&a.tbox[nid].lo[0]);
      const float2 tb1 = *reinterpret_cast<const float2*>(&a.tbox[nid].hi[1]);
      bool live = has && (double)tb0.x <= whx && (double)tb0.w >= wlx && (double)tb0.y <= why &&
                  (double)tb1.x >= wly && (double)tb0.z <= whz && (double)tb1.y >= wlz;
      if (live) {
        bool any = false;
#pragma unroll
        for (int g = 0; g < NG; g++)
          any = any || (sph_r2[g] > 0.0 &&  // 0: a group without joined lanes (its centre is not finite)
                        !(box_s(tb0.x, tb0.y, tb0.z, tb0.w, tb1.x, tb1.y, sph_c[g][0], sph_c[g][1], sph_c[g][2]) >
                          sph_r2[g]));
        live = any;
      }
      const uint32_t meta = live ? (uint32_t)topo.y : 0u;
      const uint32_t kids = (live && !(meta & kLeafBit)) ? children_in_box(nd, meta & 0xffu, wlx, wly, wlz, whx, why, whz) : 0u;
      const int lcnt = (live && (meta & kLeafBit)) ? (int)(meta & ~kLeafBit) : 0;
      if (wballot(lcnt > kWaveCandCap) != 0) return false;
      int ltot;
      const int lincl = wave_incl_scan(lcnt, &ltot);
      const bool fit = lcnt > 0 && nleaf + lincl <= kWaveCandCap;
      const bool back = lcnt > 0 && !fit;
      if (fit)
        for (int c = 0; c < lcnt; c++) plist[nleaf + lincl - lcnt + c] = first + c;
      // the points appended: the exclusive sum at the first leaf lane that did not fit
      const unsigned long long bm = wballot(back);
      const int app = bm ? __builtin_amdgcn_readlane(lincl - lcnt, __builtin_ctzll(bm)) : ltot;
      nleaf += app;
      listed += app;
      const int nch = __builtin_popcount(kids) + (back ? 1 : 0);
      int tot;
      const int incl = wave_incl_scan(nch, &tot);
      tail -= batch;  // the popped entries are in registers; pushes overwrite them
      if (tail + tot > kWideQueue) {
        if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[34], 1ull);
        return false;
      }
      int off = tail + incl - nch;
      if (back) wq[off++] = nid;
      uint32_t kk = kids;
      while (kk) {
        const uint32_t o = (uint32_t)__builtin_ctz(kk);
        kk &= kk - 1u;
        wq[off++] = first + __builtin_popcount(meta & 0xffu & ((1u << o) - 1u));
      }
      tail += tot;
      if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[5], 1ull);
      wave_lds_fence();
      if (bm != 0) {
        seg(nleaf);
        ++segs;
        nleaf = 0;
        wave_lds_fence();  // the segment's reads of the list are done before it is refilled
        // a box this dense for its balls (their bounding box cuts a surface far wider than the
        // balls do) is left to the per-query searches, with the bounds found so far
        if (segs >= (have_prev ? kWideSegs : kWideSegs0) && tail > 0) {
          if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[34], 1ull);
          return false;
        }
      }
    }
    if (nleaf > 0) {
      seg(nleaf);
      ++segs;
    }
    if (kDbg && a.dbg && lane == 0) {
      atomicAdd(&a.dbg[32], 1ull);
      atomicAdd(&a.dbg[33], (unsigned long long)segs);
      atomicAdd(&a.dbg[36], (unsigned long long)listed);
    }
    return true;
  };
  bool wstore = false, reuse = false;
  double wlx = 0.0, wly = 0.0, wlz = 0.0, whx = 0.0, why = 0.0, whz = 0.0;  // B+ of a walk
  double blx = 0.0, bly = 0.0, blz = 0.0, bhx = -1.0, bhy = -1.0, bhz = -1.0;  // B (fp64) of a walking wave
  double ocx = ox_, ocy = oy_, ocz = oz_;  // the scan frame's centre (B+'s with the cache, else B's)
  double ext = 0.0;  // >= |offset| of every point inside B and every joined query, in the frame
  auto group_spheres = [&]() {
#pragma unroll
    for (int g = 0; g < NG; g++) {
      sph_c[g][0] = uniform_d(ocx + 0.5 * ((double)gl[g][0] + (double)gh[g][0]));
      sph_c[g][1] = uniform_d(ocy + 0.5 * ((double)gl[g][1] + (double)gh[g][1]));
      sph_c[g][2] = uniform_d(ocz + 0.5 * ((double)gl[g][2] + (double)gh[g][2]));
    }
    const int gq = lane / (64 / NG);
    double cx = sph_c[0][0], cy = sph_c[0][1], cz = sph_c[0][2];
#pragma unroll
    for (int g = 1; g < NG; g++) {
      cx = gq == g ? sph_c[g][0] : cx;
      cy = gq == g ? sph_c[g][1] : cy;
      cz = gq == g ? sph_c[g][2] : cz;
    }
    const double dx = qx - cx, dy = qy - cy, dz = qz - cz;
    // |q - c| rounded up, plus the lane's radius (an upper bound already), as an fp32 key
    const double rr = (__builtin_sqrt(dx * dx + dy * dy + dz * dz) + (double)r) * (1.0 + 0x1p-40) + 0x1p-1000;
    int key = join ? __float_as_int((float)rr * (1.0f + 0x1p-22f)) : 0;  // >= 0: int order is float order
    key = rows_max_i(key);
    if (NG <= 2) key = halves_max_i(key);
    if (NG == 1) key = wave_max_from_halves(key);
#pragma unroll
    for (int g = 0; g < NG; g++) {
      const float R = __int_as_float(__builtin_amdgcn_readlane(key, (64 / NG) * g + 64 / NG - 1));
      sph_r2[g] = (double)R * (double)R * (1.0 + 0x1p-40);  // 0 for a group without joined lanes
    }
  };

  WaveBox* wb = nullptr;
  float4* wents = nullptr;
  if (jm != 0) {
    if (use_wc) {
      wb = a.wc_box + wid;
      wents = a.wc_ents + (size_t)wid * kWaveCandCap;
    }
    if (have_rec) {
      // reused while B lies inside B+ (exact: B's fp32 bounds are rounded outwards, B+'s inwards)
      // and B+ is not much larger than B (vol(B) >= the record's vmin = vol(B+) / wc_loose: a wave
      // whose box shrank, e.g. after the first iterate's descent guesses, walks again and stores a
      // tighter list)
      bool inside = true;
#pragma unroll
      for (int k = 0; k < 3; k++) inside = inside && wkl[k] >= pkl[k] && wkh[k] <= pkh[k];
      const float vb = (funkey(wkh[0]) - funkey(wkl[0])) * (funkey(wkh[1]) - funkey(wkl[1])) *
                       (funkey(wkh[2]) - funkey(wkl[2]));
      const float vmin = __int_as_float(__builtin_amdgcn_readlane((int)(unsigned)__double_as_longlong(hdr), 7));
      reuse = inside && vb >= vmin;
      if (kDbg && a.dbg && lane == 0 && !reuse) atomicAdd(&a.dbg[inside ? 25 : 24], 1ull);
    }
    if (reuse) {
      nleaf = __builtin_amdgcn_readlane((int)(unsigned)__double_as_longlong(hdr), 6);
      // the frame is o: the reduction's offsets are the scan's, its group boxes the scan's
      ext = (double)pext * (1.0 + 0x1p-20);
      if (kDbg && a.dbg && lane == 0) {
        atomicAdd(&a.dbg[12], 1ull);
        atomicAdd(&a.dbg[17], (unsigned long long)nleaf);  // entries a reusing wave streams
      }
    } else {
      // B in fp64: o + the wave's bounds, rounded outwards
      blx = uniform_d(box_lo(ox_, funkey(wkl[0])));
      bly = uniform_d(box_lo(oy_, funkey(wkl[1])));
      blz = uniform_d(box_lo(oz_, funkey(wkl[2])));
      bhx = uniform_d(box_hi(ox_, funkey(wkh[0])));
      bhy = uniform_d(box_hi(oy_, funkey(wkh[1])));
      bhz = uniform_d(box_hi(oz_, funkey(wkh[2])));
      // B+ (B itself without the cache); an overflowing B+ makes an overflowing wave (its lanes
      // take the ball search; ~0.06 % of the waves at 10M with the default margin). Wave-uniform
      // doubles are kept in scalar registers.
      // Without previous residuals (descent guesses: large, loose boxes that the next iterate
      // re-walks anyway) the wave walks B itself and stores nothing.
      const bool keep = wb && have_prev;
      const double m = keep ? a.wc_margin * 0.5 * dmax_(dmax_(bhx - blx, bhy - bly), bhz - blz) : 0.0;
      // The lead: the queries of a wave keep moving the same way for many iterates (ICP's
      // increments change slowly), so the stored B+ also covers where B will be after wc_lead
      // more iterates of this iterate's motion (the displacement of B's centre by the applied
      // transform), on the side it moves to. Any box is exact: this only sets how long the
      // record lasts against how many entries a reusing wave streams.
      double dlx = 0.0, dly = 0.0, dlz = 0.0, dhx = 0.0, dhy = 0.0, dhz = 0.0;
      if (APPLY && keep && a.wc_lead > 0.0) {
        double T[12];
        load_T(a, T);
        const double cx = (blx + bhx) * 0.5, cy = (bly + bhy) * 0.5, cz = (blz + bhz) * 0.5;
        const double ex = (((T[0] * cx + T[1] * cy) + T[2] * cz) + T[3]) - cx;
        const double ey = (((T[4] * cx + T[5] * cy) + T[6] * cz) + T[7]) - cy;
        const double ez = (((T[8] * cx + T[9] * cy) + T[10] * cz) + T[11]) - cz;
        // finite and at most twice B's largest extent per iterate (a wild increment leads nowhere)
        const double cap = 2.0 * dmax_(dmax_(bhx - blx, bhy - bly), bhz - blz);
        auto lead = [&](double e) { return (e == e && __builtin_fabs(e) <= cap) ? a.wc_lead * e : 0.0; };
        const double lx = lead(ex), ly = lead(ey), lz = lead(ez);
        dlx = lx < 0.0 ? -lx : 0.0;
        dhx = lx > 0.0 ? lx : 0.0;
        dly = ly < 0.0 ? -ly : 0.0;
        dhy = ly > 0.0 ? ly : 0.0;
        dlz = lz < 0.0 ? -lz : 0.0;
        dhz = lz > 0.0 ? lz : 0.0;
      }
      wlx = uniform_d(blx - (m + dlx));
      wly = uniform_d(bly - (m + dly));
      wlz = uniform_d(blz - (m + dlz));
      whx = uniform_d(bhx + (m + dhx));
      why = uniform_d(bhy + (m + dhy));
      whz = uniform_d(bhz + (m + dhz));
      // (the wide pass walks B in segments during its scan, phase 4)
      if (!WIDE) walk(wlx, wly, wlz, whx, why, whz);
      if (overflow && keep) {
        // B+ holds too many points: walk again with a quarter of the margin and the lead, and
        // store that list (an overflowing wave that stored nothing would overflow again at every
        // iterate)
        const double m4 = 0.25 * m;
        wlx = uniform_d(blx - (m4 + 0.25 * dlx));
        wly = uniform_d(bly - (m4 + 0.25 * dly));
        wlz = uniform_d(blz - (m4 + 0.25 * dlz));
        whx = uniform_d(bhx + (m4 + 0.25 * dhx));
        why = uniform_d(bhy + (m4 + 0.25 * dhy));
        whz = uniform_d(bhz + (m4 + 0.25 * dhz));
        walk(wlx, wly, wlz, whx, why, whz);
      }
      wstore = keep && !overflow;
      // the frame: B+'s centre with the cache (the stored record's), else B's
      if (keep) {
        ocx = (wlx + whx) * 0.5;
        ocy = (wly + why) * 0.5;
        ocz = (wlz + whz) * 0.5;
      } else {
        ocx = (blx + bhx) * 0.5;
        ocy = (bly + bhy) * 0.5;
        ocz = (blz + bhz) * 0.5;
      }
      ocx = uniform_d(ocx);
      ocy = uniform_d(ocy);
      ocz = uniform_d(ocz);
      // |offset| <= ext for every point inside B and every joined query (B lies in the frame box)
      ext = dmax_(dmax_(dmax_(bhx - ocx, ocx - blx), dmax_(bhy - ocy, ocy - bly)), dmax_(bhz - ocz, ocz - blz)) *
            (1.0 + 0x1p-40);
      if (!overflow && (WIDE || nleaf > 0)) {
        // the group boxes and the queries' offsets again, in the frame
        reduce((float)(qx - ocx), (float)(qy - ocy), (float)(qz - ocz));
        group_bounds((float)(ext * 0x1p-20));
      }
    }
  }
  // the cache record of a stored list (entries already written); vmin: the loose test's bound
  auto store_header = [&](int count) {
    if (lane == 0) {
      wb->lo[0] = wlx;
      wb->lo[1] = wly;
      wb->lo[2] = wlz;
      wb->hi[0] = whx;
      wb->hi[1] = why;
      wb->hi[2] = whz;
      wb->count = count;
      wb->gen = a.wc_gen;
      wb->vmin = (float)((whx - wlx) * (why - wly) * (whz - wlz) / a.wc_loose);
    }
    if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[13], 1ull);
  };
  // An overflowing wave (its box holds more candidates than the list takes): its joined queries
  // are searched again as two 32-query halves (k_nn_half), each with the smaller box of its own
  // balls; an overflowing half hands its queries to the ball search.
  bool deferred = false;
  if (overflow) {
    if (!kSecond && lane == 0) atomicAdd(a.fb_count + 6, 1u);  // the iteration record's n_wide
    if (!HALF && CM != 1 && a.fb_list3 != nullptr) {  // the half pass: first iterates only
      // entries (half id, mask of its deferred lanes): the half pass searches exactly these
      const unsigned long long dm = wballot(join);
      deferred = join;
      const unsigned nh = ((uint32_t)dm != 0u ? 1u : 0u) + ((dm >> 32) != 0ull ? 1u : 0u);
      if (lane == 0 && nh > 0) {
        unsigned at = atomicAdd(a.fb_count + 4, nh);
        if ((uint32_t)dm != 0u) {
          a.fb_list3[2 * at] = (int32_t)(2 * wid);
          a.fb_list3[2 * at + 1] = (int32_t)(uint32_t)dm;
          at++;
        }
        if ((dm >> 32) != 0ull) {
          a.fb_list3[2 * at] = (int32_t)(2 * wid + 1);
          a.fb_list3[2 * at + 1] = (int32_t)(uint32_t)(dm >> 32);
        }
        if (kDbg && a.dbg) atomicAdd(&a.dbg[16], (unsigned long long)nh);
      }
    } else if (!WIDE && a.fb_list4 != nullptr) {
      // the wide pass (k_nn_wide) searches the joined lanes again with the same box, walked and
      // scanned in segments: (first query of the wave or half, lane mask) per entry
      const unsigned long long dm = wballot(join);
      deferred = join;
      if (dm != 0) {
        const int fl = __builtin_ctzll(dm);
        const int32_t base = __builtin_amdgcn_readlane(i, fl) - fl;  // i = base + lane
        if (lane == 0) {
          const unsigned at = atomicAdd(a.fb_count + 5, 1u);
          a.fb_list4[3 * at] = base;
          a.fb_list4[3 * at + 1] = (int32_t)(uint32_t)dm;
          a.fb_list4[3 * at + 2] = (int32_t)(uint32_t)(dm >> 32);
        }
      }
    }
    join = false;
  }
  if (kDbg && a.dbg && lane == 0) {
    atomicAdd(&a.dbg[0], 1ull);
    if (overflow) atomicAdd(&a.dbg[1], 1ull);
  }

  PCLK(t_p3);
  PSTOP(4);
  // Phase 4: the lockstep scan: 64 candidates per chunk, the next chunk's loads in flight while
  // the current one is scanned from LDS (a reusing wave streams its cache entries; a walking wave
  // gathers the points of its list and, with the cache, stores those inside B+).
  double best = __builtin_inf(), second = __builtin_inf();
  int32_t bpos = -1;
  // streamed: the candidates are cache entries (a reusing wave's, or in the WC instance the ones a
  // walking wave stores here: the points of its list inside B+, in list order, before the scan)
  bool streamed = reuse;
  if constexpr (CM == 1) {
    if (wstore) {
      int wcount = 0;
      double4 nxtp = make_double4(0.0, 0.0, 0.0, 0.0);
      // a copy of an earlier point (TgtPt::sep's sign) is never stored: its twin is the reference's
      // answer whenever it would be (id -1 below)
      if (lane < nleaf) nxtp = load_cand(a.pts, plist[lane]);
      for (int base = 0; base < nleaf; base += 64) {
        const double4 cur = nxtp;
        const int nb = base + 64;
        if (nb + lane < nleaf) nxtp = load_cand(a.pts, plist[nb + lane]);
        const bool inp = base + lane < nleaf && cur.x >= wlx && cur.x <= whx && cur.y >= wly && cur.y <= why &&
                         cur.z >= wlz && cur.z <= whz && __double_as_longlong(cur.w) >= 0;
        const unsigned long long pm = wballot(inp);
        if (inp)
          wents[wcount + mask_rank(pm)] = make_float4((float)(cur.x - ocx), (float)(cur.y - ocy), (float)(cur.z - ocz),
                                                      __int_as_float((int)__double_as_longlong(cur.w)));
        wcount += __popcll(pm);
      }
      store_header(wcount);
      wstore = false;
      nleaf = wcount;
      // the wave's own stores, read back by other lanes of the wave (same CU: no L1 invalidate)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      ent0 = lane < wcount ? wents[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
      streamed = true;
    }
  }
  const int npts = nleaf;
  int scanned_pts = 0;
  bool need64 = wballot(join) != 0 && (WIDE || npts > 0);
  // the wide pass: lanes it leaves undecided (no certificate, or a walk that overflowed) take the
  // ball search with the tightest upper bound it found (gw: the fp64 fl(d2) of a scanned point)
  bool wide_lane = false;
  double gw = u;
  if (a.scan32 && need64) {
    if (ext >= 0x1p-40 && ext <= 0x1p60) {
      constexpr int LG = 64 / NG;  // lanes of a group
      // points of a group's segment per round: LG for a walking wave (its candidate list occupies
      // the list area); a wave that reuses its cache record leaves the list area unused, so it
      // stages up to 64 points per group (NG x 1 KB: the stack area and the list area) across its
      // chunks and scans once they would overflow (usually once per wave); slots stay below 64
      // (6 key bits)
      const int SP = streamed ? 64 : LG;
      const int gq = lane / LG;  // this lane's group
      // staging area: NG segments of SP points, in pairs [x0 x1 y0 y1 z0 z1 w0 w1] (32 B) so that
      // one packed fp32 instruction (v_pk_add/mul/fma_f32) evaluates an axis of two points.
      // Pair k of group g at k NG + g: the groups interleaved (each group's pairs contiguous costs
      // two more spilled registers)
      auto blk = [](int k, int g) { return k * NG + g; };
      // (the wide pass keeps its walk's stack through the scan: its staging area follows the list)
      float* stage32 = reinterpret_cast<float*>(wl + (WIDE ? kWaveLds : 0));
      // Selection keys: the fp32 squared distance with its low 6 bits replaced by the point's slot
      // in the segment (v_bfi), so that the two smallest are kept by two med3 per point and the
      // winner is found from its slot once per round. A key is within 63 ulps of its value, and
      // s2 & ~63 is a lower bound of the second-smallest value; keys are finite and >= 0 (offsets
      // <= ext <= 2^60, pads far but finite), so float order is key order.
      float k1 = __builtin_inff(), k2 = __builtin_inff();
      int32_t p1 = -1;
      typedef float f2 __attribute__((ext_vector_type(2)));
      typedef int v4i __attribute__((ext_vector_type(4)));
      // the queries' offsets in the frame (a reusing wave's are its reduction's, bit for bit)
      const float qx32 = (float)(qx - ocx), qy32 = (float)(qy - ocy), qz32 = (float)(qz - ocz);
      const f2 qx2 = {qx32, qx32}, qy2 = {qy32, qy32}, qz2 = {qz32, qz32};
      // ~63 in a vector register: with it (a literal cannot be a VOP3 operand on gfx9) the key is
      // one v_and_or_b32 instead of v_and_b32 + v_or_b32
      uint32_t kmask = ~63u;
      asm volatile("" : "+v"(kmask));
      // The two smallest of {k1, k2, a, b} (k1 <= k2) in three instructions per pair of points:
      // k1' = min3(k1, a, b); the second smallest is min(med3(k1, a, b), k2) (if k2 is below the
      // median of the other three it is second, as k1 <= k2; otherwise the median is). Keys are
      // never NaN, so no canonicalisation is needed; the last min is one VOP2 v_min_f32 (2/3 the
      // issue cost of a VOP3 on gfx950).
      auto sel2 = [&](float ka, float kb) {
        float m;
        asm("v_med3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(k1), "v"(ka), "v"(kb));
        asm("v_min3_f32 %0, %1, %2, %3" : "=v"(k1) : "v"(k1), "v"(ka), "v"(kb));
        asm("v_min_f32 %0, %1, %2" : "=v"(k2) : "v"(m), "v"(k2));
      };
      auto eval2 = [&](const v4i xy, const v4i zw, uint32_t sl) {
        const f2 X = {__int_as_float(xy.x), __int_as_float(xy.y)};
        const f2 Y = {__int_as_float(xy.z), __int_as_float(xy.w)};
        const f2 Z = {__int_as_float(zw.x), __int_as_float(zw.y)};
        const f2 dx = X - qx2, dy = Y - qy2, dz = Z - qz2;
        const f2 sq = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
        const float ka = __uint_as_float((__float_as_uint(sq.x) & kmask) | sl);
        const float kb = __uint_as_float((__float_as_uint(sq.y) & kmask) |
                                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(sl + 1u)));  // a scalar operand
        sel2(ka, kb);
      };
      // the same for the streamed scan's planes: an axis of the two points per 8-B read
      auto evalp = [&](const f2 X, const f2 Y, const f2 Z, uint32_t sl) {
        const f2 dx = X - qx2, dy = Y - qy2, dz = Z - qz2;
        const f2 sq = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
        const float ka = __uint_as_float((__float_as_uint(sq.x) & kmask) | sl);
        const float kb = __uint_as_float((__float_as_uint(sq.y) & kmask) |
                                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(sl + 1u)));
        sel2(ka, kb);
      };
      const v4i* st4 = reinterpret_cast<const v4i*>(stage32) + 2 * blk(0, gq);  // this group's pair 0
      constexpr int kStep = 2 * NG;                                             // v4i per pair step
      // One chunk of 64 candidates (lane = candidate base + lane; offsets vx, vy, vz, id bits vw):
      // group membership, rank among the group's points of the chunk, and (first round) the store
      // into the group's segment; `next` issues the following chunk's loads once this one is
      // staged; then the lockstep scan. Later rounds (more than S points of one group in one
      // chunk, rare) test again rather than keep NG ranks and masks live.
      int seg_n = npts;  // points of the list being scanned (the wide pass: of its segment)
      auto chunk = [&](int base, float vx, float vy, float vz, float vw, auto&& next) {
        const bool valid = base + lane < seg_n;
        int cn[NG];
        int maxc = 0;
        auto stage_round = [&](int r0, bool count) {
#pragma unroll
          for (int g = 0; g < NG; g++) {
            const bool in = valid && vx >= gl[g][0] && vx <= gh[g][0] && vy >= gl[g][1] && vy <= gh[g][1] &&
                            vz >= gl[g][2] && vz <= gh[g][2];
            const unsigned long long mk = wballot(in);
            if (count) {
              cn[g] = __popcll(mk);
              maxc = cn[g] > maxc ? cn[g] : maxc;
            }
            const int j = mask_rank(mk) - r0;
            if (in && j >= 0 && j < SP) {
              float* sp = stage32 + 8 * blk(j >> 1, g) + (j & 1);
              sp[0] = vx;
              sp[2] = vy;
              sp[4] = vz;
              sp[6] = vw;
            }
          }
        };
        wave_lds_fence();  // the previous round's reads are done before its slots are rewritten
        stage_round(0, true);
#pragma unroll
        for (int g = 0; g < NG; g++) scanned_pts += cn[g];
        next();
        for (int r0 = 0; r0 < maxc; r0 += SP) {
          if (r0 > 0) {
            wave_lds_fence();
            stage_round(r0, false);
          }
          // every segment padded to the round's even length with far points (index -1)
          int len = maxc - r0 < SP ? maxc - r0 : SP;
          len = (len + 1) & ~1;
          {
            const int pg = lane / LG;
            int c = cn[0];
#pragma unroll
            for (int g = 1; g < NG; g++) c = pg == g ? cn[g] : c;
            c -= r0;
            for (int pj = lane % LG; pj < len; pj += LG) {
              if (pj >= c) {
                float* sp = stage32 + 8 * blk(pj >> 1, pg) + (pj & 1);
                sp[0] = 0x1p62f;
                sp[2] = 0x1p62f;
                sp[4] = 0x1p62f;
                sp[6] = __int_as_float(-1);
              }
            }
          }
          wave_lds_fence();
          // lockstep over this group's staged pairs (each group's 16-B reads broadcast)
          const float k1_in = k1;
          const int mp = len >> 1;
          if (kDbg && a.dbg && lane == 0) {
            atomicAdd(&a.dbg[9], (unsigned long long)(maxc - r0 < SP ? maxc - r0 : SP));
            atomicAdd(&a.dbg[10], (unsigned long long)mp);
            atomicAdd(&a.dbg[11], 1ull);
          }
#pragma unroll 1
          for (int k = 0; k < mp; k++) eval2(st4[kStep * k], st4[kStep * k + 1], 2u * k);
          // the winner of this round, if it improved the lane's best: its index from its slot
          if (k1 != k1_in) {
            const uint32_t sl = __float_as_uint(k1) & 63u;
            p1 = __float_as_int(stage32[8 * blk((int)(sl >> 1), gq) + 6 + (sl & 1u)]);
          }
        }
      };
      wave_lds_fence();
      if (CM == 1 || streamed) {
        // Accumulate: each chunk's points are staged behind the previous chunks' (per group),
        // and a scan round runs only when a group's segment would overflow, and at the end. The
        // lockstep scan then pays max over groups of the wave's whole count once, not of every
        // chunk's count (pairs per wave 34.6 -> ~27 at NG = 4), and fewer rounds. The next
        // chunk's loads are issued before the current one is staged.
        //
        // Staged in planes (r23): x, y, z and id each in a plane of its own, a group's segment of
        // 64 points contiguous in every plane. A point's slot is then one address (the group's
        // base + the fill, scalar, + 4 x its rank: one v_lshl_add) for its four stores, which land
        // in the planes at immediate offsets; the scan reads an axis of two points as one 8-B
        // broadcast (three per pair instead of the pair blocks' 16 + 8 B). The pair blocks cost
        // five address instructions per staged point. Segments are kGS bytes apart (not 256):
        // the four groups' reads of one step fall on different banks.
        constexpr int kPl = 1280;      // bytes per plane: x, y, z, id = the wave's 5 KB
        constexpr int kGS = kPl / NG;  // a group's segment in a plane
        static_assert(4 * kPl <= kWaveLds && 64 * 4 <= kGS && kGS % 8 == 0, "planes of the streamed scan");
        unsigned char* const pl = wl;
        int fill[NG];
#pragma unroll
        for (int g = 0; g < NG; g++) fill[g] = 0;
        const unsigned char* const rp = pl + gq * kGS;  // this lane's group segment
        auto scan_round = [&]() {
          int maxf = 0;
#pragma unroll
          for (int g = 0; g < NG; g++) maxf = fill[g] > maxf ? fill[g] : maxf;
          const int len = (maxf + 1) & ~1;
          const int pg = lane / LG;
          int c = fill[0];
#pragma unroll
          for (int g = 1; g < NG; g++) c = pg == g ? fill[g] : c;
          for (int pj = lane % LG; pj < len; pj += LG) {
            if (pj >= c) {
              unsigned char* q = pl + pg * kGS + 4 * pj;
              *reinterpret_cast<float*>(q) = 0x1p62f;
              *reinterpret_cast<float*>(q + kPl) = 0x1p62f;
              *reinterpret_cast<float*>(q + 2 * kPl) = 0x1p62f;
              *reinterpret_cast<int32_t*>(q + 3 * kPl) = -1;
            }
          }
          wave_lds_fence();
          const float k1_in = k1;
          const int mp = len >> 1;
          if (kDbg && a.dbg && lane == 0) {
            atomicAdd(&a.dbg[9], (unsigned long long)maxf);
            atomicAdd(&a.dbg[10], (unsigned long long)mp);
            atomicAdd(&a.dbg[11], 1ull);
          }
#pragma unroll 1
          for (int k = 0; k < mp; k++) {
            const f2 X = *reinterpret_cast<const f2*>(rp + 8 * k);
            const f2 Y = *reinterpret_cast<const f2*>(rp + kPl + 8 * k);
            const f2 Z = *reinterpret_cast<const f2*>(rp + 2 * kPl + 8 * k);
            evalp(X, Y, Z, 2u * k);
          }
          if (k1 != k1_in) p1 = *reinterpret_cast<const int32_t*>(rp + 3 * kPl + 4 * (__float_as_uint(k1) & 63u));
          wave_lds_fence();  // the round's reads are done before the slots are rewritten
#pragma unroll
          for (int g = 0; g < NG; g++) fill[g] = 0;
        };
        float4 nx = ent0;  // loaded with the query
        for (int base = 0; base < npts; base += 64) {
          const float vx = nx.x, vy = nx.y, vz = nx.z, vw = nx.w;
          if (base + 64 + lane < npts) nx = wents[base + 64 + lane];
          const bool valid = base + lane < npts;
          // membership as lane masks (kept in scalar registers: the second pass takes its exec
          // mask and ranks from them, with no bool materialised in a vector register)
          bool ing[NG];
          unsigned long long mk[NG];
          int cn[NG];
          bool over = false;
#pragma unroll
          for (int g = 0; g < NG; g++) {
            ing[g] = valid && vx >= gl[g][0] && vx <= gh[g][0] && vy >= gl[g][1] && vy <= gh[g][1] &&
                     vz >= gl[g][2] && vz <= gh[g][2];
            mk[g] = wballot(ing[g]);
            cn[g] = __popcll(mk[g]);
            over = over || fill[g] + cn[g] > SP;
          }
          if (over) scan_round();
#pragma unroll
          for (int g = 0; g < NG; g++) {
            if (ing[g]) {
              // the slot: fill + rank (mbcnt's accumulator), one shift-add from the scalar base
              const int j = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk[g] >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)mk[g], (uint32_t)fill[g]));
              unsigned char* q = pl + g * kGS + 4 * j;
              *reinterpret_cast<float*>(q) = vx;
              *reinterpret_cast<float*>(q + kPl) = vy;
              *reinterpret_cast<float*>(q + 2 * kPl) = vz;
              *reinterpret_cast<float*>(q + 3 * kPl) = vw;
            }
            fill[g] += cn[g];
            scanned_pts += cn[g];
          }
        }
        scan_round();
      } else {
        int wcount = 0;  // entries stored to the cache (points inside B+)
        auto gather_scan = [&](const int np) {
        seg_n = np;
        double4 nxtp = make_double4(0.0, 0.0, 0.0, 0.0);
        if (lane < np) nxtp = load_cand(a.pts, plist[lane]);
        for (int base = 0; base < np; base += 64) {
          // a copy of an earlier point is staged far outside every group box (never scanned)
          const bool cp = __double_as_longlong(nxtp.w) < 0;
          const float vx = cp ? 0x1p62f : (float)(nxtp.x - ocx), vy = cp ? 0x1p62f : (float)(nxtp.y - ocy),
                      vz = cp ? 0x1p62f : (float)(nxtp.z - ocz);
          const float vw = __int_as_float((int)__double_as_longlong(nxtp.w));
          if (wstore) {
            const bool inp = base + lane < np && !cp && nxtp.x >= wlx && nxtp.x <= whx && nxtp.y >= wly &&
                             nxtp.y <= why && nxtp.z >= wlz && nxtp.z <= whz;
            const unsigned long long pm = wballot(inp);
            if (inp) wents[wcount + mask_rank(pm)] = make_float4(vx, vy, vz, vw);
            wcount += __popcll(pm);
          }
          chunk(base, vx, vy, vz, vw, [&]() {
            const int nb = base + 64;
            if (nb + lane < np) nxtp = load_cand(a.pts, plist[nb + lane]);
          });
        }
        if constexpr (WIDE) {
          // The lane's winner so far is a point: its fl(d2) bounds the nearest one's. The balls
          // shrink to the tighter bounds, and the box (in the same frame, rounded outwards) and
          // the group boxes with them: every point of a final ball lies in every earlier box, so
          // it is still listed and scanned; the rest of the walk visits less.
          if (join && p1 >= 0) {
            const TgtPt* p = a.pts + p1;
            const double dx = p->x - qx, dy = p->y - qy, dz = p->z - qz;
            const double d2 = dx * dx + dy * dy + dz * dz;
            u = d2 < u ? d2 : u;
          }
          r = join ? ball_radius32(u, amax) : 0.f;
          reduce((float)(qx - ocx), (float)(qy - ocy), (float)(qz - ocz));
          blx = uniform_d(box_lo(ocx, funkey(wkl[0])));
          bly = uniform_d(box_lo(ocy, funkey(wkl[1])));
          blz = uniform_d(box_lo(ocz, funkey(wkl[2])));
          bhx = uniform_d(box_hi(ocx, funkey(wkh[0])));
          bhy = uniform_d(box_hi(ocy, funkey(wkh[1])));
          bhz = uniform_d(box_hi(ocz, funkey(wkh[2])));
          group_bounds((float)(ext * 0x1p-20));
          group_spheres();
        }
        };
        if constexpr (WIDE) {
          // B itself (fp64, rounded outwards) in segments; a stack overflow leaves every joined
          // lane to the ball search
          group_spheres();
          if (!walk_seg(blx, bly, blz, bhx, bhy, bhz, gather_scan)) wide_lane = join;
        } else {
          gather_scan(npts);
        }
        if (wstore) {
          store_header(wcount);
          wstore = false;
        }
      }
      if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[26], (unsigned long long)scanned_pts);  // sum over groups
      const float s2 = __uint_as_float(__float_as_uint(k2) & ~63u);  // <= the second-smallest value
      // fp64 distance of the fp32 winner, exactly as the leaf scan computes it (octree.cpp:139-144)
      double b64 = __builtin_inf();
      if (join && p1 >= 0) {
        const TgtPt* p = a.pts + p1;
        const double dx = p->x - qx, dy = p->y - qy, dz = p->z - qz;
        b64 = dx * dx + dy * dy + dz * dz;
      }
      const double lb2 = scan32_lower_bound(s2, ext * (1.0 + 0x1p-19));
      // Decided lanes: nothing scanned; every point beyond the guess (the fp32 winner and the
      // bound of the rest: the per-lane search takes it, as after an fp64 scan); or a certified
      // winner within the guess. Anything else (a near tie, or a winner beyond u while another
      // point may be within it) re-scans the wave in fp64, which decides as the fp64 scan does.
      if constexpr (WIDE) {
        // no fp64 re-scan over segments: a lane that is not certified takes the ball search, with
        // its winner's fl(d2) as the bound when that is below its guess (any scanned point's is
        // an upper bound of the nearest one's)
        const bool dec = !wide_lane && join && p1 >= 0 && b64 <= u && certified(b64, lb2, a.init_best);
        if (join && p1 >= 0 && b64 < gw) gw = b64;
        wide_lane = join && !dec;
        if (kDbg && a.dbg) {
          const unsigned long long um = wballot(wide_lane);
          if (lane == 0) atomicAdd(&a.dbg[35], (unsigned long long)__popcll(um));
        }
        best = dec ? b64 : __builtin_inf();
        second = lb2;
        bpos = p1;
        need64 = false;
      }
      const bool ok = !join || p1 < 0 || (!(b64 <= u) && lb2 > u) || (b64 <= u && certified(b64, lb2, a.init_best));
      if (!WIDE && wballot(!ok) == 0) {
        best = b64;
        second = lb2;
        bpos = p1;
        need64 = false;
      }
    }
  }
  if (wstore && npts == 0) {  // an empty list (no scan below)
    store_header(0);
    wstore = false;
  }
  if (need64) {
    if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[8], 1ull);
    // Points outside B are farther than r from every joined lane (each ball lies in B), so
    // they can neither be a joined lane's nearest point nor sit in its certificate window.
    // Exact duplicates of the winner (identical coordinates) are not ties: they share its leaf
    // (identical points take the same octant at every split), where the reference's strict <
    // keeps the first in leaf order, i.e. the smallest position; `second` is the smallest fl(d2)
    // of the points that are not copies of the winner (any other equal distance stays a tie).
    // A reusing wave has no fp64 B (its reduction ran in the frame): it filters with its stored
    // B+, which holds B (a superset is exact, only the work grows; this path is rare).
    double xlx = blx, xly = bly, xlz = blz, xhx = bhx, xhy = bhy, xhz = bhz;
    if (reuse) {
      xlx = wb->lo[0];
      xly = wb->lo[1];
      xlz = wb->lo[2];
      xhx = wb->hi[0];
      xhy = wb->hi[1];
      xhz = wb->hi[2];
    }
    wave_lds_fence();
    double4 nxtp = make_double4(0.0, 0.0, 0.0, 0.0);
    bool nin = false;
    // candidate k: from the walk's list, or the id word of a reused cache entry
    auto cand_id = [&](int k) { return (CM == 1 || streamed) ? reinterpret_cast<const int32_t*>(wents + k)[3] : plist[k]; };
    if (lane < npts) {
      const int32_t g = cand_id(lane);
      const TgtPt* p = a.pts + g;
      const double2 xy = *reinterpret_cast<const double2*>(&p->x);
      nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
    }
    int wcount = 0;  // a walking wave without an fp32 pass stores its entries here
    for (int base = 0; base < npts; base += 64) {
      nin = base + lane < npts && nxtp.x >= xlx && nxtp.x <= xhx && nxtp.y >= xly && nxtp.y <= xhy &&
            nxtp.z >= xlz && nxtp.z <= xhz;
      const unsigned long long im = wballot(nin);
      const int slot = mask_rank(im);
      const double4 cur = nxtp;
      if (wstore) {
        const bool inp = base + lane < npts && cur.x >= wlx && cur.x <= whx && cur.y >= wly && cur.y <= why &&
                         cur.z >= wlz && cur.z <= whz;
        const unsigned long long pm = wballot(inp);
        if (inp)
          wents[wcount + mask_rank(pm)] = make_float4((float)(cur.x - ocx), (float)(cur.y - ocy), (float)(cur.z - ocz),
                                                      __int_as_float((int)__double_as_longlong(cur.w)));
        wcount += __popcll(pm);
      }
      const int nb = base + 64;
      if (nb + lane < npts) {
        const int32_t g = cand_id(nb + lane);
        const TgtPt* p = a.pts + g;
        const double2 xy = *reinterpret_cast<const double2*>(&p->x);
        nxtp = make_double4(xy.x, xy.y, p->z, __longlong_as_double((long long)g));
      }
      const int m = __popcll(im);
      scanned_pts += m;
      // the staging area holds 32 fp64 points: the chunk's in-B points in two halves
      for (int h = 0; h < m; h += 32) {
        wave_lds_fence();  // the previous half's reads are done before its slots are rewritten
        if (nin && slot >= h && slot < h + 32) stage[slot - h] = cur;
        wave_lds_fence();
        const int mh = m - h < 32 ? m - h : 32;
        for (int k = 0; k < mh; k++) {
          const double4 pt = stage[k];
          const double dx = pt.x - qx, dy = pt.y - qy, dz = pt.z - qz;
          const double d2 = dx * dx + dy * dy + dz * dz;
          const int32_t pi = (int32_t)__double_as_longlong(pt.w);
          bool dup = false;
          if (d2 == best) {  // rare: the winner is read back (no registers held for it)
            const TgtPt* w = a.pts + bpos;
            dup = w->x == pt.x && w->y == pt.y && w->z == pt.z;
          }
          if (d2 < best) {
            second = best;
            best = d2;
            bpos = pi;
          } else if (dup) {
            bpos = pi < bpos ? pi : bpos;  // an exact duplicate of the winner: no tie to break
          } else if (d2 < second) {
            second = d2;
          }
        }
      }
    }
    if (wstore) {
      store_header(wcount);
      wstore = false;
    }
    if (kDbg && a.dbg && lane == 0) atomicAdd(&a.dbg[4], (unsigned long long)scanned_pts);
  }
  if (kDbg && a.dbg) {
    const unsigned long long ex = wballot(cand && !join && !overflow);
    const unsigned long long cov = wballot(join && !(best <= u));
    const unsigned long long nc = wballot(active && finite_q && !safe && !cand);
    if (lane == 0) {
      atomicAdd(&a.dbg[2], (unsigned long long)__popcll(ex));
      atomicAdd(&a.dbg[3], (unsigned long long)__popcll(cov));
      atomicAdd(&a.dbg[6], (unsigned long long)__popcll(nc));
      atomicAdd(&a.dbg[7], (unsigned long long)nleaf);
    }
  }

  PCLK(t_p4);
  PSTOP(5);
  // Phase 5: certify, write, or queue.
  store_query32<APPLY>(a, i, active, qx, qy, qz);
  bool written = false, to_exact = false, to_lane = false;
  double d = 0.0;
  int32_t pos = bpos;
  if (safe) {
    qat(a.dist_out, i) = __builtin_sqrt(u);  // settled in phase 1b (the position stays)
  } else if (active) {
    if (!finite_q) {
      // NaN: every leaf distance is NaN; inf: the root's distance is inf. Either way the
      // reference keeps findNearest's default index 0 (octree.cpp:179).
      pos = a.pos0;
      d = residual_to(a.pts, pos, qx, qy, qz);
      written = true;
    } else if (WIDE && wide_lane) {
      to_lane = true;  // undecided by the wide pass (gw bounds its nearest distance)
    } else if (join && !(best <= u)) {
      to_lane = true;  // the guess did not cover the nearest point: search this one per lane
    } else if (join) {
      written = certified(best, second, a.init_best);
      to_exact = !written;
      d = __builtin_sqrt(best);
    } else if (!deferred) {
      to_lane = true;
    }
    if (written) {
      qat(a.pos_out, i) = pos;
      qat(a.dist_out, i) = d;
    }
  }
  wave_append(to_exact, i, a.fb_count, a.fb_list);
  const bool covered = !(join && !(best <= u));
  wave_append_u(to_lane, i, (WIDE && wide_lane) ? gw : covered ? u : __builtin_inf(), a.fb_count + 1, a.fb_list2,
                a.fb_u2);
  PSTOP(6);
  if (!kSecond)
    wave_record<DBG>(a, wid, lane, active, safe || written, safe ? __builtin_sqrt(u) : d, safe ? prev_pos : pos, qx,
                     qy, qz, wl);
#if ICP_PHASE_CLOCKS
  PCLK(t_p5);
  if (a.dbg && lane == 0) {
    atomicAdd(&a.dbg[16], t_p1 - t_p0);
    atomicAdd(&a.dbg[17], t_p2 - t_p1);
    atomicAdd(&a.dbg[18], t_p3 - t_p2);
    atomicAdd(&a.dbg[19], t_p4 - t_p3);
    atomicAdd(&a.dbg[20], t_p5 - t_p4);
  }
#endif
}

// Waves per SIMD the wave search is compiled for (its VGPR budget: 8 -> 64, 7 -> 72, 6 -> 80).
// 7 since r20: at 8 the frame-first setup spills (27 VGPRs, scratch reloads on the critical path:
// search 0.71 ms); at 7 it spills 6 (0.515 ms vs 0.548 for the r19 kernel at 8, 0.524 at 6;
// profiles/r20a/ab_waves_per_eu.txt). LDS (5 KB per wave) allows 8.
#ifndef ICP_WAVE_WPE
#define ICP_WAVE_WPE 7
#endif
#ifndef ICP_WAVE_WPE_WC
#define ICP_WAVE_WPE_WC ICP_WAVE_WPE
#endif
#ifndef ICP_WAVE_WPE_NC
#define ICP_WAVE_WPE_NC ICP_WAVE_WPE
#endif
// The WC instance (walking waves store their entries first, one scan path): 69 VGPRs and no
// scratch at 7 waves; search 0.473-0.477 -> 0.456-0.457 ms over 200 steps at 10M
// (profiles/r21/ab_walk_stream.txt). At 8 waves it spills 24 B and runs 0.49.
#ifndef ICP_WALK_STREAM
#define ICP_WALK_STREAM 1
#endif
#ifndef ICP_FIRST_NC
#define ICP_FIRST_NC 1
#endif
template <bool APPLY, int NG, bool CERT, bool DBG, int CM>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CM == 1 ? ICP_WAVE_WPE_WC : CM == 2 ? ICP_WAVE_WPE_NC : ICP_WAVE_WPE, CM == 1 ? ICP_WAVE_WPE_WC : CM == 2 ? ICP_WAVE_WPE_NC : ICP_WAVE_WPE))) k_nn_wave(NNLaunch a) {
  if (a.loop && a.loop->core.done) return;  // the device loop's session finished
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_raw[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int32_t i = (int32_t)(xcd_block((unsigned)a.xcd_blocks) * blockDim.x + threadIdx.x);  // n <= INT32_MAX
  wave_search<APPLY, NG, CERT, false, DBG, CM>(a, i, lane, reinterpret_cast<unsigned char*>(lds_raw) + wv * kWaveLds);
}

// The half pass: every wave takes 32-query halves of overflowed waves from the list (grid-stride;
// the list is complete when this kernel starts), lanes 0..31 each one query.
template <int NG, bool DBG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) k_nn_half(NNLaunch a) {
  if (a.loop && a.loop->core.done) return;
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_raw[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned char* wl = reinterpret_cast<unsigned char*>(lds_raw) + wv * kWaveLds;
  const unsigned cnt = a.fb_count[4];
  const unsigned waves = gridDim.x * (blockDim.x >> 6);
  for (unsigned j = blockIdx.x * (blockDim.x >> 6) + wv; j < cnt; j += waves) {
    const int32_t hb = a.fb_list3[2 * j];
    const uint32_t mask = (uint32_t)a.fb_list3[2 * j + 1];  // the lanes the first pass deferred
    const int64_t q = (int64_t)hb * 32 + lane;
    const int32_t i = (lane < 32 && ((mask >> lane) & 1u) && q < a.n) ? (int32_t)q : (int32_t)a.n;
    wave_lds_fence();  // the previous half's LDS reads are done
    wave_search<false, NG, false, true, DBG>(a, i, lane, wl);
  }
}

// The wide pass: every wave takes an overflowed wave (or half) from the list (grid-stride; the
// list is complete when this kernel starts): its deferred lanes search again with the same box,
// which the wave walks and scans in segments of up to kWaveCandCap points (walk_seg). Its LDS
// area holds the walk's stack, the list and a staging area of its own (the stack stays live
// through each segment's scan).
constexpr int kWideLds = kWaveLds + 1024 + kWideQueue * 4;
// (8 KB of LDS per wave admits 5 waves per SIMD: compiled for 5, 96 VGPRs)
#ifndef ICP_WIDE_WPE
#define ICP_WIDE_WPE 5
#endif
template <int NG, bool DBG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ICP_WIDE_WPE, ICP_WIDE_WPE))) k_nn_wide(NNLaunch a) {
  if (a.loop && a.loop->core.done) return;
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_raw[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned char* wl = reinterpret_cast<unsigned char*>(lds_raw) + wv * kWideLds;
  const unsigned cnt = a.fb_count[5];
  const unsigned waves = gridDim.x * (blockDim.x >> 6);
  for (unsigned j = blockIdx.x * (blockDim.x >> 6) + wv; j < cnt; j += waves) {
    const int64_t base = a.fb_list4[3 * j];
    const unsigned long long mask =
        (unsigned long long)(uint32_t)a.fb_list4[3 * j + 1] | (unsigned long long)(uint32_t)a.fb_list4[3 * j + 2] << 32;
    const int64_t q = base + lane;
    const int32_t i = (((mask >> lane) & 1ull) && q < a.n) ? (int32_t)q : (int32_t)a.n;
    wave_lds_fence();  // the previous entry's LDS reads are done
    wave_search<false, NG, false, false, DBG, 0, true>(a, i, lane, wl);
  }
}

// ---------------------------------------------------------------------------------------------
// The ball search: four queries per wave, one 16-lane group (a DPP row) each. The list's queries
// are latency-bound walks of a few dependent rounds, so four in flight per wave hide four times
// the latency of one. A group collects, breadth-first from the cell tables of the query's box,
// every leaf whose box distance s <= u (1 + 2^-47) (a sphere test) and scans their points one per
// lane. Leaves with s > u (1 + 2^-47) only hold points with fl(d2) > best (1 + 2^-48) (monotone
// rounding), so nothing in the certificate window is missed. Certification as in the wave search
// (best <= u and the window test). A query the group cannot decide (no usable guess, an
// overflowing candidate set, or no certificate) is finished right there by the group's first lane:
// the per-lane certified search, else the reference-order DFS (stack in the group's LDS).
// Before that, the kernel's threads take the exact list the wave search left, one query each
// (the reference-order DFS). One launch for all the follow-up searches.
constexpr int kBallGroups = 4;
constexpr int kBallGL = 64 / kBallGroups;  // lanes per query
constexpr int kBallStack = 512;
constexpr int kBallPoints = 1024;
constexpr int kBallGStack = kBallStack / kBallGroups;
constexpr int kBallGPoints = kBallPoints / kBallGroups;
constexpr int kBallLdsBytes = kBallStack * 4 + kBallPoints * 4;

// The reference-order DFS for query i (octree.cpp:128-184), its result written.
__device__ __forceinline__ void exact_query(const NNLaunch& a, int64_t i, unsigned long long* st, int bs) {
  const double qx = a.x[i], qy = a.y[i], qz = a.z[i];
  double best_d2 = a.init_best, visits = 0.0, scanned = 0.0;
  int32_t best = -1;
  exact_dfs<false>(a, qx, qy, qz, st, bs, best, best_d2, visits, scanned);
  a.pos_out[i] = best >= 0 ? best : a.pos0;
  a.dist_out[i] = best >= 0 ? __builtin_sqrt(best_d2) : residual_to(a.pts, a.pos0, qx, qy, qz);
}

// The per-lane certified search for query i; a query it cannot certify gets the reference-order
// DFS right away. budget > 0: a search that needs more node visits gives up (returns false, nothing
// written: the wave-cooperative search takes it).
// *found: the best fl(d2) it had found when it gave up (a point's: an upper bound for the next search).
// u: an upper bound of the nearest fl(d2) (inf: none), the search's initial prune bound.
__device__ __forceinline__ bool lane_query(const NNLaunch& a, int64_t i, unsigned long long* st, int bs,
                                           int budget = 0, double* found = nullptr, double u = __builtin_inf()) {
  const double qx = a.x[i], qy = a.y[i], qz = a.z[i];
  double best = __builtin_inf(), second = __builtin_inf();
  int32_t bpos = -1;
  const double thr0 = u <= 0x1p900 ? u * (1.0 + kFastPrune) : __builtin_inf();
  if (!fast_dfs(a, qx, qy, qz, st, bs, best, second, bpos, budget, thr0)) {
    if (found) *found = best;
    return false;
  }
  if (certified(best, second, a.init_best)) {
    a.pos_out[i] = bpos;
    a.dist_out[i] = __builtin_sqrt(best);
  } else {
    exact_query(a, i, st, bs);
    atomicAdd(a.fb_count + 3, 1u);  // a DFS finish of the ball search
    if (a.dbg) atomicAdd(&a.dbg[38], 1ull);
  }
  return true;
}

// Node visits a per-lane follow-up search may take before the wave-cooperative search takes over.
// A query far (relative to the local point spacing) from a dense surface needs every leaf whose
// box comes within its nearest distance: on the scene workload's outliers (metres above a ground
// sampled every few mm) up to ~30k visits of one lane, ~1 us of dependent loads each (the
// reference's DFS needs as many: tools/scene_probe.py). A wave's queue runs its lanes' searches
// together, so the longest one sets its time: the budget bounds that, and the cooperative search
// (64 nodes a step) takes the rest. Measured (profiles/r21/ab_lane_budget.txt, scene 20/5): 768
// -> 64 visits: 1M 320 -> 635 Mcorr/s, 10M 600 -> 677; config 4 and config 3 unchanged.
#ifndef ICP_LANE_BUDGET
#define ICP_LANE_BUDGET 64
#endif
constexpr int kLaneBudget = ICP_LANE_BUDGET;
constexpr int kBBStack = 2048;  // the cooperative search's node stack (int32 in LDS), the last
constexpr int kBBPts = 256;     // kBBPts entries of which hold a step's leaf points

// The wave-cooperative certified search of one query (every lane of the wave): branch and bound
// over the octree, up to 64 nodes per step (one per lane, LIFO), each node re-tested against the
// prune bound thr = best (1 + 2^-47) of the wave's best so far (exact as fast_dfs: a node is
// skipped only when its squared box distance s exceeds thr, so every point of the certificate
// window is scanned), leaves scanned by their lane, the best reduced over the wave every step.
// u: an upper bound of the query's nearest fl(d2) (inf: none). A frontier that outgrows the stack
// (a far query under a loose bound: every node within the bound is live) is searched again from
// the root with the best point found so far as the bound, which prunes the frontier to the nodes
// within the nearest distance (up to kBBPasses times while the bound shrinks). Returns false when
// it still overflows and 2 for a tie (nothing written either way: the caller runs the
// reference-order DFS), 1 after writing the certified result.
constexpr int kBBPasses = 4;
constexpr int kBBDone = 1;
__device__ __forceinline__ int wave_bb(const NNLaunch& a, int64_t i, double u, int32_t* stack, int lane) {
  const double qx = a.x[i], qy = a.y[i], qz = a.z[i];
  double best = __builtin_inf(), second = __builtin_inf();
  int32_t bpos = 0x7fffffff;
  int32_t* plist = stack + (kBBStack - kBBPts);
  double thr = (u <= 0x1p900) ? u * (1.0 + kFastPrune) : __builtin_inf();
  int steps = 0, passes = 0;
  bool over = false;
  while (true) {
    // a pass: every point it scans is counted once (best, second from this pass only)
    best = __builtin_inf();
    second = __builtin_inf();
    bpos = 0x7fffffff;
    const double thr0 = thr;
    // the start nodes: the cell-table nodes of the box q +- sqrt(thr) (every point within the
    // bound lies in it: the ball search's radius), else the root; the descent's levels skipped
    int tail = 1;
    if (a.cells && thr <= 0x1p900) {
      const double amax = __builtin_fmax(__builtin_fabs(qx), __builtin_fmax(__builtin_fabs(qy), __builtin_fabs(qz)));
      const double r = __builtin_sqrt(thr) * (1.0 + 0x1p-40) + amax * 0x1p-45;
      tail = cell_starts<64, 2>(a, qx - r, qy - r, qz - r, qx + r, qy + r, qz + r, lane, 0, stack);
    } else if (lane == 0) {
      stack[0] = 0;
    }
    over = false;
    ++passes;
    wave_lds_fence();
    while (tail > 0) {
      const int batch = tail < 64 ? tail : 64;
      const bool has = lane < batch;
      const int32_t nid = has ? stack[tail - batch + lane] : 0;
      tail -= batch;
      const NodeRec* rr = a.nodes + nid;
      const int2 topo = *reinterpret_cast<const int2*>(&rr->first);
      const uint32_t meta = (uint32_t)topo.y;
      // pushed against an older (larger) bound, and pushed by its cell: test the node's tight box
      const float4 tb0 = *reinterpret_cast<const float4*>(&a.tbox[nid].lo[0]);
      const float2 tb1 = *reinterpret_cast<const float2*>(&a.tbox[nid].hi[1]);
      const bool live = has && !(box_s(tb0.x, tb0.y, tb0.z, tb0.w, tb1.x, tb1.y, qx, qy, qz) > thr);
      const bool lf = live && (meta & kLeafBit);
      const uint32_t kids = (live && !lf) ? children_in_ball(rr, meta & 0xffu, qx, qy, qz, thr) : 0u;
      // The step's leaf points, flat: listed in LDS kBBPts at a time and scanned kBBPts / 64 per
      // lane with all their loads in flight together (a leaf scanned by its own lane was ~10
      // dependent round trips per step). Each point is scanned by one lane: the per-lane best and
      // second reduce to the wave's exactly as before.
      const int lcnt = lf ? (int)(meta & ~kLeafBit) : 0;
      int ltot;
      const int lfirst = wave_incl_scan(lcnt, &ltot) - lcnt;
      for (int base = 0; base < ltot; base += kBBPts) {
        for (int k = 0; k < lcnt; k++) {
          const int f = lfirst + k - base;
          if (f >= 0 && f < kBBPts) plist[f] = topo.x + k;
        }
        wave_lds_fence();
        const int m = ltot - base < kBBPts ? ltot - base : kBBPts;
        constexpr int P = kBBPts / 64;
        double px[P], py[P], pz[P];
        int32_t pid[P];
#pragma unroll
        for (int t = 0; t < P; t++) {
          pid[t] = t * 64 + lane < m ? plist[t * 64 + lane] : -1;
          const TgtPt* p = a.pts + (pid[t] >= 0 ? pid[t] : 0);
          const double2 pxy = *reinterpret_cast<const double2*>(&p->x);
          const double2 pzw = *reinterpret_cast<const double2*>(&p->z);
          px[t] = pxy.x;
          py[t] = pxy.y;
          pz[t] = pzw.x;
          pid[t] = tgt_copy_word(pzw.y) ? -1 : pid[t];  // a copy: its earlier twin is scanned
        }
#pragma unroll
        for (int t = 0; t < P; t++) {
          const double dx = px[t] - qx, dy = py[t] - qy, dz = pz[t] - qz;
          const double d2 = dx * dx + dy * dy + dz * dz;
          if (pid[t] >= 0) {
            if (d2 < best) {
              second = best;
              best = d2;
              bpos = pid[t];
            } else if (d2 < second) {
              second = d2;
            }
          }
        }
        wave_lds_fence();  // the list's reads are done before the next round rewrites it
      }
      const int nch = __builtin_popcount(kids);
      int tot;
      const int incl = wave_incl_scan(nch, &tot);
      if (tail + tot > kBBStack - kBBPts) {
        over = true;
        break;
      }
      wave_lds_fence();  // this step's pops are read before the pushes overwrite them
      int off = tail + incl - nch;
      uint32_t kk = kids;
      while (kk) {
        const uint32_t o = (uint32_t)__builtin_ctz(kk);
        kk &= kk - 1u;
        stack[off++] = topo.x + __builtin_popcount((meta & 0xffu) & ((1u << o) - 1u));
      }
      tail += tot;
      const double gb = wave_min_d(best);
      const double t2 = gb * (1.0 + kFastPrune);
      thr = t2 < thr ? t2 : thr;
      ++steps;
      wave_lds_fence();
    }
    wave_lds_fence();
    // again with the tighter bound (thr holds the best so far), while it shrinks
    if (!over || passes >= kBBPasses || !(thr < thr0)) break;
  }
  if (a.dbg && lane == 0) {
    atomicAdd(&a.dbg[27], 1ull);
    atomicAdd(&a.dbg[28], (unsigned long long)steps);
    if (over) atomicAdd(&a.dbg[37], 1ull);
  }
  if (over) return 0;
  // the wave's best, and its second: the smallest of the other lanes' bests and the best lane's
  // second (a best held by two lanes is its own second: a tie)
  const double gb = wave_min_d(best);
  const unsigned long long at = wballot(best == gb);
  const double gs = __popcll(at) > 1 ? gb : wave_min_d(best == gb ? second : best);
  const int32_t gp = (int32_t)__builtin_amdgcn_readlane(bpos, __builtin_ctzll(at ? at : 1ull));
  if (!certified(gb, gs, a.init_best)) return 2;
  if (lane == 0) {
    a.pos_out[i] = gp;
    a.dist_out[i] = __builtin_sqrt(gb);
  }
  return kBBDone;
}

__global__ void __launch_bounds__(64) k_nn_ball(NNLaunch a) {
  if (a.loop && a.loop->core.done) return;
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds_raw[];
  const int lane = threadIdx.x, g = lane / kBallGL, gl = lane % kBallGL, gbase = g * kBallGL;
  int32_t* stack = reinterpret_cast<int32_t*>(lds_raw) + g * kBallGStack;
  int32_t* plist = reinterpret_cast<int32_t*>(lds_raw) + kBallStack + g * kBallGPoints;
  // The exact list (queries the wave search could not certify): complete when this kernel starts,
  // one thread each, a DFS stack of `levels` entries per thread in LDS.
  {
    const unsigned n0 = a.fb_count[0];
    for (unsigned j = blockIdx.x * 64u + (unsigned)lane; j < n0; j += gridDim.x * 64u)
      exact_query(a, a.fb_list[j], lds_raw + lane, 64);
    wave_lds_fence();
  }
  // The follow-ups of the ball queries (a per-lane certified search, or the reference-order DFS)
  // are queued per wave and run 64 at a time, one query per lane with its own DFS stack column
  // (the exact list's layout), once the queue is nearly full and at the end. (One lane of the
  // query's group ran each inline before: 1 lane in 16 busy. On a dense 2.5-D scan early in a
  // registration the queries sit ~0.3 m off surfaces sampled every few mm, every ball overflows,
  // and that serial tail took 21 ms per iterate at 1M points.)
  int32_t* fq = reinterpret_cast<int32_t*>(reinterpret_cast<unsigned char*>(lds_raw) + a.ball_queue_off);
  double* fqu = reinterpret_cast<double*>(fq + 64);  // each entry's guess u (an upper bound, or inf)
  int qn = 0;  // wave-uniform
  // A per-lane search that exceeds kLaneBudget node visits is handed to the wave-cooperative
  // search (the whole wave on one query), one after the other once the lanes are done.
  auto flush = [&]() {
    wave_lds_fence();
    bool handed = false;
    int32_t e = 0;
    double qu = __builtin_inf();
    if (lane < qn) {
      e = fq[lane];
      qu = fqu[lane];
      const int64_t iq = e & 0x3fffffff;
      // an abandoned search's best so far (a point's fl(d2)) bounds the cooperative search
      double found = __builtin_inf();
      if ((e >> 30) == 1) handed = !lane_query(a, iq, lds_raw + lane, 64, kLaneBudget, &found, qu);
      else exact_query(a, iq, lds_raw + lane, 64);
      qu = found < qu ? found : qu;
    }
    wave_lds_fence();
    const unsigned long long handed_m = wballot(handed);
    if (a.dbg && lane == 0) atomicAdd(&a.dbg[29], (unsigned long long)__popcll(handed_m));
    for (unsigned long long hm = wballot(handed); hm; hm &= hm - 1) {
      const int k = __builtin_ctzll(hm);
      const int64_t iq = __builtin_amdgcn_readlane(e, k) & 0x3fffffff;
      const double uq = readlane_d(qu, k);
      // the stack in the DFS columns' area (free now); the fallback DFS after it, in the same area
      // the stack in the DFS columns' area (free now); a tie or an overflow: the reference-order
      // DFS on lane 0, in the same area
      if (wave_bb(a, iq, uq, reinterpret_cast<int32_t*>(lds_raw), lane) != kBBDone && lane == 0) {
        exact_query(a, iq, lds_raw, 1);
        atomicAdd(a.fb_count + 3, 1u);
        if (a.dbg) atomicAdd(&a.dbg[38], 1ull);
      }
      wave_lds_fence();
    }
    qn = 0;
    wave_lds_fence();
  };
  const unsigned cnt = a.fb_count[1];
  // Direct mode: each wave takes whole queries, one after the other, with all its lanes: the
  // cooperative search started from the cell tables of the query's bound (a few 64-node steps
  // instead of the 16-lane ball walk and the follow-ups after it). Used for a long list (over four
  // per wave: an unconverged registration on surface data, where most balls overflow) and after
  // the wide pass; the four-queries-per-wave ball walk takes the shorter lists, whose queries are
  // mostly easy. (Short lists, at most one query per wave, went to the direct mode too until r23:
  // since the flat leaf scans of r22 the ball walk settles them faster, config 3 6.2k -> 7.4k,
  // config 2 1.35k -> 1.41k Mcorr/s, profiles/r23/ab_ball_mode_configs23.txt.) Measured (profiles/r21/ab_ball_direct.txt): scene 10M 678 -> 1215 Mcorr/s,
  // scene 1M 624 -> 1254 (driver window), config 4 unchanged; direct at every size cost config
  // 4's window 4 % (its 15k-query lists of easy balls).
  // (icp_hip_config.ball_mode: 0 this rule, 1 the ball walk always, 2 direct always)
  if (a.ball_mode == 2 || (a.ball_mode == 0 && cnt > 4u * gridDim.x)) {
    // A query the cooperative search leaves (a tie, an overflow) is queued for the reference-order
    // DFS; the queue runs 64 at a time, one per lane, each with its DFS stack column in LDS (ties
    // come in numbers where both clouds sit on the LAS grid: the source's first iterate)
    unsigned taken = 0;
    int dq = 0;  // wave-uniform
    auto dfs_flush = [&]() {
      wave_lds_fence();
      if (lane < dq) exact_query(a, fq[lane], lds_raw + lane, 64);
      if (lane == 0) {
        atomicAdd(a.fb_count + 3, (unsigned)dq);
        if (a.dbg) atomicAdd(&a.dbg[38], (unsigned long long)dq);
      }
      dq = 0;
      wave_lds_fence();
    };
    for (unsigned j = blockIdx.x; j < cnt; j += gridDim.x, ++taken) {
      const int64_t i = a.fb_list2[j];
      const double u = a.fb_u2[j];
      if (wave_bb(a, i, u, reinterpret_cast<int32_t*>(lds_raw), lane) != kBBDone) {
        wave_lds_fence();
        if (lane == 0) fq[dq] = (int32_t)i;
        if (++dq == 64) dfs_flush();
      }
      wave_lds_fence();
    }
    if (dq > 0) dfs_flush();
    // the queries taken by the cooperative search count as follow-up searches, as after the ball
    // walk (icp_iter_stats.n_lane_search)
    if (lane == 0 && taken > 0) atomicAdd(a.fb_count + 2, taken);
    return;
  }
  for (unsigned j0 = blockIdx.x * kBallGroups; j0 < cnt; j0 += gridDim.x * kBallGroups) {
    const unsigned j = j0 + g;
    bool live = j < cnt;  // group-uniform
    int follow = 0;       // group-uniform: 1 the per-lane search, 2 the reference-order DFS
    int64_t i = 0;
    double u = 0.0, qx = 0.0, qy = 0.0, qz = 0.0;
    if (live) {
      i = a.fb_list2[j];
      u = a.fb_u2[j];
      qx = a.x[i];
      qy = a.y[i];
      qz = a.z[i];
      if (!(u <= 0x1p900)) {
        follow = 1;
        live = false;
      }
    }
    const double thr = u * (1.0 + kFastPrune);
    int tail = 0, npts = 0;
    bool overflow = false;
    wave_lds_fence();
    {
      // every point with fl(d2) <= thr lies in the box q +- r (see the wave search's radius)
      const double amax = __builtin_fmax(__builtin_fabs(qx), __builtin_fmax(__builtin_fabs(qy), __builtin_fabs(qz)));
      const double r = live ? __builtin_sqrt(thr) * (1.0 + 0x1p-40) + amax * 0x1p-45 : 0.0;
      if (a.cells) {
        const int t = cell_starts<kBallGL, 1>(a, qx - r, qy - r, qz - r, qx + r, qy + r, qz + r, gl, gbase, stack);
        tail = live ? t : 0;
      } else {
        if (gl == 0) stack[0] = 0;
        tail = live ? 1 : 0;
      }
    }
    wave_lds_fence();
    // LIFO batches of up to 16 nodes per group, sphere test s <= thr on the children
    while (wballot(tail > 0) != 0) {
      const int batch = tail < kBallGL ? tail : kBallGL;
      const bool has = gl < batch;
      bool leaf = false;
      int32_t first = 0;
      uint32_t meta = 0, kids = 0;
      if (has) {
        const NodeRec* rr = a.nodes + stack[tail - batch + gl];
        const int2 topo = *reinterpret_cast<const int2*>(&rr->first);
        first = topo.x;
        meta = (uint32_t)topo.y;
        leaf = (meta & kLeafBit) != 0;
        if (!leaf) kids = children_in_ball(rr, meta & 0xffu, qx, qy, qz, thr);
      }
      const int lcnt = (has && leaf) ? (int)(meta & ~kLeafBit) : 0;
      int ltot;
      const int lincl = row_incl_scan(lcnt, gbase, &ltot);
      const int lpos = npts + lincl - lcnt;
      if (lcnt > 0 && lpos + lcnt <= kBallGPoints)
        for (int c = 0; c < lcnt; c++) plist[lpos + c] = first + c;
      const int nch = __builtin_popcount(kids);
      int tot;
      const int incl = row_incl_scan(nch, gbase, &tot);
      if (tail > 0) {
        npts += ltot;
        tail -= batch;
        if (npts > kBallGPoints || tail + tot > kBallGStack) {
          overflow = true;
          tail = 0;
        } else {
          int off = tail + incl - nch;
          const uint32_t mask = meta & 0xffu;
          uint32_t kk = kids;
          while (kk) {
            const uint32_t o = (uint32_t)__builtin_ctz(kk);
            kk &= kk - 1u;
            stack[off++] = first + __builtin_popcount(mask & ((1u << o) - 1u));
          }
          tail += tot;
        }
      }
      wave_lds_fence();
    }
    if (a.dbg && gl == 0 && live) {
      atomicAdd(&a.dbg[14], overflow ? 1ull : 0ull);
      atomicAdd(&a.dbg[15], (unsigned long long)npts);
    }
    if (live && overflow) follow = 1;
    if (overflow) live = false;
    wave_lds_fence();
    double best = __builtin_inf(), second = __builtin_inf();
    int32_t bpos = 0x7fffffff;
    if (live) {
      for (int k = gl; k < npts; k += kBallGL) {
        const int32_t pg = plist[k];
        const TgtPt* p = a.pts + pg;
        const double2 xy = *reinterpret_cast<const double2*>(&p->x);
        const double dx = xy.x - qx, dy = xy.y - qy, dz = p->z - qz;
        const double d2 = dx * dx + dy * dy + dz * dz;
        if (d2 < best) {
          second = best;
          best = d2;
          bpos = pg;
        } else if (d2 < second) {
          second = d2;
        }
      }
    }
#pragma unroll
    for (int o = kBallGL / 2; o >= 1; o >>= 1) {
      const double ob = __shfl_xor(best, o, kWave);
      const double os = __shfl_xor(second, o, kWave);
      const int32_t op = __shfl_xor(bpos, o, kWave);
      const double lo_ = ob < best ? ob : best;
      const double hi_ = ob < best ? best : ob;
      const double ss = os < second ? os : second;
      second = hi_ < ss ? hi_ : ss;
      bpos = (ob < best || (ob == best && op < bpos)) ? op : bpos;
      best = lo_;
    }
    if (live) {
      if (!(best <= u)) {
        follow = 1;
      } else if (certified(best, second, a.init_best)) {
        if (gl == 0) {
          a.pos_out[i] = bpos;
          a.dist_out[i] = __builtin_sqrt(best);
        }
      } else {
        follow = 2;
      }
    }
    // queue the follow-ups (one entry per group: its leader lane)
    const bool fol = follow != 0 && gl == 0;
    const unsigned long long fm = wballot(fol);
    if (fol) {
      atomicAdd(a.fb_count + (follow == 1 ? 2 : 3), 1u);  // counted for the iteration record
      fq[qn + mask_rank(fm)] = (int32_t)i | (follow << 30);
      // an overflowing ball's guess bounds the nearest distance (a guess the ball did not cover
      // does not, nor does an unusable one)
      fqu[qn + mask_rank(fm)] = (overflow && u <= 0x1p900) ? u : __builtin_inf();
    }
    qn += __popcll(fm);
    if (qn > 64 - kBallGroups) flush();
    wave_lds_fence();
  }
  if (qn > 0) flush();
}

// ---------------------------------------------------------------------------------------------
// Separation of the target points (once per target): for every point p_j a lower bound S_j of its
// exact distance to every OTHER target point, stored in TgtPt::sep (fp32, rounded down; 0 when
// p_j has an exact duplicate). It turns the previous match into a certificate (k_nn_wave,
// icp_hip_config.certify_prev): a moved query q' with exact distance D* to its previous match p*
// has D(q', p) >= S - D* for every other point p (triangle inequality), so p* is the nearest with
// the reference's own certificate (nn_device.h) whenever (S - D*)^2 clears fl(d2(q', p*)) by the
// window. One thread per point (leaf order: neighbours in flight together), a branch-and-bound
// DFS for the nearest point other than itself: nearest child first, the remaining siblings of a
// level kept as one stack entry with a 16-bit lower-bound key (fast_dfs's encoding); a node is
// skipped when its squared box distance s exceeds the best (monotone rounding: every point inside
// has fl(d2) >= s), so the result is the exact minimum fl(d2) over the other points.
__global__ void __launch_bounds__(256) k_target_sep(const NodeRec* __restrict__ nodes, TgtPt* __restrict__ pts,
                                                    int64_t n) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sep_stack[];
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;  // no barriers below
  unsigned long long* st = sep_stack + threadIdx.x;
  const int bs = blockDim.x;
  const double2 qxy = *reinterpret_cast<const double2*>(&pts[j].x);
  const double qx = qxy.x, qy = qxy.y, qz = pts[j].z;
  double best = __builtin_inf();
  uint32_t thr_key = key16(best);
  int sp = 0;
  int32_t node = 0;
  double lx = nodes[0].lo[0], ly = nodes[0].lo[1], lz = nodes[0].lo[2];
  double hx = nodes[0].hi[0], hy = nodes[0].hi[1], hz = nodes[0].hi[2];
  double s = box_s(lx, ly, lz, hx, hy, hz, qx, qy, qz);
  while (true) {
    bool entered = false;
    if (!(s > best)) {
      const int2 topo = *reinterpret_cast<const int2*>(&nodes[node].first);
      const int32_t first = topo.x;
      const uint32_t meta = (uint32_t)topo.y;
      if (meta & kLeafBit) {
        const int32_t cnt = (int32_t)(meta & ~kLeafBit);
        for (int32_t k = 0; k < cnt; k++) {
          if ((int64_t)first + k == j) continue;
          const TgtPt* p = pts + first + k;
          const double2 pxy = *reinterpret_cast<const double2*>(&p->x);
          const double dx = pxy.x - qx, dy = pxy.y - qy, dz = p->z - qz;
          const double d2 = dx * dx + dy * dy + dz * dz;
          if (d2 < best) {
            best = d2;
            thr_key = key16(best);
          }
        }
      } else {
        const double mx = (lx + hx) / 2, my = (ly + hy) / 2, mz = (lz + hz) / 2;
        const double ax0 = smax(0.0, smax(lx - qx, qx - mx)), ax1 = smax(0.0, smax(mx - qx, qx - hx));
        const double ay0 = smax(0.0, smax(ly - qy, qy - my)), ay1 = smax(0.0, smax(my - qy, qy - hy));
        const double az0 = smax(0.0, smax(lz - qz, qz - mz)), az1 = smax(0.0, smax(mz - qz, qz - hz));
        const double sx[2] = {ax0 * ax0, ax1 * ax1};
        const double sy[2] = {ay0 * ay0, ay1 * ay1};
        const double sz[2] = {az0 * az0, az1 * az1};
        const uint32_t mask = meta & 0xffu;
        double bs_ = __builtin_inf();
        uint32_t o1 = 0;
#pragma unroll
        for (int o = 0; o < 8; o++) {
          const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
          const bool take = ((mask >> o) & 1u) && c < bs_;
          bs_ = take ? c : bs_;
          o1 = take ? (uint32_t)o : o1;
        }
        const uint32_t rem = mask & ~(1u << o1);
        uint32_t kmin = 0xffffu;
#pragma unroll
        for (int o = 0; o < 8; o++) {
          const double c = sx[o & 1] + sy[(o >> 1) & 1] + sz[o >> 2];
          const uint32_t kk = key16(c);
          kmin = ((rem >> o) & 1u) && kk < kmin ? kk : kmin;
        }
        if (rem) {
          st[sp * bs] = ((unsigned long long)kmin << 48) | ((unsigned long long)mask << 40) |
                        ((unsigned long long)rem << 32) | (uint32_t)first;
          sp++;
        }
        node = first + __builtin_popcount(mask & ((1u << o1) - 1u));
        if (o1 & 1u) lx = mx; else hx = mx;
        if (o1 & 2u) ly = my; else hy = my;
        if (o1 & 4u) lz = mz; else hz = mz;
        s = bs_;
        entered = true;
      }
    }
    if (entered) continue;
    bool found = false;
    while (sp > 0) {
      const unsigned long long e = st[(sp - 1) * bs];
      if ((uint32_t)(e >> 48) > thr_key) {  // key16 is monotone: every remaining child has s > best
        sp--;
        continue;
      }
      uint32_t rem = (uint32_t)(e >> 32) & 0xffu;
      const uint32_t pmask = (uint32_t)(e >> 40) & 0xffu;
      const int32_t first = (int32_t)(uint32_t)e;
      const uint32_t o = (uint32_t)__builtin_ctz(rem);
      rem &= rem - 1u;
      if (rem == 0) sp--;
      else st[(sp - 1) * bs] = (e & ~(0xffull << 32)) | ((unsigned long long)rem << 32);
      node = first + __builtin_popcount(pmask & ((1u << o) - 1u));
      const NodeRec* r = nodes + node;
      const double2 l01 = *reinterpret_cast<const double2*>(&r->lo[0]);
      const double2 l2h0 = *reinterpret_cast<const double2*>(&r->lo[2]);
      const double2 h12 = *reinterpret_cast<const double2*>(&r->hi[1]);
      lx = l01.x; ly = l01.y; lz = l2h0.x; hx = l2h0.y; hy = h12.x; hz = h12.y;
      s = box_s(lx, ly, lz, hx, hy, hz, qx, qy, qz);
      found = true;
      break;
    }
    if (!found) break;
  }
  // fl(d2) <= D^2 (1 + 5 2^-53), so D >= sqrt(best) (1 - 2^-50) (the fp64 sqrt within an ulp);
  // the fp32 conversion rounds by <= 2^-24, covered by the 2^-22 factor: sep <= D
  float sep = __builtin_inff();
  if (best < __builtin_inf()) sep = (float)(__builtin_sqrt(best) * ((1.0 - 0x1p-50) * (1.0 - 0x1p-22)));
  if (!(sep >= 0.0f)) sep = 0.0f;
  pts[j].sep = sep;
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

int nn_block_threads(int levels) {
  // LDS stack of the per-thread kernels: levels x threads x 8 B. Keep <= 64 KiB per block.
  if (levels <= 32) return 256;
  if (levels <= 64) return 128;
  return 64;
}

hipError_t launch_target_sep(const NodeRec* nodes, TgtPt* pts, int64_t n, int levels, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int lv = levels < 1 ? 1 : levels;
  const int bs = nn_block_threads(lv);
  const size_t shmem = (size_t)lv * bs * sizeof(unsigned long long);
  hipLaunchKernelGGL(k_target_sep, dim3(grid_for(n, bs)), dim3(bs), shmem, s, nodes, pts, n);
  return hipGetLastError();
}

hipError_t launch_nn(const NNLaunch& a, hipStream_t s) {
  if (a.n <= 0) return hipSuccess;
  const int levels = a.levels < 1 ? 1 : a.levels;
  const int bs = nn_block_threads(levels);
  size_t shmem = (size_t)levels * bs * sizeof(unsigned long long);
  if (shmem < 1024) shmem = 1024;  // also hosts the block reduction
  const unsigned grid = grid_for(a.n, bs);
  if (a.search == ICP_SEARCH_REFERENCE || a.count) {
    if (a.ev_start) (void)hipEventRecord(a.ev_start, s);
    if (a.apply) {
      if (a.count) hipLaunchKernelGGL((k_nn_ref<true, true>), dim3(grid), dim3(bs), shmem, s, a);
      else hipLaunchKernelGGL((k_nn_ref<true, false>), dim3(grid), dim3(bs), shmem, s, a);
    } else {
      if (a.count) hipLaunchKernelGGL((k_nn_ref<false, true>), dim3(grid), dim3(bs), shmem, s, a);
      else hipLaunchKernelGGL((k_nn_ref<false, false>), dim3(grid), dim3(bs), shmem, s, a);
    }
    if (a.ev_fast_done) (void)hipEventRecord(a.ev_fast_done, s);
    return hipGetLastError();
  }
  // wave search -> ball search -> per-lane search / exact DFS
  const unsigned wgrid = grid_for(a.n, 256);
  const size_t wshm = (size_t)(256 / 64) * kWaveLds;
  // The timing events ride on the search's own dispatch packet (no marker packets between
  // kernels). An event on a dispatch delays the next kernel by ~3-5 us (its start event carried
  // by the next kernel's dispatch instead measured no better), so the context times only every
  // config.timing_stride-th iterate (null events: plain launches).
  auto wave = [&](auto kern) {
    hipExtLaunchKernelGGL(kern, dim3(wgrid), dim3(256), (uint32_t)wshm, s, a.ev_start, a.ev_fast_done, 0u, a);
  };
  // the previous-match certificate only where it can apply (an iterate after a search)
  const bool cert = a.certify_prev != 0 && a.have_prev;
  // instances: transform, scan groups, certificate, debug counters
  auto pick = [&](auto cert_c, auto dbg_c) -> hipError_t {
    constexpr bool C = decltype(cert_c)::value, D = decltype(dbg_c)::value;
    // the cache instance where every joined wave reuses or stores (an iterate after a search)
    const bool wc = ICP_WALK_STREAM && a.apply && a.wc_box != nullptr && a.have_prev;
    // the instance without the cache for a source's first iterate (its walking waves store
    // nothing; a record is reused only after a search)
    const bool nc = ICP_FIRST_NC && !a.apply && !a.have_prev;
    switch ((wc ? 16 : 0) + (nc ? 32 : 0) + (a.apply ? 8 : 0) + a.scan_groups) {
      case 25: wave(k_nn_wave<true, 1, C, D, 1>); break;
      case 26: wave(k_nn_wave<true, 2, C, D, 1>); break;
      case 28: wave(k_nn_wave<true, 4, C, D, 1>); break;
      case 9: wave(k_nn_wave<true, 1, C, D, 0>); break;
      case 10: wave(k_nn_wave<true, 2, C, D, 0>); break;
      case 12: wave(k_nn_wave<true, 4, C, D, 0>); break;
      case 33: wave(k_nn_wave<false, 1, C, D, 2>); break;
      case 34: wave(k_nn_wave<false, 2, C, D, 2>); break;
      case 36: wave(k_nn_wave<false, 4, C, D, 2>); break;
      case 1: wave(k_nn_wave<false, 1, C, D, 0>); break;
      case 2: wave(k_nn_wave<false, 2, C, D, 0>); break;
      case 4: wave(k_nn_wave<false, 4, C, D, 0>); break;
      default: return hipErrorInvalidValue;
    }
    return hipSuccess;
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const bool dbg = a.dbg != nullptr;
  const hipError_t pe = cert ? (dbg ? pick(T_{}, T_{}) : pick(T_{}, F_{})) : (dbg ? pick(F_{}, T_{}) : pick(F_{}, F_{}));
  if (pe != hipSuccess) return pe;
  // the half pass over the overflowed waves (queries already moved: no transform, no cache)
  if (a.fb_list3) {
    NNLaunch h = a;
    h.apply = 0;
    h.wc_box = nullptr;
    h.wc_ents = nullptr;
    const int64_t halves = (a.n + 31) / 32;
    const int64_t hb = (halves + 3) / 4;
    const unsigned hgrid = (unsigned)(hb < 2048 ? hb : 2048);  // about one resident block per slot
    auto half = [&](auto kern) {
      hipExtLaunchKernelGGL(kern, dim3(hgrid), dim3(256), (uint32_t)wshm, s, nullptr, nullptr, 0u, h);
    };
    switch (a.scan_groups + (dbg ? 8 : 0)) {
      case 1: half(k_nn_half<1, false>); break;
      case 2: half(k_nn_half<2, false>); break;
      case 4: half(k_nn_half<4, false>); break;
      case 9: half(k_nn_half<1, true>); break;
      case 10: half(k_nn_half<2, true>); break;
      case 12: half(k_nn_half<4, true>); break;
      default: return hipErrorInvalidValue;
    }
  }
  // the wide pass over the overflowed waves and halves (queries already moved: no transform)
  if (a.fb_list4) {
    NNLaunch w = a;
    w.apply = 0;
    w.wc_box = nullptr;
    w.wc_ents = nullptr;
    const int64_t wb = (a.n + 255) / 256;
    const unsigned ggrid = (unsigned)(wb < 2048 ? wb : 2048);
    const size_t gshm = (size_t)(256 / 64) * kWideLds;
    auto wide = [&](auto kern) {
      hipExtLaunchKernelGGL(kern, dim3(ggrid), dim3(256), (uint32_t)gshm, s, nullptr, nullptr, 0u, w);
    };
    switch (a.scan_groups + (dbg ? 8 : 0)) {
      case 1: wide(k_nn_wide<1, false>); break;
      case 2: wide(k_nn_wide<2, false>); break;
      case 4: wide(k_nn_wide<4, false>); break;
      case 9: wide(k_nn_wide<1, true>); break;
      case 10: wide(k_nn_wide<2, true>); break;
      case 12: wide(k_nn_wide<4, true>); break;
      default: return hipErrorInvalidValue;
    }
  }
  // the follow-up lists are short (the ball list ~0.1 % of the queries, the exact list usually
  // empty): one launch of 64-thread blocks, grid-stride over them; LDS for the group stacks and
  // lists or, before them, one DFS stack of `levels` entries per thread
  const int64_t bq = (a.n + kBallGroups - 1) / kBallGroups;
  size_t bshm = (size_t)levels * 64 * sizeof(unsigned long long);
  if (bshm < (size_t)kBallLdsBytes) bshm = kBallLdsBytes;
  NNLaunch b = a;
  if (bshm < (size_t)kBBStack * sizeof(int32_t)) bshm = (size_t)kBBStack * sizeof(int32_t);  // wave_bb's stack
  b.ball_queue_off = (int32_t)bshm;  // the follow-up queue (64 entries + guesses) after the stacks and lists
  // after the wide pass the list holds what it left: far queries (lanes that joined no box, and
  // lanes the wide pass could not certify, with its bounds): whole queries per wave
  if (a.fb_list4 && b.ball_mode == 0) b.ball_mode = 2;
  bshm += 64 * (sizeof(int32_t) + sizeof(double));
  hipExtLaunchKernelGGL(k_nn_ball, dim3((unsigned)(bq < 8192 ? bq : 8192)), dim3(64), (uint32_t)bshm, s, nullptr,
                        nullptr, 0u, b);
  return hipGetLastError();
}

}  // namespace icp

#if ICP_PHASE_STOP
extern "C" int icp_hip_debug_phase_stop(int k) {
  return hipMemcpyToSymbol(HIP_SYMBOL(icp::g_phase_stop), &k, sizeof k) == hipSuccess ? 0 : -1;
}
#endif
