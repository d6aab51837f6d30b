// query_order_gpu.hip — the kd query order of query_order.cpp, built on the device.
//
// The host partition splits a range of n > bucket queries at h = n/2 rounded up to a multiple of
// 64 (of `bucket` inside a wave's 64), on the longest axis of the range's bounding box, with
// nth_element. The split positions depend on the sizes only, so every level of the recursion is a
// fixed list of segments: the host lays the segments out level by level, and per level the device
//   1. takes each splitting segment's bounding box (one workgroup per segment, fp32: the axis
//      choice needs no exact extent) and picks its longest axis;
//   2. keys every query with (segment start << 32 | order-preserving fp32 key of its coordinate on
//      the segment's axis) and radix-sorts the permutation by it (hipCUB, stable): every
//      segment ends up sorted along its axis, so its first h queries are its h smallest, which is
//      what nth_element guarantees.
// Finished segments (size <= bucket) keep their place (their start is their key). ~20 levels at
// 10M. Any kd partition gives the same correspondences (the search is exact); this one has the
// host order's bucket geometry. Non-finite coordinates count as 0, as on the host.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "query_order.h"

namespace icp {

namespace {

__device__ __forceinline__ float coord32(double v) { return __builtin_isfinite(v) ? (float)v : 0.0f; }

__device__ __forceinline__ uint32_t okey(float f) {  // order-preserving (non-NaN floats)
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

constexpr int32_t kChunk = 16384;  // segments larger than this take their box from chunks

// block-wide min/max of 3 lo + 3 hi floats into red[6][blockDim/64]; thread 0 gets the results
__device__ __forceinline__ void block_box(float lo[3], float hi[3], float (*red)[4]) {
#pragma unroll
  for (int a = 0; a < 3; a++) {
    for (int o = 32; o >= 1; o >>= 1) {
      const float l = __shfl_xor(lo[a], o, 64), h = __shfl_xor(hi[a], o, 64);
      lo[a] = l < lo[a] ? l : lo[a];
      hi[a] = h > hi[a] ? h : hi[a];
    }
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0)
    for (int a = 0; a < 3; a++) {
      red[a][w] = lo[a];
      red[3 + a][w] = hi[a];
    }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int a = 0; a < 3; a++) {
      float l = red[a][0], h = red[3 + a][0];
      for (int q = 1; q < nw; q++) {
        l = red[a][q] < l ? red[a][q] : l;
        h = red[3 + a][q] > h ? red[3 + a][q] : h;
      }
      lo[a] = l;
      hi[a] = h;
    }
  }
}

__device__ __forceinline__ uint8_t longest_axis(const float lo[3], const float hi[3]) {
  int ax = 0;
  for (int a = 1; a < 3; a++)
    if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
  return (uint8_t)ax;
}

// Big segments: the box of each chunk of kChunk slots (one workgroup each) ...
__global__ void __launch_bounds__(256) k_chunk_bbox(const double* __restrict__ xyz, const int32_t* __restrict__ perm,
                                                    const int32_t* __restrict__ cstart, const int32_t* __restrict__ clen,
                                                    float* __restrict__ cbox) {
  __shared__ float red[6][4];
  const int c = blockIdx.x;
  const int32_t s0 = cstart[c], n = clen[c];
  float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int32_t k = threadIdx.x; k < n; k += blockDim.x) {
    const int64_t j = perm[s0 + k];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const float v = coord32(xyz[3 * j + a]);
      lo[a] = v < lo[a] ? v : lo[a];
      hi[a] = v > hi[a] ? v : hi[a];
    }
  }
  block_box(lo, hi, red);
  if (threadIdx.x == 0)
    for (int a = 0; a < 3; a++) {
      cbox[6 * c + a] = lo[a];
      cbox[6 * c + 3 + a] = hi[a];
    }
}

// ... then each big segment's axis from its chunks' boxes (one thread per big segment).
__global__ void k_big_axis(const float* __restrict__ cbox, const int32_t* __restrict__ bseg,
                           const int32_t* __restrict__ bfirst, int nbig, uint8_t* __restrict__ axis) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nbig) return;
  float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int c = bfirst[b]; c < bfirst[b + 1]; c++)
    for (int a = 0; a < 3; a++) {
      lo[a] = cbox[6 * c + a] < lo[a] ? cbox[6 * c + a] : lo[a];
      hi[a] = cbox[6 * c + 3 + a] > hi[a] ? cbox[6 * c + 3 + a] : hi[a];
    }
  axis[bseg[b]] = longest_axis(lo, hi);
}

// One workgroup per segment: the longest axis of its bounding box (ties: the lower axis, as the
// host's strict > scan).
__global__ void __launch_bounds__(256) k_seg_axis(const double* __restrict__ xyz, const int32_t* __restrict__ perm,
                                                  const int32_t* __restrict__ starts,
                                                  const int32_t* __restrict__ sizes, int bucket,
                                                  uint8_t* __restrict__ axis) {
  __shared__ float red[6][4];
  const int seg = blockIdx.x;
  const int32_t s0 = starts[seg], sz = sizes[seg];
  if (sz > kChunk) return;  // a big segment: the chunk path (k_chunk_bbox, k_big_axis)
  if (sz <= bucket) {  // finished: never split again
    if (threadIdx.x == 0) axis[seg] = 0;
    return;
  }
  float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
  float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
  for (int32_t k = threadIdx.x; k < sz; k += blockDim.x) {
    const int64_t j = perm[s0 + k];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      const float v = coord32(xyz[3 * j + a]);
      lo[a] = v < lo[a] ? v : lo[a];
      hi[a] = v > hi[a] ? v : hi[a];
    }
  }
  block_box(lo, hi, red);
  if (threadIdx.x == 0) axis[seg] = longest_axis(lo, hi);
}

// Sort key of every slot: its segment's start (high word) and its coordinate on that segment's axis.
__global__ void k_seg_keys(const double* __restrict__ xyz, const int32_t* __restrict__ perm,
                           const int32_t* __restrict__ starts, int nseg, const uint8_t* __restrict__ axis,
                           int64_t n, uint64_t* __restrict__ keys) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  int lo = 0, hi = nseg;  // the last segment with start <= k
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (starts[mid] <= k) lo = mid;
    else hi = mid;
  }
  const int64_t j = perm[k];
  keys[k] = ((uint64_t)(uint32_t)starts[lo] << 32) | okey(coord32(xyz[3 * j + axis[lo]]));
}

__global__ void k_iota(int32_t* p, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) p[k] = (int32_t)k;
}

inline unsigned grid_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// The host recursion's split position (query_order.cpp: multiples of 64 while the range is
// larger than a wave, of `bucket` inside it).
inline int64_t split_at(int64_t n, int bucket) {
  const int64_t unit = n > 64 ? 64 : bucket;
  int64_t h = ((n / 2 + unit - 1) / unit) * unit;
  if (h >= n) h = n - unit;
  return h;
}

#define QO_TRY(expr)                     \
  do {                                   \
    hipError_t e_ = (expr);              \
    if (e_ != hipSuccess) {              \
      err = e_;                          \
      goto done;                         \
    }                                    \
  } while (0)

}  // namespace

hipError_t gpu_kd_query_order(const double* d_xyz, int64_t n, int bucket, int32_t* d_perm, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n > 0x7fffffff || bucket < 1 || 64 % bucket != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n, 256)), dim3(256), 0, s, d_perm, n);
  if (n <= bucket) return hipGetLastError();
  // the levels of the recursion: every segment, in position order
  std::vector<std::vector<int32_t>> lv_start, lv_size;
  {
    std::vector<int32_t> st{0}, sz{(int32_t)n};
    while (true) {
      bool splits = false;
      for (int32_t v : sz) splits = splits || v > bucket;
      if (!splits) break;
      lv_start.push_back(st);
      lv_size.push_back(sz);
      std::vector<int32_t> st2, sz2;
      st2.reserve(st.size() * 2);
      sz2.reserve(st.size() * 2);
      for (size_t k = 0; k < st.size(); k++) {
        if (sz[k] > bucket) {
          const int32_t h = (int32_t)split_at(sz[k], bucket);
          st2.push_back(st[k]);
          sz2.push_back(h);
          st2.push_back(st[k] + h);
          sz2.push_back(sz[k] - h);
        } else {
          st2.push_back(st[k]);
          sz2.push_back(sz[k]);
        }
      }
      st.swap(st2);
      sz.swap(sz2);
    }
  }
  hipError_t err = hipSuccess;
  size_t max_seg = 0;
  for (const auto& v : lv_start) max_seg = std::max(max_seg, v.size());
  int32_t *d_starts = nullptr, *d_sizes = nullptr, *perm_alt = nullptr;
  uint8_t* d_axis = nullptr;
  uint64_t *keys = nullptr, *keys_alt = nullptr;
  void* d_chunks = nullptr;  // chunk boxes + chunk / big-segment tables
  size_t chunk_cap = 0;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  int sbits = 1;
  while (((int64_t)1 << sbits) <= n) sbits++;
  const int end_bit = 32 + sbits;
  QO_TRY(hipMalloc(reinterpret_cast<void**>(&d_starts), max_seg * sizeof(int32_t)));
  QO_TRY(hipMalloc(reinterpret_cast<void**>(&d_sizes), max_seg * sizeof(int32_t)));
  QO_TRY(hipMalloc(reinterpret_cast<void**>(&d_axis), max_seg));
  QO_TRY(hipMalloc(reinterpret_cast<void**>(&perm_alt), (size_t)n * sizeof(int32_t)));
  QO_TRY(hipMalloc(reinterpret_cast<void**>(&keys), (size_t)n * sizeof(uint64_t)));
  QO_TRY(hipMalloc(reinterpret_cast<void**>(&keys_alt), (size_t)n * sizeof(uint64_t)));
  QO_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys, keys_alt, d_perm, perm_alt, (int)n, 0,
                                            end_bit, s));
  QO_TRY(hipMalloc(&tmp, tmp_bytes));
  for (size_t L = 0; L < lv_start.size(); L++) {
    const int nseg = (int)lv_start[L].size();
    QO_TRY(hipMemcpyAsync(d_starts, lv_start[L].data(), nseg * sizeof(int32_t), hipMemcpyHostToDevice, s));
    QO_TRY(hipMemcpyAsync(d_sizes, lv_size[L].data(), nseg * sizeof(int32_t), hipMemcpyHostToDevice, s));
    {
      // big segments (the top levels): their boxes from chunks of kChunk slots, many workgroups each
      std::vector<int32_t> cst, cln, bseg, bfirst{0};
      for (int k = 0; k < nseg; k++) {
        if (lv_size[L][k] <= kChunk) continue;
        for (int32_t o = 0; o < lv_size[L][k]; o += kChunk) {
          cst.push_back(lv_start[L][k] + o);
          cln.push_back(std::min(kChunk, lv_size[L][k] - o));
        }
        bseg.push_back(k);
        bfirst.push_back((int32_t)cst.size());
      }
      if (!bseg.empty()) {
        const size_t nc = cst.size(), nb = bseg.size();
        if (nc > chunk_cap) {
          if (d_chunks) (void)hipFree(d_chunks);
          d_chunks = nullptr;
          chunk_cap = nc;
          QO_TRY(hipMalloc(reinterpret_cast<void**>(&d_chunks), chunk_cap * (6 * sizeof(float) + 3 * sizeof(int32_t)) +
                                                                 2 * sizeof(int32_t)));
        }
        float* cbox = reinterpret_cast<float*>(d_chunks);
        int32_t* ci = reinterpret_cast<int32_t*>(cbox + 6 * chunk_cap);
        QO_TRY(hipMemcpyAsync(ci, cst.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, s));
        QO_TRY(hipMemcpyAsync(ci + chunk_cap, cln.data(), nc * sizeof(int32_t), hipMemcpyHostToDevice, s));
        QO_TRY(hipMemcpyAsync(ci + 2 * chunk_cap, bseg.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice, s));
        QO_TRY(hipMemcpyAsync(ci + 2 * chunk_cap + nb, bfirst.data(), (nb + 1) * sizeof(int32_t),
                              hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_chunk_bbox, dim3((unsigned)nc), dim3(256), 0, s, d_xyz, d_perm, ci, ci + chunk_cap, cbox);
        hipLaunchKernelGGL(k_big_axis, dim3(grid_for((int64_t)nb, 64)), dim3(64), 0, s, cbox, ci + 2 * chunk_cap,
                           ci + 2 * chunk_cap + nb, (int)nb, d_axis);
        QO_TRY(hipGetLastError());
        QO_TRY(hipStreamSynchronize(s));  // the host tables are read by the copies above
      }
    }
    const int32_t big = *std::max_element(lv_size[L].begin(), lv_size[L].end());
    const int bs = big <= 128 ? 64 : 256;  // deep levels: one wave per (small) segment
    hipLaunchKernelGGL(k_seg_axis, dim3((unsigned)nseg), dim3(bs), 0, s, d_xyz, d_perm, d_starts, d_sizes, bucket,
                       d_axis);
    hipLaunchKernelGGL(k_seg_keys, dim3(grid_for(n, 256)), dim3(256), 0, s, d_xyz, d_perm, d_starts, nseg, d_axis, n,
                       keys);
    QO_TRY(hipGetLastError());
    QO_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys_alt, d_perm, perm_alt, (int)n, 0, end_bit,
                                              s));
    QO_TRY(hipMemcpyAsync(d_perm, perm_alt, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToDevice, s));
    // the host tables of this level are read by the copies above: finish before they are reused
    QO_TRY(hipStreamSynchronize(s));
  }
done:
  (void)hipStreamSynchronize(s);
  for (void* p : {(void*)d_starts, (void*)d_sizes, (void*)d_axis, (void*)perm_alt, (void*)keys, (void*)keys_alt, tmp,
                  d_chunks})
    if (p) (void)hipFree(p);
  return err;
}

}  // namespace icp
