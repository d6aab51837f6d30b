// fetch_calib.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths of
// the search kernel (k_nn_wave), on gfx950. MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for
// 16-B-per-lane coalesced streaming reads (it reports half the bytes); the search kernel's reads
// are 8-B-per-lane streams (source x/y/z, previous residual) and gathers of 24 of the 32 B of a
// target point record and 56 of the 64 B of a node record. Each pattern below touches every byte
// of a 2 GiB array exactly once (8x the 256 MiB Infinity Cache), in an order that gives no line
// two separate fetches, so the true HBM bytes per dispatch are the array size; the ratio to the
// counter is the correction for that pattern.
//
// usage: fetch_calib [reps]   -> one JSON line per pattern: name, bytes per dispatch, ms
// build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                              \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

// odd multiplier mod 2^k: a bijection of the block ids that sends neighbours far apart
__device__ __forceinline__ uint64_t scramble(uint64_t b, uint64_t nblk_mask) {
  return (b * 0x9E3779B97F4A7C15ull) & nblk_mask;
}

// 16 B per lane, coalesced (the guide's calibrated case)
__global__ void k_stream16(const double2* __restrict__ a, int64_t n, double* __restrict__ sink) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double2 v = a[i];
  if (v.x == 12345.678) sink[0] = v.y;  // never true for the zero-filled array
}

// 8 B per lane, coalesced (source x/y/z, residual reads of the search)
__global__ void k_stream8(const double* __restrict__ a, int64_t n, double* __restrict__ sink) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = a[i];
  if (v == 12345.678) sink[0] = v;
}

// Target-point gathers: 32-B records, 8 consecutive records (one 256-B run, a leaf's points)
// per group of 8 lanes, runs in scrambled order; each lane loads xy (16 B) + z (8 B) as the scan.
struct Rec32 {
  double x, y, z;
  int32_t orig, pad;
};
__global__ void k_gather32(const Rec32* __restrict__ a, int64_t nrec, uint64_t nblk_mask, double* __restrict__ sink) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nrec) return;
  const uint64_t blk = scramble((uint64_t)t >> 3, nblk_mask);
  const Rec32* p = a + (blk << 3) + (t & 7);
  const double2 xy = *reinterpret_cast<const double2*>(&p->x);
  const double z = p->z;
  if (xy.x + xy.y + z == 12345.678) sink[0] = z;
}

// Node gathers: 64-B records, 4 consecutive records per group of 4 lanes (256 B), scrambled
// order; each lane loads lo[0..1], lo[2] hi[0], hi[1..2] (3 x 16 B) + first/meta (8 B).
struct Rec64 {
  double lo[3], hi[3];
  int32_t first;
  uint32_t meta;
  int32_t depth, pad;
};
__global__ void k_gather64(const Rec64* __restrict__ a, int64_t nrec, uint64_t nblk_mask, double* __restrict__ sink) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nrec) return;
  const uint64_t blk = scramble((uint64_t)t >> 2, nblk_mask);
  const Rec64* r = a + (blk << 2) + (t & 3);
  const double2 l01 = *reinterpret_cast<const double2*>(&r->lo[0]);
  const double2 l2h0 = *reinterpret_cast<const double2*>(&r->lo[2]);
  const double2 h12 = *reinterpret_cast<const double2*>(&r->hi[1]);
  const int2 topo = *reinterpret_cast<const int2*>(&r->first);
  if (l01.x + l01.y + l2h0.x + l2h0.y + h12.x + h12.y == 12345.678 || topo.x == 0x7fffffff) sink[0] = 1.0;
}

// 8-B and 4-B coalesced stores (residual and match position writes)
__global__ void k_store8(double* __restrict__ a, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = (double)i;
}
__global__ void k_store4(int32_t* __restrict__ a, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = (int32_t)i;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  const size_t bytes = (size_t)2 << 30;  // 2 GiB
  void* buf = nullptr;
  double* sink = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 0, bytes));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int bs = 256;
  auto run = [&](const char* name, auto launch) {
    for (int r = 0; r < reps; r++) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("{\"pattern\": \"%s\", \"rep\": %d, \"bytes\": %zu, \"ms\": %.4f, \"gbs\": %.1f}\n", name, r, bytes, ms,
                  bytes / (ms * 1e-3) / 1e9);
    }
  };
  {
    const int64_t n = (int64_t)(bytes / 16);
    run("k_stream16", [&] { hipLaunchKernelGGL(k_stream16, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, 0, (const double2*)buf, n, sink); });
  }
  {
    const int64_t n = (int64_t)(bytes / 8);
    run("k_stream8", [&] { hipLaunchKernelGGL(k_stream8, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, 0, (const double*)buf, n, sink); });
  }
  {
    const int64_t n = (int64_t)(bytes / 32);
    const uint64_t mask = (uint64_t)(n >> 3) - 1;
    run("k_gather32", [&] { hipLaunchKernelGGL(k_gather32, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, 0, (const Rec32*)buf, n, mask, sink); });
  }
  {
    const int64_t n = (int64_t)(bytes / 64);
    const uint64_t mask = (uint64_t)(n >> 2) - 1;
    run("k_gather64", [&] { hipLaunchKernelGGL(k_gather64, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, 0, (const Rec64*)buf, n, mask, sink); });
  }
  {
    const int64_t n = (int64_t)(bytes / 8);
    run("k_store8", [&] { hipLaunchKernelGGL(k_store8, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, 0, (double*)buf, n); });
  }
  {
    const int64_t n = (int64_t)(bytes / 4);
    run("k_store4", [&] { hipLaunchKernelGGL(k_store4, dim3((unsigned)((n + bs - 1) / bs)), dim3(bs), 0, 0, (int32_t*)buf, n); });
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
