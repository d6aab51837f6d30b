// mfma_probe.hip — does the wave search's fp32 distance scan belong on the matrix cores?
//
//  1. the lane layout of v_mfma_f32_4x4x1_16b_f32 (A, B, C/D of each 4x4 block);
//  2. four chained 4x4x1 MFMAs (C = |q|^2, then + x(-2qx), + y(-2qy), + z(-2qz), + w) against the
//     fmaf chain in the same order, bit for bit;
//  3. issue cost of one scan step (4 points per lane, 64 lanes) in three forms, many waves per
//     SIMD, the two-smallest selection included: the packed-VALU form of nn_kernels.hip (two eval2),
//     the 4x4x1 MFMA form, and one 16x16x4 MFMA (256 pairs) with a 4-value selection.
//
// build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 -o tools/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void k_layout(float* out) {
  const int l = threadIdx.x;
  const float a = (float)(l + 1), b = (float)(1000 + l);
  f4 c = {0.f, 0.f, 0.f, 0.f};
  f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; r++) out[l * 4 + r] = d[r];
}

// lane l: point (l & 3) of a step (x, y, z, w = |p|^2 fmaf), query = the lane's own
__global__ void k_chain(const float* px, const float* q, unsigned* bad, float* outm, float* outf) {
  const int l = threadIdx.x, t = blockIdx.x;
  const float* P = px + t * 16;  // 4 points x (x, y, z)
  const float* Q = q + t * 192;  // 64 queries x (x, y, z)
  const float qx = Q[3 * l], qy = Q[3 * l + 1], qz = Q[3 * l + 2];
  const float qq = __builtin_fmaf(qz, qz, __builtin_fmaf(qy, qy, qx * qx));
  const int i = l & 3;
  const float x = P[4 * i], y = P[4 * i + 1], z = P[4 * i + 2];
  const float w = __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x));
  f4 c = {qq, qq, qq, qq};
  f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(x, -2.f * qx, c, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_4x4x1f32(y, -2.f * qy, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_4x4x1f32(z, -2.f * qz, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_4x4x1f32(w, 1.f, d, 0, 0, 0);
  for (int r = 0; r < 4; r++) {
    const float X = P[4 * r], Y = P[4 * r + 1], Z = P[4 * r + 2];
    const float W = __builtin_fmaf(Z, Z, __builtin_fmaf(Y, Y, X * X));
    float f = __builtin_fmaf(X, -2.f * qx, qq);
    f = __builtin_fmaf(Y, -2.f * qy, f);
    f = __builtin_fmaf(Z, -2.f * qz, f);
    f = __builtin_fmaf(W, 1.f, f);
    outm[(t * 64 + l) * 4 + r] = d[r];
    outf[(t * 64 + l) * 4 + r] = f;
    if (__float_as_uint(f) != __float_as_uint(d[r])) atomicAdd(bad, 1u);
  }
}

constexpr int kPts = 256;  // staged points per wave (LDS), cycled

// the packed-VALU scan of nn_kernels.hip: 2 pairs (4 points) per step
__global__ void __launch_bounds__(256) k_valu(const float* pts, int steps, float* out) {
  __shared__ float st[4][kPts * 4];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int k = l; k < kPts * 4; k += 64) st[wv][k] = pts[k];
  __syncthreads();
  const float qx = pts[l], qy = pts[l + 64], qz = pts[l + 128];
  const f2 qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
  uint32_t kmask = ~63u;
  asm volatile("" : "+v"(kmask));
  float k1 = __builtin_inff(), k2 = __builtin_inff();
  const v4i* s4 = reinterpret_cast<const v4i*>(st[wv]);
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
    const float kb = __uint_as_float((__float_as_uint(sq.y) & kmask) | (uint32_t)__builtin_amdgcn_readfirstlane((int)(sl + 1u)));
    sel2(ka, kb);
  };
#pragma unroll 1
  for (int s = 0; s < steps; s++) {
    const int b = (2 * s) & (kPts / 2 - 1);
    eval2(s4[2 * b], s4[2 * b + 1], (uint32_t)(4 * s) & 63u);
    eval2(s4[2 * b + 2], s4[2 * b + 3], (uint32_t)(4 * s + 2) & 63u);
  }
  out[blockIdx.x * 256 + threadIdx.x] = k1 + k2;
}

// 4x4x1 MFMA form: lane l reads point (l & 3) of the step (x, y, z, w), 4 chained MFMAs
__global__ void __launch_bounds__(256) k_mfma4(const float* pts, int steps, float* out) {
  __shared__ f4 st[4][kPts];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int k = l; k < kPts; k += 64) st[wv][k] = f4{pts[4 * k], pts[4 * k + 1], pts[4 * k + 2], pts[4 * k + 3]};
  __syncthreads();
  const float qx = pts[l], qy = pts[l + 64], qz = pts[l + 128];
  const float bx = -2.f * qx, by = -2.f * qy, bz = -2.f * qz;
  const float qq = __builtin_fmaf(qz, qz, __builtin_fmaf(qy, qy, qx * qx));
  const f4 c = {qq, qq, qq, qq};
  uint32_t kmask = ~63u;
  asm volatile("" : "+v"(kmask));
  float k1 = __builtin_inff(), k2 = __builtin_inff();
  auto sel2 = [&](float ka, float kb) {
    float m;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(k1), "v"(ka), "v"(kb));
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(k1) : "v"(k1), "v"(ka), "v"(kb));
    asm("v_min_f32 %0, %1, %2" : "=v"(k2) : "v"(m), "v"(k2));
  };
  const int i = l & 3;
#pragma unroll 1
  for (int s = 0; s < steps; s++) {
    const f4 p = st[wv][((4 * s) & (kPts - 1)) + i];
    f4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(p.x, bx, c, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(p.y, by, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(p.z, bz, d, 0, 0, 0);
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(p.w, 1.f, d, 0, 0, 0);
    const uint32_t sl = (uint32_t)(4 * s) & 63u;
    auto sg = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };  // scalar operands
    const float ka = __uint_as_float((__float_as_uint(d[0]) & kmask) | sg(sl));
    const float kb = __uint_as_float((__float_as_uint(d[1]) & kmask) | sg(sl + 1u));
    const float kc = __uint_as_float((__float_as_uint(d[2]) & kmask) | sg(sl + 2u));
    const float kd = __uint_as_float((__float_as_uint(d[3]) & kmask) | sg(sl + 3u));
    sel2(ka, kb);
    sel2(kc, kd);
  }
  out[blockIdx.x * 256 + threadIdx.x] = k1 + k2;
}

// 16x16x4 form: one MFMA per 256 pairs (16 points x 16 queries), lane holds 4 values
__global__ void __launch_bounds__(256) k_mfma16(const float* pts, int steps, float* out) {
  __shared__ float st[4][kPts * 4];
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int k = l; k < kPts * 4; k += 64) st[wv][k] = pts[k];
  __syncthreads();
  const float bq = -2.f * pts[l];  // B[k = l >> 4][col l & 15]
  const float qq = pts[l + 64];
  const f4 c = {qq, qq, qq, qq};
  uint32_t kmask = ~63u;
  asm volatile("" : "+v"(kmask));
  float k1 = __builtin_inff(), k2 = __builtin_inff();
  auto sel2 = [&](float ka, float kb) {
    float m;
    asm("v_med3_f32 %0, %1, %2, %3" : "=v"(m) : "v"(k1), "v"(ka), "v"(kb));
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(k1) : "v"(k1), "v"(ka), "v"(kb));
    asm("v_min_f32 %0, %1, %2" : "=v"(k2) : "v"(m), "v"(k2));
  };
#pragma unroll 1
  for (int s = 0; s < steps / 4; s++) {  // one tile = 4 steps' worth of pairs
    const float a = st[wv][((64 * s) & (kPts * 4 - 1)) + l];
    f4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bq, c, 0, 0, 0);
    const uint32_t sl = (uint32_t)(16 * s) & 63u;
    auto sg = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    const float ka = __uint_as_float((__float_as_uint(d[0]) & kmask) | sg(sl));
    const float kb = __uint_as_float((__float_as_uint(d[1]) & kmask) | sg(sl + 1u));
    const float kc = __uint_as_float((__float_as_uint(d[2]) & kmask) | sg(sl + 2u));
    const float kd = __uint_as_float((__float_as_uint(d[3]) & kmask) | sg(sl + 3u));
    sel2(ka, kb);
    sel2(kc, kd);
  }
  out[blockIdx.x * 256 + threadIdx.x] = k1 + k2;
}

int main() {
  // 1. layout
  float* dl;
  CK(hipMalloc(&dl, 256 * sizeof(float)));
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dl);
  std::vector<float> hl(256);
  CK(hipMemcpy(hl.data(), dl, 256 * sizeof(float), hipMemcpyDeviceToHost));
  int layout_ok = 0, layout_n = 0;
  for (int l = 0; l < 64; l++)
    for (int r = 0; r < 4; r++) {
      const float v = hl[l * 4 + r];
      // expected: D_b[i=r][j=l&3] = a(lane 4b + r) * b(lane 4b + (l & 3))
      const int b = l >> 2;
      const float e = (float)(4 * b + r + 1) * (float)(1000 + 4 * b + (l & 3));
      layout_ok += v == e;
      layout_n++;
      if (l < 8 || v != e) {
        // decode the factors
        int fa = -1, fb = -1;
        for (int x = 0; x < 64 && fa < 0; x++)
          for (int y = 0; y < 64; y++)
            if ((float)(x + 1) * (float)(1000 + y) == v) {
              fa = x;
              fb = y;
              break;
            }
        if (l < 8) printf("lane %2d reg %d = a[lane %2d] * b[lane %2d]\n", l, r, fa, fb);
      }
    }
  printf("layout: %d / %d match D_b[r][l&3] = a(4b + r) b(4b + (l&3))\n", layout_ok, layout_n);

  // 2. chain vs fmaf
  const int T = 4096;
  std::vector<float> hp(T * 16), hq(T * 192);
  srand(7);
  auto rnd = [] { return (float)((rand() / (double)RAND_MAX) * 2.0 - 1.0); };
  for (auto& v : hp) v = rnd() * (rand() % 2 ? 1.f : 37.f);
  for (auto& v : hq) v = rnd() * (rand() % 2 ? 1.f : 37.f);
  float *dp, *dq, *om, *of;
  unsigned* dbad;
  CK(hipMalloc(&dp, hp.size() * 4));
  CK(hipMalloc(&dq, hq.size() * 4));
  CK(hipMalloc(&om, T * 256 * 4));
  CK(hipMalloc(&of, T * 256 * 4));
  CK(hipMalloc(&dbad, 4));
  CK(hipMemset(dbad, 0, 4));
  CK(hipMemcpy(dp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dq, hq.data(), hq.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_chain, dim3(T), dim3(64), 0, 0, dp, dq, dbad, om, of);
  unsigned bad = 0;
  CK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
  printf("chain: %u of %d values differ from the fmaf chain\n", bad, T * 256);

  // 3. issue cost
  std::vector<float> pts(kPts * 4);
  for (auto& v : pts) v = rnd();
  float *dpt, *dout;
  CK(hipMalloc(&dpt, pts.size() * 4));
  CK(hipMemcpy(dpt, pts.data(), pts.size() * 4, hipMemcpyHostToDevice));
  const int blocks = 256 * 7;  // 7 waves per SIMD
  CK(hipMalloc(&dout, blocks * 256 * 4));
  const int steps = 4096;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, void (*k)(const float*, int, float*)) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, dpt, steps, dout);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, dpt, steps, dout);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    // per SIMD: blocks * 4 waves / 1024 SIMDs waves, each `steps` steps
    const double wave_steps = (double)blocks * 4 * steps / 1024.0;
    printf("%-34s %8.3f ms  %6.2f ns per wave-step per SIMD (%.1f cycles at 2.4 GHz)\n", name, best,
           best * 1e6 / wave_steps, best * 1e6 / wave_steps * 2.4);
  };
  timeit("packed VALU (2 x eval2)", k_valu);
  timeit("4x4x1 MFMA x4 + selection", k_mfma4);
  timeit("16x16x4 MFMA (1/4 per step) + sel", k_mfma16);
  printf("done\n");
  return 0;
}
