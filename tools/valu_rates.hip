// Issue cost of the wave search's VALU instruction kinds on gfx950 with 8 waves per SIMD:
// each thread runs 8 independent dependency chains of one instruction kind; the chip-wide
// wave-instruction rate gives cycles per wave64 instruction per SIMD.
// build: hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIter = 4096;

template <int K>
__global__ void __launch_bounds__(256) k_rate(float* out, float b0, double bd) {
  float a[8];
  f2 p[8];
  double d[8];
  unsigned u[8];
  for (int j = 0; j < 8; j++) {
    a[j] = threadIdx.x * 0.001f + j;
    p[j] = f2{a[j], a[j] + 1.0f};
    d[j] = a[j];
    u[j] = threadIdx.x + j;
  }
  const f2 bb = {b0, b0 * 0.5f};
  const unsigned m = (unsigned)(b0 * 1000.0f);
  for (int it = 0; it < kIter; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      // inline asm: exactly one instruction of the kind per step (no packing, no folding)
      if (K == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(b0));
      if (K == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p[j]) : "v"(bb));
      if (K == 2) asm volatile("v_med3_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(b0));
      if (K == 3) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(u[j]) : "v"(m));
      if (K == 4) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[j]) : "v"(bd));
      if (K == 5) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[j]) : "v"(bd));
      if (K == 6) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[j]) : "v"(bb));
      if (K == 7) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b0));
    }
  }
  float s = 0.f;
  for (int j = 0; j < 8; j++) s += a[j] + p[j].x + p[j].y + (float)d[j] + (float)u[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int K>
float run(float* out, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.999);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 0.999);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  int dev = 0, clk = 0, cus = 0;
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  float* out = nullptr;
  if (hipMalloc(&out, sizeof(float) * blocks * 256) != hipSuccess) return 1;
  const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_med3_f32", "v_and_or_b32", "v_fma_f64", "v_add_f64",
                         "v_pk_mul_f32", "v_mul_f32"};
  float ms[8] = {run<0>(out, blocks), run<1>(out, blocks), run<2>(out, blocks), run<3>(out, blocks),
                 run<4>(out, blocks), run<5>(out, blocks), run<6>(out, blocks), run<7>(out, blocks)};
  const double waves = blocks * 4.0, instr = waves * kIter * 8.0, simds = cus * 4.0;
  for (int k = 0; k < 8; k++) {
    const double cyc = ms[k] * 1e-3 * clk * 1e3;
    printf("%-14s %8.3f ms  %.2f cycles per wave64 instruction per SIMD (clock %d MHz, %d CUs)\n", names[k], ms[k],
           cyc / (instr / simds), clk / 1000, cus);
  }
  return 0;
}
