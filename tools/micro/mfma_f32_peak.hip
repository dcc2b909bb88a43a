// Micro-benchmark: the f32 MFMA rate this chip holds with operands in registers
// (v_mfma_f32_32x32x2_f32 and v_mfma_f32_16x16x4_f32, 4 independent accumulators per wave),
// for 1..4 waves per SIMD: does the chip hold a different clock under the 16x16 shape?
// hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_f32_peak.hip -o /tmp/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void peak(float* out, int iters, float a0, float b0) {
  f32x16 c[4];
  for (int t = 0; t < 4; ++t)
    for (int v = 0; v < 16; ++v) c[t][v] = 0.f;
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c[t], 0, 0, 0);
  }
  float s = 0.f;
  for (int t = 0; t < 4; ++t)
    for (int v = 0; v < 16; ++v) s += c[t][v];
  if (s == 12345.f) out[threadIdx.x] = s;
}

typedef float f32x4v __attribute__((ext_vector_type(4)));
__global__ void peak16(float* out, int iters, float a0, float b0) {
  f32x4v c[4];
  for (int t = 0; t < 4; ++t)
    for (int v = 0; v < 4; ++v) c[t][v] = 0.f;
  float a = a0 + threadIdx.x * 1e-7f, b = b0 - threadIdx.x * 1e-7f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int t = 0; t < 4; ++t) c[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[t], 0, 0, 0);
  }
  float s = 0.f;
  for (int t = 0; t < 4; ++t)
    for (int v = 0; v < 4; ++v) s += c[t][v];
  if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 20000;
  for (int wps = 1; wps <= 4; ++wps) {
    const int blocks = cus * wps;  // 256-thread blocks: 4 waves = one per SIMD
    hipLaunchKernelGGL(peak, dim3(blocks), dim3(256), 0, 0, out, 100, 0.5f, 0.25f);
    hipEvent_t s, e;
    hipEventCreate(&s);
    hipEventCreate(&e);
    hipEventRecord(s);
    hipLaunchKernelGGL(peak, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5f, 0.25f);
    hipEventRecord(e);
    hipEventSynchronize(e);
    float ms = 0.f;
    hipEventElapsedTime(&ms, s, e);
    const double flop = (double)blocks * 4 * iters * 4 * 32 * 32 * 2 * 2;
    printf("32x32x2 waves/SIMD %d: %.3f ms, %.1f TF/s\n", wps, ms, flop / ms / 1e9);
    // the same FLOPs through 16x16x4 (2048 flop per instruction: 4x the instructions)
    hipLaunchKernelGGL(peak16, dim3(blocks), dim3(256), 0, 0, out, 100, 0.5f, 0.25f);
    hipEventRecord(s);
    hipLaunchKernelGGL(peak16, dim3(blocks), dim3(256), 0, 0, out, 4 * iters, 0.5f, 0.25f);
    hipEventRecord(e);
    hipEventSynchronize(e);
    hipEventElapsedTime(&ms, s, e);
    printf("16x16x4 waves/SIMD %d: %.3f ms, %.1f TF/s\n", wps, ms, flop / ms / 1e9);
  }
  return 0;
}
