// VALU throughput probe (gfx950): v_fma_f32 vs v_pk_fma_f32 vs v_dot2c_f32_bf16 (FMAs per CU-cycle).
// build: hipcc --offload-arch=gfx950 -O3 tools/probe/valu_rate.hip -o build/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));
constexpr int IT = 4096;

__global__ void k_fma(float* o, float s) {
  float a[8];
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_fmaf(a[j], s, 0.5f);
  float r = 0; for (int j = 0; j < 8; ++j) r += a[j];
  o[blockIdx.x * 256 + threadIdx.x] = r;
}
__global__ void k_pk(float* o, float s) {
  f2 a[8];
  const f2 ss = {s, s}, h = {0.5f, 0.5f};
  for (int j = 0; j < 8; ++j) a[j] = f2{(float)threadIdx.x, (float)j};
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_elementwise_fma(a[j], ss, h);
  float r = 0; for (int j = 0; j < 8; ++j) r += a[j][0] + a[j][1];
  o[blockIdx.x * 256 + threadIdx.x] = r;
}
__global__ void k_dot(float* o, float s) {
  float a[8];
  b2 x = {(__bf16)s, (__bf16)(s * 2)}, y = {(__bf16)0.5f, (__bf16)0.25f};
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x + j;
  for (int i = 0; i < IT; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_amdgcn_fdot2_f32_bf16(x, y, a[j], false);
  float r = 0; for (int j = 0; j < 8; ++j) r += a[j];
  o[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  float* o;
  hipMalloc(&o, 256 * 4096 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int blocks = 256 * 8;  // 8 waves/SIMD
  auto run = [&](const char* name, void (*k)(float*, float), double fma_per_it) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o, 1.0001f);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, o, 1.0001f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double fmas = 5.0 * blocks * 256 * IT * 8 * fma_per_it;
    printf("%-8s %8.3f ms  %7.1f TFMA/s  (%.1f FMA/CU/clk at 2.4 GHz)\n", name, ms, fmas / ms / 1e9,
           fmas / (ms * 1e-3) / 256 / 2.4e9);
  };
  run("fma", k_fma, 1);
  run("pk_fma", k_pk, 2);
  run("dot2bf16", k_dot, 2);
  return 0;
}
