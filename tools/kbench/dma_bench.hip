// Per-CU operand delivery into LDS on MI355X, the quantity that bounds the LDS-staged GEMM
// tiles: a GEMM-shaped stream without the MFMAs.  Each block owns a ring of D
// stages of STEP bytes; per step every thread issues its global_load_lds_dwordx4 share of the
// next stage, waits (counted vmcnt) for the oldest stage, and the block meets at a barrier --
// the k-loop of gemm_pt.h / gemm_glds.h.  Mode 1 streams with global_load_dwordx4 into VGPRs
// instead (no LDS), the plain-load rate for comparison.
//   build: hipcc -O3 --offload-arch=gfx950 -std=c++17 dma_bench.hip -o dma_bench
//   run:   ./dma_bench           (prints GB/s per CU for each configuration)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// W waves, D stages in flight (D >= 1: D - 1 stages stay in flight across the wait), STEP bytes
template <int W, int D, int STEP>
__global__ __launch_bounds__(W * 64) void dma_kernel(const char* __restrict__ src, size_t src_bytes, int steps,
                                                     unsigned* sink) {
  constexpr int PER = STEP / (W * 64 * 16);  // instructions per thread per step
  static_assert(PER >= 1 && PER * W * 64 * 16 == STEP, "step");
  __shared__ __attribute__((aligned(16))) char smem[(D + 1) * STEP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t nchunks = src_bytes / STEP;
  size_t chunk = ((size_t)blockIdx.x * 7919) % nchunks;
  auto issue = [&](int s) {
    char* st = smem + (s % (D + 1)) * STEP;
    const char* base = src + ((chunk + s) % nchunks) * STEP;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int p0 = (j * W + w) * 64;
      __builtin_amdgcn_global_load_lds((const void*)(base + (p0 + lane) * 16),
                                       (__attribute__((address_space(3))) void*)(st + p0 * 16), 16, 0, 0);
    }
  };
  for (int s = 0; s < D && s < steps; ++s) issue(s);
  unsigned acc = 0;
  for (int s = 0; s < steps; ++s) {
    if (s + D - 1 < steps) {
      if constexpr (D == 1) vmwait<0>();
      else if constexpr (D == 2) vmwait<PER>();
      else if constexpr (D == 3) vmwait<2 * PER>();
      else vmwait<3 * PER>();
    } else {
      vmwait<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + D < steps) issue(s + D);
    acc += *(const unsigned*)(smem + (s % (D + 1)) * STEP + threadIdx.x * 16);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// plain loads to VGPRs: each thread keeps D x PER 16-byte loads in flight
template <int W, int D, int STEP>
__global__ __launch_bounds__(W * 64) void vgpr_kernel(const char* __restrict__ src, size_t src_bytes, int steps,
                                                      unsigned* sink) {
  constexpr int PER = STEP / (W * 64 * 16);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const size_t nchunks = src_bytes / STEP;
  size_t chunk = ((size_t)blockIdx.x * 7919) % nchunks;
  uint4 v[D][PER];
  unsigned acc = 0;
  for (int s = 0; s < steps; s += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const char* base = src + ((chunk + s + d) % nchunks) * STEP;
#pragma unroll
      for (int j = 0; j < PER; ++j) v[d][j] = *(const uint4*)(base + ((j * W + w) * 64 + lane) * 16);
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int j = 0; j < PER; ++j) acc += v[d][j].x ^ v[d][j].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int W, int D, int STEP>
void run(const char* src, size_t bytes, const char* what, int bpc, unsigned* sink, int mode) {
  const int cus = 256, steps = 256;
  const int grid = cus * bpc;
  float ms;
  if (mode == 0)
    ms = time_it([&] { hipLaunchKernelGGL((dma_kernel<W, D, STEP>), dim3(grid), dim3(W * 64), 0, 0, src, bytes, steps, sink); }, 5);
  else
    ms = time_it([&] { hipLaunchKernelGGL((vgpr_kernel<W, D, STEP>), dim3(grid), dim3(W * 64), 0, 0, src, bytes, steps, sink); }, 5);
  const double tot = (double)grid * steps * STEP;
  printf("%-5s src %-6s waves %2d blocks/CU %d stage %3d KB in-flight %d stages: %7.1f GB/s per CU (%6.2f TB/s)\n",
         mode ? "vgpr" : "lds", what, W, bpc, STEP / 1024, D, tot / (ms * 1e-3) / cus / 1e9, tot / (ms * 1e-3) / 1e12);
}

int main() {
  const size_t big = (size_t)1 << 30, small = (size_t)2 << 20;
  char* src;
  unsigned* sink;
  CHECK(hipMalloc(&src, big));
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMemset(src, 1, big));
  for (int m = 0; m < 2; ++m) {
    const size_t bytes = m ? big : small;
    const char* what = m ? "1GiB" : "2MiB";
    run<8, 1, 32768>(src, bytes, what, 1, sink, 0);
    run<8, 2, 32768>(src, bytes, what, 1, sink, 0);
    run<8, 3, 32768>(src, bytes, what, 1, sink, 0);
    run<8, 4, 32768>(src, bytes, what, 1, sink, 0);
    run<8, 2, 49152>(src, bytes, what, 1, sink, 0);
    run<4, 2, 16384>(src, bytes, what, 4, sink, 0);
    run<4, 2, 32768>(src, bytes, what, 2, sink, 0);
    run<4, 3, 16384>(src, bytes, what, 2, sink, 0);
    run<16, 2, 32768>(src, bytes, what, 1, sink, 0);
    run<16, 3, 32768>(src, bytes, what, 1, sink, 0);
    run<8, 2, 32768>(src, bytes, what, 2, sink, 0);
    run<8, 2, 16384>(src, bytes, what, 1, sink, 1);
    run<8, 4, 16384>(src, bytes, what, 1, sink, 1);
    run<4, 4, 8192>(src, bytes, what, 4, sink, 1);
  }
  return 0;
}
