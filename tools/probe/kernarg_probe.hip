// Kernel-argument integrity probe for captured HIP graphs (tools/probe/kernarg_probe.py).
//
// canary_kernel: its by-value argument is 64 words derived from (id, k); thread 0 compares every
// word and counts mismatches into a __device__ array (no pointer in the arguments, so a corrupted
// argument block is reported, never dereferenced).  big_kernel: a by-value argument of NBIG words
// (the size of the library's grouped launches, imgcap_colsum_multi 3.3 KB / imgcap_gemm_grouped
// 3.7 KB) whose words it also checks.  Neither kernel touches memory outside __device__ arrays.
#include <hip/hip_runtime.h>

#include <cstdint>

__device__ unsigned int g_bad[4096];
__device__ unsigned int g_runs[4096];

struct Canary {
  unsigned int id;
  unsigned int w[63];
};

template <int N> struct Big {
  unsigned int id;
  unsigned int w[N - 1];
};

__host__ __device__ inline unsigned int expect(unsigned int id, int k) { return id * 2654435761u + (unsigned)k * 40503u + 7u; }

__global__ void canary_kernel(Canary c) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned int id = c.id & 4095u;
  unsigned int bad = c.id >= 4096u ? 1u : 0u;
  for (int k = 0; k < 63; ++k) bad += c.w[k] != expect(c.id, k) ? 1u : 0u;
  atomicAdd(&g_bad[id], bad);
  atomicAdd(&g_runs[id], 1u);
}

template <int N>
__global__ void big_kernel(Big<N> c) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const unsigned int id = c.id & 4095u;
  unsigned int bad = c.id >= 4096u ? 1u : 0u;
  for (int k = 0; k < N - 1; ++k) bad += c.w[k] != expect(c.id, k) ? 1u : 0u;
  atomicAdd(&g_bad[id], bad);
  atomicAdd(&g_runs[id], 1u);
}

extern "C" int probe_canary(unsigned int id, void* stream) {
  Canary c;
  c.id = id;
  for (int k = 0; k < 63; ++k) c.w[k] = expect(id, k);
  hipLaunchKernelGGL(canary_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, c);
  return (int)hipGetLastError();
}

// words: 256 (1 KB), 840 (3.3 KB) or 920 (3.6 KB)
extern "C" int probe_big(unsigned int id, int words, void* stream) {
#define BIG_(N)                                                                           \
  {                                                                                       \
    Big<N> c;                                                                             \
    c.id = id;                                                                            \
    for (int k = 0; k < N - 1; ++k) c.w[k] = expect(id, k);                               \
    hipLaunchKernelGGL(big_kernel<N>, dim3(1), dim3(64), 0, (hipStream_t)stream, c);      \
    return (int)hipGetLastError();                                                        \
  }
  if (words == 256) BIG_(256)
  if (words == 840) BIG_(840)
  if (words == 920) BIG_(920)
#undef BIG_
  return -1;
}

extern "C" int probe_read(unsigned int* bad, unsigned int* runs, int n) {
  if (hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof(unsigned int) * n) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(runs, HIP_SYMBOL(g_runs), sizeof(unsigned int) * n) != hipSuccess) return -2;
  return 0;
}
