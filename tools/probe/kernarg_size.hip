// Does a kernel argument struct over 4 KiB arrive intact?  Writes the struct's last field (and a
// field below 4 KiB) to a buffer; no pointer inside the argument is dereferenced.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int N>
struct Big {
  int head;
  char pad[N];
  uint64_t tail;
};
template <int N>
__global__ void k(Big<N> b, uint64_t* out) {
  if (threadIdx.x == 0) { out[0] = (uint64_t)b.head; out[1] = b.tail; }
}
template <int N>
int run(uint64_t* d) {
  Big<N> b{};
  b.head = 7;
  b.tail = 0x1234567890abcdefull + N;
  hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, 0, b, d);
  hipError_t e = hipDeviceSynchronize();
  uint64_t h[2] = {0, 0};
  hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("arg bytes %zu: launch %s, head %llu, tail %s\n", sizeof(Big<N>), hipGetErrorString(e),
         (unsigned long long)h[0], h[1] == b.tail ? "intact" : "WRONG");
  return 0;
}
int main() {
  uint64_t* d;
  hipMalloc(&d, 16);
  run<3000>(d);
  run<4070>(d);
  run<4100>(d);
  run<6000>(d);
  return 0;
}
