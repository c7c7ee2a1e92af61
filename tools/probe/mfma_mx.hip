// Lane map probe for v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 A and B, E8M0 block scales):
// hypothesis: lane l holds A[row l%16][k = 32*(l/16) + j] and B[k = 32*(l/16) + j][col l%16],
// j = 0..31 (bytes of its 8 VGPRs in order), and its scale register (byte 0) scales exactly
// those 32 values; C/D: col = l%16, row = 4*(l/16) + r.  Exact small-integer data.
// build: hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_mx.hip -o build/mfma_mx
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ int kmap(int L, int g, int j) {
  switch (L) {
    case 0: return 32 * g + j;
    case 1: return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);
    case 2: return 8 * g + (j % 8) + 32 * (j / 8);
    case 3: return 4 * g + (j % 4) + 16 * (j / 4);
    default: return (j % 2) + 2 * g + 8 * (j / 2);
  }
}
// unit: all scales 127 (2^0); else per-lane scales from sa/sb[(row|col) * 4 + g]
__global__ void k(int L, int unit, const unsigned char* A, const unsigned char* B, const unsigned char* sa,
                  const unsigned char* sb, float* C) {
  const int l = threadIdx.x, r = l % 16, g = l / 16;
  v8i a, b;
  unsigned char* pa = (unsigned char*)&a;
  unsigned char* pb = (unsigned char*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[r * 128 + kmap(L, g, j)];
    pb[j] = B[kmap(L, g, j) * 16 + r];
  }
  const int xa = unit ? 127 : sa[r * 4 + g], xb = unit ? 127 : sb[r * 4 + g];
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, xa, 0, xb);
  for (int i = 0; i < 4; ++i) C[(4 * g + i) * 16 + r] = c[i];
}

static unsigned char e4m3(int v) {  // small integers |v| <= 6, exact in e4m3fn
  static const unsigned char pos[7] = {0x00, 0x38, 0x40, 0x44, 0x48, 0x4A, 0x4C};
  return v < 0 ? (unsigned char)(0x80 | pos[-v]) : pos[v];
}

int main() {
  int Av[16 * 128], Bv[128 * 16];
  unsigned char A[16 * 128], B[128 * 16], sa[16 * 4], sb[16 * 4];
  srand(7);
  for (int i = 0; i < 16 * 128; ++i) { Av[i] = rand() % 13 - 6; A[i] = e4m3(Av[i]); }
  for (int i = 0; i < 128 * 16; ++i) { Bv[i] = rand() % 13 - 6; B[i] = e4m3(Bv[i]); }
  for (int i = 0; i < 64; ++i) { sa[i] = 126 + rand() % 3; sb[i] = 126 + rand() % 3; }
  double ref[256], ref1[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0, s1 = 0;
      for (int kk = 0; kk < 128; ++kk) {
        s += Av[i * 128 + kk] * std::ldexp(1.0, sa[i * 4 + kk / 32] - 127) * Bv[kk * 16 + j] *
             std::ldexp(1.0, sb[j * 4 + kk / 32] - 127);
        s1 += Av[i * 128 + kk] * Bv[kk * 16 + j];
      }
      ref[i * 16 + j] = s;
      ref1[i * 16 + j] = s1;
    }
  unsigned char *dA, *dB, *dsa, *dsb;
  float* dC;
  (void)hipMalloc(&dA, sizeof A); (void)hipMalloc(&dB, sizeof B); (void)hipMalloc(&dsa, 64); (void)hipMalloc(&dsb, 64);
  (void)hipMalloc(&dC, 256 * 4);
  (void)hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); (void)hipMemcpy(dB, B, sizeof B, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsa, sa, 64, hipMemcpyHostToDevice); (void)hipMemcpy(dsb, sb, 64, hipMemcpyHostToDevice);
  int found = -1;
  for (int unit = 1; unit >= 0; --unit)
    for (int L = 0; L < 5; ++L) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, L, unit, dA, dB, dsa, dsb, dC);
      float C[256];
      (void)hipMemcpy(C, dC, sizeof C, hipMemcpyDeviceToHost);
      const double* R = unit ? ref1 : ref;
      int bad = 0;
      for (int i = 0; i < 256; ++i)
        if (std::fabs(C[i] - R[i]) > 1e-3 * (1 + std::fabs(R[i]))) ++bad;
      printf("layout %d unit-scale %d: %d / 256 mismatches (C00 %f ref %f)\n", L, unit, bad, C[0], R[0]);
      if (!bad && !unit) found = L;
    }
  int bad = found < 0;
  return bad != 0;
}
