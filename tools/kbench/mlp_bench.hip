// Standalone timing of cnblock_mlp_kernel variants (GPU box): hipcc -O3 --offload-arch=gfx950
// -DMLP_GELU=<0|1|2> ... ; prints us per launch for the Tiny stage shapes.
#include <cstdio>
#include <vector>
#include "../../imagecaptioningconvnext_amd/csrc/cnblock_mlp.hip"
#include "../../imagecaptioningconvnext_amd/csrc/abi.cpp"

int main() {
  const int B = 32;
  const int shapes[3][2] = {{56, 96}, {28, 192}, {56, 128}};
  for (auto& sh : shapes) {
    const int H = sh[0], C = sh[1];
    const int M = B * H * H;
    bf16 *z, *x, *w1, *w2;
    float *b1, *b2, *g;
    hipMalloc(&z, (size_t)M * C * 2); hipMalloc(&x, (size_t)M * C * 2);
    hipMalloc(&w1, (size_t)4 * C * C * 2); hipMalloc(&w2, (size_t)4 * C * C * 2);
    hipMalloc(&b1, 4 * C * 4); hipMalloc(&b2, C * 4); hipMalloc(&g, C * 4);
    hipMemset(z, 0, (size_t)M * C * 2); hipMemset(x, 0, (size_t)M * C * 2);
    hipMemset(w1, 0, (size_t)4 * C * C * 2); hipMemset(w2, 0, (size_t)4 * C * C * 2);
    hipMemset(b1, 0, 4 * C * 4); hipMemset(b2, 0, C * 4); hipMemset(g, 0, C * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    // clocks ramp up under sustained load: ~0.3 s of warm-up, then the best of 5 timed runs
    for (int i = 0; i < 2000; ++i) imgcap_cnblock_mlp(M, C, z, nullptr, nullptr, w1, b1, w2, b2, g, nullptr, 1, x, nullptr);
    hipDeviceSynchronize();
    const int reps = 50;
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < reps; ++i) imgcap_cnblock_mlp(M, C, z, nullptr, nullptr, w1, b1, w2, b2, g, nullptr, 1, x, nullptr);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
#ifdef MLP_STAMPS
    {  // one more launch with phase stamps of blocks 0..63 (shader clocks)
      long long* st;
      hipMalloc(&st, 64 * 64 * 8);
      hipMemset(st, 0, 64 * 64 * 8);
      hipMemcpyToSymbol(HIP_SYMBOL(g_mlp_stamps), &st, sizeof(st));
      imgcap_cnblock_mlp(M, C, z, nullptr, nullptr, w1, b1, w2, b2, g, nullptr, 1, x, nullptr);
      hipDeviceSynchronize();
      std::vector<long long> h(64 * 64);
      hipMemcpy(h.data(), st, 64 * 64 * 8, hipMemcpyDeviceToHost);
      long long* np = nullptr;
      hipMemcpyToSymbol(HIP_SYMBOL(g_mlp_stamps), &np, sizeof(np));
      double acc[64] = {0};
      for (int b = 0; b < 64; ++b)
        for (int k = 1; k < 42; ++k)
          if (h[b * 64 + k] && h[b * 64 + k - 1]) acc[k] += (double)(h[b * 64 + k] - h[b * 64 + k - 1]) / 64;
#ifdef MLP_RES_STAMPS
      if (C == 96) {  // resident kernel: fill, barrier, then per unit: loads+LN, MFMA loop, epilogue
        printf("  C=96 res stamps (cycles, mean of 64 blocks' wave 0):");
        for (int k = 1; k < 21; ++k) printf(" %d:%.0f", k, acc[k]);
        printf("\n");
      } else
#endif
      printf("  C=%d stamps (cycles, mean of 64 blocks): zload %.0f w0 %.0f |", C, acc[1], acc[2]);
      for (int c = 0; c < 8; ++c) printf(" c%d: g1 %.0f gelu %.0f g2 %.0f st %.0f |", c, acc[3 + 4 * c], acc[4 + 4 * c], acc[5 + 4 * c], acc[6 + 4 * c]);
      printf(" epi-tile %.0f epi %.0f total %.0f\n", acc[40], acc[41], (double)0);
      hipFree(st);
    }
#endif
    const double us = best * 1e3 / reps, fl = 2.0 * 2 * M * C * 4.0 * C;
    printf("variant %s C=%4d M=%6d: %8.1f us %7.1f TFLOP/s\n", MLP_TAG, C, M, us, fl / us / 1e6);
    hipFree(z); hipFree(x); hipFree(w1); hipFree(w2); hipFree(b1); hipFree(b2); hipFree(g);
  }
  return 0;
}
