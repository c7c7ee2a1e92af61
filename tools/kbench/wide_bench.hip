// In-kernel phase stamps of the wide fused MLP (GPU box):
//   hipcc -O3 --offload-arch=gfx950 -DWIDE_STAMPS tools/kbench/wide_bench.hip -o /tmp/wb && /tmp/wb
// Per half q = 8..23 of blocks 0..63 (each wave): cycles waiting for the half's DMA + barrier, and
// the half's compute (to the next half's start); IMGCAP_WIDE_DBG as in the library.
#include <cstdio>
#include <vector>
#include "../../imagecaptioningconvnext_amd/csrc/cnblock_mlp_wide.hip"
#include "../../imagecaptioningconvnext_amd/csrc/abi.cpp"

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 6272, C = argc > 2 ? atoi(argv[2]) : 512;
  std::vector<bf16> h((size_t)M * C);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (bf16)((float)((i * 2654435761u) % 1000) / 500.f - 1.f);
  std::vector<bf16> hw((size_t)4 * C * C);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = (bf16)((float)((i * 40503u) % 1000) / 20000.f - 0.025f);
  bf16 *y, *x, *w1, *w2, *img;
  float *b1, *b2, *g, *part;
  int* sync;
  hipMalloc(&y, h.size() * 2); hipMalloc(&x, h.size() * 2);
  hipMalloc(&w1, hw.size() * 2); hipMalloc(&w2, hw.size() * 2); hipMalloc(&img, (size_t)(C / 8) * 128 * C);
  hipMalloc(&b1, 4 * C * 4); hipMalloc(&b2, C * 4); hipMalloc(&g, C * 4);
  hipMalloc(&part, (size_t)(M + 63) / 64 * 64 * C * 4); hipMalloc(&sync, (M + 63) / 64 * 8);
  hipMemcpy(y, h.data(), h.size() * 2, hipMemcpyHostToDevice); hipMemcpy(x, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(w1, hw.data(), hw.size() * 2, hipMemcpyHostToDevice); hipMemcpy(w2, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  hipMemset(b1, 0, 4 * C * 4); hipMemset(b2, 0, C * 4); hipMemset(g, 0, C * 4); hipMemset(sync, 0, (M + 63) / 64 * 8);
  imgcap_cnblock_mlp_wide_pack(C, w1, w2, img, nullptr);
  for (int i = 0; i < 200; ++i)
    imgcap_cnblock_mlp_wide(M, C, y, nullptr, nullptr, img, b1, b2, g, nullptr, 1, x, part, sync, nullptr);
  hipDeviceSynchronize();
  long long* st;
  hipMalloc(&st, 256 * 64 * 8);
  hipMemset(st, 0, 256 * 64 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_wide_stamps), &st, sizeof(st));
  imgcap_cnblock_mlp_wide(M, C, y, nullptr, nullptr, img, b1, b2, g, nullptr, 1, x, part, sync, nullptr);
  hipDeviceSynchronize();
  std::vector<long long> s(256 * 64);
  hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
  double wait = 0, comp = 0, tot = 0;
  int n = 0;
  for (int wv = 0; wv < 256; ++wv) {
    const long long* p = &s[wv * 64];
    if (!p[0] || !p[31]) continue;
    for (int k = 0; k < 15; ++k) {
      wait += p[2 * k + 1] - p[2 * k];
      comp += p[2 * k + 2] - p[2 * k + 1];
    }
    tot += p[41] - p[40];
    ++n;
  }
  printf("M=%d C=%d dbg=%s: %d waves; per half: wait+barrier %.0f, compute %.0f cycles (s_memtime); whole loop+prologue %.0f\n",
         M, C, getenv("IMGCAP_WIDE_DBG") ? getenv("IMGCAP_WIDE_DBG") : "0", n, wait / n / 15, comp / n / 15, tot / n);
  return 0;
}
