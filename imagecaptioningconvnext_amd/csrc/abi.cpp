// Error plumbing and version query of the C ABI (include/imgcap_abi.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <vector>
#include <string>

#include "../../include/imgcap_abi.h"

namespace imgcap {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
const uint64_t* g_seed_ctr = nullptr;

// Scratch for split reductions (GEMM split-K partials, colsum / LayerNorm-gradient slices).
// Two slots: work that may run concurrently on another stream (the trainer's encoder beside
// the decoder) selects slot 1 with imgcap_workspace_slot; kernels of one slot run one after
// another.  Grow-only (a captured HIP graph may reference a buffer, and no allocation may
// happen during capture: warm-up runs size them), a grown buffer never frees the old one.
struct Ws {
  void* p = nullptr;
  size_t bytes = 0;
};
static std::mutex g_ws_mu;
static Ws g_ws[2];
static std::vector<void*> g_ws_retired;
static thread_local int g_ws_slot = 0;
int set_workspace_slot(int slot) {
  const int prev = g_ws_slot;
  g_ws_slot = slot;
  return prev;
}
void* workspace(size_t bytes, hipStream_t) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Ws& w = g_ws[g_ws_slot];
  if (bytes <= w.bytes) return w.p;
  size_t sz = std::max(bytes, (size_t)16 << 20);
  void* p = nullptr;
  if (hipMalloc(&p, sz) != hipSuccess) return nullptr;
  if (w.p) g_ws_retired.push_back(w.p);
  w.p = p;
  w.bytes = sz;
  return p;
}
}  // namespace imgcap

extern "C" int imgcap_set_seed_counter(const uint64_t* counter) {
  imgcap::g_seed_ctr = counter;
  return IMGCAP_OK;
}

extern "C" const char* imgcap_last_error_string(void) { return imgcap::g_last_error.c_str(); }
extern "C" int imgcap_version(void) { return 1; }

extern "C" int imgcap_workspace_slot(int slot) {
  if (slot < 0 || slot > 1) return imgcap::fail(IMGCAP_EINVAL, "imgcap_workspace_slot: 0 or 1");
  imgcap::set_workspace_slot(slot);
  return IMGCAP_OK;
}
