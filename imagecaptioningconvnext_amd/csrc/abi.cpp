// Error plumbing and version query of the C ABI (include/imgcap_abi.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
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

// Scratch for split reductions (GEMM split-K partials, colsum row slices).  Kernels on one
// stream use it one after another.  A grown buffer never frees the old one: a captured HIP
// graph may still reference it.
static std::vector<void*> g_ws_retired;
static void* g_ws = nullptr;
static size_t g_ws_bytes = 0;
void* workspace(size_t bytes) {
  if (bytes <= g_ws_bytes) return g_ws;
  size_t sz = std::max(bytes, (size_t)16 << 20);
  void* p = nullptr;
  if (hipMalloc(&p, sz) != hipSuccess) return nullptr;
  if (g_ws) g_ws_retired.push_back(g_ws);
  g_ws = p;
  g_ws_bytes = sz;
  return p;
}
}  // namespace imgcap

extern "C" int imgcap_set_seed_counter(const uint64_t* counter) {
  imgcap::g_seed_ctr = counter;
  return IMGCAP_OK;
}

extern "C" const char* imgcap_last_error_string(void) { return imgcap::g_last_error.c_str(); }
extern "C" int imgcap_version(void) { return 1; }
