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
std::string last_error() { return g_last_error; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
const uint64_t* g_seed_ctr = nullptr;

// Scratch for split reductions (GEMM split-K partials, colsum / LayerNorm-gradient slices),
// per device and per slot.  Two slots: work that may run concurrently on another stream (the
// trainer's encoder beside the decoder) selects slot 1 with imgcap_workspace_slot, the decoder
// engines' own side streams slot 2; kernels of one slot run one after another.  The caller attaches its own buffer per (device, slot) with
// imgcap_workspace_attach (the Python side does, from the PyTorch caching allocator); a request
// larger than the attached buffer fails with IMGCAP_EWORKSPACE before anything is launched, and
// imgcap_workspace_needed reports the size to attach.  Only a (device, slot) the caller never
// attached falls back to a library-owned, grow-only allocation (a grown buffer is not freed: a
// captured HIP graph may still reference it).
// One scratch buffer serves every call of a slot, so two streams of ONE captured graph must never
// both request it: their nodes are unordered unless the code joined them, and the round-5 scratch
// race was exactly that.  Each slot remembers the capture (id) and stream of its last
// request; a request from another stream of the same capture is refused (nothing is enqueued, the
// call fails with the message below) -- a check in the library, not a convention of two callers.
constexpr int MAX_DEV = 64;
struct Ws {
  void* p = nullptr;
  size_t bytes = 0;
  size_t needed = 0;
  bool caller = false;
  unsigned long long cap_id = 0;  // capture of the last request made while capturing (0: none)
  hipStream_t cap_stream = nullptr;
};
static std::mutex g_ws_mu;
constexpr int NSLOT = 3;
static Ws g_ws[MAX_DEV][NSLOT];
static std::vector<void*> g_ws_retired;
static thread_local int g_ws_slot = 0;
int set_workspace_slot(int slot) {
  const int prev = g_ws_slot;
  g_ws_slot = slot;
  return prev;
}
static Ws* ws_entry(int slot) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return nullptr;
  return &g_ws[dev][slot];
}
void* workspace(size_t bytes, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Ws* w = ws_entry(g_ws_slot);
  if (!w) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  if (stream && hipStreamGetCaptureInfo(stream, &cs, &cid) == hipSuccess && cs == hipStreamCaptureStatusActive) {
    if (w->cap_id == cid && w->cap_stream != stream) {
      set_error("library workspace: slot " + std::to_string(g_ws_slot) +
                " scratch requested from two streams of one captured graph (unordered branches would share it; "
                "select another slot with imgcap_workspace_slot on one of them)");
      return nullptr;
    }
    w->cap_id = cid;
    w->cap_stream = stream;
  }
  w->needed = std::max(w->needed, bytes);
  if (bytes <= w->bytes) return w->p;
  if (w->caller) {
    set_error("library workspace: " + std::to_string(bytes) + " bytes needed in slot " + std::to_string(g_ws_slot) +
              ", " + std::to_string(w->bytes) + " attached (imgcap_workspace_needed / imgcap_workspace_attach)");
    return nullptr;
  }
  size_t sz = std::max(bytes, (size_t)16 << 20);
  void* p = nullptr;
  if (hipMalloc(&p, sz) != hipSuccess) return nullptr;
  if (w->p) g_ws_retired.push_back(w->p);
  w->p = p;
  w->bytes = sz;
  return p;
}
int attach_workspace(int slot, void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Ws* w = ws_entry(slot);
  if (!w) return fail(IMGCAP_EINVAL, "imgcap_workspace_attach: no current device");
  if (w->p && !w->caller) g_ws_retired.push_back(w->p);  // a library buffer may be in a captured graph
  w->p = p;
  w->bytes = p ? bytes : 0;
  w->caller = p != nullptr;
  return IMGCAP_OK;
}
size_t workspace_needed(int slot) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  Ws* w = ws_entry(slot);
  return w ? w->needed : 0;
}
}  // namespace imgcap

extern "C" int imgcap_set_seed_counter(const uint64_t* counter) {
  imgcap::g_seed_ctr = counter;
  return IMGCAP_OK;
}

extern "C" const char* imgcap_last_error_string(void) { return imgcap::g_last_error.c_str(); }
extern "C" int imgcap_version(void) { return IMGCAP_ABI_VERSION; }

extern "C" int imgcap_workspace_attach(int slot, void* ptr, uint64_t bytes) {
  if (slot < 0 || slot >= imgcap::NSLOT) return imgcap::fail(IMGCAP_EINVAL, "imgcap_workspace_attach: slot 0, 1 or 2");
  if (ptr && ((uintptr_t)ptr & 255)) return imgcap::fail(IMGCAP_EINVAL, "imgcap_workspace_attach: 256-byte alignment");
  return imgcap::attach_workspace(slot, ptr, (size_t)bytes);
}

extern "C" int imgcap_workspace_needed(int slot, uint64_t* bytes) {
  if (slot < 0 || slot >= imgcap::NSLOT || !bytes) return imgcap::fail(IMGCAP_EINVAL, "imgcap_workspace_needed: slot 0, 1 or 2");
  *bytes = imgcap::workspace_needed(slot);
  return IMGCAP_OK;
}

extern "C" int imgcap_workspace_slot(int slot) {
  if (slot < 0 || slot >= imgcap::NSLOT) return imgcap::fail(IMGCAP_EINVAL, "imgcap_workspace_slot: 0, 1 or 2");
  imgcap::set_workspace_slot(slot);
  return IMGCAP_OK;
}
