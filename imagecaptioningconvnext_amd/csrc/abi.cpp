// Error plumbing and version query of the C ABI (include/imgcap_abi.h).
#include <cstdint>
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
}  // namespace imgcap

extern "C" int imgcap_set_seed_counter(const uint64_t* counter) {
  imgcap::g_seed_ctr = counter;
  return IMGCAP_OK;
}

extern "C" const char* imgcap_last_error_string(void) { return imgcap::g_last_error.c_str(); }
extern "C" int imgcap_version(void) { return 1; }
