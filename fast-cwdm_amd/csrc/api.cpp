// Error channel and version of libcwdm.
#include <string>

#include "common.hpp"

namespace cwdm {
namespace {
thread_local std::string g_err;
}
void set_error(const std::string& msg) { g_err = msg; }
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
const char* last_error() { return g_err.c_str(); }
}  // namespace cwdm

#ifndef CWDM_SRC_HASH
#define CWDM_SRC_HASH "unknown"
#endif

extern "C" int cwdm_version(void) { return 2000; }  // 0.2.0
// sha256 prefix of the sources this library was built from (cwdm_hip/srchash.py)
extern "C" const char* cwdm_build_id(void) { return CWDM_SRC_HASH; }
extern "C" const char* cwdm_last_error(void) { return cwdm::last_error(); }
