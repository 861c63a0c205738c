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

extern "C" int cwdm_version(void) { return 1000; }  // 0.1.0
extern "C" const char* cwdm_last_error(void) { return cwdm::last_error(); }
