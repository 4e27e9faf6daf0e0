// Status / error plumbing of the C-ABI (include/hdpissa.h).
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "hdp_common.h"

namespace hdp {
static thread_local char g_err[1024] = "";

bool sync_debug() {
  static const bool on = [] {
    const char* e = getenv("HDP_SYNC_DEBUG");
    return e && e[0] == '1';
  }();
  return on;
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace hdp

extern "C" int hdp_abi_version(void) { return HDP_ABI_VERSION; }
extern "C" const char* hdp_last_error(void) { return hdp::g_err; }
