// Library-level entry points: ABI version and thread-local error reporting.
#include <stdarg.h>
#include <stdio.h>
#include "../../include/octsam.h"

namespace octsam {
static thread_local char g_err[1024] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace octsam

extern "C" int octsam_abi_version(void) { return OCTSAM_ABI_VERSION; }
extern "C" const char* octsam_last_error(void) { return octsam::g_err; }
