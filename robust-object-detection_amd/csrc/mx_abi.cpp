// mx_abi.cpp — library-wide C ABI pieces: version and thread-local error message.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mx_det.h"

namespace mx {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mx

extern "C" int mx_version(void) { return 1; }
extern "C" const char* mx_last_error(void) { return mx::g_err; }
