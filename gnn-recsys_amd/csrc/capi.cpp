// Library-level entry points of the gnnrec C ABI: version and error reporting.
#include <cstdarg>
#include <cstdio>

#include "gnnrec.h"

namespace gnnrec {

static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace gnnrec

extern "C" int gnnrec_version(void) { return 1; }

extern "C" const char* gnnrec_last_error(void) { return gnnrec::g_err; }

