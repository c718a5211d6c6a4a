// Thread-local error reporting and ABI version for the C-ABI (dfhip.h).
#include "common.h"

#include <stdarg.h>

namespace dfhip {

static thread_local char g_last_error[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

}  // namespace dfhip

extern "C" int dfhip_abi_version(void) { return 1; }
extern "C" const char *dfhip_last_error(void) { return dfhip::g_last_error; }
