// Error state + version entry points of libacme_hip.so.
#include "common.h"

#include <cstring>

namespace acme {

static thread_local char g_last_error[1024] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

}  // namespace acme

extern "C" {

const char* acme_last_error(void) { return acme::g_last_error; }

const char* acme_version(void) { return "acme_amd 0.1.0 (" __DATE__ " " __TIME__ ")"; }

const char* acme_target_arch(void) { return "gfx950"; }

}  // extern "C"
