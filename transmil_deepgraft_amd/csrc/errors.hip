// Thread-local error string and build info for the C ABI (include/transmil_hip.h).
#include "common.h"

static thread_local const char* g_tm_err = "";

const char* tm_set_error(const char* msg) {
  g_tm_err = msg;
  return msg;
}

extern "C" const char* tm_last_error(void) { return g_tm_err; }
extern "C" const char* tm_build_info(void) { return "transmil_hip gfx950 " __DATE__ " " __TIME__; }
