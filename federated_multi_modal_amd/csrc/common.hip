// C-ABI status plumbing shared by every launcher: int status (0 = ok), message via mf_last_error().
#include <string.h>
#include "mf_common.h"

static thread_local char g_err[512] = "";

extern "C" int mf_set_error(const char* msg, int code) {
  strncpy(g_err, msg ? msg : "unknown error", sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
  return code == 0 ? -1 : code;
}

extern "C" const char* mf_last_error(void) { return g_err; }

extern "C" int mf_abi_version(void) { return 1; }
