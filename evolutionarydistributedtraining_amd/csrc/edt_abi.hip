// edt_abi.hip — library-wide C ABI pieces: the thread-local error message and the version.
#include "edt_common.h"

namespace edt {
thread_local char g_err[512];
}

extern "C" {

const char* edt_last_error(void) { return g_err; }
const char* edt_version(void) { return "edt_sync 0.4.0 gfx950"; }
int edt_abi_version(void) { return EDT_ABI_VERSION; }

}  // extern "C"
