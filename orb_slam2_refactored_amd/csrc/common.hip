// Thread-local error reporting and device queries for the C-ABI.
#include <string>

#include "common.h"

namespace orbamd {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace orbamd

extern "C" {
const char* orb_last_error(void) { return orbamd::g_last_error.c_str(); }

int orb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
}
