// C-ABI plumbing of liblmi_hip.so: thread-local error text and version.
#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/lmi_hip.h"

namespace lmi {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

}  // namespace lmi

extern "C" const char* lmi_last_error(void) { return lmi::g_last_error.c_str(); }

extern "C" int32_t lmi_abi_version(void) { return LMI_ABI_VERSION; }
