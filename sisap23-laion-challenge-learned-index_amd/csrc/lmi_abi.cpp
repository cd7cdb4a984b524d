// C-ABI plumbing of liblmi_hip.so: thread-local error text and version.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/lmi_hip.h"
#include "lmi_env.hpp"

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

namespace {
int env_i(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}
bool env_b(const char* name) { return std::getenv(name) != nullptr; }
}  // namespace

EnvConfig read_env() {
    EnvConfig e{};
    e.scan_v1 = env_b("LMI_SCAN_V1");
    e.scan_v2 = env_b("LMI_SCAN_V2");
    e.scan_abl = env_i("LMI_SCAN_ABL", 0);
    e.scan_groups = env_i("LMI_SCAN_GROUPS", 0);
    e.scan_lag = env_i("LMI_SCAN_LAG", 0);
    e.scan_split = env_i("LMI_SCAN_SPLIT", 0);
    e.scan_split_parts = env_i("LMI_SCAN_SPLIT_PARTS", 2);
    e.scan_wgs = env_i("LMI_SCAN_WGS", 0);
    e.scan_no_pref = env_b("LMI_SCAN_NO_PREF");
    e.wide_passes = env_b("LMI_WIDE_PASSES");
    e.wide_no_fixup = env_b("LMI_WIDE_NO_FIXUP");
    e.router_fma = env_b("LMI_ROUTER_FMA");
    e.router_qg = env_i("LMI_ROUTER_QG", 0);
    e.refine_kb = env_i("LMI_REFINE_KB", 1);
    e.xsel_kb = env_i("LMI_XSEL_KB", 1);
    e.x_skip = env_i("LMI_X_SKIP_SHARE", 4);
    return e;
}

EnvConfig& env_store() {
    static EnvConfig c = read_env();
    return c;
}

const EnvConfig& env_config() { return env_store(); }

}  // namespace lmi

extern "C" const char* lmi_last_error(void) { return lmi::g_last_error.c_str(); }

extern "C" int32_t lmi_abi_version(void) { return LMI_ABI_VERSION; }

extern "C" int lmi_config_reload(void) {
    lmi::env_store() = lmi::read_env();
    return LMI_OK;
}
