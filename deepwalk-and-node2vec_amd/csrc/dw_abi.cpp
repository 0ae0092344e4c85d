// Library-level C ABI: error string, version, stream sync, elementwise scale.
#include <stdarg.h>
#include <string.h>

#include "dw_common.h"

namespace dw {

static thread_local char g_err[512] = "";
static thread_local const dw_step_scalars *g_step = nullptr;
static thread_local bool g_step_has_host = false;
static thread_local int64_t g_step_host = 0;

const dw_step_scalars *bound_step_scalars() { return g_step; }

int bound_step_rel(int64_t step, const dw_step_scalars **dyn, int32_t *delta, const char *what) {
    *dyn = g_step;
    *delta = 0;
    if (!g_step) return DW_OK;
    if (!g_step_has_host) {
        set_error("%s: a dw_step_scalars block is bound without its host step "
                  "(dw_step_scalars_bind_at)", what);
        return DW_E_INVALID_ARG;
    }
    const int64_t d = step - g_step_host;
    if (d < -0x7FFFFFFF || d > 0x7FFFFFFF) {
        set_error("%s: step %lld is too far from the bound block's host step %lld", what,
                  (long long)step, (long long)g_step_host);
        return DW_E_INVALID_ARG;
    }
    *delta = static_cast<int32_t>(d);
    return DW_OK;
}

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

}  // namespace dw

extern "C" {

const char *dw_last_error_string(void) { return dw::g_err; }

int dw_abi_version(void) { return 24; }

#ifndef DW_BUILD_ID
#define DW_BUILD_ID "unknown"
#endif
const char *dw_build_id(void) { return DW_BUILD_ID; }

int dw_step_scalars_bind(const dw_step_scalars *dev) {
    dw::g_step = dev;
    dw::g_step_has_host = false;
    return DW_OK;
}

int dw_step_scalars_bind_at(const dw_step_scalars *dev, int64_t host_step) {
    dw::g_step = dev;
    dw::g_step_has_host = dev != nullptr;
    dw::g_step_host = host_step;
    return DW_OK;
}

int dw_device_sync(void *stream) {
    hipError_t e = hipStreamSynchronize(dw::as_stream(stream));
    if (e != hipSuccess) {
        dw::set_error("hipStreamSynchronize: %s", hipGetErrorString(e));
        return DW_E_HIP;
    }
    return DW_OK;
}

}  // extern "C"
