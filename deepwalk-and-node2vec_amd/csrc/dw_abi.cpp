// Library-level C ABI: error string, version, stream sync, elementwise scale.
#include <stdarg.h>
#include <string.h>

#include "dw_common.h"

namespace dw {

static thread_local char g_err[512] = "";
static thread_local const dw_step_scalars *g_step = nullptr;

const dw_step_scalars *bound_step_scalars() { return g_step; }

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

}  // namespace dw

extern "C" {

const char *dw_last_error_string(void) { return dw::g_err; }

int dw_abi_version(void) { return 12; }

int dw_step_scalars_bind(const dw_step_scalars *dev) {
    dw::g_step = dev;
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
