// ABI identity and error strings for libngnn (include/ngnn.h).
#include <hip/hip_runtime_api.h>

#include "ngnn.h"

extern "C" int ngnn_abi_version(void) { return NGNN_ABI_VERSION; }

extern "C" const char *ngnn_strerror(int rc) {
    switch (rc) {
        case NGNN_OK: return "ngnn: success";
        case NGNN_E_ARG: return "ngnn: invalid argument (null pointer, negative size or bad enum)";
        case NGNN_E_DTYPE: return "ngnn: unsupported dtype";
        case NGNN_E_SHAPE: return "ngnn: unsupported shape or leading dimension";
        case NGNN_E_ALIGN: return "ngnn: unsupported pointer alignment";
        case NGNN_E_RANGE: return "ngnn: size does not fit int32 indexing";
        case NGNN_E_WORKSPACE: return "ngnn: workspace missing or too small";
        default: break;
    }
    if (rc > 0) return hipGetErrorString(static_cast<hipError_t>(rc));
    return "ngnn: unknown error";
}
