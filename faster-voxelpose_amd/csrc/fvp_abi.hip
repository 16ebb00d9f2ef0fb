// Version and status strings of the C ABI (include/fvp.h).
#include "fvp_device.h"

extern "C" int fvp_abi_version(void) { return FVP_ABI_VERSION; }

extern "C" const char *fvp_status_string(int status) {
    switch (status) {
        case FVP_OK:
            return "success";
        case FVP_ERR_NULL:
            return "fvp: a required pointer argument is NULL";
        case FVP_ERR_SHAPE:
            return "fvp: a size argument is out of range for this kernel";
        case FVP_ERR_WORKSPACE:
            return "fvp: workspace missing or smaller than fvp_voxelize_workspace_bytes()";
        default:
            return hipGetErrorString((hipError_t)status);
    }
}
