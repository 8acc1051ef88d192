// capi.hip -- version / status helpers of the C ABI (include/pcm.h).
#include "pcm_common.h"

extern "C" int pcm_version(void) { return 100; /* 0.1.0 */ }

extern "C" const char *pcm_strerror(int status) {
    switch (status) {
    case PCM_OK: return "ok";
    case PCM_ERR_INVALID_ARG: return "invalid argument (shape, size or null pointer)";
    case PCM_ERR_LAUNCH: return "HIP launch/runtime error";
    case PCM_ERR_WORKSPACE: return "workspace missing or too small";
    case PCM_ERR_UNSUPPORTED: return "size not supported by this build";
    case PCM_ERR_IO: return "file missing, unreadable or truncated";
    case PCM_ERR_FORMAT: return "not an (npoints, 3) float .npy array";
    default: return "unknown pcm status";
    }
}
