// capi.hip -- version / status helpers of the C ABI (include/pcm.h).
#include "pcm_common.h"

extern "C" int pcm_version(void) { return 100; /* 0.1.0 */ }

// ---------------------------------------------------------------------------
// Test support (tests/test_coresidency_gpu.py): a kernel that holds `blocks`
// workgroups of `threads` threads and `lds_bytes` of LDS resident for `usec`
// microseconds while issuing nothing but s_sleep -- a stand-in for another
// kernel sharing the CUs (an RCCL all-reduce beside the one-launch Chamfer
// step at N > 1).  Every wave leaves once the real-time clock (100 MHz) has
// advanced `usec`; nothing is stored.
// ---------------------------------------------------------------------------
namespace {
__global__ void pcm_occupy_kernel(unsigned long long ticks) {
    extern __shared__ int occupy_lds[];
    (void)occupy_lds;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}
}  // namespace

extern "C" int pcm_tune_occupy(int blocks, int threads, int lds_bytes, unsigned usec, void *stream) {
    if (blocks <= 0 || threads <= 0 || threads > 1024 || lds_bytes < 0 || lds_bytes > 160 * 1024 || usec > 1000000u)
        return PCM_ERR_INVALID_ARG;
    if (lds_bytes > 64 * 1024 &&
        hipFuncSetAttribute((const void *)pcm_occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds_bytes) != hipSuccess)
        return PCM_ERR_LAUNCH;
    hipLaunchKernelGGL(pcm_occupy_kernel, dim3((unsigned)blocks), dim3((unsigned)threads), (size_t)lds_bytes,
                       (hipStream_t)stream, 100ull * usec);
    return pcm_launch_status();
}

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
