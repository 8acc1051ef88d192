// capi.hip -- version / status helpers of the C ABI (include/pcm.h).
#include "pcm_common.h"

extern "C" int pcm_version(void) { return 100; /* 0.1.0 */ }

// ---------------------------------------------------------------------------
// Test support (tests/test_coresidency_gpu.py): a kernel that holds `blocks`
// workgroups of `threads` threads and `lds_bytes` of LDS resident for `usec`
// microseconds while issuing nothing but s_sleep -- a stand-in for another
// kernel sharing the CUs (an RCCL all-reduce beside the one-launch Chamfer
// step at N > 1).  Every wave leaves once the real-time clock (100 MHz) has
// advanced `usec`.  stamps (nullable, device, 3 words, caller-initialised to
// {~0, 0, 0}): the earliest workgroup start, the latest workgroup end (both
// s_memrealtime ticks) and the number of workgroups that started -- the
// evidence that the occupier was resident while another kernel ran;
// host_flag (nullable, pinned host memory): set to 1 once every workgroup
// has started.
// pcm_tune_clock_stamp writes s_memrealtime to *out from a one-thread kernel:
// on the step's stream just before and after the step it brackets the step's
// whole run (a stream runs its kernels one after the other).
// ---------------------------------------------------------------------------
namespace {
__global__ void pcm_occupy_kernel(unsigned long long ticks, unsigned long long *stamps, unsigned *host_flag) {
    extern __shared__ int occupy_lds[];
    (void)occupy_lds;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (stamps && threadIdx.x == 0) {
        atomicMin(stamps, t0);
        const unsigned long long old = atomicAdd(stamps + 2, 1ull);
        // the last workgroup to start tells the host, through pinned host
        // memory (no copy on another stream, which could share a hardware
        // queue with this kernel and wait for it)
        if (host_flag && old + 1 == (unsigned long long)gridDim.x) {
            __hip_atomic_store(host_flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    unsigned long long t = t0;
    while ((t = __builtin_amdgcn_s_memrealtime()) - t0 < ticks) __builtin_amdgcn_s_sleep(16);
    if (stamps && threadIdx.x == 0) atomicMax(stamps + 1, t);
}

__global__ void pcm_clock_stamp_kernel(unsigned long long *out) {
    // (out may be pinned host memory: a system-scope store the host can poll)
    if (threadIdx.x == 0)
        __hip_atomic_store(out, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// one wave: a dependent FMA chain between two (s_memrealtime, s_memtime)
// pairs -- the shader clock the chain ran at is the s_memtime ticks over the
// 100 MHz real-time ticks
__global__ void pcm_clock_rate_kernel(unsigned long long *out, int iters) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
    float a = (float)threadIdx.x;
    for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, 0.999f, 0.5f);
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = r1 - r0;
        out[1] = c1 - c0;
        out[2] = (unsigned long long)__float_as_uint(a);
    }
}
}  // namespace

extern "C" int pcm_tune_clock_rate(unsigned long long *out, int iters, void *stream) {
    if (!out || iters <= 0) return PCM_ERR_INVALID_ARG;
    hipLaunchKernelGGL(pcm_clock_rate_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out, iters);
    return pcm_launch_status();
}

extern "C" int pcm_tune_occupy_flagged(int blocks, int threads, int lds_bytes, unsigned usec,
                                       unsigned long long *stamps, unsigned *host_flag, void *stream) {
    if (blocks <= 0 || threads <= 0 || threads > 1024 || lds_bytes < 0 || lds_bytes > 160 * 1024 || usec > 1000000u)
        return PCM_ERR_INVALID_ARG;
    if (lds_bytes > 64 * 1024 &&
        hipFuncSetAttribute((const void *)pcm_occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            lds_bytes) != hipSuccess)
        return PCM_ERR_LAUNCH;
    hipLaunchKernelGGL(pcm_occupy_kernel, dim3((unsigned)blocks), dim3((unsigned)threads), (size_t)lds_bytes,
                       (hipStream_t)stream, 100ull * usec, stamps, host_flag);
    return pcm_launch_status();
}

extern "C" int pcm_tune_occupy_stamped(int blocks, int threads, int lds_bytes, unsigned usec,
                                       unsigned long long *stamps, void *stream) {
    return pcm_tune_occupy_flagged(blocks, threads, lds_bytes, usec, stamps, nullptr, stream);
}

extern "C" int pcm_tune_occupy(int blocks, int threads, int lds_bytes, unsigned usec, void *stream) {
    return pcm_tune_occupy_flagged(blocks, threads, lds_bytes, usec, nullptr, nullptr, stream);
}

extern "C" int pcm_tune_clock_stamp(unsigned long long *out, void *stream) {
    if (!out) return PCM_ERR_INVALID_ARG;
    hipLaunchKernelGGL(pcm_clock_stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
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
