// valu_operands.hip -- does v_pk_fma_f32 issue at full rate when all three
// operands are distinct VGPR pairs (the filtered Chamfer scan's form), or only
// with an SGPR / constant operand?  Also the scalar v_fma_f32 with three VGPRs.
// Build: hipcc -O3 --offload-arch=gfx950 -o valu_operands valu_operands.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int ITERS = 4096;

// 8 independent chains x[i] = fma(x[i], y[i], z[i]), y/z per-lane VGPR pairs
__global__ __launch_bounds__(256) void k_pk_vvv(float *out, float a, float b) {
    f2 x[8], y[8], z[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = f2{(float)threadIdx.x + i, (float)i};
        y[i] = f2{a + 1e-3f * threadIdx.x, a - 1e-3f * i};
        z[i] = f2{b * threadIdx.x, b + i};
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], y[i], z[i]);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y + y[i].x + z[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// x[i] = fma(x[i], (a, a), z[i]): one operand an SGPR pair (kernel argument)
__global__ __launch_bounds__(256) void k_pk_vsv(float *out, float a, float b) {
    f2 x[8], z[8];
    const f2 av = {a, a};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = f2{(float)threadIdx.x + i, (float)i};
        z[i] = f2{b * threadIdx.x, b + i};
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, z[i]);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y + z[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma_vvv(float *out, float a, float b) {
    float x[8], y[8], z[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        x[i] = (float)threadIdx.x + i;
        y[i] = a + 1e-3f * threadIdx.x + i;
        z[i] = b * threadIdx.x + i;
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], y[i], z[i]);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i] + y[i] + z[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// generic 8-chain scalar kernels over three per-lane VGPRs
#define SCALAR_KERNEL(NAME, EXPR)                                                   \
    __global__ __launch_bounds__(256) void NAME(float *out, float a, float b) {     \
        float x[8], y[8], z[8];                                                     \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) {                             \
            x[i] = (float)threadIdx.x + i;                                          \
            y[i] = a + 1e-3f * threadIdx.x + i;                                     \
            z[i] = b * threadIdx.x + i;                                             \
        }                                                                           \
        for (int it = 0; it < ITERS; ++it) {                                        \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) x[i] = (EXPR);            \
        }                                                                           \
        float s = 0;                                                                \
        _Pragma("unroll") for (int i = 0; i < 8; ++i) s += x[i] + y[i] + z[i];      \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                             \
    }
SCALAR_KERNEL(k_min3_vvv, __builtin_fminf(__builtin_fminf(x[i], y[i]), z[i]))
SCALAR_KERNEL(k_med3_vvv, __builtin_amdgcn_fmed3f(x[i], y[i], z[i]))
SCALAR_KERNEL(k_add_vv, x[i] + y[i])
SCALAR_KERNEL(k_mul_vv, x[i] * y[i])
SCALAR_KERNEL(k_sel_vvv, (x[i] < y[i]) ? z[i] : x[i] + 1.0f)

template <typename K>
int run(const char *name, K kern, double lane_ops_per_thread, float *buf, int blocks) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, 1.0001f, 0.5f);
    CHK(hipEventRecord(e0));
    const int reps = 20;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, 1.0001f, 0.5f);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    double t = ms / 1e3 / reps;
    double lops = lane_ops_per_thread * 256.0 * blocks;
    printf("%-10s %8.3f ms  %8.2f T lane-instr/s\n", name, t * 1e3, lops / t / 1e12);
    return 0;
}

int main() {
    const int blocks = 256 * 8;
    float *buf;
    CHK(hipMalloc(&buf, sizeof(float) * 256 * blocks));
    run("pk_fma_vvv", k_pk_vvv, 8.0 * ITERS, buf, blocks);
    run("pk_fma_vsv", k_pk_vsv, 8.0 * ITERS, buf, blocks);
    run("fma_vvv", k_fma_vvv, 8.0 * ITERS, buf, blocks);
    run("min3_vvv", k_min3_vvv, 8.0 * ITERS, buf, blocks);
    run("med3_vvv", k_med3_vvv, 8.0 * ITERS, buf, blocks);
    run("add_vv", k_add_vv, 8.0 * ITERS, buf, blocks);
    run("mul_vv", k_mul_vv, 8.0 * ITERS, buf, blocks);
    run("cmp+sel", k_sel_vvv, 8.0 * ITERS, buf, blocks);
    return 0;
}
