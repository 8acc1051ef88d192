// valu_peak.hip -- measures the fp32 VALU issue ceiling of this MI355X for the
// instruction mixes the Chamfer kernel uses (v_fma_f32 vs v_pk_fma_f32, and
// v_min3_f32), so the roofline in bench.py/DESIGN.md rests on a measurement.
// Build: hipcc -O3 --offload-arch=gfx950 -o valu_peak valu_peak.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_fma(float *out, float a, float b) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, b);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pkfma(float *out, float a, float b) {
    f2 x[8];
    const f2 av = {a, a}, bv = {b, b};
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_elementwise_fma(x[i], av, bv);
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pkadd(float *out, float a, float b) {
    f2 x[8];
    const f2 av = {a, a};
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = x[i] - av;
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i].x + x[i].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_min3(float *out, float a, float b) {
    float x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fminf(x[i], __builtin_fminf(a + it, b));
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
int run(const char *name, K kern, double lane_ops_per_thread, double flops_per_lane_op, float *buf, int blocks) {
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
    printf("%-8s %8.3f ms  %8.2f T lane-ops/s  %8.2f TFLOP/s\n", name, t * 1e3, lops / t / 1e12, lops * flops_per_lane_op / t / 1e12);
    return 0;
}

int main() {
    const int blocks = 256 * 8;
    float *buf;
    CHK(hipMalloc(&buf, sizeof(float) * 256 * blocks));
    run("fma", k_fma, 8.0 * ITERS, 2.0, buf, blocks);
    run("pk_fma", k_pkfma, 16.0 * ITERS, 2.0, buf, blocks);
    run("pk_add", k_pkadd, 16.0 * ITERS, 1.0, buf, blocks);
    run("min", k_min3, 8.0 * ITERS, 1.0, buf, blocks);
    return 0;
}
