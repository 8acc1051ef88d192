// hybrid_probe.hip -- can the matrix pipe take part of the Chamfer filter
// screen while the VALU takes the rest, on the same SIMDs?
//
// One 512-thread workgroup per CU (the one-launch step's geometry: two waves
// per SIMD; waves w and w+4 share a SIMD).  Two kinds of wave bodies:
//   VALU  one 4-candidate x 4-query group of the filtered scan exactly as
//         filt_group4 issues it: 24 v_pk_fma_f32 + 8 v_min3 (16 pairs/lane)
//   MFMA  one 16-candidate chunk against 256 queries: 16 v_mfma_f32_16x16x4_f32
//         (targets as rows, queries as columns; 4096 pairs) and, per MFMA, the
//         fold of its 4 rows (v_min3 + v_min) and the best/second/chunk
//         bookkeeping of the lane's 4-target sub-chunk (med3, cmp, cndmask, min)
// Modes: all waves VALU; all waves MFMA; waves 0-3 MFMA + 4-7 VALU (one of
// each per SIMD) with several work splits.  Prints the time and pair rate.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/hybrid_probe tools/hybrid_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void valu_group(float (&mn)[4], const f2 (&px)[4], const f2 (&py)[4], const f2 (&pz)[4],
                                           f4 X4, f4 Y4, f4 Z4, f4 W4) {
    const f2 xa = X4.xy, xb = X4.zw, ya = Y4.xy, yb = Y4.zw, za = Z4.xy, zb = Z4.zw, wa = W4.xy, wb = W4.zw;
    f2 a0, a1, a2, a3, b0, b1, b2, b3;
    asm volatile(
        "v_pk_fma_f32 %[a0], %[z0], %[za], %[wa]\n\t"
        "v_pk_fma_f32 %[b0], %[z0], %[zb], %[wb]\n\t"
        "v_pk_fma_f32 %[a1], %[z1], %[za], %[wa]\n\t"
        "v_pk_fma_f32 %[b1], %[z1], %[zb], %[wb]\n\t"
        "v_pk_fma_f32 %[a2], %[z2], %[za], %[wa]\n\t"
        "v_pk_fma_f32 %[b2], %[z2], %[zb], %[wb]\n\t"
        "v_pk_fma_f32 %[a3], %[z3], %[za], %[wa]\n\t"
        "v_pk_fma_f32 %[b3], %[z3], %[zb], %[wb]\n\t"
        "v_pk_fma_f32 %[a0], %[y0], %[ya], %[a0]\n\t"
        "v_pk_fma_f32 %[b0], %[y0], %[yb], %[b0]\n\t"
        "v_pk_fma_f32 %[a1], %[y1], %[ya], %[a1]\n\t"
        "v_pk_fma_f32 %[b1], %[y1], %[yb], %[b1]\n\t"
        "v_pk_fma_f32 %[a2], %[y2], %[ya], %[a2]\n\t"
        "v_pk_fma_f32 %[b2], %[y2], %[yb], %[b2]\n\t"
        "v_pk_fma_f32 %[a3], %[y3], %[ya], %[a3]\n\t"
        "v_pk_fma_f32 %[b3], %[y3], %[yb], %[b3]\n\t"
        "v_pk_fma_f32 %[a0], %[x0], %[xa], %[a0]\n\t"
        "v_pk_fma_f32 %[b0], %[x0], %[xb], %[b0]\n\t"
        "v_pk_fma_f32 %[a1], %[x1], %[xa], %[a1]\n\t"
        "v_pk_fma_f32 %[b1], %[x1], %[xb], %[b1]\n\t"
        "v_pk_fma_f32 %[a2], %[x2], %[xa], %[a2]\n\t"
        "v_pk_fma_f32 %[b2], %[x2], %[xb], %[b2]\n\t"
        "v_pk_fma_f32 %[a3], %[x3], %[xa], %[a3]\n\t"
        "v_pk_fma_f32 %[b3], %[x3], %[xb], %[b3]"
        : [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [b0] "=&v"(b0), [b1] "=&v"(b1),
          [b2] "=&v"(b2), [b3] "=&v"(b3)
        : [x0] "v"(px[0]), [x1] "v"(px[1]), [x2] "v"(px[2]), [x3] "v"(px[3]), [y0] "v"(py[0]), [y1] "v"(py[1]),
          [y2] "v"(py[2]), [y3] "v"(py[3]), [z0] "v"(pz[0]), [z1] "v"(pz[1]), [z2] "v"(pz[2]), [z3] "v"(pz[3]),
          [xa] "v"(xa), [xb] "v"(xb), [ya] "v"(ya), [yb] "v"(yb), [za] "v"(za), [zb] "v"(zb), [wa] "v"(wa),
          [wb] "v"(wb));
    mn[0] = __builtin_fminf(__builtin_fminf(mn[0], a0.x), a0.y);
    mn[1] = __builtin_fminf(__builtin_fminf(mn[1], a1.x), a1.y);
    mn[2] = __builtin_fminf(__builtin_fminf(mn[2], a2.x), a2.y);
    mn[3] = __builtin_fminf(__builtin_fminf(mn[3], a3.x), a3.y);
    mn[0] = __builtin_fminf(__builtin_fminf(mn[0], b0.x), b0.y);
    mn[1] = __builtin_fminf(__builtin_fminf(mn[1], b1.x), b1.y);
    mn[2] = __builtin_fminf(__builtin_fminf(mn[2], b2.x), b2.y);
    mn[3] = __builtin_fminf(__builtin_fminf(mn[3], b3.x), b3.y);
}

// kMode 0: all VALU; 1: all MFMA; 2: waves 0-3 MFMA, 4-7 VALU
template <int kMode>
__global__ __launch_bounds__(512) void probe(float *out, const float *in, int nvalu, int nmfma) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool mfma = kMode == 1 || (kMode == 2 && wave < 4);
    const float s = in[lane];
    float acc = 0.f;
    if (!mfma) {
        f2 px[4], py[4], pz[4];
        for (int q = 0; q < 4; ++q) {
            px[q] = f2{s + q, s + q};
            py[q] = f2{s - q, s - q};
            pz[q] = f2{s * q, s * q};
        }
        float best[4] = {3e38f, 3e38f, 3e38f, 3e38f}, sec[4] = {3e38f, 3e38f, 3e38f, 3e38f};
        int bc[4] = {0, 0, 0, 0};
        f4 X4 = {s, s + 1, s + 2, s + 3}, Y4 = {s, s - 1, s - 2, s - 3}, Z4 = {1, 2, 3, 4}, W4 = {s, s, s, s};
        for (int c = 0; c < nvalu; c += 4) {  // chunks of 16 candidates = 4 groups
            float mn[4] = {3e38f, 3e38f, 3e38f, 3e38f};
            for (int g = 0; g < 4; ++g) {
                valu_group(mn, px, py, pz, X4, Y4, Z4, W4);
                X4.x += 1.f;  // a new candidate group (1 VALU)
            }
            for (int q = 0; q < 4; ++q) {
                sec[q] = __builtin_amdgcn_fmed3f(mn[q], best[q], sec[q]);
                if (mn[q] < best[q]) { best[q] = mn[q]; bc[q] = c; }
            }
        }
        for (int q = 0; q < 4; ++q) acc += best[q] + sec[q] + (float)bc[q];
    } else {
        float b[16];
        for (int q = 0; q < 16; ++q) b[q] = (lane >> 4) == 3 ? 1.f : s * (float)(q + 1);
        float best[16], sec[16];
        int bc[16];
        for (int q = 0; q < 16; ++q) { best[q] = 3e38f; sec[q] = 3e38f; bc[q] = 0; }
        float a = s;
        const f4 z = {0.f, 0.f, 0.f, 0.f};
        for (int c = 0; c < nmfma; ++c) {  // one 16-candidate chunk per step
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const f4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[q], z, 0, 0, 0);
                float mn;
                // the folds as plain v_min3/v_min (no canonicalisation of the MFMA results)
                asm("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4" : "=&v"(mn) : "v"(d.x), "v"(d.y), "v"(d.z), "v"(d.w));
                sec[q] = __builtin_amdgcn_fmed3f(mn, best[q], sec[q]);
                const bool t = mn < best[q];
                bc[q] = t ? c : bc[q];
                asm("v_min_f32 %0, %0, %1" : "+v"(best[q]) : "v"(mn));
            }
            a = a * 1.0001f + 0.5f;
        }
        for (int q = 0; q < 16; ++q) acc += best[q] + sec[q] + (float)bc[q];
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

template <int kMode>
float run(int nvalu, int nmfma, float *out, float *in) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) probe<kMode><<<256, 512>>>(out, in, nvalu, nmfma);
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) probe<kMode><<<256, 512>>>(out, in, nvalu, nmfma);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / reps;
}

int main() {
    float *out, *in;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&in, 64 * 4);
    hipMemset(in, 0, 64 * 4);
    // per SIMD the real kernel screens 65,536 pairs (B=32, N=M=1024): as VALU
    // groups that is 64 groups per wave (2 waves/SIMD x 64 x 1024 pairs/wave-group / 2 ...)
    // -- here simply: VALU group = 1024 pairs per wave, MFMA chunk = 4096 pairs per wave
    const int G = 256;  // VALU groups per wave in the all-VALU run (long enough to time)
    const double pairs_valu = 8.0 * G * 1024;  // per workgroup
    float t0 = run<0>(G, 0, out, in);
    printf("all VALU   : %8.1f us  %.3e pairs/s\n", t0, 256 * pairs_valu / (t0 * 1e-6));
    const int J = G / 4;  // same pairs as MFMA chunks
    float t1 = run<1>(0, J, out, in);
    printf("all MFMA   : %8.1f us  %.3e pairs/s\n", t1, 256 * pairs_valu / (t1 * 1e-6));
    // hybrid: MFMA waves take fraction f of the pairs (total fixed)
    for (int pct = 40; pct <= 90; pct += 10) {
        const int jm = (int)(J * 2 * pct / 100.0);        // 4 MFMA waves do 2x their share
        const int gv = (int)(G * 2 * (100 - pct) / 100.0);  // 4 VALU waves
        float t2 = run<2>(gv, jm, out, in);
        const double pairs = 4.0 * jm * 4096 + 4.0 * gv * 1024;
        printf("hybrid %2d%%: %8.1f us  %.3e pairs/s (VALU waves %d groups, MFMA waves %d chunks)\n", pct, t2,
               256 * pairs / (t2 * 1e-6), gv, jm);
    }
    hipFree(out);
    hipFree(in);
    return 0;
}
