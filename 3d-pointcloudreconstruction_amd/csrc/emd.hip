// emd.hip -- auction-algorithm EMD for MI355X (gfx950, CDNA4).
//
// Replaces the reference's 7-launches-per-iteration host loop
// (metric/emd/emd_cuda.cu:256-269: clear, calc_unass_cnt, calc_unass_cnt_sum,
// calc_unass_idx, Bid, GetMax, Assign) with ONE persistent workgroup per batch
// element that runs every auction iteration in-kernel, keeping the whole
// auction state (assignment, owner, price, max increment, claim) in LDS and
// separating the phases with workgroup barriers only -- no grid barrier, no
// host round trip, 1 launch + 1 epilogue for any `iters`.
//
// Determinism: the reference's GetMax lets racing writers decide which of the
// bidders within the 1e-6 window wins (emd_cuda.cu:188-190); here the window
// is evaluated exactly as there (double compare) and the LOWEST point index
// wins via an LDS atomicMin, so results do not depend on scheduling.  The max
// increment uses an order-preserving int encoding + atomicMax (the reference
// uses a CAS loop, emd_cuda.cu:10-20) -- same value.
//
// Bid: each unassigned point is scanned by a group of G lanes (G = 1024/|U|
// rounded to a power of two, <= 64), lanes strided over the objects; value
// v = (float)((3.0 - (double)sqrtf(d)) - (double)price) as emd_cuda.cu:146
// evaluates it; per-lane top-2 merged across the group with shuffles
// (lowest index wins ties).
#include "pcm_common.h"

namespace {

constexpr int kEmdThreads = 1024;
constexpr int kEmdMaxN = 4096;  // LDS-resident state: 7 x 4 B x n

__device__ __forceinline__ int f2key(float f) {
    const int i = __float_as_int(f);
    return i ^ ((i >> 31) & 0x7fffffff);  // order-preserving for non-NaN floats
}
__device__ __forceinline__ float key2f(int k) {
    return __int_as_float(k ^ ((k >> 31) & 0x7fffffff));
}

__device__ __forceinline__ float bid_value(float x1, float y1, float z1, float qx, float qy,
                                           float qz, float price) {
    const float s = __builtin_sqrtf(pcm_sqd(qx - x1, qy - y1, qz - z1));
    const double v = (3.0 - (double)s) - (double)price;
    return (float)v;
}

// (best, better, best_i) merge: top-2 of the union, lowest index on equal best
__device__ __forceinline__ void top2_merge(float &b, float &c, int &bi, float b2, float c2, int bi2) {
    if (b2 > b || (b2 == b && bi2 >= 0 && (bi < 0 || bi2 < bi))) {
        c = fmaxf(b, c2);
        b = b2;
        bi = bi2;
    } else {
        c = fmaxf(c, b2);
    }
}

__global__ __launch_bounds__(kEmdThreads) void emd_auction_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int n, float eps, int iters,
    float *__restrict__ dist, int32_t *__restrict__ assignment_out, float *__restrict__ price_out) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    int *sAss = smem;                 // [n] assignment (point -> object)
    int *sInv = sAss + n;             // [n] owner (object -> point)
    float *sPrice = (float *)(sInv + n);  // [n]
    int *sMax = (int *)(sPrice + n);  // [n] max increment (f2key)
    int *sClaim = sMax + n;           // [n] lowest qualifying bidder
    int *sBid = sClaim + n;           // [n] bid object per point
    float *sInc = (float *)(sBid + n);  // [n] bid increment per point
    int *sU = (int *)(sInc + n);      // [n] unassigned list
    __shared__ int sNu;

    const int tid = threadIdx.x;
    const int batch = blockIdx.x;
    const float *P = xyz1 + (size_t)batch * n * 3;
    const float *Qc = xyz2 + (size_t)batch * n * 3;

    for (int j = tid; j < n; j += kEmdThreads) {
        sAss[j] = -1;
        sInv[j] = -1;
        sPrice[j] = 0.f;
        sMax[j] = f2key(0.f);  // emd_module.py:49 zero-inits max_increments
        sClaim[j] = 0x7fffffff;
    }
    if (tid == 0) sNu = 0;
    __syncthreads();

    const int lane = tid & 63;
    for (int it = 0; it < iters; ++it) {
        const bool last = (it == iters - 1);
        // ---- A: compact the unassigned points (order irrelevant downstream)
        for (int j0 = 0; j0 < n; j0 += kEmdThreads) {
            const int j = j0 + tid;
            const bool un = (j < n) && sAss[j] == -1;
            const unsigned long long bal = __ballot(un);
            const int below = __popcll(bal & ((1ull << lane) - 1ull));
            int base = 0;
            if (lane == 0 && bal) base = atomicAdd(&sNu, __popcll(bal));
            base = __shfl(base, 0, 64);
            if (un) sU[base + below] = j;
        }
        __syncthreads();
        const int nu = sNu;
        if (nu == 0) break;  // nothing left to bid: later iterations are no-ops

        // ---- B: bids.  G lanes per unassigned point.
        int G = 64;
        while (G > 1 && G * nu > kEmdThreads) G >>= 1;
        const int P_ = kEmdThreads / G;  // points in flight
        const int g = tid / G;           // group id
        const int gl = tid - g * G;      // lane in group
        for (int u0 = 0; u0 < nu; u0 += P_) {
            const int u = u0 + g;
            const bool active = u < nu;
            const int j = active ? sU[u] : 0;
            const float x1 = P[3 * (size_t)j + 0];
            const float y1 = P[3 * (size_t)j + 1];
            const float z1 = P[3 * (size_t)j + 2];
            float best = -1e9f, better = -1e9f;
            int best_i = -1;
            if (active) {
                for (int k = gl; k < n; k += G) {
                    const float d = bid_value(x1, y1, z1, Qc[3 * (size_t)k + 0], Qc[3 * (size_t)k + 1],
                                              Qc[3 * (size_t)k + 2], sPrice[k]);
                    if (d > best) { better = best; best = d; best_i = k; }
                    else if (d > better) { better = d; }
                }
            }
            for (int o = 1; o < G; o <<= 1) {
                const float b2 = __shfl_xor(best, o, 64);
                const float c2 = __shfl_xor(better, o, 64);
                const int i2 = __shfl_xor(best_i, o, 64);
                top2_merge(best, better, best_i, b2, c2, i2);
            }
            if (active && gl == 0) {
                const float inc = best - better + eps;
                sBid[j] = best_i;
                sInc[j] = inc;
                if (best_i >= 0) atomicMax(&sMax[best_i], f2key(inc));
            }
        }
        __syncthreads();

        // ---- C: claim -- lowest bidder inside the reference's 1e-6 window
        for (int u = tid; u < nu; u += kEmdThreads) {
            const int j = sU[u];
            const int k = sBid[j];
            if (k < 0) continue;
            const double bi = (double)sInc[j];
            const double mi = (double)key2f(sMax[k]);
            if (bi - 1e-6 <= mi && mi <= bi + 1e-6) atomicMin(&sClaim[k], j);
        }
        __syncthreads();

        // ---- D: assign (emd_cuda.cu:196-215).  On the last iteration every
        // bidder takes its object; prices/owners are then dead state and are
        // left as they were (the reference's racy updates are unobservable).
        for (int u = tid; u < nu; u += kEmdThreads) {
            const int j = sU[u];
            const int k = sBid[j];
            if (k < 0) continue;
            if (last) {
                sAss[j] = k;
            } else if (sClaim[k] == j) {
                const int old = sInv[k];
                if (old != -1) sAss[old] = -1;
                sInv[k] = j;
                sAss[j] = k;
                sPrice[k] += sInc[j];
                sMax[k] = f2key(-1e9f);
            }
        }
        __syncthreads();
        for (int u = tid; u < nu; u += kEmdThreads) {
            const int k = sBid[sU[u]];
            if (k >= 0) sClaim[k] = 0x7fffffff;
        }
        if (tid == 0) sNu = 0;
        __syncthreads();
    }

    // ---- CalcDist (emd_cuda.cu:217-226): deltas xyz1 - xyz2
    for (int j = tid; j < n; j += kEmdThreads) {
        const int k = sAss[j];
        float d = 0.f;
        if (k >= 0) {
            d = pcm_sqd(P[3 * (size_t)j + 0] - Qc[3 * (size_t)k + 0],
                        P[3 * (size_t)j + 1] - Qc[3 * (size_t)k + 1],
                        P[3 * (size_t)j + 2] - Qc[3 * (size_t)k + 2]);
        }
        dist[(size_t)batch * n + j] = d;
        assignment_out[(size_t)batch * n + j] = k;
        if (price_out) price_out[(size_t)batch * n + j] = sPrice[j];
    }
}

__global__ void emd_bwd_kernel(const float *__restrict__ xyz1, const float *__restrict__ xyz2, int n,
                               size_t total, const float *__restrict__ graddist,
                               const int32_t *__restrict__ assignment, float *__restrict__ grad) {
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
         t += (size_t)gridDim.x * blockDim.x) {
        const size_t batch = t / n;
        const int k = assignment[t];
        const float g = __fmul_rn(graddist[t], 2.f);
        const float *p = xyz1 + 3 * t;
        const float *q = xyz2 + 3 * (batch * n + (size_t)k);
#pragma unroll
        for (int c = 0; c < 3; ++c) grad[3 * t + c] = __fadd_rn(0.f, __fmul_rn(g, __fsub_rn(p[c], q[c])));
    }
}

size_t emd_lds_bytes(int n) { return (size_t)8 * 4 * n; }

}  // namespace

extern "C" size_t pcm_emd_workspace_bytes(int b, int n) {
    (void)b;
    (void)n;
    return 0;  // v1 keeps the whole auction state in LDS
}

extern "C" int pcm_emd_forward(const float *xyz1, const float *xyz2, int b, int n, float eps,
                               int iters, float *dist, int32_t *assignment, float *price,
                               void *workspace, size_t workspace_bytes, void *stream) {
    (void)workspace;
    (void)workspace_bytes;
    // emd_cuda.cu:236-249 (n == m is enforced by the single n here)
    if (b < 0 || n < 0 || b > 512 || n % 1024 != 0 || iters < 1) return PCM_ERR_INVALID_ARG;
    if (b == 0 || n == 0) return PCM_OK;
    if (!xyz1 || !xyz2 || !dist || !assignment) return PCM_ERR_INVALID_ARG;
    if (n > kEmdMaxN) return PCM_ERR_UNSUPPORTED;
    const size_t lds = emd_lds_bytes(n);
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)emd_auction_kernel,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return PCM_ERR_LAUNCH;
    hipLaunchKernelGGL(emd_auction_kernel, dim3(b), dim3(kEmdThreads), lds, (hipStream_t)stream, xyz1,
                       xyz2, n, eps, iters, dist, assignment, price);
    return pcm_launch_status();
}

extern "C" int pcm_emd_backward(const float *xyz1, const float *xyz2, int b, int n,
                                const float *graddist, const int32_t *assignment, float *gradxyz1,
                                void *stream) {
    if (b < 0 || n < 0) return PCM_ERR_INVALID_ARG;
    if (b == 0 || n == 0) return PCM_OK;
    if (!xyz1 || !xyz2 || !graddist || !assignment || !gradxyz1) return PCM_ERR_INVALID_ARG;
    const size_t total = (size_t)b * n;
    const unsigned blocks = (unsigned)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    hipLaunchKernelGGL(emd_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, xyz1, xyz2, n,
                       total, graddist, assignment, gradxyz1);
    return pcm_launch_status();
}
