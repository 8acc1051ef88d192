// chamfer.hip -- Chamfer3D forward/backward for MI355X (gfx950, CDNA4).
//
// Replaces the reference's NmDistanceKernel / NmDistanceGradKernel
// (metric/chamfer3D/chamfer3D.cu:12-195).  Design:
//
// Forward: ONE launch computes both directions.  A workgroup owns 64*QPT query
// points of one (direction, batch) and W waves; the opposing cloud is staged
// through LDS in SoA tiles (X[], Y[], Z[] so one ds_read_b128 broadcast yields
// four candidates' x), and each wave scans an interleaved 1/W share of the
// tile's chunks of C candidates.  Distances are evaluated two candidates at a
// time in packed-fp32 (v_pk_add/mul/fma_f32) in the pinned order
// fma(dz,dz,fma(dy,dy,dx*dx)); a chunk's minimum is folded with v_min3_f32
// and only the chunk id of the running minimum is tracked (strict '<', so the
// lowest chunk wins).  After the waves' (min, chunk) pairs are merged
// lexicographically, the single winning chunk is re-scanned to recover the
// lowest index attaining the minimum -- bit-identical to the reference's
// lowest-index first-min scan, at ~1/C of the compare/select cost.
// Non-finite coordinates (where the reference's 512-point tile boundaries
// decide NaN outcomes) divert the whole workgroup to a reference-exact scan.
//
// Backward: deterministic.  A workgroup owns up to 1024 points of one cloud;
// it gathers the direct term and sums the reverse-direction scatter terms in
// ascending source index, using an LDS counting sort of the other
// direction's argmin indices (no float atomics).
#include "pcm_common.h"

namespace {

constexpr int kFwdW = 4;      // waves per workgroup (split the candidate chunks)
constexpr int kFwdQPT = 2;    // query points per lane
constexpr int kFwdC = 32;     // candidates per chunk
constexpr int kFwdTile = 2048;  // candidates per LDS tile (3 x 8 KiB)

template <int W, int QPT, int C, int TILE>
__global__ __launch_bounds__(64 * W) void chamfer_fwd_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int b, int n, int m,
    float *__restrict__ dist1, float *__restrict__ dist2, int32_t *__restrict__ idx1,
    int32_t *__restrict__ idx2, int nblk1, int nblk2) {
    static_assert(TILE % C == 0 && C % 4 == 0, "tile must hold whole chunks");
    constexpr int QW = 64 * QPT;
    constexpr int NT = 64 * W;
    __shared__ __attribute__((aligned(16))) float sXYZ[3][TILE];
    __shared__ float sBest[W][QW];
    __shared__ int sChunk[W][QW];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    // ---- which (direction, batch, query block) this workgroup owns (uniform)
    int bid = blockIdx.x;
    const float *Q, *T;
    float *D;
    int32_t *I;
    int nq, nt, blk;
    if (bid < b * nblk1) {
        const int batch = bid / nblk1;
        blk = bid - batch * nblk1;
        Q = xyz1 + (size_t)batch * n * 3;
        T = xyz2 + (size_t)batch * m * 3;
        D = dist1 + (size_t)batch * n;
        I = idx1 + (size_t)batch * n;
        nq = n;
        nt = m;
    } else {
        bid -= b * nblk1;
        const int batch = bid / nblk2;
        blk = bid - batch * nblk2;
        Q = xyz2 + (size_t)batch * m * 3;
        T = xyz1 + (size_t)batch * n * 3;
        D = dist2 + (size_t)batch * m;
        I = idx2 + (size_t)batch * m;
        nq = m;
        nt = n;
    }
    const int qbase = blk * QW;

    // ---- this lane's query points (splatted for the packed math)
    pcm_f2 px[QPT], py[QPT], pz[QPT];
    bool nonfinite = false;
#pragma unroll
    for (int qq = 0; qq < QPT; ++qq) {
        const int qi = qbase + qq * 64 + lane;
        float x = 0.f, y = 0.f, z = 0.f;
        if (qi < nq) {
            x = Q[3 * (size_t)qi + 0];
            y = Q[3 * (size_t)qi + 1];
            z = Q[3 * (size_t)qi + 2];
            nonfinite |= !(pcm_finite(x) && pcm_finite(y) && pcm_finite(z));
        }
        px[qq] = pcm_f2{x, x};
        py[qq] = pcm_f2{y, y};
        pz[qq] = pcm_f2{z, z};
    }

    float best[QPT];
    int bchunk[QPT];
#pragma unroll
    for (int qq = 0; qq < QPT; ++qq) { best[qq] = PCM_INF; bchunk[qq] = 0; }

    for (int t0 = 0; t0 < nt; t0 += TILE) {
        const int cnt = min(TILE, nt - t0);
        const int padded = (cnt + C - 1) / C * C;
        __syncthreads();  // previous tile fully consumed
        // coalesced flat read of the AoS tile, scattered to SoA; pad = +inf
        const float *src = T + 3 * (size_t)t0;
        for (int f = tid; f < 3 * padded; f += NT) {
            const int p = f / 3;
            const int comp = f - 3 * p;
            float v = PCM_INF;
            if (p < cnt) {
                v = src[f];
                nonfinite |= !pcm_finite(v);
            }
            sXYZ[comp][p] = v;
        }
        __syncthreads();

        const int nch = padded / C;
        const int gc0 = t0 / C;
        for (int c = wave; c < nch; c += W) {
            float mn[QPT];
#pragma unroll
            for (int qq = 0; qq < QPT; ++qq) mn[qq] = PCM_INF;
            const float *cx = &sXYZ[0][c * C];
            const float *cy = &sXYZ[1][c * C];
            const float *cz = &sXYZ[2][c * C];
#pragma unroll
            for (int k = 0; k < C; k += 4) {
                const pcm_f4 X4 = *reinterpret_cast<const pcm_f4 *>(cx + k);
                const pcm_f4 Y4 = *reinterpret_cast<const pcm_f4 *>(cy + k);
                const pcm_f4 Z4 = *reinterpret_cast<const pcm_f4 *>(cz + k);
                const pcm_f2 xa = X4.xy, xb = X4.zw;
                const pcm_f2 ya = Y4.xy, yb = Y4.zw;
                const pcm_f2 za = Z4.xy, zb = Z4.zw;
#pragma unroll
                for (int qq = 0; qq < QPT; ++qq) {
                    const pcm_f2 da = pcm_sqd2(xa - px[qq], ya - py[qq], za - pz[qq]);
                    const pcm_f2 db = pcm_sqd2(xb - px[qq], yb - py[qq], zb - pz[qq]);
                    mn[qq] = __builtin_fminf(mn[qq], __builtin_fminf(da.x, da.y));
                    mn[qq] = __builtin_fminf(mn[qq], __builtin_fminf(db.x, db.y));
                }
            }
#pragma unroll
            for (int qq = 0; qq < QPT; ++qq) {
                if (mn[qq] < best[qq]) {
                    best[qq] = mn[qq];
                    bchunk[qq] = gc0 + c;
                }
            }
        }
    }

    // ---- merge the W waves' (min, chunk) per query; recover the lowest index
#pragma unroll
    for (int qq = 0; qq < QPT; ++qq) {
        sBest[wave][qq * 64 + lane] = best[qq];
        sChunk[wave][qq * 64 + lane] = bchunk[qq];
    }
    const int any_nonfinite = __syncthreads_or(nonfinite ? 1 : 0);
    if (nt == 0) return;  // reference leaves outputs untouched when m == 0

    for (int s = tid; s < QW; s += NT) {
        const int qi = qbase + s;
        if (qi >= nq) continue;
        const float x = Q[3 * (size_t)qi + 0];
        const float y = Q[3 * (size_t)qi + 1];
        const float z = Q[3 * (size_t)qi + 2];
        float d;
        int idx;
        if (any_nonfinite) {
            pcm_ref_nn_scan(x, y, z, T, nt, d, idx);
        } else {
            float fb = sBest[0][s];
            int fc = sChunk[0][s];
#pragma unroll
            for (int w = 1; w < W; ++w) {
                const float v = sBest[w][s];
                const int c = sChunk[w][s];
                if (v < fb || (v == fb && c < fc)) { fb = v; fc = c; }
            }
            const int k0 = fc * C;
            const int k1 = min(k0 + C, nt);
            idx = k0;
            for (int k = k0; k < k1; ++k) {
                const float *q = T + 3 * (size_t)k;
                if (pcm_sqd(q[0] - x, q[1] - y, q[2] - z) == fb) { idx = k; break; }
            }
            d = fb;
        }
        D[qi] = d;
        I[qi] = idx;
    }
}

// ---------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------
constexpr int kBwdThreads = 1024;   // targets per workgroup = threads
constexpr int kBwdCap = 8192;       // scatter entries sortable in LDS per workgroup

// exclusive scan of one value per thread over a 1024-thread workgroup
__device__ inline int block_exclusive_scan_1024(int v, int *wave_tot) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wave_tot[wave] = x;
    __syncthreads();
    if (wave == 0) {
        int t = lane < (kBwdThreads / 64) ? wave_tot[lane] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(t, o, 64);
            if (lane >= o) t += y;
        }
        if (lane < (kBwdThreads / 64)) wave_tot[lane] = t;  // inclusive wave prefix
    }
    __syncthreads();
    const int before = wave == 0 ? 0 : wave_tot[wave - 1];
    return before + x - v;
}

__global__ __launch_bounds__(kBwdThreads) void chamfer_bwd_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int b, int n, int m,
    const float *__restrict__ gd1, const float *__restrict__ gd2, const int32_t *__restrict__ idx1,
    const int32_t *__restrict__ idx2, float *__restrict__ grad1, float *__restrict__ grad2,
    int nblk1, int nblk2) {
    __shared__ int sCnt[kBwdThreads];
    __shared__ int sOff[kBwdThreads + 1];
    __shared__ int sTmp[kBwdCap];
    __shared__ int sSrt[kBwdCap];
    __shared__ int sWave[kBwdThreads / 64];

    const int tid = threadIdx.x;
    int bid = blockIdx.x;
    // cloud 1 (direct term first) or cloud 2 (direct term last): reference
    // kernel order chamfer3D.cu:184-185.
    const float *self, *other, *gds, *gdo;
    const int32_t *ids, *ido;
    float *grad;
    int ns, no, blk;
    bool direct_first;
    if (bid < b * nblk1) {
        const int batch = bid / nblk1;
        blk = bid - batch * nblk1;
        self = xyz1 + (size_t)batch * n * 3;
        other = xyz2 + (size_t)batch * m * 3;
        gds = gd1 + (size_t)batch * n;
        gdo = gd2 + (size_t)batch * m;
        ids = idx1 + (size_t)batch * n;
        ido = idx2 + (size_t)batch * m;
        grad = grad1 + (size_t)batch * n * 3;
        ns = n;
        no = m;
        direct_first = true;
    } else {
        bid -= b * nblk1;
        const int batch = bid / nblk2;
        blk = bid - batch * nblk2;
        self = xyz2 + (size_t)batch * m * 3;
        other = xyz1 + (size_t)batch * n * 3;
        gds = gd2 + (size_t)batch * m;
        gdo = gd1 + (size_t)batch * n;
        ids = idx2 + (size_t)batch * m;
        ido = idx1 + (size_t)batch * n;
        grad = grad2 + (size_t)batch * m * 3;
        ns = m;
        no = n;
        direct_first = false;
    }
    const int t0 = blk * kBwdThreads;
    const int T = min(kBwdThreads, ns - t0);

    // 1. histogram of the other direction's argmins that land in [t0, t0+T)
    sCnt[tid] = 0;
    __syncthreads();
    for (int j = tid; j < no; j += kBwdThreads) {
        const unsigned k = (unsigned)(ido[j] - t0);
        if (k < (unsigned)T) atomicAdd(&sCnt[k], 1);
    }
    __syncthreads();
    // 2. bucket offsets
    const int c = sCnt[tid];
    const int off = block_exclusive_scan_1024(c, sWave);
    sOff[tid] = off;
    if (tid == kBwdThreads - 1) sOff[kBwdThreads] = off + c;
    sCnt[tid] = 0;
    __syncthreads();
    const int total = sOff[kBwdThreads];
    const bool fits = total <= kBwdCap;  // uniform

    if (fits) {
        // 3. fill buckets (arbitrary order inside a bucket) ...
        for (int j = tid; j < no; j += kBwdThreads) {
            const unsigned k = (unsigned)(ido[j] - t0);
            if (k < (unsigned)T) {
                const int s = atomicAdd(&sCnt[k], 1);
                sTmp[sOff[k] + s] = j;
            }
        }
        __syncthreads();
        // 4. ... then rank each entry by source index inside its bucket
        for (int p = tid; p < total; p += kBwdThreads) {
            const int j = sTmp[p];
            const int k = ido[j] - t0;
            const int lo = sOff[k], hi = sOff[k + 1];
            int r = 0;
            for (int q = lo; q < hi; ++q) r += (sTmp[q] < j);
            sSrt[lo + r] = j;
        }
        __syncthreads();
    }

    if (tid >= T) return;
    const int i = t0 + tid;
    const float sx = self[3 * (size_t)i + 0];
    const float sy = self[3 * (size_t)i + 1];
    const float sz = self[3 * (size_t)i + 2];
    float dir[3];
    {
        const int k = ids[i];
        const float g = __fmul_rn(gds[i], 2.f);
        dir[0] = __fmul_rn(g, __fsub_rn(sx, other[3 * (size_t)k + 0]));
        dir[1] = __fmul_rn(g, __fsub_rn(sy, other[3 * (size_t)k + 1]));
        dir[2] = __fmul_rn(g, __fsub_rn(sz, other[3 * (size_t)k + 2]));
    }
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (direct_first) {
        ax = __fadd_rn(ax, dir[0]);
        ay = __fadd_rn(ay, dir[1]);
        az = __fadd_rn(az, dir[2]);
    }
    auto scatter = [&](int j) {
        const float g = __fmul_rn(gdo[j], 2.f);
        ax = __fadd_rn(ax, -__fmul_rn(g, __fsub_rn(other[3 * (size_t)j + 0], sx)));
        ay = __fadd_rn(ay, -__fmul_rn(g, __fsub_rn(other[3 * (size_t)j + 1], sy)));
        az = __fadd_rn(az, -__fmul_rn(g, __fsub_rn(other[3 * (size_t)j + 2], sz)));
    };
    if (fits) {
        const int lo = sOff[tid], hi = sOff[tid + 1];
        for (int p = lo; p < hi; ++p) scatter(sSrt[p]);
    } else {
        // degenerate clouds (many sources collapsing onto few targets): plain
        // ordered scan of the other direction's indices.
        for (int j = 0; j < no; ++j)
            if (ido[j] == i) scatter(j);
    }
    if (!direct_first) {
        ax = __fadd_rn(ax, dir[0]);
        ay = __fadd_rn(ay, dir[1]);
        az = __fadd_rn(az, dir[2]);
    }
    grad[3 * (size_t)i + 0] = ax;
    grad[3 * (size_t)i + 1] = ay;
    grad[3 * (size_t)i + 2] = az;
}

inline bool bad_dims(int b, int n, int m) { return b < 0 || n < 0 || m < 0; }

}  // namespace

extern "C" int pcm_chamfer_forward(const float *xyz1, const float *xyz2, int b, int n, int m,
                                   float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                   void *stream) {
    if (bad_dims(b, n, m)) return PCM_ERR_INVALID_ARG;
    if (b == 0 || (n == 0 && m == 0)) return PCM_OK;
    if ((n > 0 && (!xyz1 || !dist1 || !idx1)) || (m > 0 && (!xyz2 || !dist2 || !idx2)))
        return PCM_ERR_INVALID_ARG;
    constexpr int QW = 64 * kFwdQPT;
    // a direction with no targets leaves its outputs untouched: give it no blocks
    const int nblk1 = (m > 0) ? (n + QW - 1) / QW : 0;
    const int nblk2 = (n > 0) ? (m + QW - 1) / QW : 0;
    const long long blocks = (long long)b * (nblk1 + nblk2);
    if (blocks == 0) return PCM_OK;
    if (blocks > 0x7fffffffLL) return PCM_ERR_UNSUPPORTED;
    hipLaunchKernelGGL((chamfer_fwd_kernel<kFwdW, kFwdQPT, kFwdC, kFwdTile>), dim3((unsigned)blocks),
                       dim3(64 * kFwdW), 0, (hipStream_t)stream, xyz1, xyz2, b, n, m, dist1, dist2,
                       idx1, idx2, nblk1, nblk2);
    return pcm_launch_status();
}

extern "C" int pcm_chamfer_backward(const float *xyz1, const float *xyz2, int b, int n, int m,
                                    const float *graddist1, const float *graddist2,
                                    const int32_t *idx1, const int32_t *idx2, float *gradxyz1,
                                    float *gradxyz2, void *stream) {
    if (bad_dims(b, n, m)) return PCM_ERR_INVALID_ARG;
    if (b == 0 || (n == 0 && m == 0)) return PCM_OK;
    // Without targets a direction has no argmins; the reference would read
    // garbage indices.  Both clouds must be non-empty for a gradient.
    if (n == 0 || m == 0) return PCM_ERR_INVALID_ARG;
    if (!xyz1 || !xyz2 || !graddist1 || !graddist2 || !idx1 || !idx2 || !gradxyz1 || !gradxyz2)
        return PCM_ERR_INVALID_ARG;
    const int nblk1 = (n + kBwdThreads - 1) / kBwdThreads;
    const int nblk2 = (m + kBwdThreads - 1) / kBwdThreads;
    const long long blocks = (long long)b * (nblk1 + nblk2);
    if (blocks > 0x7fffffffLL) return PCM_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(chamfer_bwd_kernel, dim3((unsigned)blocks), dim3(kBwdThreads), 0,
                       (hipStream_t)stream, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2,
                       gradxyz1, gradxyz2, nblk1, nblk2);
    return pcm_launch_status();
}
