// icp.hip -- ICP alignment for the evaluation caller.
//
// Reference: utils/icp.py (numpy + sklearn) called once per sample by
// testnet.py:62-64 / test_pix.py with tolerance=1e-10, max_iterations=1024:
//   nearest_neighbor    icp.py:49-65   sklearn NearestNeighbors(1), float64
//   best_fit_transform  icp.py:4-46    centroids, H = AA^T BB, SVD, R = V U^T,
//                                      reflection fix, t = cB - R cA
//   icp                 icp.py:68-118  NN -> best fit -> src = T src until
//                                      |prev - mean(dist)| < tolerance
//
// MI355X design: a prep kernel writes B's screening rows once; then one
// 1024-thread workgroup owns one (A, B) pair and runs the whole loop in one
// launch -- the source cloud stays in LDS (float64) across iterations, so
// there is no per-iteration launch or host round trip.  Per iteration:
//   1. nearest neighbour of every source point: a float32 screen over rows
//      (-2t, |t|^2) of B streamed through SGPRs (3 FMAs + half a min3 per
//      pair; chunk minima with their second best), then an exact float64
//      decision.  The float32 value of a pair differs
//      from the exact one by at most E = 2^-21 (|q| + R)^2 (coordinates
//      centred on B's centroid, R = max |t|; the rounding analysis is in
//      DESIGN.md §3.6).  If second > best + 2E the
//      float32 winner IS the float64 winner; otherwise every candidate within
//      best + 2E is re-scored in float64 (lowest index on exact ties).  The
//      returned distance is sqrt((dx*dx + dy*dy) + dz*dz) in float64 -- the
//      expression sklearn's Euclidean rdist evaluates;
//   2. fixed-order float64 block reductions: centroids and mean distance,
//      then the 3x3 cross-covariance of the centred pairs;
//   3. thread 0: 3x3 SVD by one-sided Jacobi, R = V U^T with the reflection
//      fix, T; convergence test exactly as icp.py:111-114;
//   4. src = T src (homogeneous, float64, in LDS).
// The final transform is best_fit_transform(A, src) (icp.py:117).
#include "pcm_common.h"

namespace {

constexpr int kIcpThreads = 1024;
constexpr int kIcpWaves = kIcpThreads / 64;
constexpr int kIcpMaxN = 16384;                // 16 slices of <= 1024 points per pair
constexpr int kIcpRowsLdsMax = 96 * 1024;      // rows staged in LDS for the rescans up to this size
constexpr int kNnThreads = 256;                // one query per thread
constexpr int kPrepThreads = 256;
constexpr float kNnErr = 4.76837158203125e-07f;  // 2^-21

// ---- float64 helpers --------------------------------------------------------

// sklearn's Euclidean rdist: d = 0; d += tmp*tmp per coordinate (no fma;
// the Makefile builds with -ffp-contract=off)
template <typename P>
__device__ __forceinline__ double sqd64(double sx, double sy, double sz, P t) {
    const double dx = sx - t[0], dy = sy - t[1], dz = sz - t[2];
    return (dx * dx + dy * dy) + dz * dz;
}

// Fixed-order workgroup sum of NV doubles per thread (v is consumed); every
// thread then reads the totals from out[0..NV).  Two barriers; red/out may be
// reused by the next call.
// 64-lane sum into lane 63 by DPP moves (no LDS round trips): quad swaps,
// row_shr 4 / 8, row_bcast 15 / 31 -- a fixed pattern, so deterministic.  A
// double moves as two 32-bit halves with the same control.
template <int CTRL>
__device__ __forceinline__ double dpp_move(double v) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Fixed-order workgroup sum of NV doubles per thread (v is consumed); every
// thread then reads the totals from out[0..NV).  Two barriers; red/out may be
// reused by the next call.
template <int NV, int W>
__device__ __forceinline__ void block_sum(double (&v)[NV], double (*red)[W], double *out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0xb1>(v[i]);   // quad_perm [1,0,3,2]
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x4e>(v[i]);   // quad_perm [2,3,0,1]
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x114>(v[i]);  // row_shr:4
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x118>(v[i]);  // row_shr:8
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x142>(v[i]);  // row_bcast:15
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x143>(v[i]);  // row_bcast:31
    if (lane == 63) {
#pragma unroll
        for (int i = 0; i < NV; ++i) red[i][wave] = v[i];
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        double s = 0.0;
        for (int w = 0; w < W; ++w) s += red[threadIdx.x][w];
        out[threadIdx.x] = s;
    }
    __syncthreads();
}

template <int W>
__device__ __forceinline__ float block_max(float v, float *red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = pcm_wave_max_f32(v == v ? v : -PCM_INF);  // DPP steps; NaN counts as nothing, as fmaxf
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float r = red[0];
    for (int w = 1; w < W; ++w) r = fmaxf(r, red[w]);
    __syncthreads();
    return r;
}

// ---- Kabsch (best_fit_transform, icp.py:22-46) ------------------------------

__device__ __forceinline__ double dot3(const double *a, const double *b) {
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}

__device__ __forceinline__ void cross3(const double *a, const double *b, double *c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ void normalize3(double *a) {
    const double s = sqrt(dot3(a, a));
    if (s > 0.0) { a[0] /= s; a[1] /= s; a[2] /= s; }
}

// H (row-major, H[i][j] = sum_k AA[k][i] BB[k][j]) -> T = [R t] (3x4, row-major)
// with R = V U^T the proper rotation of H = U S V^T (the reflection fix of
// icp.py:34-36 keeps det R = +1: the smallest singular pair enters with the
// sign that makes det R = +1), t = cb - R ca.
// vwarm (optional, in/out): an orthogonal start for V -- the previous ICP
// pass's V, which nearly diagonalises this pass's H, so the Jacobi sweeps
// converge in one or two instead of four or five.
__device__ void kabsch(const double *Hin, const double *ca, const double *cb, double *T, double *vwarm = nullptr) {
    double h[3][3], v[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) v[i][j] = vwarm ? vwarm[3 * i + j] : (i == j) ? 1.0 : 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            h[i][j] = (Hin[3 * i] * v[0][j] + Hin[3 * i + 1] * v[1][j]) + Hin[3 * i + 2] * v[2][j];
    // one-sided Jacobi: rotate column pairs of h until orthogonal (h V = U S)
    // (columns count as orthogonal at |gamma| <= 1e-15 sqrt(alpha beta), ~4.5
    // ulp: a tighter test is below what rounding lets a rotation reach and
    // would spin to the sweep cap)
    for (int sweep = 0; sweep < 16; ++sweep) {
        bool rotated = false;
        for (int pq = 0; pq < 3; ++pq) {
            const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
            double alpha = 0.0, beta = 0.0, gamma = 0.0;
            for (int i = 0; i < 3; ++i) {
                alpha += h[i][p] * h[i][p];
                beta += h[i][q] * h[i][q];
                gamma += h[i][p] * h[i][q];
            }
            if (!(fabs(gamma) > 1e-15 * sqrt(alpha * beta))) continue;
            rotated = true;
            const double zeta = (beta - alpha) / (2.0 * gamma);
            const double az = fabs(zeta);
            const double t = az > 1e150 ? 0.5 / zeta : copysign(1.0, zeta) / (az + sqrt(1.0 + zeta * zeta));
            const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
            for (int i = 0; i < 3; ++i) {
                const double hp = h[i][p], hq = h[i][q];
                h[i][p] = c * hp - s * hq;
                h[i][q] = s * hp + c * hq;
                const double vp = v[i][p], vq = v[i][q];
                v[i][p] = c * vp - s * vq;
                v[i][q] = s * vp + c * vq;
            }
        }
        if (!rotated) break;
    }
    // singular values = column norms; order descending (LAPACK's order)
    // (compare-swap network on whole columns: static indices only, so the
    // arrays stay in registers)
    double sig[3];
    for (int j = 0; j < 3; ++j) sig[j] = sqrt(h[0][j] * h[0][j] + h[1][j] * h[1][j] + h[2][j] * h[2][j]);
    auto cswap = [&](int p, int q) {
        if (sig[p] < sig[q]) {
            const double s = sig[p]; sig[p] = sig[q]; sig[q] = s;
            for (int i = 0; i < 3; ++i) {
                const double x = h[i][p]; h[i][p] = h[i][q]; h[i][q] = x;
                const double y = v[i][p]; v[i][p] = v[i][q]; v[i][q] = y;
            }
        }
    };
    cswap(0, 1);
    cswap(1, 2);
    cswap(0, 1);
    double u1[3], u2[3], u3[3], v1[3], v2[3], v3[3];
    for (int i = 0; i < 3; ++i) {
        u1[i] = h[i][0]; u2[i] = h[i][1];
        v1[i] = v[i][0]; v2[i] = v[i][1]; v3[i] = v[i][2];
    }
    if (vwarm)
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) vwarm[3 * i + j] = v[i][j];
    double R[3][3];
    if (sig[0] == 0.0) {  // H == 0: numpy's SVD gives U = V = I, R = I
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R[i][j] = (i == j) ? 1.0 : 0.0;
    } else {
        normalize3(u1);
        const double pr = dot3(u2, u1);
        for (int i = 0; i < 3; ++i) u2[i] -= pr * u1[i];
        if (dot3(u2, u2) <= 1e-30 * sig[0] * sig[0]) {  // rank 1: any unit vector orthogonal to u1
            const double e[3] = {fabs(u1[0]) < 0.6 ? 1.0 : 0.0, fabs(u1[0]) < 0.6 ? 0.0 : 1.0, 0.0};
            cross3(u1, e, u2);
        }
        normalize3(u2);
        cross3(u1, u2, u3);  // det U = +1
        double vx[3];
        cross3(v2, v3, vx);
        const double sgn = dot3(v1, vx) < 0.0 ? -1.0 : 1.0;  // det V of the sorted columns
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R[i][j] = (v1[i] * u1[j] + v2[i] * u2[j]) + sgn * v3[i] * u3[j];
    }
    for (int i = 0; i < 3; ++i) {
        T[4 * i + 0] = R[i][0];
        T[4 * i + 1] = R[i][1];
        T[4 * i + 2] = R[i][2];
        T[4 * i + 3] = cb[i] - ((R[i][0] * ca[0] + R[i][1] * ca[1]) + R[i][2] * ca[2]);
    }
}

// ---- nearest neighbour: float32 screen + exact float64 decision ------------
//
// Rows: per destination cloud, rows[j] = (-2 t'_j, |t'_j|^2) with
// t' = fl32(dst_j - c) (c = the cloud's centroid), padded to a multiple of kChunk
// with (0, 0, 0, +inf).  d'(q, j) = |t'|^2 - 2 t'.q' ranks j like |q' - t'|^2.
// The rows are written by nn_prep_kernel and only read afterwards, so the scan
// reads them through the constant address space: every wave walks the same
// rows, the addresses are wave-uniform, and hipcc streams them with s_load into
// SGPRs that feed the FMAs directly (no LDS traffic; one v_min3 per two rows).

typedef const __attribute__((address_space(4))) pcm_f4 pcm_cf4;

constexpr int kChunk = 32;

struct NnHdr {      // per destination cloud, written by nn_prep_kernel
    double c[3];    // centroid
    float R;        // max |t'|
    int pad;
};

__host__ __device__ inline int nn_mpad(int m) { return (m + kChunk - 1) / kChunk * kChunk; }

__device__ __forceinline__ float row_d(const pcm_f4 t, float qx, float qy, float qz) {
    return __builtin_fmaf(t.x, qx, __builtin_fmaf(t.y, qy, __builtin_fmaf(t.z, qz, t.w)));
}

// Screen of one query against all mpad rows.  Returns d1 = min d', k1 = the
// lowest index attaining it, d2 = min over j != k1 of d'.  Chunk minima are
// tracked with their second best (med3), then the winning chunk is rescanned
// per candidate.
template <typename RowPtr, typename RowPtrV>
__device__ __forceinline__ void nn_screen(RowPtr rows, RowPtrV rows_v, int mpad, float qx,
                                          float qy, float qz, float &d1, float &d2, int &k1) {
    float b1 = PCM_INF, b2 = PCM_INF;
    int c1 = 0;
    const int nch = mpad / kChunk;
    for (int c = 0; c < nch; ++c) {
        RowPtr tk = rows + c * kChunk;
        float mn = PCM_INF;
#pragma unroll
        for (int k = 0; k < kChunk; k += 2) {
            const float da = row_d(tk[k], qx, qy, qz);
            const float db = row_d(tk[k + 1], qx, qy, qz);
            mn = __builtin_fminf(__builtin_fminf(mn, da), db);
        }
        b2 = __builtin_amdgcn_fmed3f(b1, b2, mn);  // second smallest chunk minimum (b1 <= b2)
        const bool lt = mn < b1;
        b1 = lt ? mn : b1;
        c1 = lt ? c : c1;
    }
    // rescan the winning chunk (per-lane chunk: vector loads, L1/L2 resident, or LDS)
    RowPtrV tk = rows_v + c1 * kChunk;
    float e1 = PCM_INF, e2 = PCM_INF;
    int j1 = 0;
#pragma unroll 8
    for (int k = 0; k < kChunk; ++k) {
        const float d = row_d(tk[k], qx, qy, qz);
        e2 = __builtin_amdgcn_fmed3f(e1, e2, d);
        const bool lt = d < e1;
        e1 = lt ? d : e1;
        j1 = lt ? k : j1;
    }
    d1 = e1;
    k1 = c1 * kChunk + j1;
    d2 = __builtin_fminf(e2, b2);
}

// Exact float64 decision for one query s (float64) given its screen.  The
// screened value of a pair differs from the exact |s - t|^2 - |q'|^2 by at most
// E = 2^-21 (|q'| + R)^2, so only rows with d' <= d1 + 2E can
// be the exact nearest; when d2 is above that, k1 is it.  Otherwise every
// candidate within d1 + 2E is re-scored in float64 (lowest index on exact
// ties): one more pass over the rows, taken by the whole wave when any lane
// needs it, with the rows and the float64 destination points streamed through
// SGPRs (the loop index is wave-uniform).  Returns the index; e2 = the squared
// distance in sklearn's expression.
typedef const __attribute__((address_space(4))) double pcm_cd;

template <typename RowPtr>
__device__ __forceinline__ int nn_decide(double sx, double sy, double sz, float qx, float qy, float qz, float d1,
                                         float d2, int k1, RowPtr rows, int mpad, const double *__restrict__ dst,
                                         double &e2) {
    // local bound: any row that could beat k1 lies within sqrt(D1) of q
    // (D1 = exact squared distance to k1), so |t| <= |q| + sqrt(D1) for every
    // row that matters
    const double e1 = sqd64(sx, sy, sz, dst + 3 * (size_t)k1);
    const float qn = sqrtf(__builtin_fmaf(qz, qz, __builtin_fmaf(qy, qy, qx * qx)));
    const float rr = 2.f * qn + sqrtf((float)e1) + 1e-30f;
    const float E = kNnErr * rr * rr;
    const float lim = d1 + 2.f * E;
#ifdef PCM_NN_NOFALLBACK  // A/B timing build only (tools/tune_icp.py)
    const bool fb = false;
#else
    const bool fb = !(d2 > lim);
#endif
    int bk = k1;
    if (__any(fb)) {
        // chunk by chunk as in the screen (unrolled s_load stream); only
        // chunks whose minimum is within lim are re-scored row by row
        pcm_cd *dc = (pcm_cd *)(uintptr_t)dst;
        double best = __builtin_huge_val();
        const int nch = mpad / kChunk;
        for (int c = 0; c < nch; ++c) {
            RowPtr tk = rows + c * kChunk;
            float mn = PCM_INF;
#pragma unroll
            for (int k = 0; k < kChunk; k += 2) {
                const float da = row_d(tk[k], qx, qy, qz);
                const float db = row_d(tk[k + 1], qx, qy, qz);
                mn = __builtin_fminf(__builtin_fminf(mn, da), db);
            }
            if (fb & (mn <= lim)) {
                for (int k = 0; k < kChunk; ++k) {
                    const int j = c * kChunk + k;
                    if (row_d(tk[k], qx, qy, qz) <= lim) {  // padding rows give +inf
                        const double e = sqd64(sx, sy, sz, dc + 3 * (size_t)j);
                        if (e < best) { best = e; bk = j; }
                    }
                }
            }
        }
    }
    e2 = bk == k1 ? e1 : sqd64(sx, sy, sz, dst + 3 * (size_t)bk);
    return bk;
}

template <int W>
__device__ __forceinline__ void centroid3(const double *__restrict__ p, int n, double (*red)[W], double *out,
                                          double *c) {
    double s[3] = {0.0, 0.0, 0.0};
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        s[0] += p[3 * (size_t)j];
        s[1] += p[3 * (size_t)j + 1];
        s[2] += p[3 * (size_t)j + 2];
    }
    block_sum<3, W>(s, red, out);
    c[0] = out[0] / n; c[1] = out[1] / n; c[2] = out[2] / n;
}

// One workgroup per destination cloud: centroid, rows, R.
__global__ __launch_bounds__(kPrepThreads) void nn_prep_kernel(const double *__restrict__ dst, int m,
                                                               NnHdr *__restrict__ hdr, pcm_f4 *__restrict__ rows,
                                                               unsigned *__restrict__ arrive, unsigned *__restrict__ err) {
    constexpr int W = kPrepThreads / 64;
    __shared__ double red[3][W];
    __shared__ double tot[3];
    __shared__ float redf[W];
    const int bi = blockIdx.x;
    const double *d = dst + (size_t)bi * m * 3;
    const int mpad = nn_mpad(m);
    pcm_f4 *r = rows + (size_t)bi * mpad;
    double c[3];
    centroid3<W>(d, m, red, tot, c);
    float rmax = 0.f;
    for (int j = threadIdx.x; j < mpad; j += kPrepThreads) {
        pcm_f4 t;
        if (j < m) {
            const float tx = (float)(d[3 * (size_t)j] - c[0]);
            const float ty = (float)(d[3 * (size_t)j + 1] - c[1]);
            const float tz = (float)(d[3 * (size_t)j + 2] - c[2]);
            const float w = __builtin_fmaf(tz, tz, __builtin_fmaf(ty, ty, tx * tx));
            t.x = -2.f * tx; t.y = -2.f * ty; t.z = -2.f * tz; t.w = w;
            rmax = fmaxf(rmax, sqrtf(w));
        } else {
            t.x = 0.f; t.y = 0.f; t.z = 0.f; t.w = PCM_INF;
        }
        r[j] = t;
    }
    const float R = block_max<W>(rmax, redf);
    if (threadIdx.x == 0) {
        hdr[bi].c[0] = c[0]; hdr[bi].c[1] = c[1]; hdr[bi].c[2] = c[2];
        hdr[bi].R = R;
        hdr[bi].pad = 0;
        if (arrive) arrive[(size_t)bi * 32] = 0u;  // pcm_icp's per-pair pass counter (kArriveStride)
        if (err && bi == 0) *err = 0u;
    }
}

__device__ __forceinline__ void st_sc1_d(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1_d(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- ICP kernel: K workgroups per (A, B) pair -------------------------------
//
// Workgroup (pair, k) owns the source slice [k S, min(n, (k + 1) S)) in LDS
// (float64, homogeneous).  Per pass it screens its slice, sums its 16 float64
// partials (fixed-order DPP + LDS), stores them write-through and adds to the
// pair's arrival counter; once all K partials of the pass are in (bounded
// sc1 poll), EVERY workgroup of the pair reduces them in the same fixed order
// and runs the same Kabsch on thread 0, so all K reach identical transforms
// and the same stop decision without a broadcast (MI355X_MICROARCH.md
// visibility row 1: sc1 stores, s_waitcnt vmcnt(0), agent atomic; sc1 polls
// and loads).  K = 1 skips the hand-off.  The grid (b K workgroups of at most
// 1024 threads and ~10 KB of LDS) is sized to be co-resident; a wait that
// times out sets the sticky error word and ends the loop.

struct IcpWs {
    unsigned *arrive;  // [b] arrival counter per pair (own 128-B line each), zeroed by nn_prep_kernel
    double *part;      // [2][b][K][16] partial sums, double-buffered by pass parity
    unsigned *err;     // sticky error word
};
constexpr int kArriveStride = 32;  // unsigned words per pair
constexpr unsigned kIcpMaxSpins = 1u << 22;

// partial sums of NV doubles over the workgroup (fixed order), result in out[0..NV) for every thread
// (only the first nw waves hold values: the others skip the reduction)
template <int NV>
__device__ __forceinline__ void wg_sum(double (&v)[NV], double (*red)[kIcpWaves], double *out, int nw) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave < nw) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0xb1>(v[i]);   // quad_perm [1,0,3,2]
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x4e>(v[i]);   // quad_perm [2,3,0,1]
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x114>(v[i]);  // row_shr:4
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x118>(v[i]);  // row_shr:8
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x142>(v[i]);  // row_bcast:15
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] += dpp_move<0x143>(v[i]);  // row_bcast:31
    if (lane == 63) {
#pragma unroll
        for (int i = 0; i < NV; ++i) red[i][wave] = v[i];
    }
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        double s = 0.0;
        for (int w = 0; w < nw; ++w) s += red[threadIdx.x][w];
        out[threadIdx.x] = s;
    }
    __syncthreads();
}

// the pair's totals of the NV partials: this workgroup's own when K == 1,
// else published, all K awaited and reduced in slice order.  Returns false
// on a timed-out wait.
template <int NV>
__device__ __forceinline__ bool pair_sum(double *loc, double *tot, const IcpWs &ws, int pair, int k, int K, int b,
                                         unsigned pass, int *sOk, double *stage) {
    if (K == 1) {
        if (threadIdx.x < NV) tot[threadIdx.x] = loc[threadIdx.x];
        __syncthreads();
        return true;
    }
    double *slot = ws.part + (((size_t)(pass & 1u) * b + pair) * K) * 16;
    if (threadIdx.x < NV) st_sc1_d(slot + (size_t)k * 16 + threadIdx.x, loc[threadIdx.x]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned *ctr = ws.arrive + (size_t)pair * kArriveStride;
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (pass + 1u) * (unsigned)K;
        int ok = 1;
        for (unsigned spins = 0;; ++spins) {
            if ((int)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) >= 0) break;
            if (spins >= kIcpMaxSpins) {
                ok = 0;
                __hip_atomic_store(ws.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *sOk = ok;
    }
    __syncthreads();
    // every partial by its own thread (independent loads), then fixed-order
    // sums over the K slices
    // (stage: K * 16 doubles of LDS the caller does not need here)
    if ((int)threadIdx.x < K * 16) stage[threadIdx.x] = ld_sc1_d(slot + threadIdx.x);
    __syncthreads();
    if (threadIdx.x < NV) {
        double s = 0.0;
        for (int q = 0; q < K; ++q) s += stage[q * 16 + threadIdx.x];
        tot[threadIdx.x] = s;
    }
    __syncthreads();
    return *sOk != 0;
}

#ifdef PCM_STAMPS  // profiling build: cycles per phase of workgroup 0, summed over passes (tools/tune_icp.py)
__device__ unsigned long long g_icp_stamps[8];
#define ICP_T(v) const unsigned long long v = (blockIdx.x == 0 && threadIdx.x == 0) ? __builtin_amdgcn_s_memtime() : 0
#define ICP_ACC(i, t_a, t_b) if (blockIdx.x == 0 && threadIdx.x == 0) acc[i] += (t_b) - (t_a)
#else
#define ICP_T(v)
#define ICP_ACC(i, t_a, t_b)
#endif

// Row-split screen of the workgroup's query slice: all 16 waves hold the same
// queries (QPT per lane: query r*64 + lane), wave w screens the 32-row chunks
// c = w, w + 16, ... (SGPR stream, as nn_screen), rescans its best chunk per
// query, and the waves' results meet in LDS: a 64-bit atomicMin of
// (order-preserving key of d1, row) gives the lowest-index minimum, then every
// non-winning wave offers its d1 and every wave its second best to the d2 slot.
// Per wave that is n/16 rows instead of n: the screen is a latency chain per
// row, so splitting the rows over the waves is what shortens it.
__device__ __forceinline__ unsigned f2ukey(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // order-preserving, unsigned
}
__device__ __forceinline__ float ukey2f(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <int QPT>
__device__ __forceinline__ void nn_screen_split(pcm_cf4 *rows, const pcm_f4 *__restrict__ rows_v, int mpad,
                                                const float (&qx)[QPT], const float (&qy)[QPT],
                                                const float (&qz)[QPT], unsigned long long *mk, unsigned *m2,
                                                int nq) {
    // wave index made provably uniform: the chunk index must live in an SGPR for
    // the rows to stream through s_load (a VGPR index turns every row into a
    // per-lane vector load)
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float b1[QPT], b2[QPT];
    int c1[QPT];
#pragma unroll
    for (int r = 0; r < QPT; ++r) { b1[r] = PCM_INF; b2[r] = PCM_INF; c1[r] = 0; }
    const int nch = mpad / kChunk;
    for (int c = wave; c < nch; c += kIcpWaves) {
        pcm_cf4 *tk = rows + c * kChunk;
        float mn[QPT];
#pragma unroll
        for (int r = 0; r < QPT; ++r) mn[r] = PCM_INF;
#pragma unroll
        for (int k = 0; k < kChunk; k += 2) {
            const pcm_f4 ta = tk[k], tb = tk[k + 1];
#pragma unroll
            for (int r = 0; r < QPT; ++r) {
                const float da = row_d(ta, qx[r], qy[r], qz[r]);
                const float db = row_d(tb, qx[r], qy[r], qz[r]);
                mn[r] = __builtin_fminf(__builtin_fminf(mn[r], da), db);
            }
        }
#pragma unroll
        for (int r = 0; r < QPT; ++r) {
            b2[r] = __builtin_amdgcn_fmed3f(b1[r], b2[r], mn[r]);
            const bool lt = mn[r] < b1[r];
            b1[r] = lt ? mn[r] : b1[r];
            c1[r] = lt ? c : c1[r];
        }
    }
    unsigned long long key[QPT];
#pragma unroll
    for (int r = 0; r < QPT; ++r) {
        float e1 = PCM_INF, e2 = PCM_INF;
        int j1 = 0;
        if (b1[r] < PCM_INF) {  // this wave saw a finite row for the query
            const pcm_f4 *tk = rows_v + c1[r] * kChunk;
#pragma unroll 8
            for (int k = 0; k < kChunk; ++k) {
                const float d = row_d(tk[k], qx[r], qy[r], qz[r]);
                e2 = __builtin_amdgcn_fmed3f(e1, e2, d);
                const bool lt = d < e1;
                e1 = lt ? d : e1;
                j1 = lt ? k : j1;
            }
        }
        const int i = r * 64 + lane;
        key[r] = ((unsigned long long)f2ukey(e1) << 32) | (unsigned)(c1[r] * kChunk + j1);
        if (i < nq) {
            atomicMin(mk + i, key[r]);
            atomicMin(m2 + i, f2ukey(__builtin_fminf(e2, b2[r])));
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < QPT; ++r) {  // the non-winning waves' minima are second-best candidates
        const int i = r * 64 + lane;
        if (i < nq && mk[i] != key[r]) atomicMin(m2 + i, (unsigned)(key[r] >> 32));
    }
    __syncthreads();
}

template <int QPT, bool kLdsRows>
__global__ __launch_bounds__(kIcpThreads) void icp_kernel(const double *__restrict__ A, const double *__restrict__ B,
                                                          int b, int pair0, int n, int K, int S,
                                                          const double *__restrict__ init_pose, int max_it,
                                                          double tol, const NnHdr *__restrict__ hdr,
                                                          const pcm_f4 *__restrict__ rows_all, IcpWs ws,
                                                          double *__restrict__ T_out, double *__restrict__ dist_out,
                                                          int32_t *__restrict__ iters_out) {
    extern __shared__ __align__(16) unsigned char smem[];
    pcm_f4 *sRows = reinterpret_cast<pcm_f4 *>(smem);                      // [mpad] rows, for the rescans
    unsigned long long *mk =
        reinterpret_cast<unsigned long long *>(smem + (kLdsRows ? (size_t)nn_mpad(n) * 16 : 0));  // [S]
    unsigned *m2 = reinterpret_cast<unsigned *>(mk + S);                   // [S] merged d2 key
    double *sx = reinterpret_cast<double *>(m2 + ((S + 1) & ~1));
    double *sy = sx + S, *sz = sy + S, *sw = sz + S;
    __shared__ double red[16][kIcpWaves];
    __shared__ double loc[16];
    __shared__ double tot[16];
    __shared__ double sT[12];
    __shared__ int sDone, sOk;

    // pairs [pair0, pair0 + gridDim.x / K) in this launch: K * pairs <= 256
    // workgroups, all co-resident (the pair's slices wait on each other)
    const int bl = blockIdx.x / K, k = blockIdx.x - bl * K, bi = pair0 + bl, tid = threadIdx.x, lane = tid & 63;
    const int j0 = k * S, j1 = min(n, j0 + S), ns = j1 - j0;  // this workgroup's slice
    const double *a = A + (size_t)bi * n * 3;
    const double *bb = B + (size_t)bi * n * 3;
    const double *P = init_pose ? init_pose + (size_t)bi * 16 : nullptr;
    const int mpad = nn_mpad(n);
    const pcm_f4 *rows_g = rows_all + (size_t)bi * mpad;
    pcm_cf4 *rows = (pcm_cf4 *)(uintptr_t)rows_g;  // the screen: SGPR stream (wave-uniform)
    // the rescans: per-lane chunks, from LDS (or global memory for large clouds)
    const pcm_f4 *rows_v = kLdsRows ? (const pcm_f4 *)sRows : rows_g;
    if constexpr (kLdsRows) pcm_dma_to_lds(sRows, rows_g, 16 * mpad, tid >> 6, kIcpWaves);
    const double c[3] = {hdr[bi].c[0], hdr[bi].c[1], hdr[bi].c[2]};
    const int nwq = min(kIcpWaves, (ns + 63) / 64);  // waves holding queries in the per-query loops

    // src = init_pose @ [A^T; 1] (icp.py:89-96), kept homogeneous
    for (int j = tid; j < ns; j += kIcpThreads) {
        const double *pa = a + 3 * (size_t)(j0 + j);
        const double x = pa[0], y = pa[1], z = pa[2];
        if (P) {
            sx[j] = ((P[0] * x + P[1] * y) + P[2] * z) + P[3];
            sy[j] = ((P[4] * x + P[5] * y) + P[6] * z) + P[7];
            sz[j] = ((P[8] * x + P[9] * y) + P[10] * z) + P[11];
            sw[j] = ((P[12] * x + P[13] * y) + P[14] * z) + P[15];
        } else {
            sx[j] = x; sy[j] = y; sz[j] = z; sw[j] = 1.0;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rows have landed
    __syncthreads();

    double prev = 0.0;
    int it = 0;
    unsigned pass = 0;
    bool ok = true;
    double vw[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};  // thread 0's warm start
#ifdef PCM_STAMPS
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
#endif
    for (;; ++it) {
        ICP_T(t0);
        // 1. nearest neighbours of the slice (screen split over the waves),
        //    then per query (thread tid) the exact decision and, in the same
        //    sweep, the sums for best_fit_transform (icp.py:23-29):
        //    S = sum of (a - c)(b - c)^T about B's centroid c, so that
        //    H = S - n (ca - c)(cb - c)^T is the centred cross-covariance
        //    without a second pass
        for (int i = tid; i < ns; i += kIcpThreads) {
            mk[i] = ~0ull;
            m2[i] = ~0u;
        }
        float qx[QPT], qy[QPT], qz[QPT];
#pragma unroll
        for (int r = 0; r < QPT; ++r) {
            const int q = min(r * 64 + lane, ns - 1);
            qx[r] = (float)(sx[q] - c[0]);
            qy[r] = (float)(sy[q] - c[1]);
            qz[r] = (float)(sz[q] - c[2]);
        }
        __syncthreads();
        nn_screen_split<QPT>(rows, rows_v, mpad, qx, qy, qz, mk, m2, ns);
        ICP_T(t0b);
        double s16[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) s16[i] = 0.0;
        for (int q = tid; q < ns; q += kIcpThreads) {
            const unsigned long long key = mk[q];
            const float d1 = ukey2f((unsigned)(key >> 32)), d2 = ukey2f(m2[q]);
            const int k1 = (int)(unsigned)key;
            const float fx = (float)(sx[q] - c[0]), fy = (float)(sy[q] - c[1]), fz = (float)(sz[q] - c[2]);
            double e2;
            const int kk = nn_decide(sx[q], sy[q], sz[q], fx, fy, fz, d1, d2, k1, rows, mpad, bb, e2);
            const double dist = sqrt(e2);
            dist_out[(size_t)bi * n + j0 + q] = dist;
            const double ax = sx[q], ay = sy[q], az = sz[q];
            const double bx = bb[3 * (size_t)kk], by = bb[3 * (size_t)kk + 1], bz = bb[3 * (size_t)kk + 2];
            s16[0] += ax; s16[1] += ay; s16[2] += az;
            s16[3] += bx; s16[4] += by; s16[5] += bz;
            s16[6] += dist;
            const double ux = ax - c[0], uy = ay - c[1], uz = az - c[2];
            const double vx = bx - c[0], vy = by - c[1], vz = bz - c[2];
            s16[7] += ux * vx; s16[8] += ux * vy; s16[9] += ux * vz;
            s16[10] += uy * vx; s16[11] += uy * vy; s16[12] += uy * vz;
            s16[13] += uz * vx; s16[14] += uz * vy; s16[15] += uz * vz;
        }
        ICP_T(t1);
        wg_sum<16>(s16, red, loc, nwq);
        ICP_T(t2);
        ok = pair_sum<16>(loc, tot, ws, bi, k, K, b, pass++, &sOk, &red[0][0]);
        ICP_T(t3);
        const double ca[3] = {tot[0] / n, tot[1] / n, tot[2] / n};
        const double cb[3] = {tot[3] / n, tot[4] / n, tot[5] / n};
        const double mean = tot[6] / n;
        // 3. SVD / transform / convergence (icp.py:105-114), identical in all K
        if (tid == 0) {
            const double ea[3] = {ca[0] - c[0], ca[1] - c[1], ca[2] - c[2]};
            const double eb[3] = {cb[0] - c[0], cb[1] - c[1], cb[2] - c[2]};
            double H[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) H[3 * i + j] = tot[7 + 3 * i + j] - n * (ea[i] * eb[j]);
            kabsch(H, ca, cb, sT, vw);
            sDone = (fabs(prev - mean) < tol) || (it + 1 >= max_it) || !ok;
        }
        __syncthreads();
        ICP_T(t4);
        // 4. src = T src
        for (int j = tid; j < ns; j += kIcpThreads) {
            const double x = sx[j], y = sy[j], z = sz[j], w = sw[j];
            sx[j] = ((sT[0] * x + sT[1] * y) + sT[2] * z) + sT[3] * w;
            sy[j] = ((sT[4] * x + sT[5] * y) + sT[6] * z) + sT[7] * w;
            sz[j] = ((sT[8] * x + sT[9] * y) + sT[10] * z) + sT[11] * w;
        }
        prev = mean;
        ICP_T(t5);
        ICP_ACC(0, t0, t0b);
        ICP_ACC(5, t0b, t1);
        ICP_ACC(1, t1, t2);
        ICP_ACC(2, t2, t3);
        ICP_ACC(3, t3, t4);
        ICP_ACC(4, t4, t5);
        if (sDone) break;  // uniform: written before the barrier above, rewritten only after two more
        __syncthreads();   // the update is read by the next pass's query loads
    }
#ifdef PCM_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int i = 0; i < 6; ++i) g_icp_stamps[i] = acc[i];
#endif
    __syncthreads();
    // final: best_fit_transform(A, src) (icp.py:117): centroids of A and src,
    // then H about them -- two pair-wide sums
    double s6[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) s6[i] = 0.0;
    for (int j = tid; j < ns; j += kIcpThreads) {
        const double *pa = a + 3 * (size_t)(j0 + j);
        s6[0] += pa[0]; s6[1] += pa[1]; s6[2] += pa[2];
        s6[3] += sx[j]; s6[4] += sy[j]; s6[5] += sz[j];
    }
    wg_sum<16>(s6, red, loc, nwq);
    ok = pair_sum<6>(loc, tot, ws, bi, k, K, b, pass++, &sOk, &red[0][0]) && ok;
    const double ca[3] = {tot[0] / n, tot[1] / n, tot[2] / n};
    const double cs[3] = {tot[3] / n, tot[4] / n, tot[5] / n};
    double h[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) h[i] = 0.0;
    for (int j = tid; j < ns; j += kIcpThreads) {
        const double *pa = a + 3 * (size_t)(j0 + j);
        const double ax = pa[0] - ca[0], ay = pa[1] - ca[1], az = pa[2] - ca[2];
        const double bx = sx[j] - cs[0], by = sy[j] - cs[1], bz = sz[j] - cs[2];
        h[0] += ax * bx; h[1] += ax * by; h[2] += ax * bz;
        h[3] += ay * bx; h[4] += ay * by; h[5] += ay * bz;
        h[6] += az * bx; h[7] += az * by; h[8] += az * bz;
    }
    wg_sum<16>(h, red, loc, nwq);
    ok = pair_sum<9>(loc, tot, ws, bi, k, K, b, pass++, &sOk, &red[0][0]) && ok;
    if (k == 0 && tid == 0) {
        double T[12];
        kabsch(tot, ca, cs, T);
        double *o = T_out + (size_t)bi * 16;
        for (int i = 0; i < 12; ++i) o[i] = ok ? T[i] : __builtin_nan("");
        o[12] = 0.0; o[13] = 0.0; o[14] = 0.0; o[15] = 1.0;
        iters_out[bi] = it;
    }
}

// ---- standalone nearest neighbour and best fit -----------------------------

__global__ __launch_bounds__(kNnThreads) void nn_kernel(const double *__restrict__ src, const double *__restrict__ dst,
                                                        int n, int m, const NnHdr *__restrict__ hdr,
                                                        const pcm_f4 *__restrict__ rows_all,
                                                        double *__restrict__ dist, int32_t *__restrict__ idx) {
    const int bi = blockIdx.y;
    const int q0 = blockIdx.x * kNnThreads + threadIdx.x;
    const int q = min(q0, n - 1);
    const double *s = src + (size_t)bi * n * 3;
    const double *d = dst + (size_t)bi * m * 3;
    const int mpad = nn_mpad(m);
    const pcm_f4 *rows_v = rows_all + (size_t)bi * mpad;
    pcm_cf4 *rows = (pcm_cf4 *)(uintptr_t)rows_v;
    const double c0 = hdr[bi].c[0], c1 = hdr[bi].c[1], c2 = hdr[bi].c[2];
    const double sx = s[3 * (size_t)q], sy = s[3 * (size_t)q + 1], sz = s[3 * (size_t)q + 2];
    const float qx = (float)(sx - c0), qy = (float)(sy - c1), qz = (float)(sz - c2);
    float d1, d2;
    int k1;
    nn_screen(rows, rows_v, mpad, qx, qy, qz, d1, d2, k1);
    if (q0 < n) {
        double e2;
        const int k = nn_decide(sx, sy, sz, qx, qy, qz, d1, d2, k1, rows, mpad, d, e2);
        dist[(size_t)bi * n + q0] = sqrt(e2);
        idx[(size_t)bi * n + q0] = k;
    }
}

__global__ __launch_bounds__(kPrepThreads) void best_fit_kernel(const double *__restrict__ A,
                                                                const double *__restrict__ B, int n,
                                                                double *__restrict__ T_out) {
    constexpr int W = kPrepThreads / 64;
    __shared__ double red[9][W];
    __shared__ double tot[9];
    const int bi = blockIdx.x;
    const double *a = A + (size_t)bi * n * 3;
    const double *b = B + (size_t)bi * n * 3;
    double ca[3], cb[3];
    centroid3<W>(a, n, red, tot, ca);
    centroid3<W>(b, n, red, tot, cb);
    double h[9] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int j = threadIdx.x; j < n; j += kPrepThreads) {
        const double ax = a[3 * (size_t)j] - ca[0], ay = a[3 * (size_t)j + 1] - ca[1], az = a[3 * (size_t)j + 2] - ca[2];
        const double bx = b[3 * (size_t)j] - cb[0], by = b[3 * (size_t)j + 1] - cb[1], bz = b[3 * (size_t)j + 2] - cb[2];
        h[0] += ax * bx; h[1] += ax * by; h[2] += ax * bz;
        h[3] += ay * bx; h[4] += ay * by; h[5] += ay * bz;
        h[6] += az * bx; h[7] += az * by; h[8] += az * bz;
    }
    block_sum<9, W>(h, red, tot);
    if (threadIdx.x == 0) {
        double T[12];
        kabsch(tot, ca, cb, T);
        double *o = T_out + (size_t)bi * 16;
        for (int i = 0; i < 12; ++i) o[i] = T[i];
        o[12] = 0.0; o[13] = 0.0; o[14] = 0.0; o[15] = 1.0;
    }
}

size_t nn_ws_bytes(int b, int m) {
    return (size_t)b * sizeof(NnHdr) + (size_t)b * nn_mpad(m) * sizeof(pcm_f4);
}

// pcm_icp: the rows, then the pass counters, the error word and the partials
constexpr int kIcpMaxSlices = 16;
size_t icp_ws_bytes(int b, int m) {
    const size_t base = (nn_ws_bytes(b, m) + 127) / 128 * 128;
    return base + (size_t)b * kArriveStride * 4 + 128 + (size_t)2 * b * kIcpMaxSlices * 16 * 8;
}
IcpWs icp_ws(void *workspace, int b, int m) {
    char *p = (char *)workspace + (nn_ws_bytes(b, m) + 127) / 128 * 128;
    IcpWs w;
    w.arrive = (unsigned *)p;
    w.err = (unsigned *)(p + (size_t)b * kArriveStride * 4);
    w.part = (double *)(p + (size_t)b * kArriveStride * 4 + 128);
    return w;
}

int launch_prep(const double *dst, int b, int m, void *workspace, hipStream_t s, const NnHdr **hdr,
                const pcm_f4 **rows, unsigned *arrive = nullptr, unsigned *err = nullptr) {
    NnHdr *h = reinterpret_cast<NnHdr *>(workspace);
    pcm_f4 *r = reinterpret_cast<pcm_f4 *>(h + b);
    hipLaunchKernelGGL(nn_prep_kernel, dim3(b), dim3(kPrepThreads), 0, s, dst, m, h, r, arrive, err);
    *hdr = h;
    *rows = r;
    return pcm_launch_status();
}

// slices per pair: fill the chip (K b <= 256 one-per-CU workgroups), at least
// 64 points each, at most 1024 (16 per lane)
int icp_slices(int b, int n) {
    int K = pcm_device_cus() / b;  // one workgroup per CU across the batch
    K = K < 1 ? 1 : (K > kIcpMaxSlices ? kIcpMaxSlices : K);
    const int most = (n + 63) / 64, least = (n + 1023) / 1024;
    K = K < most ? K : most;
    return K > least ? K : least;
}

}  // namespace

extern "C" size_t pcm_icp_workspace_bytes(int b, int m) {
    if (b <= 0 || m <= 0) return 0;
    return icp_ws_bytes(b, m);
}

extern "C" int pcm_icp(const double *A, const double *B, int b, int n, const double *init_pose, int max_iterations,
                       double tolerance, double *T_out, double *distances, int32_t *iterations, void *workspace,
                       size_t workspace_bytes, void *stream) {
    if (b < 0 || n < 0 || max_iterations < 1) return PCM_ERR_INVALID_ARG;
    if (b == 0) return PCM_OK;
    if (n == 0 || !A || !B || !T_out || !distances || !iterations) return PCM_ERR_INVALID_ARG;
    if (n > kIcpMaxN || b > 65535) return PCM_ERR_UNSUPPORTED;
    if (!workspace || workspace_bytes < icp_ws_bytes(b, n)) return PCM_ERR_WORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    const NnHdr *hdr;
    const pcm_f4 *rows;
    const IcpWs ws = icp_ws(workspace, b, n);
    if (launch_prep(B, b, n, workspace, s, &hdr, &rows, ws.arrive, ws.err) != PCM_OK) return PCM_ERR_LAUNCH;
    const int K = icp_slices(b, n);
    const int S = (n + K - 1) / K;  // points per slice (<= 1024)
    const int qpt = S <= 64 ? 1 : S <= 128 ? 2 : S <= 256 ? 4 : S <= 512 ? 8 : 16;
    const bool lds_rows = (size_t)nn_mpad(n) * 16 <= (size_t)kIcpRowsLdsMax;
    const size_t lds = (lds_rows ? (size_t)nn_mpad(n) * 16 : 0) + (size_t)S * (8 + 4 + 32) + 8;
    // pairs per launch: every slice of a pair must be resident while the
    // others wait on it, so a launch holds at most one workgroup per CU of
    // this device (256 on a whole MI355X)
    const int cus = pcm_device_cus();
    const int per_launch = K <= cus ? cus / K : 1;
    auto launch = [&](auto kfn) -> int {
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return PCM_ERR_LAUNCH;
        for (int p0 = 0; p0 < b; p0 += per_launch) {
            const int np = b - p0 < per_launch ? b - p0 : per_launch;
            hipLaunchKernelGGL(kfn, dim3((unsigned)(np * K)), dim3(kIcpThreads), lds, s, A, B, b, p0, n, K, S,
                               init_pose, max_iterations, tolerance, hdr, rows, ws, T_out, distances, iterations);
        }
        return PCM_OK;
    };
    int rc;
    if (lds_rows) {
        switch (qpt) {
            case 1: rc = launch(icp_kernel<1, true>); break;
            case 2: rc = launch(icp_kernel<2, true>); break;
            case 4: rc = launch(icp_kernel<4, true>); break;
            case 8: rc = launch(icp_kernel<8, true>); break;
            default: rc = launch(icp_kernel<16, true>); break;
        }
    } else {  // above 96 KB of rows: N > 6144, so S >= 384 (QPT 8 or 16)
        rc = qpt <= 8 ? launch(icp_kernel<8, false>) : launch(icp_kernel<16, false>);
    }
    if (rc != PCM_OK) return rc;
    return pcm_launch_status();
}

#ifdef PCM_STAMPS
extern "C" int pcm_tune_read_icp_stamps(unsigned long long *host, int n) {
    if (n > 8) n = 8;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_icp_stamps), n * sizeof(unsigned long long)) == hipSuccess
               ? PCM_OK : PCM_ERR_LAUNCH;
}
#endif

// sticky device-side error of the last pcm_icp on `workspace` (a timed-out
// wait between the workgroups of a pair): PCM_OK or PCM_ERR_LAUNCH; synchronises.
extern "C" int pcm_icp_workspace_status(const void *workspace, size_t workspace_bytes, int b, int n, void *stream) {
    if (b <= 0 || n <= 0) return PCM_OK;
    if (!workspace || workspace_bytes < icp_ws_bytes(b, n)) return PCM_ERR_WORKSPACE;
    unsigned err = 0;
    const IcpWs ws = icp_ws(const_cast<void *>(workspace), b, n);
    if (hipMemcpyAsync(&err, ws.err, 4, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return PCM_ERR_LAUNCH;
    return err ? PCM_ERR_LAUNCH : PCM_OK;
}

extern "C" int pcm_nearest_neighbor(const double *src, const double *dst, int b, int n, int m, double *distances,
                                    int32_t *indices, void *workspace, size_t workspace_bytes, void *stream) {
    if (b < 0 || n < 0 || m < 0) return PCM_ERR_INVALID_ARG;
    if (b == 0 || n == 0) return PCM_OK;
    if (m == 0 || !src || !dst || !distances || !indices) return PCM_ERR_INVALID_ARG;
    if (b > 65535) return PCM_ERR_UNSUPPORTED;
    if (!workspace || workspace_bytes < nn_ws_bytes(b, m)) return PCM_ERR_WORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    const NnHdr *hdr;
    const pcm_f4 *rows;
    if (launch_prep(dst, b, m, workspace, s, &hdr, &rows) != PCM_OK) return PCM_ERR_LAUNCH;
    const unsigned gx = (unsigned)((n + kNnThreads - 1) / kNnThreads);
    hipLaunchKernelGGL(nn_kernel, dim3(gx, b), dim3(kNnThreads), 0, s, src, dst, n, m, hdr, rows, distances,
                       indices);
    return pcm_launch_status();
}


extern "C" int pcm_best_fit_transform(const double *A, const double *B, int b, int n, double *T_out, void *stream) {
    if (b < 0 || n < 0) return PCM_ERR_INVALID_ARG;
    if (b == 0) return PCM_OK;
    if (n == 0 || !A || !B || !T_out) return PCM_ERR_INVALID_ARG;
    if (b > 65535) return PCM_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(best_fit_kernel, dim3(b), dim3(kPrepThreads), 0, (hipStream_t)stream, A, B, n, T_out);
    return pcm_launch_status();
}
