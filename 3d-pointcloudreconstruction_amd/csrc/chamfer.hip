// chamfer.hip -- Chamfer3D forward/backward for MI355X (gfx950, CDNA4).
//
// Replaces the reference's NmDistanceKernel / NmDistanceGradKernel
// (metric/chamfer3D/chamfer3D.cu:12-195).  DESIGN.md section 3 has the full
// rationale and the roofline; in short:
//
// Forward: ONE launch computes both directions.  A workgroup owns 64*QPT query
// points of one (direction, batch) and W waves; the opposing cloud is staged
// through LDS in SoA tiles (X[], Y[], Z[]: one ds_read_b128 broadcast yields
// four candidates' x), and each wave scans an interleaved 1/W share of the
// tile's chunks of C candidates.  Distances are evaluated two candidates at a
// time in packed fp32 (v_pk_add/mul/fma_f32 -- measured 2x the scalar rate on
// MI355X) in the pinned order fma(dz,dz,fma(dy,dy,dx*dx)); a chunk's minimum
// is folded with v_min3_f32 and only the chunk id of the running minimum is
// tracked (strict '<': the lowest chunk wins).  After the waves' (min, chunk)
// pairs are merged lexicographically, the single winning chunk is re-scanned
// (from LDS, all threads, branch-free) for the lowest index attaining the
// minimum -- bit-identical to the reference's lowest-index first-min scan at
// ~1/C of its compare/select cost.  Non-finite coordinates (where the
// reference's 512-point tile boundaries decide NaN outcomes) divert the
// workgroup to a reference-exact scan.  Optionally (kLoss) the epilogue also
// produces mean(dist1), mean(dist2) (loss/loss.py:36) deterministically:
// per-workgroup partial sums + an arrival ticket, the last workgroup sums the
// partials in a fixed order.
//
// Backward: deterministic.  A workgroup owns kBwdT points of one cloud; it
// gathers the direct term and sums the reverse-direction scatter terms in
// ascending source index (LDS counting sort of the other direction's argmins,
// no float atomics), in the reference's kernel order (chamfer3D.cu:184-185).
#include "pcm_common.h"
#include "pcm_internal.h"
#include "chamfer_loss.h"

using namespace pcm_loss;

namespace {

constexpr int kTile = 2048;  // candidates per LDS tile (3 x 8 KiB SoA)
constexpr int kChunk = 32;   // candidates per chunk (rescan granularity)

template <typename TIn, int W, int QPT, int C, int TILE, bool kLoss>
__global__ __launch_bounds__(64 * W) void chamfer_fwd_kernel(
    const TIn *__restrict__ xyz1, const TIn *__restrict__ xyz2, int b, int n, int m,
    float *__restrict__ dist1, float *__restrict__ dist2, int32_t *__restrict__ idx1,
    int32_t *__restrict__ idx2, int nblk1, int nblk2, float *__restrict__ partials,
    unsigned *__restrict__ ticket, float *__restrict__ mean_out) {
    static_assert(TILE % C == 0 && C % 4 == 0, "tile must hold whole chunks");
    constexpr int QW = 64 * QPT;
    constexpr int NT = 64 * W;
    constexpr int PARTS = (NT / QW) > 0 ? (NT / QW) : 1;  // rescan splits per query
    constexpr int CP = C / PARTS;
    static_assert(C % PARTS == 0, "chunk must split evenly");
    __shared__ __attribute__((aligned(16))) float sXYZ[3][TILE];
    __shared__ float sBest[W][QW];
    __shared__ int sChunk[W][QW];
    __shared__ int sHit[PARTS][QW];
    __shared__ float sRed[2][W];
    __shared__ int sLast;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    // ---- which (direction, batch, query block) this workgroup owns (uniform)
    int bid = pcm_xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int slot = bid;  // logical block id (partials are stored in this order)
    const TIn *Q, *T;
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
            x = pcm_ld(Q + 3 * (size_t)qi + 0);
            y = pcm_ld(Q + 3 * (size_t)qi + 1);
            z = pcm_ld(Q + 3 * (size_t)qi + 2);
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
        if (t0 > 0) __syncthreads();  // previous tile fully consumed
        // coalesced flat read of the AoS tile, scattered to SoA; pad = +inf.
        // All of a thread's loads are issued before any LDS write, so the
        // tile costs one memory latency, not one per element.
        const TIn *src = T + 3 * (size_t)t0;
        constexpr int kFill = (3 * TILE + NT - 1) / NT;
        float v[kFill];
#pragma unroll
        for (int r = 0; r < kFill; ++r) {
            const int f = tid + r * NT;
            v[r] = (f < 3 * cnt) ? pcm_ld(src + f) : PCM_INF;
        }
#pragma unroll
        for (int r = 0; r < kFill; ++r) {
            const int f = tid + r * NT;
            if (f < 3 * padded) {
                const int p = f / 3;
                nonfinite |= (f < 3 * cnt) && !pcm_finite(v[r]);
                sXYZ[f - 3 * p][p] = v[r];
            }
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
                    // written so that hipcc forms two v_min3_f32 per 4 candidates
                    mn[qq] = __builtin_fminf(__builtin_fminf(mn[qq], da.x), da.y);
                    mn[qq] = __builtin_fminf(__builtin_fminf(mn[qq], db.x), db.y);
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

    // ---- merge the W waves' (min, chunk) per query
#pragma unroll
    for (int qq = 0; qq < QPT; ++qq) {
        sBest[wave][qq * 64 + lane] = best[qq];
        sChunk[wave][qq * 64 + lane] = bchunk[qq];
    }
    __shared__ int sNF[W];
    const int any_nonfinite = pcm_wg_or(nonfinite, sNF, W);

    float my_d = 0.f;  // dist of the query this thread finalises (kLoss sum)
    if (!any_nonfinite) {
        // ---- rescan the winning chunk for the lowest index attaining the min.
        // Every thread takes one (query, part) pair; candidates come from the
        // LDS tile when the whole target cloud was one tile, else from global.
        const bool resident = nt <= TILE;
        for (int item = tid; item < QW * PARTS; item += NT) {
            const int s = item % QW;
            const int part = item / QW;
            const int qi = qbase + s;
            int hit = 0x7fffffff;
            if (qi < nq) {
                float fb = sBest[0][s];
                int fc = sChunk[0][s];
#pragma unroll
                for (int w = 1; w < W; ++w) {
                    const float v = sBest[w][s];
                    const int c = sChunk[w][s];
                    pcm_lexmin(fb, fc, v, c);
                }
                // item % 64 == lane, so query s is this lane's register copy
                // number (item / 64) % QPT -- wave-uniform, no reload
                const int qsel = (item >> 6) % QPT;
                float x = px[0].x, y = py[0].x, z = pz[0].x;
#pragma unroll
                for (int qq = 1; qq < QPT; ++qq)
                    if (qsel == qq) { x = px[qq].x; y = py[qq].x; z = pz[qq].x; }
                const int k0 = fc * C + part * CP;
                if (resident) {
#pragma unroll
                    for (int k = 0; k < CP; ++k) {
                        const int kk = k0 + k;
                        const float d = pcm_sqd(sXYZ[0][kk] - x, sXYZ[1][kk] - y, sXYZ[2][kk] - z);
                        hit = (d == fb && hit == 0x7fffffff && kk < nt) ? kk : hit;
                    }
                } else {
                    for (int k = 0; k < CP; ++k) {
                        const int kk = k0 + k;
                        if (kk >= nt) break;
                        const TIn *q = T + 3 * (size_t)kk;
                        const float d = pcm_sqd(pcm_ld(q) - x, pcm_ld(q + 1) - y, pcm_ld(q + 2) - z);
                        if (d == fb) { hit = kk; break; }
                    }
                }
            }
            sHit[part][s] = hit;
        }
        __syncthreads();
        for (int s = tid; s < QW; s += NT) {
            const int qi = qbase + s;
            if (qi >= nq) continue;
            float fb = sBest[0][s];
#pragma unroll
            for (int w = 1; w < W; ++w) fb = __builtin_fminf(fb, sBest[w][s]);
            int idx = sHit[0][s];
#pragma unroll
            for (int p = 1; p < PARTS; ++p) idx = min(idx, sHit[p][s]);
            my_d = fb;
            D[qi] = my_d;
            I[qi] = idx;
        }
    } else {
        for (int s = tid; s < QW; s += NT) {
            const int qi = qbase + s;
            if (qi >= nq) continue;
            float d;
            int idx;
            pcm_ref_nn_scan(pcm_ld(Q + 3 * (size_t)qi + 0), pcm_ld(Q + 3 * (size_t)qi + 1),
                            pcm_ld(Q + 3 * (size_t)qi + 2), T, nt,
                            d, idx);
            my_d = d;
            D[qi] = d;
            I[qi] = idx;
        }
    }

    if constexpr (kLoss) {
        // deterministic workgroup sum -> partials[block]; last block reduces
        const float ws = wave_sum(my_d);
        if (lane == 0) sRed[0][wave] = ws;
        __syncthreads();
        if (tid == 0) {
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < W; ++w) s += sRed[0][w];
            // hand-off without fences (MI355X_MICROARCH.md, visibility table
            // row 1): write-through (sc1) partial, drain, agent atomic ticket;
            // the last arriver reads every partial with sc1 loads.
            __hip_atomic_store(&partials[slot], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sLast = (t == gridDim.x - 1);
        }
        __syncthreads();
        if (sLast) {
            const int nb1 = b * nblk1;
            const int nbt = (int)gridDim.x;
            float s1 = 0.f, s2 = 0.f;
            for (int i = tid; i < nbt; i += NT) {
                const float v = __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (i < nb1) s1 += v; else s2 += v;
            }
            s1 = wave_sum(s1);
            s2 = wave_sum(s2);
            if (lane == 0) { sRed[0][wave] = s1; sRed[1][wave] = s2; }
            __syncthreads();
            if (tid == 0) {
                float a1 = 0.f, a2 = 0.f;
#pragma unroll
                for (int w = 0; w < W; ++w) { a1 += sRed[0][w]; a2 += sRed[1][w]; }
                mean_out[0] = a1 / ((float)b * (float)n);
                mean_out[1] = a2 / ((float)b * (float)m);
                __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Forward, SGPR-stream form.  Same algorithm and results as above, but the
// candidates are not staged through LDS for the scan: a wave's chunk index is
// wave-uniform, so hipcc reads the AoS candidates with s_load (scalar cache)
// and feeds them to v_pk_add_f32 as an SGPR operand broadcast with op_sel --
// packing runs over two QUERIES per lane instead of two candidates.  No LDS
// reads or barriers in the main loop.  (Any memory-writing intrinsic or
// volatile asm placed before the scan -- e.g. an LDS-DMA prefetch -- makes
// hipcc fall back to per-lane vector loads of the candidates: measured 35%
// slower, so the epilogue reads global memory instead.)  With kLoss the
// workgroup's partial sum is published right after the merge and the arrival
// ticket's round trip overlaps the rescan.
// ---------------------------------------------------------------------------

constexpr int kFwdChk = 8;  // target floats per thread loaded up front (finiteness check + rescan copy)

template <int W, int QPT, int C, int kLoss>
__global__ __launch_bounds__(64 * W) void chamfer_fwd_sgpr_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int b, int n, int m,
    float *__restrict__ dist1, float *__restrict__ dist2, int32_t *__restrict__ idx1,
    int32_t *__restrict__ idx2, int nblk1, int nblk2, float *__restrict__ partials,
    unsigned *__restrict__ ticket, float *__restrict__ mean_out) {
    static_assert(QPT % 2 == 0, "queries are packed in pairs");
    static_assert(C % 2 == 0, "candidates are consumed in pairs");
    static_assert(W <= 16, "sRed holds 16 waves");
    constexpr int QW = 64 * QPT;
    constexpr int NT = 64 * W;
    static_assert(NT >= QW, "one thread per query slot in the merge");
    constexpr int QP = QPT / 2;        // packed query pairs per lane
    constexpr int PARTS = NT / QW;     // rescan splits per query
    constexpr int CP = C / PARTS;
    static_assert(C % PARTS == 0, "chunk must split evenly");
    __shared__ float sBest[W][QW];
    __shared__ int sChunk[W][QW];
    __shared__ float sFb[QW];
    __shared__ int sFc[QW];
    __shared__ int sHit[PARTS][QW];
    __shared__ float sRed[2][16];
    __shared__ int sLast[4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    int nprod = (int)gridDim.x;  // producer workgroups
    unsigned epoch = 0;
    if constexpr (kLoss == 3) {
        nprod -= 1;
        if ((int)blockIdx.x == nprod) {  // the grid's last workgroup polls
            poll_loss(b * nblk1, nprod, b, n, m, reinterpret_cast<const unsigned long long *>(partials), ticket,
                      mean_out);
            return;
        }
        epoch = ticket[kEpochWord] + 1u;  // plain load: written by an earlier launch
    }
    int bid = pcm_xcd_remap((int)blockIdx.x, nprod);
    const int slot = bid;  // logical block id (partials are stored in this order)
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

    // ---- queries: pair pp holds the lane's queries (2pp)*64+lane, (2pp+1)*64+lane
    pcm_f2 px[QP], py[QP], pz[QP];
    bool nonfinite = false;
#pragma unroll
    for (int pp = 0; pp < QP; ++pp) {
        float c3[2][3];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int qi = qbase + (2 * pp + h) * 64 + lane;
#pragma unroll
            for (int d = 0; d < 3; ++d) c3[h][d] = 0.f;
            if (qi < nq) {
#pragma unroll
                for (int d = 0; d < 3; ++d) c3[h][d] = Q[3 * (size_t)qi + d];
                nonfinite |= !(pcm_finite(c3[h][0]) && pcm_finite(c3[h][1]) && pcm_finite(c3[h][2]));
            }
        }
        px[pp] = pcm_f2{c3[0][0], c3[1][0]};
        py[pp] = pcm_f2{c3[0][1], c3[1][1]};
        pz[pp] = pcm_f2{c3[0][2], c3[1][2]};
    }
    // finiteness of the target cloud: issue the loads now, test after the scan
    // (kChk per thread covers 3*nt <= kChk*NT; larger clouds loop at the end)
    constexpr int kChk = kFwdChk;
    float chk[kChk];
    const bool chk_all = 3 * nt <= kChk * NT;
#pragma unroll
    for (int r = 0; r < kChk; ++r) {
        const int f = tid + r * NT;
        chk[r] = (chk_all && f < 3 * nt) ? T[f] : 0.f;
    }

    float best[QPT];
    int bchunk[QPT];
#pragma unroll
    for (int q = 0; q < QPT; ++q) { best[q] = PCM_INF; bchunk[q] = 0; }

    // ---- main scan: chunks c = wave, wave+W, ... ; candidates via SGPRs
    const int nfull = nt / C;
    for (int c = wave; c < nfull; c += W) {
        float mn[QPT];
#pragma unroll
        for (int q = 0; q < QPT; ++q) mn[q] = PCM_INF;
        const float *tk = T + 3 * (size_t)c * C;
#pragma unroll
        for (int k = 0; k < C; k += 2) {
            const float ax = tk[3 * k + 0], ay = tk[3 * k + 1], az = tk[3 * k + 2];
            const float bx = tk[3 * k + 3], by = tk[3 * k + 4], bz = tk[3 * k + 5];
#pragma unroll
            for (int pp = 0; pp < QP; ++pp) {
                const pcm_f2 da = pcm_sqd2(pcm_f2{ax, ax} - px[pp], pcm_f2{ay, ay} - py[pp],
                                           pcm_f2{az, az} - pz[pp]);
                const pcm_f2 db = pcm_sqd2(pcm_f2{bx, bx} - px[pp], pcm_f2{by, by} - py[pp],
                                           pcm_f2{bz, bz} - pz[pp]);
                mn[2 * pp] = __builtin_fminf(__builtin_fminf(mn[2 * pp], da.x), db.x);
                mn[2 * pp + 1] = __builtin_fminf(__builtin_fminf(mn[2 * pp + 1], da.y), db.y);
            }
        }
#pragma unroll
        for (int q = 0; q < QPT; ++q) {
            if (mn[q] < best[q]) { best[q] = mn[q]; bchunk[q] = c; }
        }
    }
    // tail chunk (nt % C candidates), owned by the wave that owns chunk nfull
    if (nfull * C < nt && (nfull % W) == wave) {
        float mn[QPT];
#pragma unroll
        for (int q = 0; q < QPT; ++q) mn[q] = PCM_INF;
        for (int k = nfull * C; k < nt; ++k) {
            const float ax = T[3 * (size_t)k], ay = T[3 * (size_t)k + 1], az = T[3 * (size_t)k + 2];
#pragma unroll
            for (int pp = 0; pp < QP; ++pp) {
                const pcm_f2 da = pcm_sqd2(pcm_f2{ax, ax} - px[pp], pcm_f2{ay, ay} - py[pp],
                                           pcm_f2{az, az} - pz[pp]);
                mn[2 * pp] = __builtin_fminf(mn[2 * pp], da.x);
                mn[2 * pp + 1] = __builtin_fminf(mn[2 * pp + 1], da.y);
            }
        }
#pragma unroll
        for (int q = 0; q < QPT; ++q) {
            if (mn[q] < best[q]) { best[q] = mn[q]; bchunk[q] = nfull; }
        }
    }

    // ---- per-wave results to LDS; finish the finiteness check
#pragma unroll
    for (int q = 0; q < QPT; ++q) {
        sBest[wave][q * 64 + lane] = best[q];
        sChunk[wave][q * 64 + lane] = bchunk[q];
    }
    if (chk_all) {
#pragma unroll
        for (int r = 0; r < kChk; ++r) nonfinite |= !pcm_finite(chk[r]);
    } else {
        // large clouds: 8 independent loads in flight per step
        for (int f0 = tid; f0 < 3 * nt; f0 += kChk * NT) {
            float v[kChk];
#pragma unroll
            for (int r = 0; r < kChk; ++r) {
                const int f = f0 + r * NT;
                v[r] = f < 3 * nt ? T[f] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < kChk; ++r) nonfinite |= !pcm_finite(v[r]);
        }
    }
    __shared__ int sNF[W];
    const int any_nonfinite = pcm_wg_or(nonfinite, sNF, W);
    unsigned tk = 0;  // arrival ticket (thread 0, kLoss)

    if (!any_nonfinite) {
        // ---- merge: thread s < QW owns query slot s
        float fbv = 0.f;
        if (tid < QW) {
            float vb[W];
            int vc[W];
#pragma unroll
            for (int w = 0; w < W; ++w) {  // every load first, then branch-free selects
                vb[w] = sBest[w][tid];
                vc[w] = sChunk[w][tid];
            }
            float fb = vb[0];
            int fc = vc[0];
#pragma unroll
            for (int w = 1; w < W; ++w) pcm_lexmin(fb, fc, vb[w], vc[w]);
            sFb[tid] = fb;
            sFc[tid] = fc;
            if (qbase + tid < nq) fbv = fb;
        }
        if constexpr (kLoss != 0) tk = publish_partial<kLoss>(fbv, slot, partials, ticket, sRed, epoch);  // has a barrier
        else __syncthreads();
        // ---- rescan the winning chunk: item -> (query s, part)
#pragma unroll
        for (int r = 0; r < (QW * PARTS + NT - 1) / NT; ++r) {
            const int item = tid + r * NT;
            if (item >= QW * PARTS) break;
            const int s = item % QW;
            const int part = item / QW;
            int hit = 0x7fffffff;
            if (qbase + s < nq) {
                const float fb = sFb[s];
                const int fc = sFc[s];
                // query s is this lane's register copy q = (item/64) % QPT
                const int qsel = (item >> 6) % QPT;
                float x = px[0].x, y = py[0].x, z = pz[0].x;
#pragma unroll
                for (int q = 1; q < QPT; ++q) {
                    if (qsel == q) {
                        x = (q & 1) ? px[q / 2].y : px[q / 2].x;
                        y = (q & 1) ? py[q / 2].y : py[q / 2].x;
                        z = (q & 1) ? pz[q / 2].y : pz[q / 2].x;
                    }
                }
                const int k0 = fc * C + part * CP;
                // (measured and rejected: the up-front finiteness loads parked in
                // LDS and rescanned from there -- every SGPR variant 0.6-1.5 us
                // slower at B=32, N=M=1024)
#pragma unroll
                for (int k = 0; k < CP; ++k) {
                    const int kk = k0 + k;
                    if (kk < nt) {
                        const float *t = T + 3 * (size_t)kk;
                        const float d = pcm_sqd(t[0] - x, t[1] - y, t[2] - z);
                        hit = (d == fb && hit == 0x7fffffff) ? kk : hit;
                    }
                }
            }
            sHit[part][s] = hit;
        }
        __syncthreads();
        if (tid < QW && qbase + tid < nq) {
            int idx = sHit[0][tid];
#pragma unroll
            for (int p = 1; p < PARTS; ++p) idx = min(idx, sHit[p][tid]);
            D[qbase + tid] = sFb[tid];
            I[qbase + tid] = idx;
        }
    } else {
        float myd = 0.f;
        for (int s = tid; s < QW; s += NT) {
            const int qi = qbase + s;
            if (qi >= nq) continue;
            float d;
            int idx;
            pcm_ref_nn_scan(Q[3 * (size_t)qi + 0], Q[3 * (size_t)qi + 1], Q[3 * (size_t)qi + 2], T, nt,
                            d, idx);
            myd = d;
            D[qi] = d;
            I[qi] = idx;
        }
        if constexpr (kLoss != 0) tk = publish_partial<kLoss>(myd, slot, partials, ticket, sRed, epoch);
    }
    if constexpr (kLoss == 1) {
        if (tid == 0) sLast[0] = tk;
        __syncthreads();
        if (sLast[0]) finish_loss(b * nblk1, b, n, m, partials, ticket, mean_out, sRed);
    }
}

// Loss mode 2: the forward kernel only stores its workgroup partials; this
// one-workgroup kernel, next on the stream, sums them in the same fixed order
// as finish_loss (no atomics, no write-through: the kernel boundary is the
// hand-off).
__global__ __launch_bounds__(512) void chamfer_loss_finalize_kernel(const float *__restrict__ partials,
                                                                    int nb1, int nbt, int b, int n, int m,
                                                                    float *__restrict__ mean_out) {
    __shared__ float sRed[2][16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float s1 = 0.f, s2 = 0.f;
    for (int i = threadIdx.x; i < nbt; i += blockDim.x) {
        const float v = partials[i];
        if (i < nb1) s1 += v; else s2 += v;
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) { sRed[0][wave] = s1; sRed[1][wave] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a1 = 0.f, a2 = 0.f;
        const int nw = blockDim.x >> 6;
        for (int w = 0; w < nw; ++w) { a1 += sRed[0][w]; a2 += sRed[1][w]; }
        mean_out[0] = a1 / ((float)b * (float)n);
        mean_out[1] = a2 / ((float)b * (float)m);
    }
}

// ---------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------
constexpr int kBwdT = 256;     // targets per workgroup = threads
constexpr int kBwdCap = 4096;  // scatter entries sortable in LDS per workgroup

template <int NT>
__device__ inline int block_exclusive_scan(int v, int *wave_tot) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = pcm_wave_incl_scan(v);  // DPP steps, no LDS round trips
    if (lane == 63) wave_tot[wave] = x;
    __syncthreads();
    int before = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) before += (w < wave) ? wave_tot[w] : 0;
    return before + x - v;
}

// NT targets per workgroup (= threads): every workgroup reads the whole
// other direction's argmins, so large clouds take NT = 1024 (4x less of that)
template <typename TIn, int NT = kBwdT, int CAP = kBwdCap>
__global__ __launch_bounds__(NT) void chamfer_bwd_kernel(
    const TIn *__restrict__ xyz1, const TIn *__restrict__ xyz2, int b, int n, int m,
    const float *__restrict__ gd1, const float *__restrict__ gd2, const int32_t *__restrict__ idx1,
    const int32_t *__restrict__ idx2, TIn *__restrict__ grad1, TIn *__restrict__ grad2,
    int nblk1, int nblk2, int lay1 = 0, int lay2 = 0, PcmGdStr GS = PcmGdStr()) {
    __shared__ int sCnt[NT];
    __shared__ int sOff[NT + 1];
    __shared__ int sTmp[CAP];
    __shared__ int sSrt[CAP];
    __shared__ int sWave[NT / 64];

    const int tid = threadIdx.x;
    int bid = pcm_xcd_remap((int)blockIdx.x, (int)gridDim.x);
    // cloud 1 (direct term first) or cloud 2 (direct term last): reference
    // kernel order chamfer3D.cu:184-185.
    const TIn *self, *other;
    const float *gds, *gdo;
    const int32_t *ids, *ido;
    TIn *grad;
    int ns, no, blk, gps, gpo;
    bool direct_first;
    int batch;  // batch-major placement: both directions of an element on one XCD (pcm_split_bm)
    bool first_dir;
    pcm_split_bm(bid, nblk1, nblk2, batch, first_dir, blk);
    if (first_dir) {
        self = xyz1 + (size_t)batch * n * 3;
        other = xyz2 + (size_t)batch * m * 3;
        gds = gd1 + (size_t)batch * (GS.bs1 < 0 ? n : GS.bs1);
        gdo = gd2 + (size_t)batch * (GS.bs2 < 0 ? m : GS.bs2);
        gps = GS.ps1;
        gpo = GS.ps2;
        ids = idx1 + (size_t)batch * n;
        ido = idx2 + (size_t)batch * m;
        grad = grad1 + (size_t)batch * n * 3;
        ns = n;
        no = m;
        direct_first = true;
    } else {
        self = xyz2 + (size_t)batch * m * 3;
        other = xyz1 + (size_t)batch * n * 3;
        gds = gd2 + (size_t)batch * (GS.bs2 < 0 ? m : GS.bs2);
        gdo = gd1 + (size_t)batch * (GS.bs1 < 0 ? n : GS.bs1);
        gps = GS.ps2;
        gpo = GS.ps1;
        ids = idx2 + (size_t)batch * m;
        ido = idx1 + (size_t)batch * n;
        grad = grad2 + (size_t)batch * m * 3;
        ns = m;
        no = n;
        direct_first = false;
    }
    // layouts (pcm_common.h PcmLay): the gradient takes its cloud's layout
    const PcmLay LS = direct_first ? pcm_lay(lay1, n) : pcm_lay(lay2, m);
    const PcmLay LO = direct_first ? pcm_lay(lay2, m) : pcm_lay(lay1, n);
    const int t0 = blk * NT;
    const int T = min(NT, ns - t0);

    // direct term first: its loads overlap the histogram pass
    const int i = t0 + tid;
    const bool own = tid < T;
    float sx = 0.f, sy = 0.f, sz = 0.f, dir0 = 0.f, dir1 = 0.f, dir2 = 0.f;
    if (own) {
        sx = pcm_ld(self + pcm_at(LS, i, 0));
        sy = pcm_ld(self + pcm_at(LS, i, 1));
        sz = pcm_ld(self + pcm_at(LS, i, 2));
        const int k = ids[i];
        const float g = __fmul_rn(gds[(size_t)i * gps], 2.f);
        dir0 = __fmul_rn(g, __fsub_rn(sx, pcm_ld(other + pcm_at(LO, k, 0))));
        dir1 = __fmul_rn(g, __fsub_rn(sy, pcm_ld(other + pcm_at(LO, k, 1))));
        dir2 = __fmul_rn(g, __fsub_rn(sz, pcm_ld(other + pcm_at(LO, k, 2))));
    }

    // 1. histogram of the other direction's argmins that land in [t0, t0+T)
    sCnt[tid] = 0;
    __syncthreads();
    for (int j = tid; j < no; j += NT) {
        const unsigned k = (unsigned)(ido[j] - t0);
        if (k < (unsigned)T) atomicAdd(&sCnt[k], 1);
    }
    __syncthreads();
    // 2. bucket offsets
    const int c = sCnt[tid];
    const int off = block_exclusive_scan<NT>(c, sWave);
    sOff[tid] = off;
    if (tid == NT - 1) sOff[NT] = off + c;
    sCnt[tid] = 0;
    __syncthreads();
    const int total = sOff[NT];
    const bool fits = total <= CAP;  // uniform

    if (fits && total > 0) {
        // 3. fill buckets (arbitrary order inside a bucket) ...
        for (int j = tid; j < no; j += NT) {
            const unsigned k = (unsigned)(ido[j] - t0);
            if (k < (unsigned)T) {
                const int s = atomicAdd(&sCnt[k], 1);
                sTmp[sOff[k] + s] = j;
            }
        }
        __syncthreads();
        // 4. ... then rank each entry by source index inside its bucket
        for (int p = tid; p < total; p += NT) {
            const int j = sTmp[p];
            const int k = ido[j] - t0;
            const int lo = sOff[k], hi = sOff[k + 1];
            int r = 0;
            for (int q = lo; q < hi; ++q) r += (sTmp[q] < j);
            sSrt[lo + r] = j;
        }
        __syncthreads();
    }

    if (!own) return;
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (direct_first) {
        ax = __fadd_rn(ax, dir0);
        ay = __fadd_rn(ay, dir1);
        az = __fadd_rn(az, dir2);
    }
    auto scatter = [&](int j) {
        const float g = __fmul_rn(gdo[(size_t)j * gpo], 2.f);
        ax = __fadd_rn(ax, -__fmul_rn(g, __fsub_rn(pcm_ld(other + pcm_at(LO, j, 0)), sx)));
        ay = __fadd_rn(ay, -__fmul_rn(g, __fsub_rn(pcm_ld(other + pcm_at(LO, j, 1)), sy)));
        az = __fadd_rn(az, -__fmul_rn(g, __fsub_rn(pcm_ld(other + pcm_at(LO, j, 2)), sz)));
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
        ax = __fadd_rn(ax, dir0);
        ay = __fadd_rn(ay, dir1);
        az = __fadd_rn(az, dir2);
    }
    pcm_st(grad + pcm_at(LS, i, 0), ax);
    pcm_st(grad + pcm_at(LS, i, 1), ay);
    pcm_st(grad + pcm_at(LS, i, 2), az);
}

// ---------------------------------------------------------------------------
// Backward, LDS-resident: one workgroup per batch element computes BOTH
// clouds' gradients with the whole batch (points, graddists, argmins, the two
// inverse-index counting sorts) in LDS: one coalesced load phase, LDS-only
// work, one store phase.  Used when 36*(n+m) bytes fit (n = m <= 2048).
// ---------------------------------------------------------------------------
constexpr int kBwdLdsT = 1024;

__host__ __device__ inline size_t bwd_lds_bytes(int n, int m) { return (size_t)36 * (n + m) + 64; }
constexpr size_t kBwdLdsMax = 150 * 1024;

// copy `count` 4-byte words global -> LDS, loads batched ahead of the stores
template <int NT, typename Tp>
__device__ inline void lds_copy(Tp *__restrict__ dst, const Tp *__restrict__ src, int count) {
    constexpr int U = 4;
    for (int base = 0; base < count; base += U * NT) {
        Tp v[U];
#pragma unroll
        for (int r = 0; r < U; ++r) {
            const int i = base + r * NT + (int)threadIdx.x;
            if (i < count) v[r] = src[i];
        }
#pragma unroll
        for (int r = 0; r < U; ++r) {
            const int i = base + r * NT + (int)threadIdx.x;
            if (i < count) dst[i] = v[r];
        }
    }
}

// exclusive scan of cnt[0..len) into off[0..len] (off[len] = total), NT threads
template <int NT>
__device__ inline void block_scan_array(const int *cnt, int *off, int len, int *wave_tot) {
    const int per = (len + NT - 1) / NT;
    const int lo = min(len, (int)threadIdx.x * per), hi = min(len, lo + per);
    int local = 0;
    for (int i = lo; i < hi; ++i) local += cnt[i];
    const int before = block_exclusive_scan<NT>(local, wave_tot);
    int run = before;
    for (int i = lo; i < hi; ++i) { off[i] = run; run += cnt[i]; }
    if (threadIdx.x == NT - 1) off[len] = run;
}

// counting sort of sources j (0..ns) by key[j] in [0, nk): off[0..nk], srt[]
// ascending j inside every bucket.  cnt is scratch [nk]; tmp scratch [ns].
template <int NT>
__device__ inline void inverse_index(const int *key, int ns, int nk, int *cnt, int *off, int *tmp,
                                     int *srt, int *wave_tot) {
    for (int i = threadIdx.x; i < nk; i += NT) cnt[i] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < ns; j += NT) atomicAdd(&cnt[key[j]], 1);
    __syncthreads();
    block_scan_array<NT>(cnt, off, nk, wave_tot);
    __syncthreads();
    for (int i = threadIdx.x; i < nk; i += NT) cnt[i] = 0;
    __syncthreads();
    for (int j = threadIdx.x; j < ns; j += NT) {
        const int k = key[j];
        tmp[off[k] + atomicAdd(&cnt[k], 1)] = j;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < ns; p += NT) {
        const int j = tmp[p];
        const int k = key[j];
        const int lo = off[k], hi = off[k + 1];
        int r = 0;
        for (int q = lo; q < hi; ++q) r += (tmp[q] < j);
        srt[lo + r] = j;
    }
}

__global__ __launch_bounds__(kBwdLdsT) void chamfer_bwd_lds_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int n, int m,
    const float *__restrict__ gd1, const float *__restrict__ gd2, const int32_t *__restrict__ idx1,
    const int32_t *__restrict__ idx2, float *__restrict__ grad1, float *__restrict__ grad2) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int sWave[kBwdLdsT / 64];
    const int batch = blockIdx.x;
    float *P1 = lds;                 // [3n] AoS
    float *P2 = P1 + 3 * n;          // [3m]
    float *G1 = P2 + 3 * m;          // [n]
    float *G2 = G1 + n;              // [m]
    int *I1 = (int *)(G2 + m);       // [n] argmin in cloud 2
    int *I2 = I1 + n;                // [m] argmin in cloud 1
    int *cnt = I2 + m;               // [max(n,m)] scratch
    int *off1 = cnt + max(n, m);     // [n+1] buckets of cloud-2 sources per cloud-1 point
    int *off2 = off1 + n + 1;        // [m+1]
    int *tmp = off2 + m + 1;         // [max(n,m)] scratch
    int *srt1 = tmp + max(n, m);     // [m]
    int *srt2 = srt1 + m;            // [n]

    lds_copy<kBwdLdsT>(P1, xyz1 + (size_t)batch * n * 3, 3 * n);
    lds_copy<kBwdLdsT>(P2, xyz2 + (size_t)batch * m * 3, 3 * m);
    lds_copy<kBwdLdsT>(G1, gd1 + (size_t)batch * n, n);
    lds_copy<kBwdLdsT>(G2, gd2 + (size_t)batch * m, m);
    lds_copy<kBwdLdsT>(I1, idx1 + (size_t)batch * n, n);
    lds_copy<kBwdLdsT>(I2, idx2 + (size_t)batch * m, m);
    __syncthreads();
    // cloud-1 points receive scatter terms from cloud-2 sources (key idx2)
    inverse_index<kBwdLdsT>(I2, m, n, cnt, off1, tmp, srt1, sWave);
    __syncthreads();
    inverse_index<kBwdLdsT>(I1, n, m, cnt, off2, tmp, srt2, sWave);
    __syncthreads();

    // cloud 1: direct term first (chamfer3D.cu:184), then cloud-2 scatters
    float *g1o = grad1 + (size_t)batch * n * 3;
    for (int i = threadIdx.x; i < n; i += kBwdLdsT) {
        const float sx = P1[3 * i], sy = P1[3 * i + 1], sz = P1[3 * i + 2];
        const int k = I1[i];
        const float g = __fmul_rn(G1[i], 2.f);
        float ax = __fadd_rn(0.f, __fmul_rn(g, __fsub_rn(sx, P2[3 * k])));
        float ay = __fadd_rn(0.f, __fmul_rn(g, __fsub_rn(sy, P2[3 * k + 1])));
        float az = __fadd_rn(0.f, __fmul_rn(g, __fsub_rn(sz, P2[3 * k + 2])));
        for (int p = off1[i]; p < off1[i + 1]; ++p) {
            const int j = srt1[p];
            const float h = __fmul_rn(G2[j], 2.f);
            ax = __fadd_rn(ax, -__fmul_rn(h, __fsub_rn(P2[3 * j], sx)));
            ay = __fadd_rn(ay, -__fmul_rn(h, __fsub_rn(P2[3 * j + 1], sy)));
            az = __fadd_rn(az, -__fmul_rn(h, __fsub_rn(P2[3 * j + 2], sz)));
        }
        g1o[3 * i] = ax;
        g1o[3 * i + 1] = ay;
        g1o[3 * i + 2] = az;
    }
    // cloud 2: cloud-1 scatters first (kernel 1 ran before kernel 2), then direct
    float *g2o = grad2 + (size_t)batch * m * 3;
    for (int i = threadIdx.x; i < m; i += kBwdLdsT) {
        const float sx = P2[3 * i], sy = P2[3 * i + 1], sz = P2[3 * i + 2];
        float ax = 0.f, ay = 0.f, az = 0.f;
        for (int p = off2[i]; p < off2[i + 1]; ++p) {
            const int j = srt2[p];
            const float h = __fmul_rn(G1[j], 2.f);
            ax = __fadd_rn(ax, -__fmul_rn(h, __fsub_rn(P1[3 * j], sx)));
            ay = __fadd_rn(ay, -__fmul_rn(h, __fsub_rn(P1[3 * j + 1], sy)));
            az = __fadd_rn(az, -__fmul_rn(h, __fsub_rn(P1[3 * j + 2], sz)));
        }
        const int k = I2[i];
        const float g = __fmul_rn(G2[i], 2.f);
        ax = __fadd_rn(ax, __fmul_rn(g, __fsub_rn(sx, P1[3 * k])));
        ay = __fadd_rn(ay, __fmul_rn(g, __fsub_rn(sy, P1[3 * k + 1])));
        az = __fadd_rn(az, __fmul_rn(g, __fsub_rn(sz, P1[3 * k + 2])));
        g2o[3 * i] = ax;
        g2o[3 * i + 1] = ay;
        g2o[3 * i + 2] = az;
    }
}

// ---------------------------------------------------------------------------
// Backward, staged: the 256-target workgroup layout of chamfer_bwd_kernel, but
// the other cloud's argmins, points and graddists (everything the histogram,
// fill, rank and scatter phases touch) arrive by one asynchronous LDS-DMA, so
// the phases run on LDS instead of re-reading global memory.  The own
// targets' direct terms load meanwhile.  Used when 20*no bytes fit.
// ---------------------------------------------------------------------------
constexpr int kBwdStageMax = 2048;  // sources staged (20 B each + sort scratch)

__global__ __launch_bounds__(kBwdT) void chamfer_bwd_staged_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int b, int n, int m,
    const float *__restrict__ gd1, const float *__restrict__ gd2, const int32_t *__restrict__ idx1,
    const int32_t *__restrict__ idx2, float *__restrict__ grad1, float *__restrict__ grad2,
    int nblk1, int nblk2, int lay1 = 0, int lay2 = 0, PcmGdStr GS = PcmGdStr()) {
    __shared__ __attribute__((aligned(16))) float sO[3 * kBwdStageMax];   // other cloud, AoS
    __shared__ __attribute__((aligned(16))) float sG[kBwdStageMax];       // other graddist
    __shared__ __attribute__((aligned(16))) int sK[kBwdStageMax];         // other argmins
    __shared__ int sCnt[kBwdT];
    __shared__ int sOff[kBwdT + 4];
    __shared__ int sTmp[kBwdStageMax];
    __shared__ int sSrt[kBwdStageMax];
    __shared__ int sWave[kBwdT / 64];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    int bid = pcm_xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const float *self, *other, *gds, *gdo;
    const int32_t *ids, *ido;
    float *grad;
    int ns, no, blk, gps, gpo;
    bool direct_first;
    int batch;  // batch-major placement: both directions of an element on one XCD (pcm_split_bm)
    bool first_dir;
    pcm_split_bm(bid, nblk1, nblk2, batch, first_dir, blk);
    if (first_dir) {
        self = xyz1 + (size_t)batch * n * 3;
        other = xyz2 + (size_t)batch * m * 3;
        gds = gd1 + (size_t)batch * (GS.bs1 < 0 ? n : GS.bs1);
        gdo = gd2 + (size_t)batch * (GS.bs2 < 0 ? m : GS.bs2);
        gps = GS.ps1;
        gpo = GS.ps2;
        ids = idx1 + (size_t)batch * n;
        ido = idx2 + (size_t)batch * m;
        grad = grad1 + (size_t)batch * n * 3;
        ns = n;
        no = m;
        direct_first = true;
    } else {
        self = xyz2 + (size_t)batch * m * 3;
        other = xyz1 + (size_t)batch * n * 3;
        gds = gd2 + (size_t)batch * (GS.bs2 < 0 ? m : GS.bs2);
        gdo = gd1 + (size_t)batch * (GS.bs1 < 0 ? n : GS.bs1);
        gps = GS.ps2;
        gpo = GS.ps1;
        ids = idx2 + (size_t)batch * m;
        ido = idx1 + (size_t)batch * n;
        grad = grad2 + (size_t)batch * m * 3;
        ns = m;
        no = n;
        direct_first = false;
    }
    const int t0 = blk * kBwdT;
    const int T = min(kBwdT, ns - t0);
    // layouts (pcm_common.h PcmLay): either is the element's 12 no contiguous
    // bytes, so the other cloud's LDS copy keeps its layout; the gradient
    // takes its own cloud's
    const PcmLay LS = direct_first ? pcm_lay(lay1, n) : pcm_lay(lay2, m);
    const PcmLay LO = direct_first ? pcm_lay(lay2, m) : pcm_lay(lay1, n);

    pcm_dma_to_lds(sK, ido, 4 * no, wave, kBwdT / 64);
    pcm_dma_to_lds(sO, other, 12 * no, wave, kBwdT / 64);
    if (gpo == 1)
        pcm_dma_to_lds(sG, gdo, 4 * no, wave, kBwdT / 64);
    else
        for (int j = threadIdx.x; j < no; j += kBwdT) sG[j] = gdo[(size_t)j * gpo];

    const int i = t0 + tid;
    const bool own = tid < T;
    float sx = 0.f, sy = 0.f, sz = 0.f, gself = 0.f;
    int kself = 0;
    if (own) {
        sx = self[pcm_at(LS, i, 0)];
        sy = self[pcm_at(LS, i, 1)];
        sz = self[pcm_at(LS, i, 2)];
        kself = ids[i];
        gself = gds[(size_t)i * gps];
    }
    sCnt[tid] = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // 1. histogram of the other direction's argmins landing in [t0, t0+T)
    for (int j = tid; j < no; j += kBwdT) {
        const unsigned k = (unsigned)(sK[j] - t0);
        if (k < (unsigned)T) atomicAdd(&sCnt[k], 1);
    }
    __syncthreads();
    const int c = sCnt[tid];
    const int off = block_exclusive_scan<kBwdT>(c, sWave);
    sOff[tid] = off;
    if (tid == kBwdT - 1) sOff[kBwdT] = off + c;
    sCnt[tid] = 0;
    __syncthreads();
    const int total = sOff[kBwdT];
    // 2. fill buckets, 3. rank by source index inside each bucket
    for (int j = tid; j < no; j += kBwdT) {
        const unsigned k = (unsigned)(sK[j] - t0);
        if (k < (unsigned)T) sTmp[sOff[k] + atomicAdd(&sCnt[k], 1)] = j;
    }
    __syncthreads();
    for (int p = tid; p < total; p += kBwdT) {
        const int j = sTmp[p];
        const int k = sK[j] - t0;
        const int lo = sOff[k], hi = sOff[k + 1];
        int r = 0;
        for (int q = lo; q < hi; ++q) r += (sTmp[q] < j);
        sSrt[lo + r] = j;
    }
    __syncthreads();
    if (!own) return;

    // 4. accumulate in the reference's kernel order
    const float g = __fmul_rn(gself, 2.f);
    const float d0 = __fmul_rn(g, __fsub_rn(sx, sO[pcm_at(LO, kself, 0)]));
    const float d1 = __fmul_rn(g, __fsub_rn(sy, sO[pcm_at(LO, kself, 1)]));
    const float d2 = __fmul_rn(g, __fsub_rn(sz, sO[pcm_at(LO, kself, 2)]));
    float ax = 0.f, ay = 0.f, az = 0.f;
    if (direct_first) {
        ax = __fadd_rn(ax, d0);
        ay = __fadd_rn(ay, d1);
        az = __fadd_rn(az, d2);
    }
    for (int p = sOff[tid]; p < sOff[tid + 1]; ++p) {
        const int j = sSrt[p];
        const float h = __fmul_rn(sG[j], 2.f);
        ax = __fadd_rn(ax, -__fmul_rn(h, __fsub_rn(sO[pcm_at(LO, j, 0)], sx)));
        ay = __fadd_rn(ay, -__fmul_rn(h, __fsub_rn(sO[pcm_at(LO, j, 1)], sy)));
        az = __fadd_rn(az, -__fmul_rn(h, __fsub_rn(sO[pcm_at(LO, j, 2)], sz)));
    }
    if (!direct_first) {
        ax = __fadd_rn(ax, d0);
        ay = __fadd_rn(ay, d1);
        az = __fadd_rn(az, d2);
    }
    grad[pcm_at(LS, i, 0)] = ax;
    grad[pcm_at(LS, i, 1)] = ay;
    grad[pcm_at(LS, i, 2)] = az;
}

inline bool bad_dims(int b, int n, int m) { return b < 0 || n < 0 || m < 0; }

// ---- forward variant table (tuning: tools/tune_chamfer.py) -----------------
typedef pcm_fwd_kernel_t fwd_kernel_t;
typedef PcmFwdVariant FwdVariant;
#define PCM_FWD_LDS(W, Q)                                                              \
    FwdVariant{chamfer_fwd_kernel<float, W, Q, kChunk, kTile, false>,                  \
               chamfer_fwd_kernel<float, W, Q, kChunk, kTile, true>, nullptr, nullptr, W, Q, false}
#define PCM_FWD_SGPR(W, Q, C)                                                          \
    FwdVariant{chamfer_fwd_sgpr_kernel<W, Q, C, 0>, chamfer_fwd_sgpr_kernel<W, Q, C, 1>, \
               chamfer_fwd_sgpr_kernel<W, Q, C, 2>, chamfer_fwd_sgpr_kernel<W, Q, C, 3>, W, Q, true}
const FwdVariant kFwdVariants[] = {
    PCM_FWD_LDS(8, 2),       // 0: LDS-tile form
    PCM_FWD_LDS(8, 4),       // 1
    PCM_FWD_SGPR(8, 2, 32),  // 2: SGPR-stream form
    PCM_FWD_SGPR(8, 4, 32),  // 3
    PCM_FWD_SGPR(4, 2, 32),  // 4
    PCM_FWD_SGPR(16, 2, 32), // 5
    PCM_FWD_SGPR(4, 4, 32),  // 6
    PCM_FWD_SGPR(16, 4, 32), // 7
    PCM_FWD_SGPR(8, 2, 16),  // 8
    PCM_FWD_SGPR(16, 2, 16), // 9
};
constexpr int kNumBaseFwdVariants = sizeof(kFwdVariants) / sizeof(kFwdVariants[0]);
// variant ids >= kNumBaseFwdVariants index the filtered-scan table (chamfer_filt.hip)
inline int num_fwd_variants() { return kNumBaseFwdVariants + kPcmNumFiltVariants; }
inline const FwdVariant &fwd_variant(int i) {
    return i < kNumBaseFwdVariants ? kFwdVariants[i] : kPcmFiltVariants[i - kNumBaseFwdVariants];
}
// Default policy from tools/tune_chamfer.py on MI355X (profiles/r01): the
// SGPR-stream form wins everywhere; 2 queries per lane and 16-candidate chunks
// for ShapeNet-size clouds (B=32, N=M=1024: 12.7 us vs 13.5 us LDS-tile), 4
// queries per lane once a batch has >= 4M pairs (B=8, N=M=16384: 453 us).
constexpr int kDefaultLossMode = 3;  // tools/tune_chamfer.py (profiles/r01): mode 3 vs 2 vs 1
// With chamfer_filt.hip's filtered form (profiles/r01/tune_chamfer_r01e.txt): at
// B=8, N=M=16384 the filtered W=8 QPT=4 C=32 variant takes 344-356 us against
// 457-471 us for the best exact-scan form; at B=32, N=M=1024 the two are level
// (12.2 vs 12.4 us) and the SGPR form keeps the small sizes.
// Round 2 (near-tie scans split over the waves, DPP reductions): the
// filtered W=8 QPT=4 C=32 form leads at config 2 as well -- 11.96 us against
// 12.45 us for the SGPR form -- so it is the default at every size.
// Round 5 (tools/ab_ref_call.py, profiles/r05): clouds of at most 1024 points
// take the one-launch step's geometry, C 16 with 1024-point tiles -- 11.07
// against 11.43 us at config 2, bit-identical.
inline int default_fwd_variant(int n, int m) { return kNumBaseFwdVariants + ((n <= 1024 && m <= 1024) ? 8 : 3); }

int fwd_grid(const FwdVariant &v, int b, int n, int m, int &nblk1, int &nblk2, long long &blocks) {
    const int QW = 64 * v.qpt;
    // a direction with no targets leaves its outputs untouched: give it no blocks
    nblk1 = (m > 0) ? (n + QW - 1) / QW : 0;
    nblk2 = (n > 0) ? (m + QW - 1) / QW : 0;
    blocks = (long long)b * (nblk1 + nblk2);
    return blocks > 0x7ffffffeLL ? PCM_ERR_UNSUPPORTED : PCM_OK;  // + 1 polling workgroup (mode 3)
}

// loss_mode (mean_out != nullptr): 1 = in-kernel arrival ticket + last-workgroup
// reduction; 2 = workgroup partials + chamfer_loss_finalize_kernel; 3 = granules
// swept by one extra polling workgroup (poll_loss).
int launch_fwd(int variant, const float *xyz1, const float *xyz2, int b, int n, int m, float *dist1,
               float *dist2, int32_t *idx1, int32_t *idx2, float *mean_out, void *ws, size_t ws_bytes,
               void *stream, int loss_mode = kDefaultLossMode) {
    if (bad_dims(b, n, m)) return PCM_ERR_INVALID_ARG;
    if (variant < 0 || variant >= num_fwd_variants()) return PCM_ERR_INVALID_ARG;
    const FwdVariant &v = fwd_variant(variant);
    const bool loss = mean_out != nullptr;
    if (loss && (b == 0 || n == 0 || m == 0)) return PCM_ERR_INVALID_ARG;
    if (b == 0 || (n == 0 && m == 0)) return PCM_OK;
    if ((n > 0 && (!xyz1 || !dist1 || !idx1)) || (m > 0 && (!xyz2 || !dist2 || !idx2)))
        return PCM_ERR_INVALID_ARG;
    int nblk1, nblk2;
    long long blocks;
    if (fwd_grid(v, b, n, m, nblk1, nblk2, blocks) != PCM_OK) return PCM_ERR_UNSUPPORTED;
    if (blocks == 0) return PCM_OK;
    float *partials = nullptr;
    unsigned *ticket = nullptr;
    if (loss) {
        const size_t need = pcm_chamfer_workspace_bytes(b, n, m);
        if (!ws || ws_bytes < need) return PCM_ERR_WORKSPACE;
        ticket = (unsigned *)ws;
        partials = (float *)((char *)ws + kTicketBytes);
    }
    if (loss && loss_mode == 2 && !v.loss2) loss_mode = 1;
    if (loss && loss_mode == 3 && !v.loss3) loss_mode = 1;
    if (loss && loss_mode == 1 && !v.loss) loss_mode = 3;  // filtered variants: granules only
    if (loss && (loss_mode < 1 || loss_mode > 3)) return PCM_ERR_INVALID_ARG;
    fwd_kernel_t k = !loss ? v.plain : (loss_mode == 3 ? v.loss3 : (loss_mode == 2 ? v.loss2 : v.loss));
    const long long grid = blocks + ((loss && loss_mode == 3) ? 1 : 0);  // + the polling workgroup
    hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * v.waves), 0, (hipStream_t)stream, xyz1, xyz2,
                       b, n, m, dist1, dist2, idx1, idx2, nblk1, nblk2, partials, ticket, mean_out);
    if (loss && loss_mode == 2)
        hipLaunchKernelGGL(chamfer_loss_finalize_kernel, dim3(1), dim3(512), 0, (hipStream_t)stream,
                           partials, b * nblk1, (int)blocks, b, n, m, mean_out);
    return pcm_launch_status();
}

}  // namespace

size_t pcm_chamfer_loss_ws_offset(int b, int n, int m) {
    if (b <= 0 || n < 0 || m < 0) return kTicketBytes;
    long long most = 0;
    for (int i = 0; i < num_fwd_variants(); ++i) {
        int n1, n2;
        long long blocks;
        fwd_grid(fwd_variant(i), b, n, m, n1, n2, blocks);
        most = blocks > most ? blocks : most;
    }
    const size_t bytes = kTicketBytes + (size_t)most * sizeof(unsigned long long);  // 8-B granules (mode 3)
    return (bytes + 127) / 128 * 128;
}

extern "C" size_t pcm_chamfer_workspace_bytes(int b, int n, int m) {
    return pcm_chamfer_loss_ws_offset(b, n, m) + pcm_chamfer_grad_ws_bytes(b, n, m);
}

// sticky device-side error words of the fused-loss kernels (a bounded wait
// that timed out): PCM_ERR_LAUNCH when either is set.  Synchronises `stream`.
extern "C" int pcm_chamfer_workspace_status(const void *workspace, size_t workspace_bytes, int b, int n, int m,
                                            void *stream) {
    if (b <= 0 || n <= 0 || m <= 0) return PCM_OK;
    if (!workspace || workspace_bytes < pcm_chamfer_workspace_bytes(b, n, m)) return PCM_ERR_WORKSPACE;
    unsigned words[2] = {0u, 0u};
    const char *base = (const char *)workspace;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemcpyAsync(&words[0], base + 4 * pcm_loss::kErrWord, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&words[1], base + pcm_chamfer_loss_ws_offset(b, n, m) + 4 * pcm_chamfer_grad_err_word(), 4,
                       hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return PCM_ERR_LAUNCH;
    return (words[0] || words[1]) ? PCM_ERR_LAUNCH : PCM_OK;
}

// byte offsets in the workspace of the two sticky error words read above
// (which = 0: the fused-loss forward's, 1: the one-launch step's), for the
// Python wrappers' asynchronous copy (metric/pcm_hip.py _StickyWatch)
extern "C" size_t pcm_tune_chamfer_err_offset(int which, int b, int n, int m) {
    return which == 0 ? 4 * (size_t)pcm_loss::kErrWord
                      : pcm_chamfer_loss_ws_offset(b, n, m) + 4 * (size_t)pcm_chamfer_grad_err_word();
}

extern "C" int pcm_chamfer_forward(const float *xyz1, const float *xyz2, int b, int n, int m,
                                   float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                   void *stream) {
    return launch_fwd(default_fwd_variant(n, m), xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, nullptr,
                      nullptr, 0, stream);
}

extern "C" int pcm_chamfer_forward_loss(const float *xyz1, const float *xyz2, int b, int n, int m,
                                        float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                        float *mean_out, void *workspace, size_t workspace_bytes,
                                        void *stream) {
    if (!mean_out) return PCM_ERR_INVALID_ARG;
    return launch_fwd(default_fwd_variant(n, m), xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, mean_out,
                      workspace, workspace_bytes, stream);
}

extern "C" int pcm_tune_chamfer_forward(int variant, const float *xyz1, const float *xyz2, int b, int n,
                                        int m, float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                        void *stream) {
    return launch_fwd(variant, xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, nullptr, nullptr, 0,
                      stream);
}

extern "C" int pcm_tune_chamfer_forward_loss(int variant, int loss_mode, const float *xyz1,
                                             const float *xyz2, int b, int n, int m, float *dist1,
                                             float *dist2, int32_t *idx1, int32_t *idx2, float *mean_out,
                                             void *workspace, size_t workspace_bytes, void *stream) {
    if (!mean_out) return PCM_ERR_INVALID_ARG;
    if (variant < 0) variant = default_fwd_variant(n, m);
    return launch_fwd(variant, xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, mean_out, workspace,
                      workspace_bytes, stream, loss_mode);
}

extern "C" int pcm_tune_num_chamfer_variants(void) { return num_fwd_variants(); }

namespace {
constexpr int kBwdWideT = 1024;    // targets per workgroup for large clouds
constexpr int kBwdWideCap = 8192;  // their sortable scatter entries (64 KiB of LDS)
inline bool wide_bwd(int n, int m) { return n >= 4096 && m >= 4096; }

int launch_bwd(int variant, const float *xyz1, const float *xyz2, int b, int n, int m,
               const float *graddist1, const float *graddist2, const int32_t *idx1,
               const int32_t *idx2, float *gradxyz1, float *gradxyz2, void *stream, int lay1 = 0, int lay2 = 0,
               PcmGdStr GS = PcmGdStr()) {
    if (bad_dims(b, n, m)) return PCM_ERR_INVALID_ARG;
    if (b == 0 || (n == 0 && m == 0)) return PCM_OK;
    // Without targets a direction has no argmins; the reference would read
    // garbage indices.  Both clouds must be non-empty for a gradient.
    if (n == 0 || m == 0) return PCM_ERR_INVALID_ARG;
    if (!xyz1 || !xyz2 || !graddist1 || !graddist2 || !idx1 || !idx2 || !gradxyz1 || !gradxyz2)
        return PCM_ERR_INVALID_ARG;
    const int nblk1 = (n + kBwdT - 1) / kBwdT;
    const int nblk2 = (m + kBwdT - 1) / kBwdT;
    const long long blocks = (long long)b * (nblk1 + nblk2);
    if (blocks > 0x7fffffffLL) return PCM_ERR_UNSUPPORTED;
    if (variant == 0 && pcm_bwd_slots_fits(n, m))
        return pcm_launch_bwd_slots(xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2, lay1,
                                    lay2, GS, (hipStream_t)stream);
    if (variant == 4 && n <= kBwdStageMax && m <= kBwdStageMax) {  // round 4's default (staged passes)
        hipLaunchKernelGGL(chamfer_bwd_staged_kernel, dim3((unsigned)blocks), dim3(kBwdT), 0,
                           (hipStream_t)stream, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1,
                           idx2, gradxyz1, gradxyz2, nblk1, nblk2, lay1, lay2, GS);
        return pcm_launch_status();
    }
    const bool strided = GS.bs1 >= 0 || GS.bs2 >= 0 || GS.ps1 != 1 || GS.ps2 != 1;
    if (lay1 != 0 || lay2 != 0 || (strided && !wide_bwd(n, m)) || variant == 4) {
        // channel planes or strided graddists: the staged kernel's forms, else the global-memory kernel's
        hipLaunchKernelGGL(chamfer_bwd_kernel<float>, dim3((unsigned)blocks), dim3(kBwdT), 0, (hipStream_t)stream,
                           xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2, nblk1, nblk2,
                           lay1, lay2, GS);
        return pcm_launch_status();
    }
    const size_t lds = bwd_lds_bytes(n, m);
    if (variant == 2 && lds <= kBwdLdsMax && !strided) {
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute((const void *)chamfer_bwd_lds_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return PCM_ERR_LAUNCH;
        hipLaunchKernelGGL(chamfer_bwd_lds_kernel, dim3((unsigned)b), dim3(kBwdLdsT), lds,
                           (hipStream_t)stream, xyz1, xyz2, n, m, graddist1, graddist2, idx1, idx2,
                           gradxyz1, gradxyz2);
        return pcm_launch_status();
    }
    if (variant == 3 || (variant == 0 && wide_bwd(n, m))) {
        const int w1 = (n + kBwdWideT - 1) / kBwdWideT, w2 = (m + kBwdWideT - 1) / kBwdWideT;
        hipLaunchKernelGGL((chamfer_bwd_kernel<float, kBwdWideT, kBwdWideCap>), dim3((unsigned)(b * (w1 + w2))),
                           dim3(kBwdWideT), 0, (hipStream_t)stream, xyz1, xyz2, b, n, m, graddist1, graddist2,
                           idx1, idx2, gradxyz1, gradxyz2, w1, w2, 0, 0, GS);
        return pcm_launch_status();
    }
    hipLaunchKernelGGL(chamfer_bwd_kernel<float>, dim3((unsigned)blocks), dim3(kBwdT), 0,
                       (hipStream_t)stream, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2,
                       gradxyz1, gradxyz2, nblk1, nblk2);
    return pcm_launch_status();
}
}  // namespace

extern "C" int pcm_chamfer_backward(const float *xyz1, const float *xyz2, int b, int n, int m,
                                    const float *graddist1, const float *graddist2,
                                    const int32_t *idx1, const int32_t *idx2, float *gradxyz1,
                                    float *gradxyz2, void *stream) {
    return launch_bwd(0, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2,
                      stream);
}

extern "C" int pcm_chamfer_backward_layout(const float *xyz1, const float *xyz2, int b, int n, int m, int layout1,
                                           int layout2, const float *graddist1, const float *graddist2,
                                           const int32_t *idx1, const int32_t *idx2, float *gradxyz1,
                                           float *gradxyz2, void *stream) {
    if ((unsigned)layout1 > 1u || (unsigned)layout2 > 1u) return PCM_ERR_INVALID_ARG;
    return launch_bwd(0, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2, stream, layout1,
                      layout2);
}

extern "C" int pcm_chamfer_backward_strided(const float *xyz1, const float *xyz2, int b, int n, int m, int layout1,
                                            int layout2, const float *graddist1, long long gd1_batch_stride,
                                            long long gd1_point_stride, const float *graddist2,
                                            long long gd2_batch_stride, long long gd2_point_stride,
                                            const int32_t *idx1, const int32_t *idx2, float *gradxyz1,
                                            float *gradxyz2, void *stream) {
    if ((unsigned)layout1 > 1u || (unsigned)layout2 > 1u) return PCM_ERR_INVALID_ARG;
    const long long lim = 0x7fffffffLL;
    if (gd1_batch_stride < 0 || gd1_point_stride < 0 || gd2_batch_stride < 0 || gd2_point_stride < 0 ||
        gd1_batch_stride > lim || gd1_point_stride > lim || gd2_batch_stride > lim || gd2_point_stride > lim)
        return PCM_ERR_INVALID_ARG;
    PcmGdStr GS;  // contiguous graddists keep the default (unstrided) routing
    const bool c1 = gd1_point_stride == 1 && gd1_batch_stride == n, c2 = gd2_point_stride == 1 && gd2_batch_stride == m;
    GS.bs1 = c1 ? -1 : (int)gd1_batch_stride;
    GS.ps1 = c1 ? 1 : (int)gd1_point_stride;
    GS.bs2 = c2 ? -1 : (int)gd2_batch_stride;
    GS.ps2 = c2 ? 1 : (int)gd2_point_stride;
    return launch_bwd(0, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2, stream, layout1,
                      layout2, GS);
}

extern "C" int pcm_tune_chamfer_backward(int variant, const float *xyz1, const float *xyz2, int b,
                                         int n, int m, const float *graddist1,
                                         const float *graddist2, const int32_t *idx1,
                                         const int32_t *idx2, float *gradxyz1, float *gradxyz2,
                                         void *stream) {
    return launch_bwd(variant, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1,
                      gradxyz2, stream);
}

// ---------------------------------------------------------------------------
// fp16 clouds (BASELINE config 5, an extension: the reference read
// Tensor::data<float>() only).  Coordinates are widened to fp32 on load
// (exact), so every result equals the fp32 path on the widened clouds; the
// gradients are rounded to fp16 once, at the store.  The forward uses the
// LDS-tile form, which widens each tile as it stages it (one cvt per loaded
// coordinate per workgroup); the SGPR-stream form would convert every
// candidate in every wave (3 more VALU per candidate per wave).
// ---------------------------------------------------------------------------
namespace {
typedef PcmFwd16Variant Fwd16Variant;
const Fwd16Variant kFwd16Variants[] = {
    {chamfer_fwd_kernel<pcm_h, 8, 2, kChunk, kTile, false>, 8, 2},  // 0
    {chamfer_fwd_kernel<pcm_h, 8, 4, kChunk, kTile, false>, 8, 4},  // 1
};
constexpr int kNumBaseFwd16Variants = sizeof(kFwd16Variants) / sizeof(kFwd16Variants[0]);
// ids >= kNumBaseFwd16Variants: the filtered form on fp16 clouds (chamfer_filt.hip)
inline int num_fwd16_variants() { return kNumBaseFwd16Variants + kPcmNumFilt16Variants; }
inline const Fwd16Variant &fwd16_variant(int i) {
    return i < kNumBaseFwd16Variants ? kFwd16Variants[i] : kPcmFilt16Variants[i - kNumBaseFwd16Variants];
}
// tools/tune_chamfer.py on MI355X (profiles/r01): the filtered form wins once
// a batch element has >= 4M pairs (B=8, N=M=16384); round 2: also at B=32,
// N=M=1024 (12.25 us against 13.46 us for the LDS-tile form), so at every size
inline int default_fwd16_variant(int, int) { return kNumBaseFwd16Variants + 1; }

int launch_fwd16(int variant, const pcm_h *xyz1, const pcm_h *xyz2, int b, int n, int m, float *dist1,
                 float *dist2, int32_t *idx1, int32_t *idx2, void *stream) {
    if (bad_dims(b, n, m)) return PCM_ERR_INVALID_ARG;
    if (variant < 0 || variant >= num_fwd16_variants()) return PCM_ERR_INVALID_ARG;
    if (b == 0 || (n == 0 && m == 0)) return PCM_OK;
    if ((n > 0 && (!xyz1 || !dist1 || !idx1)) || (m > 0 && (!xyz2 || !dist2 || !idx2)))
        return PCM_ERR_INVALID_ARG;
    const Fwd16Variant &v = fwd16_variant(variant);
    const int QW = 64 * v.qpt;
    const int nblk1 = (m > 0) ? (n + QW - 1) / QW : 0;
    const int nblk2 = (n > 0) ? (m + QW - 1) / QW : 0;
    const long long blocks = (long long)b * (nblk1 + nblk2);
    if (blocks > 0x7fffffffLL) return PCM_ERR_UNSUPPORTED;
    if (blocks == 0) return PCM_OK;
    hipLaunchKernelGGL(v.k, dim3((unsigned)blocks), dim3(64 * v.waves), 0, (hipStream_t)stream, xyz1, xyz2, b,
                       n, m, dist1, dist2, idx1, idx2, nblk1, nblk2, nullptr, nullptr, nullptr);
    return pcm_launch_status();
}
}  // namespace

extern "C" int pcm_chamfer_forward_f16(const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                                       float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                       void *stream) {
    return launch_fwd16(default_fwd16_variant(n, m), (const pcm_h *)xyz1, (const pcm_h *)xyz2, b, n, m, dist1,
                        dist2, idx1, idx2, stream);
}

extern "C" int pcm_tune_chamfer_forward_f16(int variant, const uint16_t *xyz1, const uint16_t *xyz2, int b,
                                            int n, int m, float *dist1, float *dist2, int32_t *idx1,
                                            int32_t *idx2, void *stream) {
    if (variant < 0) variant = default_fwd16_variant(n, m);
    return launch_fwd16(variant, (const pcm_h *)xyz1, (const pcm_h *)xyz2, b, n, m, dist1, dist2, idx1, idx2,
                        stream);
}

extern "C" int pcm_tune_num_chamfer_f16_variants(void) { return num_fwd16_variants(); }

namespace {
int launch_bwd16(int variant, const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m, const float *graddist1,
                 const float *graddist2, const int32_t *idx1, const int32_t *idx2, uint16_t *gradxyz1,
                 uint16_t *gradxyz2, void *stream) {
    if (bad_dims(b, n, m)) return PCM_ERR_INVALID_ARG;
    if (b == 0 || (n == 0 && m == 0)) return PCM_OK;
    if (n == 0 || m == 0) return PCM_ERR_INVALID_ARG;
    if (!xyz1 || !xyz2 || !graddist1 || !graddist2 || !idx1 || !idx2 || !gradxyz1 || !gradxyz2)
        return PCM_ERR_INVALID_ARG;
    if (variant == 3 || (variant == 0 && wide_bwd(n, m))) {
        const int w1 = (n + kBwdWideT - 1) / kBwdWideT, w2 = (m + kBwdWideT - 1) / kBwdWideT;
        hipLaunchKernelGGL((chamfer_bwd_kernel<pcm_h, kBwdWideT, kBwdWideCap>), dim3((unsigned)(b * (w1 + w2))),
                           dim3(kBwdWideT), 0, (hipStream_t)stream, (const pcm_h *)xyz1, (const pcm_h *)xyz2, b, n,
                           m, graddist1, graddist2, idx1, idx2, (pcm_h *)gradxyz1, (pcm_h *)gradxyz2, w1, w2);
        return pcm_launch_status();
    }
    const int nblk1 = (n + kBwdT - 1) / kBwdT;
    const int nblk2 = (m + kBwdT - 1) / kBwdT;
    const long long blocks = (long long)b * (nblk1 + nblk2);
    if (blocks > 0x7fffffffLL) return PCM_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(chamfer_bwd_kernel<pcm_h>, dim3((unsigned)blocks), dim3(kBwdT), 0, (hipStream_t)stream,
                       (const pcm_h *)xyz1, (const pcm_h *)xyz2, b, n, m, graddist1, graddist2, idx1, idx2,
                       (pcm_h *)gradxyz1, (pcm_h *)gradxyz2, nblk1, nblk2);
    return pcm_launch_status();
}
}  // namespace

extern "C" int pcm_chamfer_backward_f16(const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                                        const float *graddist1, const float *graddist2,
                                        const int32_t *idx1, const int32_t *idx2, uint16_t *gradxyz1,
                                        uint16_t *gradxyz2, void *stream) {
    return launch_bwd16(0, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2, stream);
}

// variant 0 = default, 1 = 256-target workgroups, 3 = 1024-target workgroups
extern "C" int pcm_tune_chamfer_backward_f16(int variant, const uint16_t *xyz1, const uint16_t *xyz2, int b, int n,
                                             int m, const float *graddist1, const float *graddist2,
                                             const int32_t *idx1, const int32_t *idx2, uint16_t *gradxyz1,
                                             uint16_t *gradxyz2, void *stream) {
    return launch_bwd16(variant, xyz1, xyz2, b, n, m, graddist1, graddist2, idx1, idx2, gradxyz1, gradxyz2,
                        stream);
}
