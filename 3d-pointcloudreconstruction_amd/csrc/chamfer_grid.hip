// chamfer_grid.hip -- exact bidirectional nearest neighbour for large clouds
// through a uniform grid (BASELINE config 5: B=8, N=M=16384 fp16).
//
// Same outputs as pcm_chamfer_forward (chamfer3D.cu:12-154: squared distance
// in the pinned fma order, lowest argmin index), bit for bit; only the set of
// candidates a query evaluates shrinks from the whole cloud to the points of
// the grid cells around its block, plus a proof that nothing outside can win:
//
//   grid_build_kernel  one workgroup per (cloud, slab of 4 cell layers): a
//                      G^3 grid of cubic cells (G = 16, or 32 from 12k
//                      points) over the cloud's bounding box and two sorted
//                      (x, y, z, index) float4 copies: by row-major cell --
//                      the target copy, where one row of cells is one
//                      contiguous range -- and by serpentine brick order --
//                      the query copy, where 64 consecutive points are
//                      spatially compact.  No global atomics, no waits.
//   grid_nn_kernel     one wave per 64 consecutive query-order points of one
//                      direction.  The wave's bounding box in the target grid,
//                      widened by `margin` cells, is gathered row range by row
//                      range into the wave's LDS slice (512 candidates per
//                      round) and every query keeps the lexicographic minimum
//                      of (distance bits, index) -- one 64-bit compare, exact
//                      because distances are non-negative.  A query whose best
//                      distance is not below the squared distance to the
//                      region's inner faces (minus rounding slack) stays
//                      pending; the next round gathers around the pending
//                      queries only, 3x wider, and the last round takes the
//                      whole grid (always proven).  Elements with a non-finite
//                      coordinate take the reference's 512-point tile scan
//                      (pcm_ref_nn_scan) per query, as the dense kernels do.
//
// The margin is sized from the target's point count so that on uniform clouds
// a query's nearest neighbour lies beyond it with probability ~e^-12: at
// N=16384, G=32, margin 2, a wave gathers ~10^3 cells, ~450 candidates per
// query -- 36x fewer than the dense scan.  The order of points inside a cell
// depends on atomics, but no result does (the lexicographic minimum is
// order-free).
#include "pcm_common.h"
#include "pcm_internal.h"

namespace {

constexpr int kMaxGBits = 5;
constexpr int kMaxCells = 1 << (3 * kMaxGBits);  // 32768
constexpr int kFineMin = 12000;  // clouds from this size get G = 32
constexpr int kNnT = 1024;       // 16 waves (one workgroup per CU), each an independent block of 64 queries
constexpr int kWaveCap = 512;    // candidates staged per wave and round (8 KiB of LDS)
constexpr int kGeo = 8;          // floats per cloud: lo.xyz, h, 1/h, non-finite flag, G, margin
constexpr int kGridMinPoints = 4096;  // smaller clouds take the dense kernels

// Query order: bricks of 4x4x4 cells visited in a serpentine (boustrophedon)
// order -- consecutive bricks always share a face, so any run of consecutive
// points spans a few neighbouring bricks (a Z-order curve jumps across the
// grid at its octant seams) -- and the cells of a brick in row-major order
// (cell_query_key below).
// cell coordinate along one axis: floor((v - lo) / h) clamped to the grid
// (NaN -> 0; only reached for clouds flagged non-finite, whose results come
// from the reference scan)
__device__ __forceinline__ int cell_axis(float v, float lo, float inv_h, int G) {
    return (int)fminf(fmaxf((v - lo) * inv_h, 0.f), (float)(G - 1));
}

// wave-wide reductions and scans on DPP row shifts / broadcasts (VALU operand
// modifiers: no LDS round trip per step); results are taken from lane 63
template <int CTRL, int ROWMASK, bool BC>
__device__ __forceinline__ int dpp(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xf, BC);
}
template <bool kMax>
__device__ __forceinline__ float wave_extf(float v) {
    auto f = [](float a, float b) { return kMax ? fmaxf(a, b) : fminf(a, b); };
    int x = __float_as_int(v);
    x = __float_as_int(f(__int_as_float(x), __int_as_float(dpp<0x111, 0xf, false>(x, x))));  // row_shr:1
    x = __float_as_int(f(__int_as_float(x), __int_as_float(dpp<0x112, 0xf, false>(x, x))));  // row_shr:2
    x = __float_as_int(f(__int_as_float(x), __int_as_float(dpp<0x114, 0xf, false>(x, x))));  // row_shr:4
    x = __float_as_int(f(__int_as_float(x), __int_as_float(dpp<0x118, 0xf, false>(x, x))));  // row_shr:8
    x = __float_as_int(f(__int_as_float(x), __int_as_float(dpp<0x142, 0xa, false>(x, x))));  // row_bcast:15
    x = __float_as_int(f(__int_as_float(x), __int_as_float(dpp<0x143, 0xc, false>(x, x))));  // row_bcast:31
    return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}
__device__ __forceinline__ float wave_minf(float v) { return wave_extf<false>(v); }
__device__ __forceinline__ float wave_maxf(float v) { return wave_extf<true>(v); }
// inclusive prefix sum over the wave (shifted-in lanes read 0)
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += dpp<0x111, 0xf, true>(0, x);  // row_shr:1
    x += dpp<0x112, 0xf, true>(0, x);  // row_shr:2
    x += dpp<0x114, 0xf, true>(0, x);  // row_shr:4
    x += dpp<0x118, 0xf, true>(0, x);  // row_shr:8
    x += dpp<0x142, 0xa, false>(0, x); // row_bcast:15 into rows 1 and 3
    x += dpp<0x143, 0xc, false>(0, x); // row_bcast:31 into rows 2 and 3
    return x;
}

// LDS hand-off inside one wave: the wave's LDS operations complete in order,
// so waiting for them (and fencing the compiler) is all a wave needs
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// the wave's LDS-DMA copies have landed
__device__ __forceinline__ void wave_vm_sync() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// (distance bits, index) key of candidate t for query (qx, qy, qz)
__device__ __forceinline__ unsigned long long nn_key(pcm_f4 t, float qx, float qy, float qz) {
    const float d = pcm_sqd(t.x - qx, t.y - qy, t.z - qz);
    return ((unsigned long long)__float_as_uint(d) << 32) | __float_as_uint(t.w);
}

// ---- build: one workgroup per (cloud, slab of 4 cell layers in z).  Both
// orders (row-major cells; serpentine bricks, whose bricks are 4 layers
// thick) put whole slabs in z order, so a slab's points occupy one contiguous
// range of either sorted copy, whose offset is the count of points in lower
// slabs.  Every workgroup of a cloud reads the whole cloud (L2-resident after
// the first): bounding box, then slab counts and its own slab's two cell
// histograms in LDS, then its own points' positions -- no global atomics
// (device-scope atomics leave the XCD: 13 us for config 5's counts alone)
// and no workgroup waits on another.
constexpr int kSlabT = 1024;
constexpr int kSlabK = 16;   // points per thread and pass chunk (16384 per chunk)
constexpr int kSlabMax = 8;  // slabs per cloud: G / 4
constexpr int kSlabCells = 4 * 32 * 32;  // cells of one slab at G = 32

__device__ __forceinline__ int grid_dim(int np) { return np >= kFineMin ? 32 : 16; }

// cell (x, y, z) -> its key in the query (serpentine brick) order
__device__ __forceinline__ int cell_query_key(int x, int y, int z, int G) {
    const int nb = G >> 2;
    const int bx = x >> 2, by = y >> 2, bz = z >> 2;
    const int r = bz * nb + ((bz & 1) ? nb - 1 - by : by);
    const int bi = r * nb + ((r & 1) ? nb - 1 - bx : bx);
    return (bi << 6) + (((z & 3) * 4 + (y & 3)) << 2) + (x & 3);
}

template <typename TIn>
__global__ __launch_bounds__(kSlabT) void grid_build_kernel(const TIn *__restrict__ xyz1, const TIn *__restrict__ xyz2,
                                                            int b, int n, int m, pcm_f4 *__restrict__ tpts,
                                                            pcm_f4 *__restrict__ qpts, int *__restrict__ start,
                                                            float *__restrict__ geo) {
    constexpr int kW = kSlabT / 64;
    __shared__ int hT[kSlabCells], hQ[kSlabCells];  // own slab: row-major / query-order histograms -> cursors
    __shared__ float red[7][kW];
    __shared__ int sBelow;  // points of the cloud in lower slabs
    __shared__ int sw[2][kW];
    // a cloud's slab workgroups share one XCD (pcm_xcd_remap): the cloud they
    // all read twice is fetched into that L2 only, not into all eight
    const int L = pcm_xcd_remap((int)blockIdx.x, (int)gridDim.x);
    const int c = L / kSlabMax, slab = L % kSlabMax;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const bool two = c >= b;
    const int e = two ? c - b : c, np = two ? m : n;
    const int G = grid_dim(np), NS = G >> 2, scells = 4 * G * G;
    if (np == 0 || slab >= NS) return;
    const TIn *src = two ? xyz2 + 3 * (size_t)e * m : xyz1 + 3 * (size_t)e * n;
    const size_t off = two ? (size_t)b * n + (size_t)e * m : (size_t)e * n;
    int *st = start + (size_t)c * (kMaxCells + 1);

    float px[kSlabK], py[kSlabK], pz[kSlabK];
    auto load = [&](int c0) {  // the chunk's loads issued together (clamped: unconditional)
#pragma unroll
        for (int k = 0; k < kSlabK; ++k) {
            const int i = min(c0 + k * kSlabT + tid, np - 1);
            px[k] = pcm_ld(src + 3 * i);
            py[k] = pcm_ld(src + 3 * i + 1);
            pz[k] = pcm_ld(src + 3 * i + 2);
        }
    };

    // 1. the grid's box (every workgroup of the cloud computes the same
    // bits): over the whole cloud when it is one chunk -- loaded here, once,
    // for the box and passes 2 and 4 -- else over a strided sample of kSlabT
    // points.  Any box is exact: a point outside it is clamped into a boundary
    // cell, which only moves it farther inside the cell range than it is, and
    // the region proof holds for it as for every other point of that cell
    // (search kernel).  The non-finite flag needs every point: pass 2.
    const bool one = np <= kSlabK * kSlabT;
    float mn[3] = {PCM_INF, PCM_INF, PCM_INF}, mx[3] = {-PCM_INF, -PCM_INF, -PCM_INF}, bad = 0.f;
    if (one) {
        load(0);  // (clamped: padding repeats the last point, which the box holds anyway)
#pragma unroll
        for (int k = 0; k < kSlabK; ++k) {
            mn[0] = fminf(mn[0], px[k]);
            mn[1] = fminf(mn[1], py[k]);
            mn[2] = fminf(mn[2], pz[k]);
            mx[0] = fmaxf(mx[0], px[k]);
            mx[1] = fmaxf(mx[1], py[k]);
            mx[2] = fmaxf(mx[2], pz[k]);
        }
    } else {
        const int i = (int)(((long long)tid * np) / kSlabT);
        const float x = pcm_ld(src + 3 * i), y = pcm_ld(src + 3 * i + 1), z = pcm_ld(src + 3 * i + 2);
        mn[0] = mx[0] = x;
        mn[1] = mx[1] = y;
        mn[2] = mx[2] = z;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        mn[a] = wave_minf(mn[a]);
        mx[a] = wave_maxf(mx[a]);
    }
    if (lane == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            red[a][w] = mn[a];
            red[3 + a][w] = mx[a];
        }
    }
    for (int i = tid; i < scells; i += kSlabT) {
        hT[i] = 0;
        hQ[i] = 0;
    }
    if (tid == 0) sBelow = 0;
    __syncthreads();
    float lo[3], ext = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float l = PCM_INF, hgh = -PCM_INF;
        for (int i = 0; i < kW; ++i) {
            l = fminf(l, red[a][i]);
            hgh = fmaxf(hgh, red[3 + a][i]);
        }
        lo[a] = l;
        ext = fmaxf(ext, hgh - l);
    }
    float h = ext / (float)G, inv = 1.f / h;
    if (!(h > 0.f) || !(inv < 1e30f)) {  // one point, coincident points or a tiny extent: unit cells
        h = 1.f;
        inv = 1.f;
    }
    const int z0 = 4 * slab, kbase = slab * (G / 4) * (G / 4) * 64;  // first cell layer / query key of the slab

    // 2. the count of points in lower slabs (one ballot per point: only the
    // own slab's offset is needed) and the own slab's histograms
    int below = 0;
    // a cloud of one chunk stays in this thread's registers for pass 4, with
    // its own-slab points' cells (packed x | y << 5 | z << 10; -1: not own)
    int ck[kSlabK];
    for (int c0 = 0; c0 < np; c0 += kSlabK * kSlabT) {
        if (!one) load(c0);
#pragma unroll
        for (int k = 0; k < kSlabK; ++k) {
            const bool v = c0 + k * kSlabT + tid < np;
            bad = (!v || (pcm_finite(px[k]) && pcm_finite(py[k]) && pcm_finite(pz[k]))) ? bad : 1.f;
            const int ix = cell_axis(px[k], lo[0], inv, G), iy = cell_axis(py[k], lo[1], inv, G),
                      iz = cell_axis(pz[k], lo[2], inv, G);
            const int sl = iz >> 2;
            below += __popcll(__ballot(v && sl < slab));
            ck[k] = (v && sl == slab) ? (ix | (iy << 5) | (iz << 10)) : -1;
            if (v && sl == slab) {
                atomicAdd(&hT[((iz - z0) * G + iy) * G + ix], 1);
                atomicAdd(&hQ[cell_query_key(ix, iy, iz, G) - kbase], 1);
            }
        }
    }
    bad = wave_maxf(bad);
    if (lane == 0) {
        if (below) atomicAdd(&sBelow, below);
        red[6][w] = bad;  // read after the next barrier only
    }
    __syncthreads();
    const int soff = sBelow;
    for (int i = 0; i < kW; ++i) bad = fmaxf(bad, red[6][i]);

    // 3. exclusive scans of both histograms (wave w: rows [w R, w R + R) of
    // 64 bins, DPP scans with a carry; one barrier for the waves' offsets);
    // the row-major starts go to global for the search
    const int R = scells / kSlabT;  // 4 (G = 32) or 1 (G = 16)
    int tv[4], qv[4], tcarry = 0, qcarry = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (r < R) {
            const int i = (w * R + r) * 64 + lane;
            const int a1 = hT[i], a2 = hQ[i];
            const int i1 = wave_incl_scan(a1), i2 = wave_incl_scan(a2);
            tv[r] = tcarry + i1 - a1;
            qv[r] = qcarry + i2 - a2;
            tcarry += __builtin_amdgcn_readlane(i1, 63);
            qcarry += __builtin_amdgcn_readlane(i2, 63);
        }
    }
    if (lane == 0) {
        sw[0][w] = tcarry;
        sw[1][w] = qcarry;
    }
    __syncthreads();
    int toff = soff, qoff = soff;
    for (int i = 0; i < w; ++i) {
        toff += sw[0][i];
        qoff += sw[1][i];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (r < R) {
            const int i = (w * R + r) * 64 + lane;
            hT[i] = tv[r] + toff;  // cursors (absolute positions in the cloud's range)
            hQ[i] = qv[r] + qoff;
            st[z0 * G * G + i] = tv[r] + toff;
        }
    }
    if (slab == NS - 1 && tid == 0) st[G * G * G] = np;
    __syncthreads();

    // 4. the own slab's points into both copies
    if (one) {
#pragma unroll
        for (int k = 0; k < kSlabK; ++k) {
            if (ck[k] >= 0) {
                const int ix = ck[k] & 31, iy = (ck[k] >> 5) & 31, iz = ck[k] >> 10;
                const pcm_f4 v = pcm_f4{px[k], py[k], pz[k], __int_as_float(k * kSlabT + tid)};
                tpts[off + atomicAdd(&hT[((iz - z0) * G + iy) * G + ix], 1)] = v;
                qpts[off + atomicAdd(&hQ[cell_query_key(ix, iy, iz, G) - kbase], 1)] = v;
            }
        }
    }
    for (int c0 = 0; c0 < (one ? 0 : np); c0 += kSlabK * kSlabT) {
        load(c0);
#pragma unroll
        for (int k = 0; k < kSlabK; ++k) {
            const int i = c0 + k * kSlabT + tid;
            const int ix = cell_axis(px[k], lo[0], inv, G), iy = cell_axis(py[k], lo[1], inv, G),
                      iz = cell_axis(pz[k], lo[2], inv, G);
            if (i < np && (iz >> 2) == slab) {
                const pcm_f4 v = pcm_f4{px[k], py[k], pz[k], __int_as_float(i)};
                tpts[off + atomicAdd(&hT[((iz - z0) * G + iy) * G + ix], 1)] = v;
                qpts[off + atomicAdd(&hQ[cell_query_key(ix, iy, iz, G) - kbase], 1)] = v;
            }
        }
    }
    if (slab == 0 && tid == 0) {
        // margin (cells): the nearest neighbour of a uniform cloud of np points
        // lies beyond r with probability exp(-np 4/3 pi r^3); r = 1.43 np^-1/3
        // of the extent makes that ~e^-12
        const float mg = ceilf(1.43f * (float)G * cbrtf(1.f / (float)np));
        float *gg = geo + (size_t)c * kGeo;
        gg[0] = lo[0];
        gg[1] = lo[1];
        gg[2] = lo[2];
        gg[3] = h;
        gg[4] = inv;
        gg[5] = bad;
        gg[6] = (float)G;
        gg[7] = fminf(fmaxf(mg, 1.f), 4.f);
    }
}

// exact scan: every candidate's (distance, index) key
__device__ __forceinline__ void scan_exact(const pcm_f4 *cand, int lo, int hi, float qx, float qy, float qz,
                                           unsigned long long &best) {
    for (int j = lo; j < hi; ++j) {
        const unsigned long long key = nn_key(cand[j], qx, qy, qz);
        best = key < best ? key : best;
    }
}

// screened scan: distances only, min per 8-candidate chunk, the chunk that
// first reaches the window minimum remembered; then the exact keys of that
// chunk alone.  If a later chunk equals the window minimum (a tie across
// chunks: which index is lower is unknown) the window is scanned exactly.
// Same distances as scan_exact (same operations), so the same result.
template <bool kScreen>
__device__ __forceinline__ void scan_cands(const pcm_f4 *cand, int cnt, float qx, float qy, float qz,
                                           unsigned long long &best) {
    if (!kScreen) {
        int j = 0;
        for (; j + 4 <= cnt; j += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const unsigned long long key = nn_key(cand[j + u], qx, qy, qz);
                best = key < best ? key : best;
            }
        }
        scan_exact(cand, j, cnt, qx, qy, qz, best);
        return;
    }
    const int c8 = cnt & ~7;
    float wb = PCM_INF;
    int wc = -1;
    bool tie = false;
    for (int j = 0; j < c8; j += 8) {
        float d[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const pcm_f4 t = cand[j + u];
            d[u] = pcm_sqd(t.x - qx, t.y - qy, t.z - qz);
        }
        const float mc = __builtin_fminf(
            __builtin_fminf(__builtin_fminf(d[0], d[1]), __builtin_fminf(d[2], d[3])),
            __builtin_fminf(__builtin_fminf(d[4], d[5]), __builtin_fminf(d[6], d[7])));
        const bool lt = mc < wb;
        tie = lt ? false : (tie | (mc == wb));
        wc = lt ? j : wc;
        wb = lt ? mc : wb;
    }
    if (tie) scan_exact(cand, 0, c8, qx, qy, qz, best);
    else if (wc >= 0) scan_exact(cand, wc, wc + 8, qx, qy, qz, best);
    scan_exact(cand, c8, cnt, qx, qy, qz, best);
}

// filtered window scan (kFilter): the csrc/chamfer_filt.hip screen on the
// wave's window.  The raw candidates are transformed once per window into
// pair-interleaved (u, w) = (-2 t', |t'|^2), t' = t - c (c = the wave's query
// box centre): fu[2k] = {ux, ux', uy, uy'}, fu[2k + 1] = {uz, uz', w, w'} for
// candidates 2k, 2k + 1, so each lane evaluates a = |t'|^2 - 2 q'.t' for two
// candidates with three packed FMAs.  Per 8-candidate chunk the minimum; the
// best chunk and the best of the other chunks (v_med3); proof as
// chamfer_filt.hip step 2 (E = 16u (R + |q'|)^2, narrowed by the best
// chunk's distance); then the exact keys of the best chunk, or of the whole
// window when the proof fails (near-ties).
constexpr float kGridU16 = 9.5367431640625e-07f;  // 16 u = 2^-20

__device__ __forceinline__ void scan_filter(const pcm_f4 *__restrict__ cand, pcm_f4 *__restrict__ fu, int cnt,
                                            const float (&c)[3], float qx, float qy, float qz,
                                            unsigned long long &best) {
    const int lane = threadIdx.x & 63;
    const int npair = (cnt + 1) >> 1, c8 = (cnt + 7) & ~7;
    float rt2 = 0.f;
    for (int k = lane; k < (c8 >> 1); k += 64) {
        float u[2][3], wv[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = 2 * k + h;
            if (j < cnt) {
                const pcm_f4 t = cand[j];
                const float x = t.x - c[0], y = t.y - c[1], z = t.z - c[2];
                wv[h] = __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x));
                rt2 = fmaxf(rt2, wv[h]);
                u[h][0] = -2.f * x;
                u[h][1] = -2.f * y;
                u[h][2] = -2.f * z;
            } else {  // padding: a = +inf
                wv[h] = PCM_INF;
                u[h][0] = u[h][1] = u[h][2] = 0.f;
            }
        }
        fu[2 * k] = pcm_f4{u[0][0], u[1][0], u[0][1], u[1][1]};
        fu[2 * k + 1] = pcm_f4{u[0][2], u[1][2], wv[0], wv[1]};
    }
    (void)npair;
    const float rmax2 = wave_maxf(rt2);
    wave_lds_sync();
    const float qxp = qx - c[0], qyp = qy - c[1], qzp = qz - c[2];
    const pcm_f2 px = {qxp, qxp}, py = {qyp, qyp}, pz = {qzp, qzp};
    float fb = PCM_INF, fs = PCM_INF;
    int fc = 0;
    for (int j = 0; j < c8; j += 8) {
        float mn = PCM_INF;
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
            const pcm_f4 A = fu[j + 2 * pp], Bv = fu[j + 2 * pp + 1];
            const pcm_f2 a = __builtin_elementwise_fma(
                px, A.xy, __builtin_elementwise_fma(py, A.zw, __builtin_elementwise_fma(pz, Bv.xy, Bv.zw)));
            mn = __builtin_fminf(__builtin_fminf(mn, a.x), a.y);
        }
        fs = __builtin_amdgcn_fmed3f(mn, fb, fs);
        const bool lt = mn < fb;
        fc = lt ? j : fc;
        fb = lt ? mn : fb;
    }
    const float qn2 = __builtin_fmaf(qzp, qzp, __builtin_fmaf(qyp, qyp, qxp * qxp));
    const float sq = __builtin_amdgcn_sqrtf(qn2);
    const float rr = __builtin_amdgcn_sqrtf(rmax2) + sq;
    const float eR = kGridU16 * (rr * rr) * 1.001f;
    const float db = __builtin_fmaxf((fb + qn2) * 1.0001f + 2.f * eR, 0.f);
    const float rq = 2.f * sq + __builtin_amdgcn_sqrtf(db);
    const float e2 = 2.f * kGridU16 * __builtin_fminf(rr * rr, rq * rq) * 1.001f;
    const bool proven = (fs - fb) > e2;  // false for NaN / +inf - +inf
    if (proven) scan_exact(cand, fc, min(fc + 8, cnt), qx, qy, qz, best);
    else scan_exact(cand, 0, cnt, qx, qy, qz, best);
}

template <typename TIn, bool kScreen, int NT, bool kDma = true, bool kFilter = false>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void grid_nn_kernel(const pcm_f4 *__restrict__ tpts,
                                                       const pcm_f4 *__restrict__ qpts, const int *__restrict__ start,
                                                       const float *__restrict__ geo, const TIn *__restrict__ xyz1,
                                                       const TIn *__restrict__ xyz2, int b, int n, int m, int nb1,
                                                       int nb2, float *__restrict__ dist1, float *__restrict__ dist2,
                                                       int32_t *__restrict__ idx1, int32_t *__restrict__ idx2,
                                                       int *__restrict__ stats, unsigned *__restrict__ stamps) {
    constexpr int kW = NT / 64;
    constexpr int kCap = kFilter ? kWaveCap / 2 : kWaveCap;  // candidates per window
    __shared__ pcm_f4 cand_all[kW][kCap];
    __shared__ pcm_f4 fu_all[kFilter ? kW : 1][kFilter ? kCap : 1];
    __shared__ int spre_all[kW][65];
    __shared__ int sst_all[kW][64];

    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int per = nb1 + nb2;
    const long long blk_all = (long long)pcm_xcd_remap(blockIdx.x, gridDim.x) * kW + w;
    if (blk_all >= (long long)b * per) return;  // whole wave; no workgroup barriers below
    auto stamp = [&](int i) {
        if (stamps != nullptr && lane == 0) stamps[8 * blk_all + i] = (unsigned)__builtin_amdgcn_s_memrealtime();
    };
    stamp(0);
    const int e = (int)(blk_all / per), r = (int)(blk_all % per);
    const bool dir2 = r >= nb1;
    const int blk = dir2 ? r - nb1 : r;
    const int nq = dir2 ? m : n, nt = dir2 ? n : m;
    const int cq = dir2 ? b + e : e, ct = dir2 ? e : b + e;
    const size_t qoff = dir2 ? (size_t)b * n + (size_t)e * m : (size_t)e * n;
    const pcm_f4 *T = tpts + (dir2 ? (size_t)e * n : (size_t)b * n + (size_t)e * m);
    const int *Ts = start + (size_t)ct * (kMaxCells + 1);
    float *dout = dir2 ? dist2 + (size_t)e * m : dist1 + (size_t)e * n;
    int32_t *iout = dir2 ? idx2 + (size_t)e * m : idx1 + (size_t)e * n;
    const int q0 = blk * 64, qi = q0 + lane;
    const bool valid = qi < nq;
    const pcm_f4 q = qpts[qoff + (valid ? qi : q0)];
    const float *gt = geo + (size_t)ct * kGeo;

    if (geo[(size_t)cq * kGeo + 5] != 0.f || gt[5] != 0.f) {
        // non-finite coordinates in this element: the reference's tile scan
        if (valid) {
            const int oid = __float_as_int(q.w);
            const TIn *Qo = dir2 ? xyz2 + 3 * (size_t)e * m : xyz1 + 3 * (size_t)e * n;
            const TIn *To = dir2 ? xyz1 + 3 * (size_t)e * n : xyz2 + 3 * (size_t)e * m;
            float d;
            int k;
            pcm_ref_nn_scan(pcm_ld(Qo + 3 * (size_t)oid), pcm_ld(Qo + 3 * (size_t)oid + 1),
                            pcm_ld(Qo + 3 * (size_t)oid + 2), To, nt, d, k);
            dout[oid] = d;
            iout[oid] = k;
        }
        return;
    }

    pcm_f4 *cand = cand_all[w];
    pcm_f4 *fu = fu_all[kFilter ? w : 0];
    int *spre = spre_all[w], *sst = sst_all[w];
    stamp(1);
    const float lo[3] = {gt[0], gt[1], gt[2]}, h = gt[3], inv = gt[4];
    const int G = (int)gt[6], margin = (int)gt[7];
    const float qc[3] = {q.x, q.y, q.z};
    float cen[3];  // the filter's centre: midpoint of the wave's query box
#pragma unroll
    for (int a = 0; a < 3; ++a) cen[a] = 0.5f * (wave_minf(qc[a]) + wave_maxf(qc[a]));
    unsigned long long best = ~0ull;
    auto scan_window = [&](int cnt) {
        if constexpr (kFilter) scan_filter(cand, fu, cnt, cen, q.x, q.y, q.z, best);
        else scan_cands<kScreen>(cand, cnt, q.x, q.y, q.z, best);
    };
    bool pending = valid;
    int nround = 0, cand0 = 0, candall = 0;  // diagnostics (stats != nullptr)
    for (int round = 0; __ballot(pending) != 0; ++round) {
        const bool full = round >= 2;  // the last round gathers the whole grid
        const int mg = round == 0 ? margin : 3 * margin;
        // cell box of the pending queries, widened by mg cells
        int cl[3], ch[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float mn = wave_minf(pending ? qc[a] : PCM_INF), mx = wave_maxf(pending ? qc[a] : -PCM_INF);
            const float fl = fminf(fmaxf((mn - lo[a]) * inv, -2.f), (float)(G + 1));
            const float fh = fminf(fmaxf((mx - lo[a]) * inv, -2.f), (float)(G + 1));
            cl[a] = full ? 0 : min(max((int)floorf(fl) - mg, 0), G - 1);
            ch[a] = full ? G - 1 : min(max((int)floorf(fh) + mg, 0), G - 1);
        }
        const int ny = ch[1] - cl[1] + 1, nrows = ny * (ch[2] - cl[2] + 1);
        int filled = 0;
        for (int r0 = 0; r0 < nrows; r0 += 64) {  // 64 rows of cells (contiguous ranges) at a time
            const int row = r0 + lane;
            int cnt = 0, cs = 0;
            if (row < nrows) {
                const int base = ((cl[2] + row / ny) * G + cl[1] + row % ny) * G;
                cs = Ts[base + cl[0]];
                cnt = Ts[base + ch[0] + 1] - cs;
            }
            if (round == 0 && r0 == 0) stamp(2);
            const int inc = wave_incl_scan(cnt);
            const int tot = __builtin_amdgcn_readlane(inc, 63);  // SGPR, not an LDS permute
            candall += tot;
            cand0 += round == 0 ? tot : 0;
            spre[lane] = inc - cnt;
            sst[lane] = cs;
            if (lane == 63) spre[64] = inc;
            wave_lds_sync();
            for (int w0 = 0; w0 < tot;) {
                const int take = min(tot - w0, kCap - filled);
                // candidate copies global -> LDS by LDS-DMA (lane l of a batch
                // lands at slot base + l): every batch's loads in flight at once
                // the row of slot v: the last row whose prefix is <= v (it
                // holds v); the batches' searches interleaved (independent
                // LDS chains)
                constexpr int kB = kCap / 64;
                int v[kB], a[kB];
#pragma unroll
                for (int bt = 0; bt < kB; ++bt) {
                    v[bt] = w0 + bt * 64 + lane;
                    a[bt] = 0;
                }
#pragma unroll
                for (int step = 32; step > 0; step >>= 1) {
#pragma unroll
                    for (int bt = 0; bt < kB; ++bt) a[bt] = spre[a[bt] + step] <= v[bt] ? a[bt] + step : a[bt];
                }
                if constexpr (kDma) {
#pragma unroll
                    for (int bt = 0; bt < kB; ++bt) {
                        if (bt * 64 < take && bt * 64 + lane < take)
                            __builtin_amdgcn_global_load_lds((const void *)(T + sst[a[bt]] + (v[bt] - spre[a[bt]])),
                                                             (pcm_lds_void *)(cand + filled + bt * 64), 16, 0, 0);
                    }
                } else {  // through registers: all loads, then all LDS writes
                    pcm_f4 g[kB];
#pragma unroll
                    for (int bt = 0; bt < kB; ++bt)
                        if (bt * 64 < take && bt * 64 + lane < take) g[bt] = T[sst[a[bt]] + (v[bt] - spre[a[bt]])];
#pragma unroll
                    for (int bt = 0; bt < kB; ++bt)
                        if (bt * 64 < take && bt * 64 + lane < take) cand[filled + bt * 64 + lane] = g[bt];
                }
                filled += take;
                w0 += take;
                if (filled == kCap) {
                    wave_vm_sync();
                    scan_window(kCap);
                    wave_lds_sync();
                    filled = 0;
                }
            }
            wave_lds_sync();  // spre / sst are rewritten by the next 64 rows
        }
        wave_vm_sync();
        if (round == 0) stamp(3);
        scan_window(filled);
        wave_lds_sync();
        if (round == 0) stamp(4);

        // proof: every target outside the gathered cells is at least `gap`
        // away along some axis.  Cell boundaries carry the rounding of
        // (v - lo) * (1/h) (a few ulps of |lo| + G h), covered by `tol`; the
        // pinned distance of a point `gap` away is >= gap^2 (1 - 6u), covered
        // by the 2^-18 factor.
        float gap = PCM_INF;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float tol = 0x1p-18f * (fabsf(lo[a]) + (float)G * h + fabsf(qc[a]));
            if (cl[a] > 0) gap = fminf(gap, qc[a] - (lo[a] + (float)cl[a] * h) - tol);
            if (ch[a] < G - 1) gap = fminf(gap, (lo[a] + (float)(ch[a] + 1) * h) - qc[a] - tol);
        }
        const float bd = __uint_as_float((unsigned)(best >> 32));
        const bool ok = gap > 0.f && bd < gap * gap * (1.f - 0x1p-18f);
        pending = pending && !ok && !full;
        nround = round + 1;
    }
    if (stats != nullptr && lane == 0) {
        stats[4 * blk_all + 0] = nround;
        stats[4 * blk_all + 1] = cand0;
        stats[4 * blk_all + 2] = candall;
        stats[4 * blk_all + 3] = e * 2 + (dir2 ? 1 : 0);
    }
    if (valid) {
        const int oid = __float_as_int(q.w);
        dout[oid] = __uint_as_float((unsigned)(best >> 32));
        iout[oid] = (int32_t)(unsigned)best;
    }
    stamp(5);
    if (stamps != nullptr && lane == 0) {  // placement: HW_ID and XCC_ID registers
        stamps[8 * blk_all + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        stamps[8 * blk_all + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
}

inline size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

struct GridLayout {
    size_t tpts, qpts, start, geo, total;
};
inline GridLayout grid_layout(int b, int n, int m) {
    GridLayout L;
    const size_t pts = align256(16 * (size_t)b * ((size_t)n + m));
    L.tpts = 0;
    L.qpts = pts;
    L.start = 2 * pts;
    L.geo = L.start + align256(4 * (size_t)2 * b * (kMaxCells + 1));
    L.total = L.geo + align256(4 * (size_t)2 * b * kGeo);
    return L;
}

inline bool bad_dims(int b, int n, int m) { return b < 0 || n < 0 || m < 0; }

template <typename TIn>
int launch_grid(const TIn *xyz1, const TIn *xyz2, int b, int n, int m, float *dist1, float *dist2, int32_t *idx1,
                int32_t *idx2, void *workspace, size_t workspace_bytes, void *stream, bool screen = true,
                int *stats = nullptr, bool build = true, bool nn = true, bool small_wg = false,
                bool reg_gather = false, bool filter = true) {
    if (bad_dims(b, n, m)) return PCM_ERR_INVALID_ARG;
    if (b == 0 || (n == 0 && m == 0)) return PCM_OK;
    if ((n > 0 && (!xyz1 || !dist1 || !idx1)) || (m > 0 && (!xyz2 || !dist2 || !idx2)))
        return PCM_ERR_INVALID_ARG;
    const GridLayout L = grid_layout(b, n, m);
    if (!workspace || workspace_bytes < L.total || ((uintptr_t)workspace & 15)) return PCM_ERR_WORKSPACE;
    const int nb1 = m > 0 ? (n + 63) / 64 : 0;
    const int nb2 = n > 0 ? (m + 63) / 64 : 0;
    const long long waves = (long long)b * (nb1 + nb2);
    if (waves == 0) return PCM_OK;
    // threads per search workgroup: 16 waves (one workgroup per CU, fewer to
    // dispatch) when the waves fill the chip in one round, else 4 (finer
    // balance over several rounds; r04 grid_diag: config 5 45.5 vs 49.2 us,
    // B=4 N=M=65536 147 vs 127 us)
    {
        const long long full = (long long)(kNnT / 64) * pcm_device_cus();
        if (waves < full * 3 / 4 || waves > full) small_wg = true;
    }
    const int nt_wg = small_wg ? 256 : kNnT;
    const long long blocks = (waves + nt_wg / 64 - 1) / (nt_wg / 64);
    if (blocks > 0x7fffffffLL || 2LL * b > 0x7fffffffLL) return PCM_ERR_UNSUPPORTED;
    char *base = (char *)workspace;
    pcm_f4 *tpts = (pcm_f4 *)(base + L.tpts);
    pcm_f4 *qpts = (pcm_f4 *)(base + L.qpts);
    int *start = (int *)(base + L.start);
    float *geo = (float *)(base + L.geo);
    hipStream_t st = (hipStream_t)stream;
    // diagnostics layout: [waves][4] stats, then [waves][8] search stamps
    unsigned *sst = stats ? (unsigned *)(stats + 4 * waves) : nullptr;
    if (build)
        hipLaunchKernelGGL(grid_build_kernel<TIn>, dim3((unsigned)(2 * b * kSlabMax)), dim3(kSlabT), 0, st, xyz1,
                           xyz2, b, n, m, tpts, qpts, start, geo);
    // default: the filtered window scan (r04: config 5 search 42.4 us against
    // 45.5 screened-exact, 55.8 with the register gather)
    auto nnk = small_wg ? grid_nn_kernel<TIn, true, 256, true, true> : grid_nn_kernel<TIn, true, kNnT, true, true>;
    if (!filter) nnk = small_wg ? (screen ? grid_nn_kernel<TIn, true, 256> : grid_nn_kernel<TIn, false, 256>)
                                : (screen ? grid_nn_kernel<TIn, true, kNnT> : grid_nn_kernel<TIn, false, kNnT>);
    if (reg_gather) nnk = small_wg ? grid_nn_kernel<TIn, true, 256, false> : grid_nn_kernel<TIn, true, kNnT, false>;
    if (nn)
        hipLaunchKernelGGL(nnk, dim3((unsigned)blocks), dim3(nt_wg), 0, st, tpts, qpts, start, geo, xyz1, xyz2, b, n,
                           m, nb1, nb2, dist1, dist2, idx1, idx2, stats, sst);
    return pcm_launch_status();
}

// the dense forward costs ~1.6e-13 s per (b n m) pair beyond ~20 us; the grid
// ~25 us plus ~0.35 ns per point, but needs ~2k search waves to fill the chip
// (tools/ab_grid.py, r04: B=2 N=M=4096 dense 29 us / grid 52 us; B=32 N=M=4096
// 107 / 66 us; config 5 340 / 117 us)
inline bool grid_pays(int b, int n, int m) {
    return n >= kGridMinPoints && m >= kGridMinPoints && (double)b * n * m >= 268435456.0;
}

}  // namespace

// 0 when the problem takes the dense kernels (no workspace used)
extern "C" size_t pcm_chamfer_forward_ws_bytes(int b, int n, int m) {
    if (bad_dims(b, n, m) || !grid_pays(b, n, m)) return 0;
    return grid_layout(b, n, m).total;
}

// the grid path's workspace at any size (pcm_tune_chamfer_forward_grid)
extern "C" size_t pcm_tune_chamfer_forward_grid_ws_bytes(int b, int n, int m) {
    if (bad_dims(b, n, m)) return 0;
    return grid_layout(b, n, m).total;
}

extern "C" int pcm_chamfer_forward_ws(const float *xyz1, const float *xyz2, int b, int n, int m, float *dist1,
                                      float *dist2, int32_t *idx1, int32_t *idx2, void *workspace,
                                      size_t workspace_bytes, void *stream) {
    if (!grid_pays(b, n, m)) return pcm_chamfer_forward(xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, stream);
    return launch_grid(xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, workspace, workspace_bytes, stream);
}

extern "C" int pcm_chamfer_forward_ws_f16(const uint16_t *xyz1, const uint16_t *xyz2, int b, int n, int m,
                                          float *dist1, float *dist2, int32_t *idx1, int32_t *idx2, void *workspace,
                                          size_t workspace_bytes, void *stream) {
    if (!grid_pays(b, n, m)) return pcm_chamfer_forward_f16(xyz1, xyz2, b, n, m, dist1, dist2, idx1, idx2, stream);
    return launch_grid((const pcm_h *)xyz1, (const pcm_h *)xyz2, b, n, m, dist1, dist2, idx1, idx2, workspace,
                       workspace_bytes, stream);
}

// the grid path at any size (tests and A/B): mode bit 0 = binary16 clouds,
// bit 1 = exact scan of every candidate instead of the screened scan, bit 2 =
// the build kernel only, bit 3 = the search kernel only (on the workspace of a
// previous call with the same clouds), bit 4 = 256-thread search workgroups,
// bit 5 = candidate gather through registers instead of LDS-DMA (screened
// scan), bit 6 = the screened exact-distance scan instead of the filtered
// scan (the default); stats (nullable): per wave of the
// search, {rounds, candidates of round 0, candidates of all rounds,
// 2 * element + direction}, then s_memrealtime stamps: 8 per cloud of the
// build, 8 per search wave
extern "C" int pcm_tune_chamfer_forward_grid(int mode, const void *xyz1, const void *xyz2, int b, int n, int m,
                                             float *dist1, float *dist2, int32_t *idx1, int32_t *idx2,
                                             void *workspace, size_t workspace_bytes, void *stream, int *stats) {
    const bool screen = !(mode & 2), build = !(mode & 8), nn = !(mode & 4), small_wg = (mode & 16) != 0;
    const bool reg_gather = (mode & 32) != 0, filter = !(mode & 66);  // exact (2) or screened (64): no filter
    if (mode & 1)
        return launch_grid((const pcm_h *)xyz1, (const pcm_h *)xyz2, b, n, m, dist1, dist2, idx1, idx2, workspace,
                           workspace_bytes, stream, screen, stats, build, nn, small_wg, reg_gather, filter);
    return launch_grid((const float *)xyz1, (const float *)xyz2, b, n, m, dist1, dist2, idx1, idx2, workspace,
                       workspace_bytes, stream, screen, stats, build, nn, small_wg, reg_gather, filter);
}
