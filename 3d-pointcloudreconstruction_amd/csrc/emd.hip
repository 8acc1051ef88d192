// emd.hip -- auction-algorithm EMD for MI355X (gfx950, CDNA4).
//
// Replaces the reference's 7-launches-per-iteration host loop
// (metric/emd/emd_cuda.cu:256-269: clear, calc_unass_cnt, calc_unass_cnt_sum,
// calc_unass_idx, Bid, GetMax, Assign) by two launches for any `iters` and any
// n % 1024 == 0 (the reference's contract, emd_cuda.cu:236-249):
//
//  1. emd_seed_kernel (all CUs, one wave per point, target cloud staged in
//     LDS per workgroup): iteration 0's bids.  With every price 0 the bid value
//     v = (float)((3.0 - (double)sqrtf(d)) - 0.0) is a monotone non-increasing
//     function of the squared distance d, so the nearest candidates by d are
//     the top of the value list.  Each lane keeps its top-3 keys; the cache is
//     every lane top-2 entry above K* = max over lanes of the 3rd keys (ballot
//     compaction, <= kL entries), and every uncached object has v <= T = v(-K*).
//     If the cached second-best value exceeds T nothing outside the cache can
//     enter the top two, so the bid is exact; otherwise the point is flagged
//     for a full scan.  A cache entry is (object id, s = sqrtf(d)) packed in 8
//     bytes: s does not depend on prices.
//
//  2. emd_auction_kernel: one persistent MASTER workgroup per batch element
//     runs every auction iteration in-kernel with workgroup barriers only.  Its
//     state (assignment, owner, price, max increment, claim key, bids, the two
//     bidder lists, the miss list) lives in LDS for n <= 2048 and in the
//     workspace (L2) for larger n.  An unassigned point re-bids from its cache
//     at CURRENT prices (two double subtractions per entry, G lanes per point,
//     DPP row reductions): prices only rise, so uncached values stay <= T and
//     the same proof applies.  Points whose cache cannot prove the top two get
//     a full scan: selection on an fp32 approximation with a proven error
//     bound, exact values of the chosen entries, cache rebuilt (exact scan as
//     fallback).  At n = 1024 a miss first tries the seed's reserve (every
//     object within a radius ~8x the cache's) before a full scan.  Few
//     bidders (<= 16) run as tail mode (each bid an exact scan split over
//     16 / bidders waves), one bidder as chain mode (bid, resolve, assign of
//     the evicted owner, two barriers per step).
//
//     HELPER workgroups (the rest of the grid, up to 31 per batch element, on
//     the master's XCD where the dispatcher allows) take the full scans of
//     heavy iterations: the master publishes the miss list and a price
//     snapshot; items are split statically (groups of 16 consecutive items
//     round-robin over the master and the helpers, one item per wave), so no
//     claim atomic sits on anyone's critical path.  A helper writes the
//     rebuilt cache and the bid write-through (sc1) and raises a per-item done
//     word; the master polls those words (bounded), then places the bids.  An
//     item whose done word does not arrive in time is scanned by the master
//     itself, so the result never depends on how many helpers are resident.
//     (MI355X_MICROARCH.md, inter-workgroup visibility, row 1: sc1 stores,
//     s_waitcnt vmcnt(0), sc1 flag; sc1 polls and sc1 loads.)
//
// Per iteration: bids -> barrier -> [full scans -> barrier] -> claim ->
// barrier -> assign (+ next bidder list) -> barrier.  Claims carry the
// iteration in their key ((~it) << 32 | j with atomicMin), so no reset pass.
//
// The cache only skips evaluations that provably cannot change the bid, so
// the results are identical to scanning every object every iteration (the
// oracle does exactly that).  Tie rules: argbest = lowest index among equal
// best values (the reference's strict '>' scan, emd_cuda.cu:147); `better` is
// the second largest value of the multiset; GetMax's 1e-6 window is evaluated
// in double exactly as emd_cuda.cu:188 and the LOWEST qualifying point index
// wins (the reference lets a racing writer win); max increments use an
// order-preserving int encoding + atomicMax (the reference's CAS loop,
// emd_cuda.cu:10-20).  Non-finite inputs are outside the reference's
// contract (coordinates in [0, 1], emd_module.py:9).
#include "pcm_common.h"
#include "pcm_internal.h"

namespace {

constexpr int kL = 64;               // cache slots per point (unused slots: id -1)
constexpr int kSelectSteps = 8;      // bisection steps when > kL entries clear K3
constexpr int kSectionSteps = 4;     // quarter-section steps of the reserve thresholds (1/256 of the range)
#ifndef PCM_SEED_THREADS
#define PCM_SEED_THREADS 256
#endif
constexpr int kSeedThreads = PCM_SEED_THREADS;  // 4 waves
constexpr int kSeedPtsPerWave = 1;   // 4 points per seed workgroup (2: seed 2.2 us slower at config 3, 4: 3.9 us, 8: 15 us)
constexpr int kSeedPts = kSeedThreads / 64 * kSeedPtsPerWave;
constexpr int kEmdThreads = 1024;    // auction workgroup (16 waves)
constexpr int kWaves = kEmdThreads / 64;
constexpr int kLdsStateMaxN = 2048;  // master state in LDS up to here (48 B x n)
constexpr int kStageMaxN = 8192;     // target cloud copied to LDS up to here (12 B x n)
constexpr int kHelperMaxN = 32768;   // helpers keep a price snapshot in LDS (4 B x n)
constexpr int kMaxHelpers = 31;
constexpr int kBoardWords = 32;      // per batch element: gen, quit, jn, err (128-B line each group)
constexpr int kSpinLimit = 1 << 22;  // bounded polls (sticky error word on timeout)
constexpr int kStagePN = 1024;          // the n of the LDS-state, staged-bidder auction form
constexpr int kDefaultOffloadMin = 24;  // misses above which an iteration is offloaded
constexpr int kDefaultTailMax = 16;     // bidders at or below which an iteration runs in tail mode
#ifndef PCM_CHAIN_W
#define PCM_CHAIN_W 16
#endif
constexpr int kChainW = PCM_CHAIN_W;    // waves a chain-mode bid is split over
constexpr int kDefaultWsplit = 1;       // most waves one miss's scan is split over (2, 4: measured slower at config 3 and the training call)
// Reserve (n == kStagePN): every object closer than a radius, built by the
// seed at zero prices, up to kR entries of {object id, d}.  Radius^2 starts at
// kResGrow x the cache bound's d (about 4^1.5 = 8x the cache's objects in a
// locally uniform cloud) and shrinks by kResShrink until kR fit.  The
// workspace keeps only the 16-bit object ids (n = 1024): the reserve bid
// recomputes d from the LDS-staged clouds, the same pinned arithmetic.
constexpr int kR = 256;
constexpr float kResGrow = 6.f, kResShrink = 0.85f;
#ifndef PCM_RES_FILL
#define PCM_RES_FILL 0.8f
#endif
constexpr float kResFill = PCM_RES_FILL * kR;  // reserve size aimed at by the first shrink
constexpr int kResTries = 16;           // 6 * 0.85^11 < 1: the radius reaches dK (<= 128 objects inside)

typedef unsigned long long centry;   // low 32 bits: object id (-1 unused), high 32: s bits
typedef unsigned long long ckey;     // claim key: (~it) << 32 | point

__device__ __forceinline__ centry cpack(int id, float s) {
    return (unsigned)id | ((centry)__float_as_uint(s) << 32);
}

template <typename T>
__device__ __forceinline__ T ld_sc1(const T *p) {
    return __hip_atomic_load(const_cast<T *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_sc1(T *p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <bool kSc1>
__device__ __forceinline__ void st_entry(centry *p, centry v) {
    if constexpr (kSc1) st_sc1(p, v); else *p = v;
}
template <bool kSc1>
__device__ __forceinline__ void st_float(float *p, float v) {
    if constexpr (kSc1) st_sc1(p, v); else *p = v;
}

__device__ __forceinline__ int f2key(float f) {
    const int i = __float_as_int(f);
    return i ^ ((i >> 31) & 0x7fffffff);  // order-preserving for non-NaN floats
}
__device__ __forceinline__ float key2f(int k) {
    return __int_as_float(k ^ ((k >> 31) & 0x7fffffff));
}

// emd_cuda.cu:142-146: x2 = xyz2 - xyz1 ...; v = 3.0 - sqrtf(d) - price in double
__device__ __forceinline__ float sqd_to(float x1, float y1, float z1, const float *q) {
    return pcm_sqd(q[0] - x1, q[1] - y1, q[2] - z1);
}
__device__ __forceinline__ float value_from_s(float s, float price) {
    const double v = (3.0 - (double)s) - (double)price;
    return (float)v;
}
__device__ __forceinline__ float value_of(float d, float price) {
    return value_from_s(__builtin_sqrtf(d), price);  // correctly rounded sqrtf
}

// ---- DPP cross-lane steps (VALU operand modifiers: no LDS crossbar round
// trip).  Hillis-Steele: row_shr 1,2,4,8 leaves each 16-lane row's result in
// its lane 15; row_bcast 15 and 31 then carry it across rows so lane 63 holds
// the wave's result.

// full-wave reductions: result returned wave-uniform (read from lane 63).
// Each Hillis-Steele step is ONE v_{max,min}_i32_dpp: a lane the pattern
// does not feed is not written (no bound_ctrl), so it keeps its own value --
// an idempotent no-op.  Written as inline asm: through update_dpp + fmaxf
// hipcc emitted a mov_dpp, a canonicalising max and the max for every step.
// s_nop 1 before each step: a DPP read of a VGPR the previous VALU
// instruction wrote needs two wait states (asm is not hazard-checked).
#define PCM_WAVE_RED_STEPS(OP)                                                   \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"   \
    "s_nop 1\n\t" OP " %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
__device__ __forceinline__ int wave_max_i(int v) {
    asm volatile(PCM_WAVE_RED_STEPS("v_max_i32_dpp") : "+v"(v));
    return __builtin_amdgcn_readlane(v, 63);
}
// max of the wave's finite / -inf values (a NaN counts as -inf, as fmaxf
// skips it), through the order-preserving int key
__device__ __forceinline__ float wave_max(float v) {
    return key2f(wave_max_i(f2key(v == v ? v : -PCM_INF)));
}

// ===========================================================================
// Candidate scan + cache selection by ONE wave (64 lanes) for one point.
//
// Selection (no sorting, no extraction rounds): with key = "larger is better,
// lower object index on ties", each lane keeps its top-2 (key, k, d) and its
// 3rd-best key.  Cache = every lane-top-2 entry strictly above K3 = max over
// lanes of the 3rd-best keys: every other object lies at or below K3 -- it is
// either outside its lane's top-2 (<= that lane's 3rd <= K3) or a top-2 entry
// not above K3.  If more than kL qualify, the threshold is raised by
// bisection between K3 and the largest key until at most kL lane-top-2
// entries lie above it; the bound then stays exact for every uncached key.
// ===========================================================================
struct LaneTop {
    float a1, a2, a3;  // the lane's three largest keys (multiset order)
    int q1, q2;        // object ids of the top-2
};

__device__ __forceinline__ void lane_top_init(LaneTop &t) {
    t.a1 = t.a2 = t.a3 = -PCM_INF;
    t.q1 = t.q2 = 0x7fffffff;
}
// Insertion into a sorted triple with v_med3: a1' = max(a1, key),
// a2' = med3(a1, a2, key), a3' = med3(a2, a3, key).  Ids follow with strict
// '>' while k ascends, so equal keys keep the lower index.  The id selects
// are spelled out as v_cmp/v_cndmask in one asm block: written as ternaries,
// hipcc turns them into exec-mask branches inside the scan loop.  gfx950
// needs two wait states between a VALU SGPR write and a v_cndmask reading it
// as the lane mask (s_nop 1).
__device__ __forceinline__ void lane_top_push(LaneTop &t, float key, int k) {
    unsigned long long c1, c2;
    int tmp;
    asm("v_cmp_gt_f32_e64 %[c1], %[key], %[a1]\n\t"
        "v_cmp_gt_f32_e64 %[c2], %[key], %[a2]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[tmp], %[k], %[q1], %[c1]\n\t"   // c1 ? q1 : k
        "v_cndmask_b32_e64 %[q2], %[q2], %[tmp], %[c2]\n\t"  // c2 ? tmp : q2 (c1 implies c2)
        "v_cndmask_b32_e64 %[q1], %[q1], %[k], %[c1]"         // c1 ? k : q1
        : [q1] "+v"(t.q1), [q2] "+v"(t.q2), [tmp] "=&v"(tmp), [c1] "=&s"(c1), [c2] "=&s"(c2)
        : [key] "v"(key), [a1] "v"(t.a1), [a2] "v"(t.a2), [k] "v"(k));
    t.a3 = __builtin_amdgcn_fmed3f(t.a2, t.a3, key);
    t.a2 = __builtin_amdgcn_fmed3f(t.a1, t.a2, key);
    t.a1 = __builtin_amdgcn_fmed3f(t.a1, key, 3.4028235e38f);  // max (keys are finite)
}
// Merge of another lane top over a LATER (higher-index) object range into t:
// the result is the lane top of the union scanned in ascending order.
__device__ __forceinline__ void lane_top_merge(LaneTop &t, float o1, int r1, float o2, int r2, float o3) {
    lane_top_push(t, o1, r1);
    lane_top_push(t, o2, r2);
    t.a3 = __builtin_amdgcn_fmed3f(t.a2, t.a3, o3);  // o3 <= o2 <= a2 already
}

// squared distance of a lane's entry (recomputed in the pinned order, so it
// is bit-identical to the value the scan used)
__device__ __forceinline__ float entry_d(float x1, float y1, float z1, const float *Qc, int n, int q) {
    return (unsigned)q < (unsigned)n ? sqd_to(x1, y1, z1, Qc + 3 * (size_t)q) : 0.f;
}

// picks the cache entries; writes (id, s = sqrtf(d)) of the chosen entries
// into cache[0..kL) (unused slots: id -1).  Returns K* (every uncached key
// <= K*) or +inf when nothing could be cached.  s1/s2: this lane's entries
// chosen; d1/d2: their squared distances.
template <bool kSc1>
__device__ __forceinline__ float select_cache(const LaneTop &t, float d1, float d2, centry *__restrict__ cache,
                                              bool &s1, bool &s2, int n) {
    const int lane = threadIdx.x & 63;
    float Kstar = wave_max(t.a3);
    s1 = t.a1 > Kstar;
    s2 = t.a2 > Kstar;
    unsigned long long m1 = __ballot(s1), m2 = __ballot(s2);
    int cnt = __popcll(m1) + __popcll(m2);
    if (cnt > kL) {  // wave-uniform: raise the threshold by bisection
        // invariant: count(> lo) > kL >= count(> hi); every uncached key is
        // <= max(K3, hi) = hi, so hi is a valid bound at every step
        float lo = Kstar, hi = wave_max(t.a1);
#pragma unroll 1
        for (int step = 0; step < kSelectSteps; ++step) {
            const float mid = lo + 0.5f * (hi - lo);
            const int c = __popcll(__ballot(t.a1 > mid)) + __popcll(__ballot(t.a2 > mid));
            if (c > kL) lo = mid; else hi = mid;
        }
        Kstar = hi;
        s1 = t.a1 > Kstar;
        s2 = t.a2 > Kstar;
        m1 = __ballot(s1);
        m2 = __ballot(s2);
        cnt = __popcll(m1) + __popcll(m2);
    }
    const unsigned long long below = (1ull << lane) - 1ull;
    if (lane < kL && lane >= cnt) st_entry<kSc1>(cache + lane, cpack(n, 0.f));  // unused slots: the sentinel
    if (s1) st_entry<kSc1>(cache + __popcll(m1 & below), cpack(t.q1, __builtin_sqrtf(d1)));
    if (s2) st_entry<kSc1>(cache + __popcll(m1) + __popcll(m2 & below), cpack(t.q2, __builtin_sqrtf(d2)));
    return Kstar;
}

__device__ __forceinline__ int wave_min_i(int v) {
    asm volatile(PCM_WAVE_RED_STEPS("v_min_i32_dpp") : "+v"(v));
    return __builtin_amdgcn_readlane(v, 63);
}

// exact (best, argbest, better) over the wave: each lane offers up to two
// (value, id) entries; result wave-uniform.  Three single-instruction DPP
// reductions instead of a top-2 merge per step: best = max, argbest = the
// lowest id among the entries equal to best, better = best again when two
// entries tie at best, else the max of the rest (the multiset's second).
__device__ __forceinline__ void wave_top2(float v1, int k1, float v2, int k2, float &b1, int &kb, float &b2) {
    b1 = wave_max(fmaxf(v1, v2));
    const bool e1 = v1 == b1, e2 = v2 == b1;
    kb = wave_min_i(min(e1 ? k1 : 0x7fffffff, e2 ? k2 : 0x7fffffff));
    const int ties = __popcll(__ballot(e1)) + __popcll(__ballot(e2));
    b2 = ties >= 2 ? b1 : wave_max(fmaxf(e1 ? -PCM_INF : v1, e2 ? -PCM_INF : v2));
}

// ---- all-reduce inside aligned groups of G lanes (G = 4, 8, 16) with
// butterfly DPP permutations: every lane of the group gets the result.  Every
// lane has a source lane in these patterns, so the permuted copy needs no
// "old" value (mov_dpp, bound_ctrl) and hipcc folds each step into ONE
// v_{max,min,add}_i32_dpp; float maxima go through the order-preserving int
// key (fmaxf would add a canonicalising v_max per step).
constexpr int kQuadXor1 = 0xB1, kQuadXor2 = 0x4E, kRowHalfMirror = 0x141, kRowMirror = 0x140;
template <int CTRL>
__device__ __forceinline__ int dpp_all(int x) {
    return __builtin_amdgcn_mov_dpp(x, CTRL, 0xf, 0xf, true);
}
template <int G>
__device__ __forceinline__ int group_max_i(int v) {
    v = max(v, dpp_all<kQuadXor1>(v));
    v = max(v, dpp_all<kQuadXor2>(v));
    if constexpr (G >= 8) v = max(v, dpp_all<kRowHalfMirror>(v));
    if constexpr (G >= 16) v = max(v, dpp_all<kRowMirror>(v));
    return v;
}
// max over the group of finite / -inf values (a NaN counts as -inf, as fmaxf
// skips it)
template <int G>
__device__ __forceinline__ float group_max(float v) {
    return key2f(group_max_i<G>(f2key(v == v ? v : -PCM_INF)));
}
template <int G>
__device__ __forceinline__ int group_min_i(int v) {
    v = min(v, dpp_all<kQuadXor1>(v));
    v = min(v, dpp_all<kQuadXor2>(v));
    if constexpr (G >= 8) v = min(v, dpp_all<kRowHalfMirror>(v));
    if constexpr (G >= 16) v = min(v, dpp_all<kRowMirror>(v));
    return v;
}
template <int G>
__device__ __forceinline__ int group_add_i(int v) {
    v += dpp_all<kQuadXor1>(v);
    v += dpp_all<kQuadXor2>(v);
    if constexpr (G >= 8) v += dpp_all<kRowHalfMirror>(v);
    if constexpr (G >= 16) v += dpp_all<kRowMirror>(v);
    return v;
}

// ---- seed: key = -d (every price is 0: the bid value is monotone
// non-increasing in d).  T = v(-K*) bounds every uncached value.  The bid is
// exact whenever b2 > T (caller checks).
__device__ __forceinline__ void scan_seed(float x1, float y1, float z1, const float *Qc, int n,
                                          centry *__restrict__ cache, float &b1, int &kb, float &b2, float &T) {
    const int lane = threadIdx.x & 63;
    LaneTop t;
    lane_top_init(t);
    for (int k0 = lane; k0 < n; k0 += 4 * 64) {  // n % 1024 == 0 (launch_emd)
        float key[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) key[r] = -sqd_to(x1, y1, z1, Qc + 3 * (size_t)(k0 + 64 * r));
#pragma unroll
        for (int r = 0; r < 4; ++r) lane_top_push(t, key[r], k0 + 64 * r);
    }
    bool s1, s2;
    const float d1 = -t.a1, d2 = -t.a2;  // negation is exact
    const float Kstar = select_cache<false>(t, d1, d2, cache, s1, s2, n);
    T = Kstar == PCM_INF ? PCM_INF : value_of(-Kstar, 0.f);
    wave_top2(s1 ? value_of(d1, 0.f) : -PCM_INF, s1 ? t.q1 : 0x7fffffff,
              s2 ? value_of(d2, 0.f) : -PCM_INF, s2 ? t.q2 : 0x7fffffff, b1, kb, b2);
}

// ---- seed at n = kStagePN, one wave per point, the 16 squared distances per
// lane kept in registers.
//  1. dK = min over lanes of the lane's 3rd smallest d: every lane holds at
//     most 2 objects closer than dK (<= 128 in all).
//  2. RESERVE: every object with d < th, th starting at kResGrow * dK and
//     shrinking towards dK until at most kR qualify.  Every other object has
//     d >= th, so at ANY prices (p >= 0, only rising) its value is <=
//     rT = value_of(th, 0): the cache's proof against a bound ~8x further out.
//     Entries {id, d bits} go to R (global) and to this wave's LDS slot sR.
//  3. CACHE: the exact nearest kL of the reserve (threshold K on d by
//     bisection over the compacted entries, two per lane), bound
//     T = value_of(K, 0); the iteration-0 bid is their top two.
// rn = 0: no reserve (degenerate or non-finite cloud; the cache is then the
// lane-top form of scan_seed).
__device__ __forceinline__ float wave_min(float v) { return -wave_max(-v); }

__device__ __forceinline__ void scan_seed_res(float x1, float y1, float z1, const float *Qc, centry *__restrict__ cache,
                                              uint16_t *__restrict__ R, centry *sR, float &b1, int &kb, float &b2,
                                              float &T, int &rn, float &rT) {
    constexpr int n = kStagePN, S = n / 256;
    const int lane = threadIdx.x & 63;
    float dd[4 * S];
    float m1 = PCM_INF, m2 = PCM_INF, m3 = PCM_INF;  // the lane's 3 smallest d
#pragma unroll
    for (int i = 0; i < 4 * S; ++i) {
        dd[i] = sqd_to(x1, y1, z1, Qc + 3 * (size_t)(lane + 256 * (i / 4) + 64 * (i % 4)));
        m3 = __builtin_amdgcn_fmed3f(m2, m3, dd[i]);
        m2 = __builtin_amdgcn_fmed3f(m1, m2, dd[i]);
        m1 = fminf(m1, dd[i]);
    }
    const float dK = wave_min(m3);
    rn = 0;
    rT = PCM_INF;
    float th = kResGrow * dK;
    int cnt = 0;
    const bool ok = dK > 0.f && dK < PCM_INF;
    if (ok) {
#pragma unroll 1
        for (int tr = 0; tr < kResTries; ++tr) {
            cnt = 0;
#pragma unroll
            for (int i = 0; i < 4 * S; ++i) cnt += __popcll(__ballot(dd[i] < th));
            if (cnt <= kR) break;
            // each count is 16 ballot -> s_bcnt1 round trips (most of the
            // seed's SALU): the first miss jumps to the radius a locally
            // uniform cloud (count ~ th^1.5) predicts for kResFill objects,
            // later ones shrink geometrically (any th >= dK is valid: only
            // the reserve's size, never a result, depends on it)
            const float f = tr == 0 ? fminf(kResShrink, __builtin_amdgcn_exp2f(
                                                            (2.f / 3.f) * __builtin_amdgcn_logf(kResFill / (float)cnt)))
                                    : kResShrink;
            th = fmaxf(dK, f * th);
        }
    }
    if (!ok || cnt > kR) {  // no reserve: the lane-top cache of scan_seed
        scan_seed(x1, y1, z1, Qc, n, cache, b1, kb, b2, T);
        return;
    }
    const unsigned long long below = (1ull << lane) - 1ull;
    int pos = 0;
#pragma unroll
    for (int i = 0; i < 4 * S; ++i) {
        const bool in = dd[i] < th;
        const unsigned long long m = __ballot(in);
        if (in) {
            const centry e = cpack(lane + 256 * (i / 4) + 64 * (i % 4), dd[i]);
            R[pos + __popcll(m & below)] = (uint16_t)(lane + 256 * (i / 4) + 64 * (i % 4));
            sR[pos + __popcll(m & below)] = e;
        }
        pos += __popcll(m);
    }
    rn = cnt;
    rT = value_of(th, 0.f);
    // sR is written by this wave's lanes and read across them: a wave's LDS
    // accesses complete in order; the asm keeps the compiler from moving the
    // reads above the writes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    constexpr int RPL = kR / 64;
    float d[RPL];
    int k[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        const bool h = lane + 64 * i < rn;
        const centry e = sR[lane + 64 * i];
        d[i] = h ? __uint_as_float((unsigned)(e >> 32)) : PCM_INF;
        k[i] = (int)(unsigned)e;
    }
    auto count_below = [&](float t) {
        int c = 0;
#pragma unroll
        for (int i = 0; i < RPL; ++i) c += __popcll(__ballot(d[i] < t));
        return c;
    };
    float K = th;  // rn <= kL: the whole reserve
    if (rn > kL) {
        // invariant: count(d < lo) <= kL < count(d < hi); quarter sections
        // (three independent counts per step: a quarter of the dependent
        // VALU -> SALU round trips of halving)
        float lo = 0.f, hi = th;
#pragma unroll 1
        for (int step = 0; step < kSectionSteps; ++step) {
            const float w = 0.25f * (hi - lo);
            const float t1 = lo + w, t2 = lo + 2.f * w, t3 = lo + 3.f * w;
            const int c1 = count_below(t1), c2 = count_below(t2), c3 = count_below(t3);
            if (c3 <= kL) lo = t3;
            else if (c2 <= kL) { lo = t2; hi = t3; }
            else if (c1 <= kL) { lo = t1; hi = t2; }
            else hi = t1;
        }
        K = lo;
    }
    float lmax = -PCM_INF;
    float v[RPL];
    int cpos = 0;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        const bool c = d[i] < K;
        const unsigned long long m = __ballot(c);
        if (c) cache[cpos + __popcll(m & below)] = cpack(k[i], __builtin_sqrtf(d[i]));
        cpos += __popcll(m);
        v[i] = c ? value_of(d[i], 0.f) : -PCM_INF;
        lmax = fmaxf(lmax, v[i]);
    }
    if (lane < kL && lane >= cpos) cache[lane] = cpack(n, 0.f);
    T = value_of(K, 0.f);
    b1 = wave_max(lmax);
    int lk = 0x7fffffff, lc = 0;
    float lrest = -PCM_INF;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        const bool eq = v[i] == b1;
        lk = eq ? min(lk, k[i]) : lk;
        lc += __popcll(__ballot(eq));
        lrest = eq ? lrest : fmaxf(lrest, v[i]);
    }
    kb = wave_min_i(lk);
    b2 = lc >= 2 ? b1 : wave_max(lrest);
}


// ---- reserve bid (one wave): the exact top-2 over the rn reserve entries at
// current prices, proven when its second best exceeds rT.  Then the cache is
// rebuilt from the reserve: the <= kL largest values (threshold K by bisection
// as in select_cache), bound T = max(rT, K).  Returns false when not proven.
// Results by value; the master runs it in a loop of its own (B2a), apart
// from the full scans (B2b): inlined into the same loop body it pushed the
// kernel past 128 VGPRs into scratch.
typedef const __attribute__((address_space(3))) float *lds_cfp;
struct ResBid {
    float b1, b2, T;
    int kb, ok;
};
template <typename Stamp>
__device__ __forceinline__ ResBid reserve_bid(const uint16_t *__restrict__ R, int rn, float rT, lds_cfp price,
                                           float x1, float y1, float z1, const float *Qc, centry *__restrict__ cache,
                                           Stamp stamp) {
    constexpr int RPL = kR / 64;  // reserve entries per lane: lane + 64 i
    const int lane = threadIdx.x & 63;
    ResBid r;
    r.ok = 0;
    r.T = PCM_INF;
    bool h[RPL];
    int k[RPL];
    float sv[RPL], v[RPL];
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        h[i] = lane + 64 * i < rn;
        k[i] = h[i] ? (int)R[lane + 64 * i] : 0;
    }
    unsigned dep = 0;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        sv[i] = __builtin_sqrtf(sqd_to(x1, y1, z1, Qc + 3 * (size_t)k[i]));  // as the seed's d, pinned order
        dep += (unsigned)k[i];
    }
    stamp(6, dep);
    float lmax = -PCM_INF, lmin = PCM_INF;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        v[i] = h[i] ? value_from_s(sv[i], price[k[i]]) : -PCM_INF;
        lmax = fmaxf(lmax, v[i]);
        lmin = h[i] ? fminf(lmin, v[i]) : lmin;
    }
    // exact top-2 (lowest id at the best; better = best on a tie)
    const float b1 = wave_max(lmax);
    int lk = 0x7fffffff, lc = 0;
    float lrest = -PCM_INF;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        const bool eq = v[i] == b1;
        lk = eq ? min(lk, k[i]) : lk;
        lc += __popcll(__ballot(eq));
        lrest = eq ? lrest : fmaxf(lrest, v[i]);
    }
    r.b1 = b1;
    r.kb = wave_min_i(lk);
    r.b2 = lc >= 2 ? b1 : wave_max(lrest);
    stamp(7, 0u);
    if (!(r.b2 > rT)) return r;
    auto count_above = [&](float t) {
        int c = 0;
#pragma unroll
        for (int i = 0; i < RPL; ++i) c += __popcll(__ballot(v[i] > t));
        return c;
    };
    float K = -PCM_INF;
    if (rn > kL) {
        float lo = wave_min(lmin);
        if (count_above(lo) <= kL) {
            K = lo;  // ties at the minimum: everything above it fits
        } else {
            // invariant: count(> lo) > kL >= count(> hi); quarter sections
            float hi = b1;
#pragma unroll 1
            for (int step = 0; step < kSectionSteps; ++step) {
                const float w = 0.25f * (hi - lo);
                const float t1 = lo + w, t2 = lo + 2.f * w, t3 = lo + 3.f * w;
                const int c1 = count_above(t1), c2 = count_above(t2), c3 = count_above(t3);
                if (c1 <= kL) hi = t1;
                else if (c2 <= kL) { lo = t1; hi = t2; }
                else if (c3 <= kL) { lo = t2; hi = t3; }
                else lo = t3;
            }
            K = hi;
        }
    }
    stamp(11, 0u);
    const unsigned long long below = (1ull << lane) - 1ull;
    int pos = 0;
#pragma unroll
    for (int i = 0; i < RPL; ++i) {
        const bool c = v[i] > K;
        const unsigned long long m = __ballot(c);
        if (c) cache[pos + __popcll(m & below)] = cpack(k[i], sv[i]);
        pos += __popcll(m);
    }
    if (lane < kL && lane >= pos) cache[lane] = cpack(kStagePN, 0.f);  // the reserve form: n == kStagePN
    r.T = fmaxf(rT, K);
    r.ok = 1;
    return r;
}

// ---- auction full scan, exact: key = the exact bid value.  Always exact
// bid (the lanes' top-2 hold the global top-2); T = K*.  Out of line (the
// rare fallback), so its results come back BY VALUE: through reference
// parameters every caller kept b1/kb/b2/T in scratch memory, a store and a
// dependent reload on the fast path of every full scan.
struct ScanBid {
    float b1, b2, T;
    int kb;
};
template <bool kSc1>
__device__ __noinline__ ScanBid scan_exact_bid(float x1, float y1, float z1, const float *Qc, const float *price,
                                               int n, centry *__restrict__ cache) {
    const int lane = threadIdx.x & 63;
    LaneTop t;
    lane_top_init(t);
    for (int k0 = lane; k0 < n; k0 += 4 * 64) {
        float key[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = k0 + 64 * r;
            key[r] = value_of(sqd_to(x1, y1, z1, Qc + 3 * (size_t)k), price[k]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) lane_top_push(t, key[r], k0 + 64 * r);
    }
    bool s1, s2;
    ScanBid r;
    r.T = select_cache<kSc1>(t, entry_d(x1, y1, z1, Qc, n, t.q1), entry_d(x1, y1, z1, Qc, n, t.q2), cache, s1, s2,
                             n);
    wave_top2(t.a1, t.q1, t.a2, t.q2, r.b1, r.kb, r.b2);
    return r;
}
template <bool kSc1>
__device__ __forceinline__ void scan_exact(float x1, float y1, float z1, const float *Qc, const float *price, int n,
                                           centry *__restrict__ cache, float &b1, int &kb, float &b2, float &T) {
    const ScanBid r = scan_exact_bid<kSc1>(x1, y1, z1, Qc, price, n, cache);
    b1 = r.b1;
    kb = r.kb;
    b2 = r.b2;
    T = r.T;
}

// ---- auction full scan, fast: selection on an fp32 approximation
//   v' = (3 - s') - p,  s' = v_sqrt_f32(d) (<= 1 ulp; sqrtf is 0.5 ulp)
// With u = 2^-23, s >= 0 and p >= 0 (prices start at 0 and only rise):
//   |v - v'| <= 1.5us + 0.5u(3+s) + 2 * 0.5u(3+s+p) <= u(3(s+p) + 4.5)
// and s + p = 3 - v (up to rounding), so v <= (v' + 13.5u) / (1 - 3u).  For
// every uncached object v' <= K*', hence
//   v <= T = K*' + 4u(6 + |K*'|)      (>= 1.7x margin on both terms)
// independently of the object.  Exact values are computed for the cached
// entries only; if their second best does not exceed T the exact scan runs
// instead.  Keys of objects [kbeg, kend) (a multiple of 256 long) into t.
// Software-pipelined: the next block's coordinates and prices are loaded
// before the current block's keys are computed, so a lone wave (one miss per
// wave, the others at the barrier) waits on one LDS round trip per block
// instead of several.  Same keys, same push order.
__device__ __forceinline__ void scan_fast_keys(LaneTop &t, float x1, float y1, float z1, const float *Qc,
                                               const float *price, int kbeg, int kend) {
    const int lane = threadIdx.x & 63;
    for (int k0 = kbeg + lane; k0 < kend; k0 += 4 * 64) {
        float key[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = k0 + 64 * r;
            key[r] = (3.f - __builtin_amdgcn_sqrtf(sqd_to(x1, y1, z1, Qc + 3 * (size_t)k))) - price[k];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) lane_top_push(t, key[r], k0 + 64 * r);
    }
}

// selection, bound and exact bid from the lanes' approximate-key tops;
// returns false when the exact scan is needed
template <bool kSc1>
__device__ __forceinline__ bool scan_fast_finish(const LaneTop &t, float x1, float y1, float z1, const float *Qc,
                                                 const float *price, int n, centry *__restrict__ cache, float &b1,
                                                 int &kb, float &b2, float &T) {
    bool s1, s2;
    const float d1 = entry_d(x1, y1, z1, Qc, n, t.q1), d2 = entry_d(x1, y1, z1, Qc, n, t.q2);
    const float Kp = select_cache<kSc1>(t, d1, d2, cache, s1, s2, n);
    T = Kp + 4.f * 1.1920929e-7f * (6.f + fabsf(Kp));  // +inf stays +inf
    const float v1 = s1 ? value_of(d1, price[t.q1]) : -PCM_INF;
    const float v2 = s2 ? value_of(d2, price[t.q2]) : -PCM_INF;
    wave_top2(v1, s1 ? t.q1 : 0x7fffffff, v2, s2 ? t.q2 : 0x7fffffff, b1, kb, b2);
    return b2 > T;
}

// one wave's part of a split exact bid: objects r*64 + lane + 64*W*i (every
// lane ascending), exact values, the wave's (best, argbest, better)
// returned wave-uniform.  The top-2 of the whole cloud is the top-2 of the
// parts' top-2s (part_merge).
__device__ __forceinline__ void part_top2(float x1, float y1, float z1, const float *Qc, const float *price, int n,
                                          int r, int W, float &b1, int &kb, float &b2) {
    const int lane = threadIdx.x & 63;
    LaneTop t;
    lane_top_init(t);
    for (int k = r * 64 + lane; k < n; k += 64 * W) lane_top_push(t, value_of(sqd_to(x1, y1, z1, Qc + 3 * (size_t)k), price[k]), k);
    wave_top2(t.a1, t.q1, t.a2, t.q2, b1, kb, b2);
}
// merge of W parts' results (lanes < W read part i's slot); the second
// entries carry no id: a tie at the best already lists the lowest id first
__device__ __forceinline__ void part_merge(const float *pb1, const int *pkb, const float *pb2, int W, float &b1,
                                           int &kb, float &b2) {
    const int lane = threadIdx.x & 63;
    const bool in = lane < W;
    wave_top2(in ? pb1[lane] : -PCM_INF, in ? pkb[lane] : 0x7fffffff, in ? pb2[lane] : -PCM_INF, 0x7fffffff, b1, kb,
              b2);
}

// ---- the reference's order among EXACTLY equal best values (emd_cuda.cu:
// 108-110, 136-139, 165-173).  Bid splits every 2048-object tile over
// tpu = 1024 / ceil(nu / (n / 1024)) threads per bidder (nu: unassigned
// points this iteration); thread r scans [r delta, (r + 1) delta) of each tile
// in turn (delta = ceil(tile width / tpu)), keeping its first maximum, and the
// bidder's threads are merged in thread order with strict '>'.  Among objects
// of equal value the winner is therefore the lowest (r, tile, k): key
// (r << 21) | k.  With tpu == 1, or n <= 2048 (one tile: r grows with k), that
// is the lowest k -- every path below keeps the lowest k and, only when the
// top two values are equal (a tie at the best) and the order differs, the
// bidder's winner is re-chosen by this key.  The top-2 VALUES never depend on
// the order.
constexpr int kTieKBits = 21;  // object ids < 2^21 (launch_emd)
struct TieRank {
    int on, dfull, dlast;  // order differs from the lowest k; delta of full tiles / the last tile
};
__device__ __forceinline__ TieRank tie_rank(int n, int nu) {
    TieRank t;
    const int bc = n / 1024, upb = (nu + bc - 1) / bc;
    const int tpu = 1024 / (upb > 0 ? upb : 1);
    const int lastw = (n & 2047) ? (n & 2047) : 2048;
    t.on = n > 2048 && tpu > 1;
    t.dfull = (2048 + tpu - 1) / tpu;
    t.dlast = (lastw + tpu - 1) / tpu;
    return t;
}
__device__ __forceinline__ int tie_key(const TieRank &t, int k, int n) {
    const int d = (k >> 11) == ((n - 1) >> 11) ? t.dlast : t.dfull;
    return (((k & 2047) / d) << kTieKBits) | k;
}
// wave: the reference's winner among the objects whose exact value equals
// b1 (every object re-evaluated: rare -- exact ties at the best)
__device__ __noinline__ int tie_rescan(float x1, float y1, float z1, const float *Qc, const float *price, int n,
                                       float b1, TieRank t) {
    const int lane = threadIdx.x & 63;
    int best = 0x7fffffff;
    for (int k = lane; k < n; k += 64) {
        const float v = value_of(sqd_to(x1, y1, z1, Qc + 3 * (size_t)k), price[k]);
        if (v == b1) best = min(best, tie_key(t, k, n));
    }
    return wave_min_i(best) & ((1 << kTieKBits) - 1);
}
template <bool kG>
__device__ __forceinline__ int tie_fix(int kb, float b1, float b2, float x1, float y1, float z1, const float *Qc,
                                       const float *price, int n, const TieRank &t) {
    if constexpr (kG) {
        if (t.on && b1 == b2 && (unsigned)kb < (unsigned)n) return tie_rescan(x1, y1, z1, Qc, price, n, b1, t);
    }
    return kb;
}

// one wave: the full bid of point (x1, y1, z1) with a rebuilt cache
template <bool kSc1>
__device__ __forceinline__ void scan_full(float x1, float y1, float z1, const float *Qc, const float *price, int n,
                                          centry *__restrict__ cache, float &b1, int &kb, float &b2, float &T) {
    LaneTop t;
    lane_top_init(t);
    scan_fast_keys(t, x1, y1, z1, Qc, price, 0, n);
    if (!scan_fast_finish<kSc1>(t, x1, y1, z1, Qc, price, n, cache, b1, kb, b2, T))
        scan_exact<kSc1>(x1, y1, z1, Qc, price, n, cache, b1, kb, b2, T);
}

// ===========================================================================
// Workspace
// ===========================================================================
// Two cache regions: A is written by the seed kernel and the master only
// (plain stores and loads, L2-resident); B by the helpers only (sc1 stores,
// read by the master with sc1 loads), so no XCD ever holds a dirty line of
// the other's region.  CT[j] == kInB marks a point whose cache is in B.
struct EmdWs {
    centry *cache;   // [b*n*kL] region A
    float *CT;       // [b*n] cache bound (A) or the kInB marker
    centry *cacheB;  // [b*n*kL] region B
    float *CTB;      // [b*n] cache bound (B)
    int32_t *bid0;   // [b*n] iteration-0 bid (-2: full scan needed)
    float *inc0;     // [b*n]
    int32_t *board;  // [b*kBoardWords]: gen, quit, jn, err (one 128-B line each)
    int32_t *ml;     // [b*n] job: miss list
    int32_t *idone;  // [b*n] job: per-item done generation
    int32_t *rbid;   // [b*n] job results
    float *rinc;     // [b*n]
    float *pp;       // [b*n] job: price snapshot
    // reserve (n == kStagePN only, else null): seed-written, read by the master
    uint16_t *res;   // [b*n*kR] object ids
    float *RT;       // [b*n] reserve bound
    int32_t *RN;     // [b*n] reserve entries (0: none)
    // master state in global memory (n > kLdsStateMaxN), per batch element n words each
    int32_t *g_ass, *g_inv, *g_max, *g_bid, *g_u0, *g_u1, *g_miss;
    float *g_price, *g_inc;
    ckey *g_claim;
};
constexpr int kBoardGen = 0, kBoardQuit = 8, kBoardJn = 16, kBoardNu = 20, kBoardErr = 24;
constexpr unsigned kInB = 0x7fc0b00bu;  // a quiet NaN no bound ever equals

#ifdef PCM_STAMPS
// profiling build: the XCD (XCC_ID) that ran each batch element's first seed
// workgroup ([i]) and its auction master ([512 + i])
__device__ int g_emd_xcc[1024];
__device__ __forceinline__ int pcm_xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15; }
#endif

// ===========================================================================
// 1. seed kernel: iteration-0 bids + caches, one wave per point, 16 points
//    per workgroup, the target cloud staged in LDS (kStage)
// ===========================================================================
template <bool kStage, bool kRes>
__global__ __launch_bounds__(kSeedThreads) void emd_seed_kernel(const float *__restrict__ xyz1,
                                                                const float *__restrict__ xyz2, int b, int n,
                                                                float eps, EmdWs ws) {
    extern __shared__ __attribute__((aligned(16))) float sQs[];
    const int wgs_per_batch = n / kSeedPts;
    // batch element i's workgroups go to the XCD its master (block i of the
    // auction launch) runs on, so the caches are written into the L2 the
    // master reads them from (round-robin placement: speed only)
    int batch, chunk;
    if (b % 8 == 0) {
        const int x = (int)blockIdx.x, sx = x / 8;
        batch = (x % 8) + 8 * (sx / wgs_per_batch);
        chunk = sx % wgs_per_batch;
    } else {
        const int blk = pcm_xcd_remap((int)blockIdx.x, (int)gridDim.x);
        batch = blk / wgs_per_batch;
        chunk = blk - batch * wgs_per_batch;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#ifdef PCM_STAMPS
    if (chunk == 0 && threadIdx.x == 0) g_emd_xcc[batch] = pcm_xcc_id();
#endif
    const float *Pg = xyz1 + (size_t)batch * n * 3;
    const float *Qg = xyz2 + (size_t)batch * n * 3;
    // this wave's query points, loaded (scalar) while the target cloud lands
    const int j0 = chunk * kSeedPts + __builtin_amdgcn_readfirstlane(wave) * kSeedPtsPerWave;
    float qp[kSeedPtsPerWave][3];
#pragma unroll
    for (int p = 0; p < kSeedPtsPerWave; ++p)
#pragma unroll
        for (int c = 0; c < 3; ++c) qp[p][c] = Pg[3 * (j0 + p) + c];
    if constexpr (kStage) {
        pcm_dma_to_lds(sQs, Qg, 12 * n, wave, kSeedThreads / 64);
        vm_drain();
        __syncthreads();
    }
    const float *Qc = kStage ? (const float *)sQs : Qg;
#pragma unroll
    for (int p = 0; p < kSeedPtsPerWave; ++p) {
        const int j = j0 + p;
        const size_t pt = (size_t)batch * n + j;
        float b1, b2, T;
        int kb;
        if constexpr (kRes) {  // n == kStagePN (launch_emd)
            int rn;
            float rT;
            centry *sR = reinterpret_cast<centry *>(sQs + 3 * kStagePN) + wave * kR;  // this wave's reserve copy
            scan_seed_res(qp[p][0], qp[p][1], qp[p][2], Qc, ws.cache + pt * kL, ws.res + pt * kR, sR, b1, kb, b2,
                          T, rn, rT);
            if (lane == 0) {
                ws.RN[pt] = rn;
                ws.RT[pt] = rT;
            }
        } else {
            scan_seed(qp[p][0], qp[p][1], qp[p][2], Qc, n, ws.cache + pt * kL, b1, kb, b2, T);
        }
        if (lane == 0) {
            ws.CT[pt] = T;
            const bool proven = b2 > T && (unsigned)kb < (unsigned)n;
            ws.bid0[pt] = proven ? kb : -2;  // -2: needs a full scan in the auction kernel
            ws.inc0[pt] = b1 - b2 + eps;
            ws.idone[pt] = 0;  // done words of this launch start at 0
            if (j == 0) {
                ws.board[(size_t)batch * kBoardWords + kBoardGen] = 0;
                ws.board[(size_t)batch * kBoardWords + kBoardQuit] = 0;
                ws.board[(size_t)batch * kBoardWords + kBoardJn] = 0;
                ws.board[(size_t)batch * kBoardWords + kBoardErr] = 0;
            }
        }
    }
}

// ===========================================================================
// 2. auction kernel
// ===========================================================================

// Master state: LDS arrays (kG = false) or the workspace (kG = true).  Words
// updated by atomics are re-read with L1-bypassing sc1 loads in the global
// form (a plain load could hit a stale L1 line).
template <bool kG>
struct AState {
    int *ass, *inv, *mx, *bid, *U0, *U1, *miss;
    float *price, *inc;
    ckey *claim;
    __device__ __forceinline__ int ld_max(int k) const {
        if constexpr (kG) return ld_sc1(mx + k); else return mx[k];
    }
    __device__ __forceinline__ ckey ld_claim(int k) const {
        if constexpr (kG) return ld_sc1(claim + k); else return claim[k];
    }
};

// Cache bids: G lanes per bidder, kL/G cached (id, s) entries per lane at
// current prices, a row_shr reduction over the G lanes (G divides the 16-lane
// DPP row); the group's last lane places the bid or lists a full scan.
#ifndef PCM_G16_MAX
#define PCM_G16_MAX 64
#endif
#ifndef PCM_G8_MAX
#define PCM_G8_MAX 256
#endif
constexpr int kG16Max = PCM_G16_MAX, kG8Max = PCM_G8_MAX;  // bidder counts up to which 16 / 8 lanes bid each
__device__ __forceinline__ int cache_bid_lanes(int nu) {
    // measured per bidder count on MI355X (tools/tune_emd.py, profiles/r01):
    // few bidders are latency-bound (more lanes per bidder), many are
    // VALU-bound (fewer lanes, fewer reduction steps per bidder)
    return nu <= kG16Max ? 16 : (nu <= kG8Max ? 8 : 4);
}

// the reference's winner among a group's cached entries of value b1 (rare:
// exact ties at the best, global-state form): lane gl re-reads its slots
template <int G>
__device__ __noinline__ int cache_tie_winner(const centry *cj, bool sc1, const float *price, float b1, TieRank tr,
                                             int n) {
    constexpr int E = kL / G;
    const int gl = threadIdx.x % G;
    int lr = 0x7fffffff;
    for (int e = 0; e < E; ++e) {
        const int slot = 2 * (gl + G * (e >> 1)) + (e & 1);
        const centry c = sc1 ? ld_sc1(cj + slot) : cj[slot];
        const int k = (int)(unsigned)c;
        if ((unsigned)k >= (unsigned)n) continue;  // unused slot (the sentinel n)
        if (value_from_s(__uint_as_float((unsigned)(c >> 32)), price[k]) == b1) lr = min(lr, tie_key(tr, k, n));
    }
    return group_min_i<G>(lr) & ((1 << kTieKBits) - 1);
}

// A bid on object k.  Maxima persisted from earlier iterations are <= 0
// (0 initially, -1e9 once assigned), and with eps > 0 every increment is > 0,
// so an old maximum above 0 means a second bid on k in this iteration: the
// claim phase is needed only when some object saw that (coll[0]).
//
// The claim phase itself is needed only when a bidder other than the maximum's
// holder lies inside GetMax's 1e-6 window of the maximum (emd_cuda.cu:188):
// otherwise the holder -- the bidder whose increment equals the maximum --
// wins.  Every such pair is seen by one of its two atomicMax calls: a bidder
// arriving after the holder gets the maximum back; a holder arriving after
// it gets back an earlier maximum that lies between the two increments.  So
// coll[1] is raised (conservatively, 2e-6) whenever an atomicMax returns a
// same-iteration value that close to the caller's increment; equal
// increments raise it too.
// Bids and increments are kept by the bidder's slot s in the current bidder
// list, not by point id, so the claim and assign passes (which walk the list)
// read them in the same LDS round trip as the point id.
template <bool kG>
__device__ __forceinline__ void bid_on(const AState<kG> &st, int s, int k, float inc, int *coll) {
    st.bid[s] = k;
    st.inc[s] = inc;
    const int old = atomicMax(&st.mx[k], f2key(inc));
    if (old > 0) {
        coll[0] = 1;
        if (fabs((double)inc - (double)key2f(old)) <= 2e-6) coll[1] = 1;
    }
}

// resT/resN (reserve form, else null): a miss whose cache bound is not above
// its reserve bound cannot be bid from the reserve (every value outside the
// cache is <= the bound, so the reserve's second best is too): its reserve
// is retired here and the miss goes straight to the full scan.
// profiling build: sub-phase stamps of the first pass by thread 0 of the
// timed element (slots 4..8 of the phase timers: bidder id, entries, values,
// reductions, bid placed; slot 0 keeps the rest of B1)
#ifdef PCM_STAMPS
#define PCM_B1_STAMP(slot, dep)                                                         \
    if (tm && threadIdx.x == 0 && u0 == 0) {                                            \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::"v"(dep) : "memory");            \
        const unsigned long long tn = __builtin_amdgcn_s_memtime();                     \
        tm[slot] += tn - tm[12];                                                        \
        tm[12] = tn;                                                                    \
    }
#else
#define PCM_B1_STAMP(slot, dep)
#endif
template <int G, bool kG>
__device__ __forceinline__ void cache_bids(int nu, float eps, const int *Ucur, const centry *C, const float *CT,
                                           const centry *CB, const float *CTB, const AState<kG> &st, int *sNm,
                                           int *coll, const float *resT, int *resN, int n, TieRank tr,
                                           unsigned long long *tm = nullptr) {
    (void)tm;
    static_assert(G == 4 || G == 8 || G == 16, "G lanes inside one DPP row");
    constexpr int E = kL / G;
    static_assert(E % 2 == 0, "slot pairs");
    const int gi = threadIdx.x / G, gl = threadIdx.x % G;
    for (int u0 = 0; u0 < nu; u0 += kEmdThreads / G) {
        const int u = u0 + gi;
        const bool act = u < nu;
        PCM_B1_STAMP(4, 0u);  // slot 4: from the barrier to the pass start
        const int j = act ? Ucur[u] : 0;
        PCM_B1_STAMP(5, j);
        // region A (the master's own, plain, L2-resident) is loaded together
        // with the bound; a point whose cache a helper rebuilt (marker) is
        // re-read from region B (sc1)
        float tj = CT[j];
        centry ce[E];
        // lane gl evaluates the slot pairs 2 (gl + G e') + {0, 1}: one 16-byte
        // load per pair (any partition of the kL slots over the group works)
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int e = 0; e < E / 2; ++e) {
            const u64x2 w = *reinterpret_cast<const u64x2 *>(C + (size_t)j * kL + 2 * (gl + G * e));
            ce[2 * e] = w.x;
            ce[2 * e + 1] = w.y;
        }
        PCM_B1_STAMP(6, (unsigned)ce[0] ^ (unsigned)ce[E - 1] ^ __float_as_uint(tj));
        if (__float_as_uint(tj) == kInB) {
            tj = ld_sc1(CTB + j);
#pragma unroll
            for (int e = 0; e < E / 2; ++e) {
                ce[2 * e] = ld_sc1(CB + (size_t)j * kL + 2 * (gl + G * e));
                ce[2 * e + 1] = ld_sc1(CB + (size_t)j * kL + 2 * (gl + G * e) + 1);
            }
        }
        // values at current prices.  An unused slot names the sentinel
        // object n with s = 0: in the LDS-state form price[n] = +inf, so its
        // value is -inf with no masking (and it never equals a best); the
        // global-state form (prices of the next element follow) masks it to
        // (-inf, INT_MAX)
        float v[E];
        int kk[E];
        // the lane's two largest values (multiset: a repeated best is kept
        // twice), two instructions per entry (values are never NaN: cached
        // entries have finite s, prices are finite or +inf)
        float m1 = -PCM_INF, m2 = -PCM_INF;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int k = (int)(unsigned)ce[e];
            const float s = __uint_as_float((unsigned)(ce[e] >> 32));
            if constexpr (kG) {
                const bool bad = (unsigned)k >= (unsigned)n;
                const float v0 = value_from_s(s, st.price[bad ? 0 : k]);
                v[e] = bad ? -PCM_INF : v0;
                kk[e] = bad ? 0x7fffffff : k;
            } else {
                v[e] = value_from_s(s, st.price[k]);
                kk[e] = k;
            }
            m2 = __builtin_amdgcn_fmed3f(m1, m2, v[e]);
            m1 = fmaxf(m1, v[e]);
        }
        PCM_B1_STAMP(7, __float_as_uint(m1));
        // group top-2: best = max, argbest = lowest id at best, better = best
        // when two entries hold it (two lanes' maxima, or a lane's two), else
        // the max of the best lane's second and the other lanes' maxima
        const float b1 = group_max<G>(m1);
        int lk = 0x7fffffff;
#pragma unroll
        for (int e = 0; e < E; ++e) lk = v[e] == b1 ? min(lk, kk[e]) : lk;
        int kb = group_min_i<G>(lk);
        const bool top = m1 == b1;
        const int ntop = group_add_i<G>(top ? 1 : 0);
        const float rest = group_max<G>(top ? m2 : m1);
        const float b2 = ntop >= 2 ? b1 : rest;
        const int ties = b2 == b1 ? 2 : 1;  // a tie at the best
        PCM_B1_STAMP(8, __float_as_uint(b2) ^ (unsigned)kb);
        if constexpr (kG) {
            // a tie at the best (group-uniform): the reference's order
            // decides.  When the bid is proven (b2 > bound) every object of
            // value b1 is cached, so the cached entries hold the winner (out
            // of line: the entries are re-read rather than kept live)
            if (tr.on && ties >= 2 && b2 > tj)
                kb = cache_tie_winner<G>(__float_as_uint(CT[j]) == kInB ? CB + (size_t)j * kL : C + (size_t)j * kL,
                                         __float_as_uint(CT[j]) == kInB, st.price, b1, tr, n);
        }
        if (act && gl == G - 1) {
            if (b2 > tj) {
                bid_on(st, u, kb, b1 - b2 + eps, coll);
            } else {
                st.miss[atomicAdd(sNm, 1)] = u;  // list slots: the point is Ucur[u]
                if (resN && !(tj > resT[j])) resN[j] = 0;
            }
        }
        PCM_B1_STAMP(9, (unsigned)kb);
    }
}

// a bid produced by a full scan, placed by the scanning wave's lane 0 (s:
// the bidder's slot in the current list)
template <bool kG>
__device__ __forceinline__ void place_bid(const AState<kG> &st, int s, int kb, float inc, int n, int *coll) {
    if ((unsigned)kb < (unsigned)n) {
        bid_on(st, s, kb, inc, coll);
    } else {  // all-NaN values: no bid (oracle: best_i = -1)
        st.bid[s] = -1;
        st.inc[s] = inc;
    }
}

// Items of a job are split statically: groups of kWaves consecutive items go
// round-robin to the master (group 0, H + 1, ...) and helpers 0 .. H - 1, one
// item per wave of the group -- no claim atomics on anyone's critical path.
// Owner of item i: (i / kWaves) % (H + 1), 0 = the master, r + 1 = helper r.

// helper side of a job item: full scan with the snapshot prices, cache into
// region B, result words, then the done word (sc1 throughout)
template <bool kG>
__device__ __forceinline__ void helper_item(const EmdWs &ws, size_t base, int i, int g, const float *P,
                                            const float *Qc, const float *price, int n, float eps,
                                            const TieRank &tr) {
    const int lane = threadIdx.x & 63;
    const int j = __builtin_amdgcn_readfirstlane(ld_sc1(ws.ml + base + i));
    float b1, b2, T;
    int kb;
    scan_full<true>(P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, price, n, ws.cacheB + (base + j) * kL, b1, kb, b2,
                    T);
    kb = tie_fix<kG>(kb, b1, b2, P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, price, n, tr);
    if (lane == 0) {
        st_sc1(ws.CTB + base + j, T);
        st_sc1(ws.rbid + base + i, (int)kb);
        st_sc1(ws.rinc + base + i, b1 - b2 + eps);
    }
    vm_drain();  // every store of this wave (cache entries included) has left the CU
    if (lane == 0) st_sc1(ws.idone + base + i, g);
}

struct KArgs {
    const float *xyz1, *xyz2;
    int b, n, iters, H, offload_min, diag, wmax, tail_max;
    int spin_limit;  // bound of every poll (kSpinLimit; tests force 0)
    float eps;
    float *dist;
    int32_t *ass_out;
    float *price_out;
    int32_t *stats;
};

// diagnostics (stats != nullptr): diag 1 = per-iteration (unassigned, full
// scans) summed over the batch plus job counters (atomics: they perturb the
// timing); diag 2 = phase timers of batch 0 in registers, written at the end
constexpr int kDiagHist = 1, kDiagTimers = 2;

// helper role: take full scans of the master's jobs until it quits
template <bool kG, bool kStage, int kN>
__device__ void helper_loop(const KArgs &a, const EmdWs &ws, int batch, int rank, int *smem) {
    __shared__ int sGen;
    const int n = kN > 0 ? kN : a.n;  // kN: the cloud size fixed at compile time
    const int tid = threadIdx.x, wave = tid >> 6;
    float *sQ = (float *)smem;                                       // [3n] (kStage)
    float *sPH = (float *)smem + (kStage ? 3 * (size_t)n : 0);       // [n] price snapshot
    const size_t base = (size_t)batch * n;
    const float *P = a.xyz1 + base * 3;
    const float *Qg = a.xyz2 + base * 3;
    int32_t *bw = ws.board + (size_t)batch * kBoardWords;
    if constexpr (kStage) pcm_dma_to_lds(sQ, Qg, 12 * n, wave, kWaves);
    const float *Qc = kStage ? (const float *)sQ : Qg;
    int last = 0;
    for (;;) {
        if (tid == 0) {
            int g = -1;  // no job within the bound: this helper leaves (the master scans what it would have)
            for (int spin = 0; spin < a.spin_limit; ++spin) {
                if (ld_sc1(bw + kBoardQuit)) break;
                const int gv = ld_sc1(bw + kBoardGen);
                if (gv != last) { g = gv; break; }
                __builtin_amdgcn_s_sleep(2);
            }
            sGen = g;
        }
        if constexpr (kStage) vm_drain();  // the staged cloud has landed (first pass)
        __syncthreads();
        const int g = sGen;
        if (g < 0) return;
        const int jn = ld_sc1(bw + kBoardJn);
        const TieRank tr = tie_rank(n, ld_sc1(bw + kBoardNu));  // the job's iteration
        for (int k = tid; k < n; k += kEmdThreads) sPH[k] = ld_sc1(ws.pp + base + k);
        __syncthreads();
        for (int g0 = rank + 1; g0 * kWaves < jn; g0 += a.H + 1) {  // this helper's groups (owner rank + 1)
            const int i = g0 * kWaves + wave;
            if (i < jn) helper_item<kG>(ws, base, i, g, P, Qc, sPH, n, a.eps, tr);
        }
        if (a.diag == kDiagHist && tid == 0) atomicAdd(&a.stats[2 * a.iters + 12], 1);  // helper wake-ups
        last = g;
        __syncthreads();
    }
}

// master role: the auction of one batch element
template <bool kG, bool kStage, bool kStageP, int kN>
__device__ void master_loop(const KArgs &a, const EmdWs &ws, int batch, int *smem) {
    __shared__ int sNu[2], sNm, sColl[2], sChainJ;  // sColl: [0] some object saw 2 bids, [1] a window contention
    __shared__ float sPb1[kWaves], sPb2[kWaves];  // split bids: one part per wave
    __shared__ int sPkb[kWaves];
    const int n = kN > 0 ? kN : a.n, iters = a.iters;
    const float eps = a.eps;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t base = (size_t)batch * n;
    const float *Pg = a.xyz1 + base * 3;
    const float *Qg = a.xyz2 + base * 3;
    int32_t *bw = ws.board + (size_t)batch * kBoardWords;
    centry *C = ws.cache + base * kL;
    float *CT = ws.CT + base;  // region-A bounds (LDS copy in the LDS-state forms, below)
    const bool hist = a.diag == kDiagHist;
    // diag >= 2: timers of batch element diag - 2
    const bool timers = a.diag >= kDiagTimers && batch == a.diag - kDiagTimers && tid == 0;
#ifdef PCM_STAMPS
    if (tid == 0) g_emd_xcc[512 + batch] = pcm_xcc_id();
#endif

    AState<kG> st;
    char *lp = (char *)smem;
    if constexpr (!kG) {
        st.ass = (int *)lp; lp += 4 * (size_t)n;
        st.inv = (int *)lp; lp += 4 * (size_t)n;
        st.price = (float *)lp; lp += 4 * (size_t)n + 8;  // + the sentinel price[n] = +inf (8: claim alignment)
        st.mx = (int *)lp; lp += 4 * (size_t)n;
        st.claim = (ckey *)lp; lp += 8 * (size_t)n;
        st.bid = (int *)lp; lp += 4 * (size_t)n;
        st.inc = (float *)lp; lp += 4 * (size_t)n;
        st.U0 = (int *)lp; lp += 4 * (size_t)n;
        st.U1 = (int *)lp; lp += 4 * (size_t)n;
        st.miss = (int *)lp; lp += 4 * (size_t)n;
        CT = (float *)lp; lp += 4 * (size_t)n;  // the bound is read first in every cache bid: LDS, not L2
    } else {
        st.ass = ws.g_ass + base; st.inv = ws.g_inv + base; st.price = ws.g_price + base;
        st.mx = ws.g_max + base; st.claim = ws.g_claim + base; st.bid = ws.g_bid + base;
        st.inc = ws.g_inc + base; st.U0 = ws.g_u0 + base; st.U1 = ws.g_u1 + base;
        st.miss = ws.g_miss + base;
    }
    float *sQ = (float *)lp;  // [3n] staged target cloud (kStage)
    if constexpr (kStage) lp += 12 * (size_t)n;
    float *sP = (float *)lp;  // [3n] staged bidder cloud (kStageP)
    if constexpr (kStageP) lp += 12 * (size_t)n;
    // lane tops of the split scans: 5 words x 64 lanes x 16 waves
    float *xA1 = (float *)lp, *xA2 = xA1 + kEmdThreads, *xA3 = xA2 + kEmdThreads;
    int *xQ1 = (int *)(xA3 + kEmdThreads), *xQ2 = xQ1 + kEmdThreads;
    // reserve form (n == kStagePN, LDS state): bounds and entry counts of the
    // seed's reserves; a point's count drops to 0 once its reserve fails a proof
    constexpr bool kRes = !kG && kN == kStagePN;
    float *sRT = (float *)(xQ2 + kEmdThreads);  // [n] (kRes)
    int *sRN = (int *)(sRT + n);                // [n] (kRes)
    const bool res_on = eps >= 0.f;             // prices never fall: the reserve bounds hold

    if constexpr (kStage) pcm_dma_to_lds(sQ, Qg, 12 * n, wave, kWaves);
    if constexpr (kStageP) pcm_dma_to_lds(sP, Pg, 12 * n, wave, kWaves);
    const float *Qc = kStage ? (const float *)sQ : Qg;
    const float *P = kStageP ? (const float *)sP : Pg;

    for (int j = tid; j < n; j += kEmdThreads) {
        st.ass[j] = -1;
        st.inv[j] = -1;
        st.price[j] = 0.f;
        if constexpr (!kG) if (j == 0) st.price[n] = PCM_INF;  // the unused cache slots' object
        st.mx[j] = f2key(0.f);  // emd_module.py:49 zero-inits max_increments
        st.claim[j] = ~0ull;
        st.U0[j] = j;           // iteration 0: every point bids
        if constexpr (!kG) CT[j] = ws.CT[base + j];  // the seed's bounds
        if constexpr (kRes) {
            sRT[j] = ws.RT[base + j];
            sRN[j] = res_on ? ws.RN[base + j] : 0;
        }
    }
    if (tid == 0) { sNu[0] = n; sNu[1] = 0; sNm = 0; sColl[0] = sColl[1] = 0; }
    vm_drain();  // the DMA has landed
    __syncthreads();

    TieRank tr = tie_rank(n, n);  // the current iteration's exact-tie order
    int gen = 0;   // jobs posted so far
    int H = a.H;   // helpers still taking jobs (0 after a timed-out job)
    // timers (diag >= 2): cycles per phase, kept by thread 0 in LDS (not in
    // registers the whole kernel would reserve)
    __shared__ unsigned long long sTm[13];  // [12] = the previous stamp
    if (timers) {
        for (int i = 0; i < 12; ++i) sTm[i] = 0;
        sTm[12] = __builtin_amdgcn_s_memtime();
    }
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#define PCM_EMD_PHASE(i)                                                  \
    if (timers) {                                                         \
        const unsigned long long tn = __builtin_amdgcn_s_memtime();      \
        sTm[i] += tn - sTm[12];                                           \
        sTm[12] = tn;                                                     \
    }
    // the master's own full scan of point j: cache region A, bid placed
    // (profiling build: wave 0's key scan, proof and exact fallback timed
    // in slots 6, 7, 11 and the exact fallbacks counted)
    // the reserve bid of miss q (kRes): two entries per lane instead of n / 64
    // objects; on success the miss entry is cleared (-1) so B2b skips it
    auto own_reserve = [&](int q, const int *Ucur) {
        const int u = st.miss[q];
        const int j = Ucur[u];
        const int rn = __builtin_amdgcn_readfirstlane(sRN[j]);
        if (rn <= 0) return;
#ifdef PCM_STAMPS
        PCM_EMD_PHASE(5);  // profiling build: B1 end -> wave 0's first reserve bid (slot 5), the bid (slot 4)
#endif
#ifdef PCM_STAMPS
        // slots 6 (entries loaded), 7 (values + top-2), 11 (cache threshold)
        auto stamp = [&](int i, unsigned dep) {
            if (timers) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::"v"(dep) : "memory");
                const unsigned long long tn = __builtin_amdgcn_s_memtime();
                sTm[i] += tn - sTm[12];
                sTm[12] = tn;
            }
        };
#else
        auto stamp = [](int, unsigned) {};
#endif
        const ResBid rb = reserve_bid(ws.res + (base + j) * kR, rn, sRT[j], (lds_cfp)st.price, P[3 * j],
                                      P[3 * j + 1], P[3 * j + 2], Qc, C + (size_t)j * kL, stamp);
#ifdef PCM_STAMPS
        PCM_EMD_PHASE(4);
#endif
        if (lane == 0) {
            if (rb.ok) {
                CT[j] = rb.T;
                place_bid(st, u, rb.kb, rb.b1 - rb.b2 + eps, n, sColl);
                st.miss[q] = -1;
                if (hist) atomicAdd(&a.stats[2 * iters + 13], 1);  // reserve bids
            } else {
                sRN[j] = 0;  // exhausted: j's later misses scan directly
            }
        }
    };
    auto own_scan = [&](int u, int j) {
        float b1, b2, T;
        int kb;
        centry *cj = C + (size_t)j * kL;
        const float x1 = P[3 * j], y1 = P[3 * j + 1], z1 = P[3 * j + 2];
#ifdef PCM_STAMPS
        LaneTop t;
        lane_top_init(t);
        scan_fast_keys(t, x1, y1, z1, Qc, st.price, 0, n);
        PCM_EMD_PHASE(6);
        const bool ok = scan_fast_finish<false>(t, x1, y1, z1, Qc, st.price, n, cj, b1, kb, b2, T);
        PCM_EMD_PHASE(7);
        if (!ok) {
            scan_exact<false>(x1, y1, z1, Qc, st.price, n, cj, b1, kb, b2, T);
            if (hist && lane == 0) atomicAdd(&a.stats[2 * iters + 15], 1);  // exact fallbacks
            PCM_EMD_PHASE(11);
        }
#else
        scan_full<false>(x1, y1, z1, Qc, st.price, n, cj, b1, kb, b2, T);
#endif
        kb = tie_fix<kG>(kb, b1, b2, x1, y1, z1, Qc, st.price, n, tr);
        if (lane == 0) {
            CT[j] = T;
            place_bid(st, u, kb, b1 - b2 + eps, n, sColl);
        }
    };
    int active = 0, chain_its = 0, tail_its = 0;
    for (int it = 0; it < iters; ++it) {
        const bool last = (it == iters - 1);
        // timers: this iteration's start (cycles) and B1 total so far
        unsigned long long it_t0 = 0, it_b1 = 0;
        if (timers) { it_t0 = __builtin_amdgcn_s_memtime(); it_b1 = sTm[0]; }
        const int cur = it & 1;
        const int nu = sNu[cur];
        if (nu == 0) break;  // nothing left to bid: later iterations are no-ops
        ++active;
        tr = tie_rank(n, nu);
        // (two named arrays, not an indexed pair: the selected pointer keeps
        // its address space and the list reads stay ds_read, not flat loads)
        const int *Ucur = cur ? st.U1 : st.U0;
        int *Unext = cur ? st.U0 : st.U1;
        // the other list's counter was last read at the start of iteration it-1
        if (tid == 0) sNu[cur ^ 1] = 0;

        // ---- chain mode: a single bidder.  Its bid can only collide with
        // itself, so every later iteration is bid -> resolve -> assign of one
        // point, and the evicted owner (if any) is the next iteration's only
        // bidder.  The bid is split over kChainW waves (each scans every
        // kChainW-th 64-object chunk); wave 0 merges, resolves (solo rule,
        // else the 1e-6 window) and assigns: two barriers per iteration and no
        // list handling.  (One wave scanning all n objects alone took 4.3k
        // cycles per iteration against 1.9k: the 16 dependent per-lane steps
        // of its lane top-2 are latency-bound.)
        if (it > 0 && nu == 1 && a.tail_max > 0) {
            int j = Ucur[0];
            for (; it < iters; ++it) {
                ++active;
                ++chain_its;
                PCM_EMD_PHASE(8);
                if (hist && tid == 0) {
                    atomicAdd(&a.stats[2 * it], 1);
                    atomicAdd(&a.stats[2 * it + 1], 1);
                }
                if (wave < kChainW) {
                    float b1, b2;
                    int kb;
                    part_top2(P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, st.price, n, wave, kChainW, b1, kb, b2);
                    if (lane == 0) { sPb1[wave] = b1; sPkb[wave] = kb; sPb2[wave] = b2; }
                }
                __syncthreads();
                PCM_EMD_PHASE(9);
                if (wave == 0) {
                    float b1, b2;
                    int kb;
                    part_merge(sPb1, sPkb, sPb2, kChainW, b1, kb, b2);
                    kb = tie_fix<kG>(kb, b1, b2, P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, st.price, n, tr);
                    int next = j;  // no bid / not won: j bids again
                    if ((unsigned)kb < (unsigned)n && lane == 0) {
                        if (it == iters - 1) {
                            st.ass[j] = kb;
                        } else {
                            const float inc = b1 - b2 + eps;
                            const bool coll = atomicMax(&st.mx[kb], f2key(inc)) > 0;
                            bool won = true;
                            if (coll || !(eps > 0.f)) {
                                const double bi = (double)inc, mi = (double)key2f(st.ld_max(kb));
                                won = bi - 1e-6 <= mi && mi <= bi + 1e-6;
                            }
                            if (won) {
                                const int old = st.inv[kb];
                                if (old != -1) st.ass[old] = -1;
                                st.inv[kb] = j;
                                st.ass[j] = kb;
                                st.price[kb] += inc;
                                st.mx[kb] = f2key(-1e9f);
                                next = old;  // -1: nobody left to bid
                            }
                        }
                    }
                    if (lane == 0) sChainJ = next;
                }
                __syncthreads();
                PCM_EMD_PHASE(10);
                j = sChainJ;
                if (j < 0) break;
            }
            break;
        }

        // ---- tail mode (few bidders; the count never grows): one wave per
        // bidder, full scan without a cache, no cache-bid phase
        if (it > 0 && nu <= a.tail_max) {
            ++tail_its;
            // W waves per bidder (16 / the next power of two >= nu), each
            // scanning every W-th 64-object chunk; the bidder's first wave merges
            const int W = nu <= 1 ? 16 : (nu <= 2 ? 8 : (nu <= 4 ? 4 : (nu <= 8 ? 2 : 1)));
            const int q = wave / W, r = wave - q * W;
            if (W == 1) {  // whole bids, one wave each (more than 8 bidders)
                for (int u = wave; u < nu; u += kWaves) {
                    const int j = Ucur[u];
                    float b1, b2;
                    int kb;
                    part_top2(P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, st.price, n, 0, 1, b1, kb, b2);
                    kb = tie_fix<kG>(kb, b1, b2, P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, st.price, n, tr);
                    if (lane == 0) place_bid(st, u, kb, b1 - b2 + eps, n, sColl);
                }
            } else if (q < nu) {
                const int j = Ucur[q];
                float b1, b2;
                int kb;
                part_top2(P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, st.price, n, r, W, b1, kb, b2);
                if (lane == 0) { sPb1[wave] = b1; sPkb[wave] = kb; sPb2[wave] = b2; }
            }
            if (hist && tid == 0) {
                atomicAdd(&a.stats[2 * it], nu);
                atomicAdd(&a.stats[2 * it + 1], nu);
            }
            __syncthreads();
            if (W > 1 && q < nu && r == 0) {
                float b1, b2;
                int kb;
                part_merge(sPb1 + wave, sPkb + wave, sPb2 + wave, W, b1, kb, b2);
                const int j = Ucur[q];
                kb = tie_fix<kG>(kb, b1, b2, P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, st.price, n, tr);
                if (lane == 0) place_bid(st, q, kb, b1 - b2 + eps, n, sColl);
            }
            __syncthreads();
            PCM_EMD_PHASE(1);
        } else {
        // ---- B1: bids from the seed (iteration 0) or the caches; misses listed
        if (it == 0) {
            for (int u = tid; u < nu; u += kEmdThreads) {
                const int j = Ucur[u];
                const int k = ws.bid0[base + j];
                if (k >= 0) {
                    bid_on(st, u, k, ws.inc0[base + j], sColl);
                } else {
                    st.miss[atomicAdd(&sNm, 1)] = u;
                }
            }
        } else {
            const centry *CB = ws.cacheB + base * kL;
            const float *CTB = ws.CTB + base;
            const int G = cache_bid_lanes(nu);
            const float *rT = kRes ? sRT : nullptr;
            int *rN = kRes ? sRN : nullptr;
            unsigned long long *tm = timers ? sTm : nullptr;
            if (G == 16) cache_bids<16>(nu, eps, Ucur, C, CT, CB, CTB, st, &sNm, sColl, rT, rN, n, tr, tm);
            else if (G == 8) cache_bids<8>(nu, eps, Ucur, C, CT, CB, CTB, st, &sNm, sColl, rT, rN, n, tr, tm);
            else cache_bids<4>(nu, eps, Ucur, C, CT, CB, CTB, st, &sNm, sColl, rT, rN, n, tr, tm);
        }
        __syncthreads();
        PCM_EMD_PHASE(0);

        // ---- B2: full scans of the misses, caches rebuilt
        const int nm = sNm;
        if (hist && tid == 0) {
            atomicAdd(&a.stats[2 * it], nu);
            atomicAdd(&a.stats[2 * it + 1], nm);
        }
        if (nm > 0) {
            if (H > 0 && nm > a.offload_min) {
                // publish the job: miss list, price snapshot, size
                ++gen;
                for (int i = tid; i < nm; i += kEmdThreads) st_sc1(ws.ml + base + i, Ucur[st.miss[i]]);
                for (int k = tid; k < n; k += kEmdThreads) st_sc1(ws.pp + base + k, st.price[k]);
                if (tid == 0) {
                    st_sc1(bw + kBoardJn, nm);
                    st_sc1(bw + kBoardNu, nu);
                }
                vm_drain();
                __syncthreads();
                if (tid == 0) st_sc1(bw + kBoardGen, gen);
                PCM_EMD_PHASE(4);
                // the master's own groups (owner 0); an item it scans itself
                // goes to region A and is marked (miss entry negated) so the
                // collection skips it
                for (int g0 = 0; g0 * kWaves < nm; g0 += a.H + 1) {
                    const int i = g0 * kWaves + wave;
                    if (i >= nm) break;
                    const int u = st.miss[i];
                    own_scan(u, Ucur[u]);
                    if (lane == 0) st.miss[i] = -1 - u;
                }
                __syncthreads();
                PCM_EMD_PHASE(5);
                // collect the helpers' items once their done words show this
                // job.  An item whose done word does not arrive within the
                // bound (a helper that is not resident, or left) keeps its
                // miss entry: the master scans it below itself, so a timeout
                // costs time, never correctness
                bool late = false;
                for (int i = tid; i < nm; i += kEmdThreads) {
                    const int u = st.miss[i];
                    if (u < 0) continue;
                    const int j = Ucur[u];
                    int spin = 0;
                    while (!late && ld_sc1(ws.idone + base + i) != gen) {
                        if (++spin > a.spin_limit) late = true;
                        else __builtin_amdgcn_s_sleep(1);
                    }
                    if (late) continue;
                    CT[j] = __uint_as_float(kInB);
                    place_bid(st, u, ld_sc1(ws.rbid + base + i), ld_sc1(ws.rinc + base + i), n, sColl);
                    st.miss[i] = -1 - u;
                }
                __shared__ int sLate[kWaves];
                if (pcm_wg_or(late, sLate, kWaves)) {
                    // region A rebuilt for the unanswered items, bids placed;
                    // no further jobs in this call (the word is a diagnostic)
                    H = 0;
                    if (tid == 0) st_sc1(bw + kBoardErr, 1);
                    for (int i = wave; i < nm; i += kWaves) {
                        const int u = __builtin_amdgcn_readfirstlane(st.miss[i]);
                        if (u >= 0) own_scan(u, Ucur[u]);
                    }
                }
                if (hist && tid == 0) {
                    atomicAdd(&a.stats[2 * iters + 10], 1);   // jobs
                    atomicAdd(&a.stats[2 * iters + 11], nm);  // items
                }
            } else {
                // W waves per miss for a few misses (each scans n/W objects, the
                // lane tops are merged in object order), one wave per miss else
                const int W = (nm <= 4 && a.wmax >= 4) ? 4 : ((nm <= 8 && a.wmax >= 2) ? 2 : 1);
                if (W == 1) {
                    if constexpr (kRes) {
                        // B2a: reserve bids; B2b: full scans of the rest (the
                        // same wave's misses: no barrier between the two)
                        for (int q = wave; q < nm; q += kWaves) own_reserve(q, Ucur);
                        for (int q = wave; q < nm; q += kWaves) {
                            const int u = __builtin_amdgcn_readfirstlane(st.miss[q]);
                            if (u >= 0) own_scan(u, Ucur[u]);
                        }
                    } else {
                        for (int q = wave; q < nm; q += kWaves) {
                            const int u = st.miss[q];
                            own_scan(u, Ucur[u]);
                        }
                    }
                } else {
                    const int q = wave / W, r = wave - q * W;
                    const bool act = q < nm;
                    const int uq = act ? st.miss[q] : 0;
                    const int j = Ucur[uq];
                    const float x1 = P[3 * j], y1 = P[3 * j + 1], z1 = P[3 * j + 2];
                    LaneTop t;
                    lane_top_init(t);
                    const int part = n / W;  // a multiple of 256
                    if (act) scan_fast_keys(t, x1, y1, z1, Qc, st.price, r * part, (r + 1) * part);
                    if (act && r != 0) {
                        xA1[tid] = t.a1; xA2[tid] = t.a2; xA3[tid] = t.a3; xQ1[tid] = t.q1; xQ2[tid] = t.q2;
                    }
                    PCM_EMD_PHASE(4);
                    __syncthreads();
                    PCM_EMD_PHASE(5);
                    if (act && r == 0) {
                        for (int rr = 1; rr < W; ++rr) {
                            const int o = tid + 64 * rr;
                            lane_top_merge(t, xA1[o], xQ1[o], xA2[o], xQ2[o], xA3[o]);
                        }
                        PCM_EMD_PHASE(6);
                        float b1, b2, T;
                        int kb;
                        centry *cj = C + (size_t)j * kL;
                        if (!scan_fast_finish<false>(t, x1, y1, z1, Qc, st.price, n, cj, b1, kb, b2, T))
                            scan_exact<false>(x1, y1, z1, Qc, st.price, n, cj, b1, kb, b2, T);
                        kb = tie_fix<kG>(kb, b1, b2, x1, y1, z1, Qc, st.price, n, tr);
                        if (lane == 0) {
                            CT[j] = T;
                            place_bid(st, uq, kb, b1 - b2 + eps, n, sColl);
                        }
                        PCM_EMD_PHASE(7);
                    }
                }
            }
            __syncthreads();
        }
        PCM_EMD_PHASE(1);
        }  // not tail mode

        // ---- C: claim -- lowest bidder inside the reference's 1e-6 window
        //      (emd_cuda.cu:181-194); the key carries the iteration.  Skipped
        //      when every bid object has a single bidder (it then wins).
        const ckey itag = (ckey)(~(unsigned)it) << 32;
        // solo: no object saw two bids; by_max: no bidder other than the
        // maximum's holder inside the window (see bid_on) -- the holder wins
        const bool solo = sColl[0] == 0 && eps > 0.f;
        const bool by_max = sColl[1] == 0 && eps > 0.f;
        if (!last && !by_max) {
            for (int u = tid; u < nu; u += kEmdThreads) {
                const int j = Ucur[u];
                const int k = st.bid[u];
                if (k < 0) continue;
                const double bi = (double)st.inc[u];
                const double mi = (double)key2f(st.ld_max(k));
                if (bi - 1e-6 <= mi && mi <= bi + 1e-6) atomicMin(&st.claim[k], itag | (unsigned)j);
            }
            __syncthreads();
        }
        PCM_EMD_PHASE(2);

        // ---- D: assign (emd_cuda.cu:196-215) and the next bidder list.  On
        // the last iteration every bidder takes its object; prices/owners are
        // then dead state and are left as they were (the reference's racy
        // updates are unobservable).
        for (int u0 = 0; u0 < nu; u0 += kEmdThreads) {
            const int u = u0 + tid;
            int push = -1;
            if (u < nu) {
                // point, bid and increment in one LDS round trip (slot-indexed
                // bids); then the owner, maximum and price of the object in one
                const int j = Ucur[u];
                const int k = st.bid[u];
                const float inc = st.inc[u];
                const int kc = k < 0 ? 0 : k;
                const int old = st.inv[kc];
                const int mxk = by_max ? st.ld_max(kc) : 0;
                const float pk = st.price[kc];
                if (k < 0) {
                    push = j;  // no bid: stays unassigned
                } else if (last) {
                    st.ass[j] = k;
                } else if (solo || (by_max ? inc == key2f(mxk) : st.ld_claim(k) == (itag | (unsigned)j))) {
                    if (old != -1) { st.ass[old] = -1; push = old; }
                    st.inv[k] = j;
                    st.ass[j] = k;
                    st.price[k] = pk + inc;
                    st.mx[k] = f2key(-1e9f);
                } else {
                    push = j;  // outbid
                }
            }
            if (tid == 0) { sNm = 0; sColl[0] = sColl[1] = 0; }  // read before the last barrier
            if (!last) {
                const unsigned long long bal = __ballot(push >= 0);
                int pos = 0;
                if (lane == 0 && bal) pos = atomicAdd(&sNu[cur ^ 1], __popcll(bal));
                pos = __builtin_amdgcn_readlane(pos, 0);  // lane 0's slot, no LDS round trip
                if (push >= 0) Unext[pos + __popcll(bal & ((1ull << lane) - 1ull))] = push;
            }
        }
        __syncthreads();
        PCM_EMD_PHASE(3);
        if (timers) {  // per iteration: cycles / 16, B1 cycles / 16, bidders
            a.stats[2 * it] = (int)((__builtin_amdgcn_s_memtime() - it_t0) >> 4);
            a.stats[2 * it + 1] = (int)((sTm[0] - it_b1) >> 4);
            a.stats[2 * iters + 16 + it] = nu;
        }
    }
#undef PCM_EMD_PHASE
    if (a.H > 0 && tid == 0) st_sc1(bw + kBoardQuit, 1);  // helpers exit
    if (a.stats && tid == 0)  // diagnostics: whole-auction wall time per batch element
        a.stats[3 * iters + 16 + batch] = (int)(__builtin_amdgcn_s_memrealtime() - t_start);
    if (timers) {
        for (int i = 0; i < 12; ++i) a.stats[2 * iters + i] = (int)(sTm[i] >> 4);  // units of 16 cycles
        a.stats[2 * iters + 12] = active;
        a.stats[2 * iters + 13] = tail_its;
        a.stats[2 * iters + 14] = chain_its;
    }

    // ---- CalcDist (emd_cuda.cu:217-226): deltas xyz1 - xyz2
    for (int j = tid; j < n; j += kEmdThreads) {
        const int k = st.ass[j];
        float d = 0.f;
        if (k >= 0) {
            d = pcm_sqd(P[3 * (size_t)j + 0] - Qc[3 * (size_t)k + 0], P[3 * (size_t)j + 1] - Qc[3 * (size_t)k + 1],
                        P[3 * (size_t)j + 2] - Qc[3 * (size_t)k + 2]);
        }
        a.dist[base + j] = d;
        a.ass_out[base + j] = k;
        if (a.price_out) a.price_out[base + j] = st.price[j];
    }
}

// Grid: b masters (blocks 0..b-1) then b*H helpers.  Helper x serves the
// batch element on its own XCD when b % 8 == 0 (blocks x and x + 8 share one
// under round-robin dispatch -- speed only, nothing depends on it).
// The LDS-state form with the bidder cloud staged runs exactly n = 1024 (the
// launcher's stage_p), so that instantiation fixes n at compile time: loop
// bounds fold and the master spills fewer scalars.
template <bool kG, bool kStage, bool kStageP>
__global__ __launch_bounds__(kEmdThreads) void emd_auction_kernel(KArgs a, EmdWs ws) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    constexpr int kN = (!kG && kStageP) ? kStagePN : 0;
    const int x = (int)blockIdx.x;
    if (x < a.b) {
        master_loop<kG, kStage, kStageP, kN>(a, ws, x, smem);
        return;
    }
    const int h = x - a.b;
    int batch, rank;
    if (a.b % 8 == 0) {
        const int per = a.b / 8;
        batch = (h % 8) + 8 * ((h / 8) % per);
        rank = (h / 8) / per;
    } else {
        batch = h % a.b;
        rank = h / a.b;
    }
    if (rank >= a.H) return;
    helper_loop<kG, kStage, kN>(a, ws, batch, rank, smem);
}

__global__ void emd_bwd_kernel(const float *__restrict__ xyz1, const float *__restrict__ xyz2, int n,
                               size_t total, const float *__restrict__ graddist,
                               const int32_t *__restrict__ assignment, float *__restrict__ grad) {
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
         t += (size_t)gridDim.x * blockDim.x) {
        const size_t batch = t / n;
        const int k = assignment[t];
        const float *p = xyz1 + 3 * t;
        if ((unsigned)k >= (unsigned)n) {
            // a point the forward left unassigned (all-NaN bid values): no
            // partner to pull towards -- zero gradient, no out-of-range read
#pragma unroll
            for (int c = 0; c < 3; ++c) grad[3 * t + c] = 0.f;
            continue;
        }
        const float g = __fmul_rn(graddist[t], 2.f);
        const float *q = xyz2 + 3 * (batch * n + (size_t)k);
#pragma unroll
        for (int c = 0; c < 3; ++c) grad[3 * t + c] = __fadd_rn(0.f, __fmul_rn(g, __fsub_rn(p[c], q[c])));
    }
}

// ---- workspace layout
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t ws_layout(int b, int n, EmdWs *w, char *basep) {
    const size_t pts = (size_t)b * n;
    size_t off = 0;
    auto take = [&](size_t bytes) -> char * {
        char *p = basep ? basep + off : nullptr;
        off = align256(off + bytes);
        return p;
    };
    EmdWs t{};
    t.cache = (centry *)take(pts * kL * sizeof(centry));
    t.CT = (float *)take(pts * 4);
    t.cacheB = (centry *)take(pts * kL * sizeof(centry));
    t.CTB = (float *)take(pts * 4);
    t.bid0 = (int32_t *)take(pts * 4);
    t.inc0 = (float *)take(pts * 4);
    t.board = (int32_t *)take((size_t)b * kBoardWords * 4);
    t.ml = (int32_t *)take(pts * 4);
    t.idone = (int32_t *)take(pts * 4);
    t.rbid = (int32_t *)take(pts * 4);
    t.rinc = (float *)take(pts * 4);
    t.pp = (float *)take(pts * 4);
    if (n == kStagePN) {
        t.res = (uint16_t *)take(pts * kR * sizeof(uint16_t));
        t.RT = (float *)take(pts * 4);
        t.RN = (int32_t *)take(pts * 4);
    }
    if (n > kLdsStateMaxN) {
        t.g_ass = (int32_t *)take(pts * 4);
        t.g_inv = (int32_t *)take(pts * 4);
        t.g_max = (int32_t *)take(pts * 4);
        t.g_bid = (int32_t *)take(pts * 4);
        t.g_u0 = (int32_t *)take(pts * 4);
        t.g_u1 = (int32_t *)take(pts * 4);
        t.g_miss = (int32_t *)take(pts * 4);
        t.g_price = (float *)take(pts * 4);
        t.g_inc = (float *)take(pts * 4);
        t.g_claim = (ckey *)take(pts * 8);
    }
    if (w) *w = t;
    return off;
}

}  // namespace

extern "C" size_t pcm_emd_workspace_bytes(int b, int n) {
    if (b <= 0 || n <= 0) return 0;
    return ws_layout(b, n, nullptr, nullptr);
}

namespace {
// helpers per batch element: every master and helper gets a CU of its own
// (the launch pads LDS to one workgroup per CU), sized from the device's CU
// count (a compute partition or a CU-masked device has fewer than 256).  A
// helper that is not resident only costs time: the master scans the items
// it would have taken itself.
int default_helpers(int b, int n) {
    if (n > kHelperMaxN) return 0;
    const int h = pcm_device_cus() / b - 1;
    return h < 0 ? 0 : (h > kMaxHelpers ? kMaxHelpers : h);
}

int launch_emd(const float *xyz1, const float *xyz2, int b, int n, float eps, int iters, float *dist,
               int32_t *assignment, float *price, void *workspace, size_t workspace_bytes, int helpers,
               int offload_min, int diag, int wsplit, int tail_max, int32_t *stats, void *stream,
               int spin_limit = kSpinLimit) {
    // emd_cuda.cu:236-249 (n == m is enforced by the single n here)
    if (b < 0 || n < 0 || b > 512 || n % 1024 != 0 || iters < 1) return PCM_ERR_INVALID_ARG;
    if (b == 0 || n == 0) return PCM_OK;
    if (n > (1 << kTieKBits)) return PCM_ERR_UNSUPPORTED;  // object ids in the tie keys
    if (!xyz1 || !xyz2 || !dist || !assignment) return PCM_ERR_INVALID_ARG;
    const size_t need = ws_layout(b, n, nullptr, nullptr);
    if (!workspace || workspace_bytes < need) return PCM_ERR_WORKSPACE;
    EmdWs ws;
    ws_layout(b, n, &ws, (char *)workspace);
    hipStream_t s = (hipStream_t)stream;

    // seed
    const bool seed_stage = n <= kStageMaxN;
    const unsigned seed_blocks = (unsigned)((size_t)b * n / kSeedPts);
    const size_t seed_lds = seed_stage ? 12 * (size_t)n + (n == kStagePN ? kSeedThreads / 64 * kR * 8 : 0) : 0;
    if (seed_stage) {
        if (seed_lds > 64 * 1024 &&
            hipFuncSetAttribute((const void *)emd_seed_kernel<true, false>,  // n > 5461: not the reserve form
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)seed_lds) != hipSuccess)
            return PCM_ERR_LAUNCH;
        if (n == kStagePN)
            hipLaunchKernelGGL((emd_seed_kernel<true, true>), dim3(seed_blocks), dim3(kSeedThreads), seed_lds, s,
                               xyz1, xyz2, b, n, eps, ws);
        else
            hipLaunchKernelGGL((emd_seed_kernel<true, false>), dim3(seed_blocks), dim3(kSeedThreads), seed_lds, s,
                               xyz1, xyz2, b, n, eps, ws);
    } else {
        hipLaunchKernelGGL((emd_seed_kernel<false, false>), dim3(seed_blocks), dim3(kSeedThreads), 0, s, xyz1, xyz2,
                           b, n, eps, ws);
    }

    // auction
    int H = helpers >= 0 ? helpers : default_helpers(b, n);
    if (n > kHelperMaxN) H = 0;
    if (H > kMaxHelpers) H = kMaxHelpers;
    const bool g_state = n > kLdsStateMaxN;
    const bool stage = n <= (g_state ? kStageMaxN : kLdsStateMaxN);
    const size_t xchg = 5 * (size_t)kEmdThreads * 4;
    const bool stage_p = n <= (g_state ? 4096 : kStagePN);  // !g_state: n == kStagePN exactly
    const bool res = !g_state && stage_p;  // n == kStagePN: the reserve form (bounds + counts in LDS)
    const size_t m_lds = (g_state ? 0 : 48 * (size_t)n + 8) + (stage ? 12 * (size_t)n : 0) + (stage_p ? 12 * (size_t)n : 0) +
                         xchg + (res ? 8 * (size_t)n : 0);
    const size_t h_lds = H > 0 ? (stage ? 12 * (size_t)n : 0) + 4 * (size_t)n : 0;
    size_t lds = m_lds > h_lds ? m_lds : h_lds;
    // one workgroup per CU when helpers run: a master never shares its SIMDs
    if (H > 0 && lds < 84 * 1024) lds = 84 * 1024;
    KArgs ka{xyz1, xyz2, b, n, iters, H, offload_min >= 0 ? offload_min : kDefaultOffloadMin,
             stats ? (diag >= kDiagTimers ? diag : kDiagHist) : 0,
             wsplit > 0 ? wsplit : kDefaultWsplit, tail_max >= 0 ? tail_max : kDefaultTailMax,
             spin_limit >= 0 ? spin_limit : kSpinLimit, eps, dist, assignment, price, stats};
    const unsigned grid = (unsigned)(b * (1 + H));
    auto launch = [&](auto kfn) -> int {
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
                hipSuccess)
            return PCM_ERR_LAUNCH;
        hipLaunchKernelGGL(kfn, dim3(grid), dim3(kEmdThreads), lds, s, ka, ws);
        return PCM_OK;
    };
    int rc;
    if (!g_state) rc = stage_p ? launch(emd_auction_kernel<false, true, true>)
                               : launch(emd_auction_kernel<false, true, false>);
    else if (stage) rc = stage_p ? launch(emd_auction_kernel<true, true, true>)
                                 : launch(emd_auction_kernel<true, true, false>);
    else rc = launch(emd_auction_kernel<true, false, false>);
    if (rc != PCM_OK) return rc;
    return pcm_launch_status();
}
}  // namespace

extern "C" int pcm_emd_forward(const float *xyz1, const float *xyz2, int b, int n, float eps,
                               int iters, float *dist, int32_t *assignment, float *price,
                               void *workspace, size_t workspace_bytes, void *stream) {
    return launch_emd(xyz1, xyz2, b, n, eps, iters, dist, assignment, price, workspace, workspace_bytes, -1, -1, 0,
                      0, -1, nullptr, stream);
}

// Tuning / diagnostics entry.  helpers, offload_min < 0: the defaults.
// stats (caller zero-fills 3*iters + 16 + b int32) with diag 1: stats[2*it] +=
// unassigned points, stats[2*it+1] += full scans (summed over the batch),
// stats[2*iters + 10/11/12] = jobs / offloaded items / helper wake-ups,
// stats[2*iters + 13] = misses bid from the reserve (no full scan); with
// diag 2: stats[2*iters + 0..7] = batch-0 phase cycles / 16 (bids, full scans,
// claim, assign; sub-phases 4..7), stats[2*iters + 8] = iterations with
// bidders.  Both: stats[3*iters + 16 + i] = auction wall time of batch
// element i (10 ns units).  (diag 1's atomics perturb the timing.)
extern "C" int pcm_tune_emd_forward_cfg(const float *xyz1, const float *xyz2, int b, int n, float eps, int iters,
                                        float *dist, int32_t *assignment, float *price, void *workspace,
                                        size_t workspace_bytes, int helpers, int offload_min, int diag,
                                        int wsplit, int tail_max, int spin_limit, int32_t *stats, void *stream) {
    return launch_emd(xyz1, xyz2, b, n, eps, iters, dist, assignment, price, workspace, workspace_bytes, helpers,
                      offload_min, diag, wsplit, tail_max, stats, stream, spin_limit);
}

namespace {
// batch elements of the last forward on `workspace` whose master timed out
// on a helper job (and scanned those items itself); synchronises `stream`
int emd_timeouts(const void *workspace, size_t workspace_bytes, int b, int n, void *stream) {
    if (b <= 0 || n <= 0) return 0;
    if (!workspace || workspace_bytes < ws_layout(b, n, nullptr, nullptr)) return PCM_ERR_WORKSPACE;
    EmdWs ws;
    ws_layout(b, n, &ws, (char *)workspace);
    int count = 0;
    for (int i = 0; i < b; ++i) {
        int32_t err = 0;
        if (hipMemcpyAsync(&err, ws.board + (size_t)i * kBoardWords + kBoardErr, 4, hipMemcpyDeviceToHost,
                           (hipStream_t)stream) != hipSuccess ||
            hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
            return PCM_ERR_LAUNCH;
        count += err ? 1 : 0;
    }
    return count;
}
}  // namespace

// Status of the last pcm_emd_forward on this workspace; synchronises `stream`.
// Every wait between the auction's workgroups is bounded and a timed-out
// helper job is scanned by the master itself, so the outputs never depend on
// helper residency: PCM_OK unless reading the workspace fails.
extern "C" int pcm_emd_workspace_status(const void *workspace, size_t workspace_bytes, int b, int n,
                                        void *stream) {
    const int t = emd_timeouts(workspace, workspace_bytes, b, n, stream);
    return t < 0 ? t : PCM_OK;
}

// diagnostics: how many batch elements of the last forward had a helper job
// time out (>= 0), or a negative pcm_status
extern "C" int pcm_tune_emd_timeouts(const void *workspace, size_t workspace_bytes, int b, int n, void *stream) {
    return emd_timeouts(workspace, workspace_bytes, b, n, stream);
}

#ifdef PCM_STAMPS
extern "C" int pcm_tune_emd_xcc(int *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_emd_xcc), sizeof(int) * 1024, 0, hipMemcpyDeviceToHost) == hipSuccess
               ? 0 : PCM_ERR_LAUNCH;
}
#endif

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
