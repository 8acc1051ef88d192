// emd.hip -- auction-algorithm EMD for MI355X (gfx950, CDNA4).
//
// Replaces the reference's 7-launches-per-iteration host loop
// (metric/emd/emd_cuda.cu:256-269: clear, calc_unass_cnt, calc_unass_cnt_sum,
// calc_unass_idx, Bid, GetMax, Assign) by two launches for any `iters`:
//
//  1. emd_seed_kernel (all CUs, one wave per point): iteration 0's bids.  With
//     every price 0 the bid value v = (float)((3.0 - (double)sqrtf(d)) - 0.0)
//     is a monotone non-increasing function of the squared distance d, so the
//     nearest candidates by d are the top of the value list.  Each lane keeps
//     its top-3 keys (v_med3 insertion); the cache is every lane top-2 entry
//     above K* = max over lanes of the 3rd keys (ballot compaction, <= kL = 32
//     entries), and every uncached object has v <= T = v(-K*).  If the cached
//     second-best value exceeds T nothing outside the cache can enter the top
//     two, so the bid is exact; otherwise the point is flagged for a full scan.
//     A cache entry is (object id, s = sqrtf(d)): s does not depend on prices.
//
//  2. emd_auction_kernel (one persistent workgroup per batch element): every
//     auction iteration in-kernel with the whole auction state (assignment,
//     owner, price, max increment, claim) and both clouds in LDS, and
//     workgroup barriers only.  An unassigned point re-bids from its cache at
//     CURRENT prices (two double subtractions per entry; 16, 8 or 4 lanes per
//     point by bidder count, reduced with DPP row shifts): prices only rise,
//     so uncached values are still <= T and the same proof applies.  Points whose cache cannot prove the top two are
//     re-scanned by one wave each: selection on an fp32 approximation of the
//     values with a proven error bound, exact evaluation of the chosen
//     entries, cache rebuilt (exact scan as fallback).  (Measured and
//     rejected: a lock-free LDS queue letting waves start full scans before
//     every cache bid is placed, 408 -> 421 us; fewer lanes per point for
//     large bidder sets, 421 -> 436 us.)
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

#ifndef PCM_EMD_KL
#define PCM_EMD_KL 32
#endif
constexpr int kL = PCM_EMD_KL;     // cache slots per point (unused slots hold -1); <= 64
constexpr int kSelectSteps = 8;    // bisection steps when > kL entries clear K3
typedef int16_t cid_t;             // cached object id (n <= kEmdMaxN = 4096), -1 = unused
constexpr int kSeedThreads = 256;  // one wave per point, 4 points per workgroup
constexpr int kEmdThreads = 1024;  // auction workgroup (16 waves)
constexpr int kEmdMaxN = 4096;     // LDS-resident auction state: 9 x 4 B x n
constexpr int kEmdStageMaxN = 2048;  // + 24 B x n copies of both clouds up to here

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

// (a better than b) in bid order: larger value, then lower index
__device__ __forceinline__ bool vk_better(float va, int ka, float vb, int kb) {
    return va > vb || (va == vb && ka < kb);
}

// Top-2 triples (b1, k1, b2): best value, its (lowest) id, second largest
// value of the multiset.  Written as one asm block each: as C++ ternaries
// hipcc emits exec-mask branches plus NaN-canonicalising v_max pairs here.
// "Better" = larger value, then lower id (vk_better).  The trailing s_nop
// covers the VALU-write -> DPP-read hazard of the next reduction step, and
// the one before v_cndmask the VALU/SALU-SGPR-write -> lane-mask read.
//
// merge of two triples: b2 = max(min(b1, o1), max(b2, o2)), b1 = max(b1, o1)
__device__ __forceinline__ void top2_merge(float &b1, int &k1, float &b2, float o1, int ok1, float o2) {
    unsigned long long g, e, l;
    float t, u, n1, n2;
    asm("v_cmp_gt_f32_e64 %[g], %[o1], %[b1]\n\t"
        "v_cmp_eq_f32_e64 %[e], %[o1], %[b1]\n\t"
        "v_cmp_lt_i32_e64 %[l], %[ok1], %[k1]\n\t"
        "v_min_f32 %[t], %[b1], %[o1]\n\t"
        "v_max_f32 %[u], %[b2], %[o2]\n\t"
        "v_max_f32 %[n1], %[b1], %[o1]\n\t"
        "v_max_f32 %[n2], %[t], %[u]\n\t"
        "s_and_b64 %[e], %[e], %[l]\n\t"
        "s_or_b64 %[g], %[g], %[e]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[k1], %[k1], %[ok1], %[g]\n\t"
        "s_nop 1"
        : [k1] "+v"(k1), [t] "=&v"(t), [u] "=&v"(u), [n1] "=&v"(n1), [n2] "=&v"(n2), [g] "=&s"(g),
          [e] "=&s"(e), [l] "=&s"(l)
        : [o1] "v"(o1), [ok1] "v"(ok1), [o2] "v"(o2), [b1] "v"(b1), [b2] "v"(b2));
    b1 = n1;
    b2 = n2;
}
// push of one entry (v, k): b2 = med3(b1, b2, v), b1 = max(b1, v)
__device__ __forceinline__ void top2_push(float &b1, int &k1, float &b2, float v, int k) {
    unsigned long long g, e, l;
    float n1, n2;
    asm("v_cmp_gt_f32_e64 %[g], %[v], %[b1]\n\t"
        "v_cmp_eq_f32_e64 %[e], %[v], %[b1]\n\t"
        "v_cmp_lt_i32_e64 %[l], %[k], %[k1]\n\t"
        "v_med3_f32 %[n2], %[b1], %[b2], %[v]\n\t"
        "v_max_f32 %[n1], %[b1], %[v]\n\t"
        "s_and_b64 %[e], %[e], %[l]\n\t"
        "s_or_b64 %[g], %[g], %[e]\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %[k1], %[k1], %[k], %[g]\n\t"
        "s_nop 1"
        : [k1] "+v"(k1), [n1] "=&v"(n1), [n2] "=&v"(n2), [g] "=&s"(g), [e] "=&s"(e), [l] "=&s"(l)
        : [v] "v"(v), [k] "v"(k), [b1] "v"(b1), [b2] "v"(b2));
    b1 = n1;
    b2 = n2;
}

// ---- DPP cross-lane steps (VALU operand modifiers: no LDS crossbar round trip).
// Lanes the DPP pattern does not feed keep their own value (old = self), so a
// combine with it is a no-op for idempotent selections.  Hillis-Steele:
// row_shr 1,2,4,8 leaves each 16-lane row's result in its lane 15; row_bcast
// 15 and 31 then carry it across rows so lane 63 holds the wave's result.
constexpr int kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118;
constexpr int kDppRowBcast15 = 0x142, kDppRowBcast31 = 0x143;

template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i(int x) {
    return __builtin_amdgcn_update_dpp(x, x, CTRL, ROWMASK, 0xf, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL, ROWMASK,
                                                      0xf, false));
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ void dpp_top2_step(float &b1, int &k1, float &b2) {
    const float ob1 = dpp_f<CTRL, ROWMASK>(b1);
    const int ok1 = dpp_i<CTRL, ROWMASK>(k1);
    const float ob2 = dpp_f<CTRL, ROWMASK>(b2);
    top2_merge(b1, k1, b2, ob1, ok1, ob2);
}

// full-wave reductions: result returned wave-uniform (read from lane 63)
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_f<kDppRowShr1, 0xf>(v));
    v = fmaxf(v, dpp_f<kDppRowShr2, 0xf>(v));
    v = fmaxf(v, dpp_f<kDppRowShr4, 0xf>(v));
    v = fmaxf(v, dpp_f<kDppRowShr8, 0xf>(v));
    v = fmaxf(v, dpp_f<kDppRowBcast15, 0xa>(v));
    v = fmaxf(v, dpp_f<kDppRowBcast31, 0xc>(v));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// ===========================================================================
// Candidate scan + cache selection by ONE wave (64 lanes) for one point.
//
// A cache entry is (object id, s = sqrtf(d)): s does not depend on prices, so
// re-evaluating a cached object later costs the two double subtractions of
// emd_cuda.cu:146 and nothing else.
//
// Selection (no sorting, no extraction rounds): with key = "larger is better,
// lower object index on ties", each lane keeps its top-2 (key, k, d) and its
// 3rd-best key.  Cache = every lane-top-2 entry strictly above K3 = max over
// lanes of the 3rd-best keys (~30 on random clouds): every other object lies
// at or below K3 -- it is either outside its lane's top-2 (<= that lane's 3rd
// <= K3) or a top-2 entry not above K3.  If more than kL qualify (common:
// ~30 is the typical count), the threshold is raised by bisection between K3
// and the largest key until at most kL lane-top-2 entries lie above it; the
// bound then stays exact for every uncached key.  (The earlier fallback -- the
// lane-top-1 entries above K2 = max of the 2nd keys -- loses the global
// second best whenever it shares a lane with the best, which sent ~4% of the
// auction's full scans to the exact re-scan.)  Ballots, popcounts, mbcnt.
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
// '>' while k ascends, so equal keys keep the lower index.  (fmed3 takes its
// operands as they are: no NaN-canonicalising v_max per loop-carried value.)
// The id selects are spelled out as v_cmp/v_cndmask in one asm block:
// written as ternaries, hipcc turns them into exec-mask branches inside the
// scan loop.  gfx950 needs two wait states between a VALU SGPR write and a
// v_cndmask reading it as the lane mask (s_nop 1).
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

// squared distance of a lane's entry (recomputed in the pinned order, so it
// is bit-identical to the value the scan used)
__device__ __forceinline__ float entry_d(float x1, float y1, float z1, const float *Qc, int n, int q) {
    return (unsigned)q < (unsigned)n ? sqd_to(x1, y1, z1, Qc + 3 * (size_t)q) : 0.f;
}

// picks the cache entries; writes the ids and s = sqrtf(d) of the chosen
// entries into cidx/cs (unused slots: id -1).  Returns K* (every uncached
// key <= K*) or +inf when nothing could be cached.  s1/s2: this lane's
// entries chosen; d1/d2: their squared distances.
__device__ __forceinline__ float select_cache(const LaneTop &t, float d1, float d2, cid_t *__restrict__ cidx,
                                              float *__restrict__ cs, bool &s1, bool &s2) {
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
    if (lane < kL && lane >= cnt) cidx[lane] = -1;  // unused slots
    if (s1) {
        const int p = __popcll(m1 & below);
        cidx[p] = (cid_t)t.q1;
        if (cs) cs[p] = __builtin_sqrtf(d1);
    }
    if (s2) {
        const int p = __popcll(m1) + __popcll(m2 & below);
        cidx[p] = (cid_t)t.q2;
        if (cs) cs[p] = __builtin_sqrtf(d2);
    }
    return Kstar;
}

// exact (best, argbest, better) over the wave: each lane offers up to two
// (value, id) entries; result wave-uniform
__device__ __forceinline__ void wave_top2(float v1, int k1, float v2, int k2, float &b1, int &kb, float &b2) {
    if (vk_better(v2, k2, v1, k1)) {
        const float tv = v1; v1 = v2; v2 = tv;
        const int tk = k1; k1 = k2; k2 = tk;
    }
    b1 = v1; kb = k1; b2 = v2;
    dpp_top2_step<kDppRowShr1, 0xf>(b1, kb, b2);
    dpp_top2_step<kDppRowShr2, 0xf>(b1, kb, b2);
    dpp_top2_step<kDppRowShr4, 0xf>(b1, kb, b2);
    dpp_top2_step<kDppRowShr8, 0xf>(b1, kb, b2);
    dpp_top2_step<kDppRowBcast15, 0xa>(b1, kb, b2);
    dpp_top2_step<kDppRowBcast31, 0xc>(b1, kb, b2);
    b1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b1), 63));
    kb = __builtin_amdgcn_readlane(kb, 63);
    b2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b2), 63));
}

// ---- seed: key = -d (every price is 0: the bid value is monotone
// non-increasing in d).  T = v(-K*) bounds every uncached value.  The bid is
// exact whenever b2 > T (caller checks).
__device__ __forceinline__ void scan_seed(float x1, float y1, float z1, const float *Qc, int n,
                                          cid_t *__restrict__ cidx, float *__restrict__ cs,
                                          float &b1, int &kb, float &b2, float &T) {
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
    const float Kstar = select_cache(t, d1, d2, cidx, cs, s1, s2);
    T = Kstar == PCM_INF ? PCM_INF : value_of(-Kstar, 0.f);
    wave_top2(s1 ? value_of(d1, 0.f) : -PCM_INF, s1 ? t.q1 : 0x7fffffff,
              s2 ? value_of(d2, 0.f) : -PCM_INF, s2 ? t.q2 : 0x7fffffff, b1, kb, b2);
}

// ---- auction full scan, exact: key = the exact bid value.  Always exact
// bid (the lanes' top-2 hold the global top-2); T = K*.
__device__ __noinline__ void scan_exact(float x1, float y1, float z1, const float *Qc,
                                        const float *sPrice, int n, cid_t *__restrict__ cidx,
                                        float *__restrict__ cs, float &b1, int &kb, float &b2,
                                        float &T) {
    const int lane = threadIdx.x & 63;
    LaneTop t;
    lane_top_init(t);
    for (int k0 = lane; k0 < n; k0 += 4 * 64) {
        float key[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = k0 + 64 * r;
            key[r] = value_of(sqd_to(x1, y1, z1, Qc + 3 * (size_t)k), sPrice[k]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) lane_top_push(t, key[r], k0 + 64 * r);
    }
    bool s1, s2;
    T = select_cache(t, entry_d(x1, y1, z1, Qc, n, t.q1), entry_d(x1, y1, z1, Qc, n, t.q2), cidx, cs, s1, s2);
    wave_top2(t.a1, t.q1, t.a2, t.q2, b1, kb, b2);
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
// instead (~4% of scans).  Returns false when that fallback is needed.
// approximate keys of objects [kbeg, kend) (a multiple of 256 long) into t
__device__ __forceinline__ void scan_fast_keys(LaneTop &t, float x1, float y1, float z1, const float *Qc,
                                               const float *sPrice, int kbeg, int kend) {
    const int lane = threadIdx.x & 63;
    for (int k0 = kbeg + lane; k0 < kend; k0 += 4 * 64) {
        float key[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = k0 + 64 * r;
            key[r] = (3.f - __builtin_amdgcn_sqrtf(sqd_to(x1, y1, z1, Qc + 3 * (size_t)k))) - sPrice[k];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) lane_top_push(t, key[r], k0 + 64 * r);
    }
}

// selection, bound and exact bid from the lanes' approximate-key tops
__device__ __forceinline__ bool scan_fast_finish(const LaneTop &t, float x1, float y1, float z1,
                                                 const float *Qc, const float *sPrice, int n,
                                                 cid_t *__restrict__ cidx, float *__restrict__ cs, float &b1,
                                                 int &kb, float &b2, float &T) {
    bool s1, s2;
    const float d1 = entry_d(x1, y1, z1, Qc, n, t.q1), d2 = entry_d(x1, y1, z1, Qc, n, t.q2);
    const float Kp = select_cache(t, d1, d2, cidx, cs, s1, s2);
    T = Kp + 4.f * 1.1920929e-7f * (6.f + fabsf(Kp));  // +inf stays +inf
    // exact values of this lane's cached entries
    const float v1 = s1 ? value_of(d1, sPrice[t.q1]) : -PCM_INF;
    const float v2 = s2 ? value_of(d2, sPrice[t.q2]) : -PCM_INF;
    wave_top2(v1, s1 ? t.q1 : 0x7fffffff, v2, s2 ? t.q2 : 0x7fffffff, b1, kb, b2);
    return b2 > T;
}

__device__ __forceinline__ bool scan_fast(float x1, float y1, float z1, const float *Qc,
                                          const float *sPrice, int n, cid_t *__restrict__ cidx,
                                          float *__restrict__ cs, float &b1, int &kb, float &b2,
                                          float &T) {
    LaneTop t;
    lane_top_init(t);
    scan_fast_keys(t, x1, y1, z1, Qc, sPrice, 0, n);
    return scan_fast_finish(t, x1, y1, z1, Qc, sPrice, n, cidx, cs, b1, kb, b2, T);
}

// ===========================================================================
// 1. seed kernel: iteration-0 bids + caches, one wave per point
// ===========================================================================
__global__ __launch_bounds__(kSeedThreads) void emd_seed_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int n, float eps,
    cid_t *__restrict__ cache_idx, float *__restrict__ cache_s, float *__restrict__ cache_T,
    int32_t *__restrict__ bid0, float *__restrict__ inc0) {
    const int pt = pcm_xcd_remap((int)blockIdx.x, (int)gridDim.x) * (kSeedThreads / 64) + (threadIdx.x >> 6);
    const int batch = pt / n;
    const int j = pt - batch * n;
    const float *P = xyz1 + (size_t)batch * n * 3;
    const float *Qc = xyz2 + (size_t)batch * n * 3;
    float b1, b2, T;
    int kb;
    scan_seed(P[3 * j], P[3 * j + 1], P[3 * j + 2], Qc, n, cache_idx + (size_t)pt * kL,
              cache_s + (size_t)pt * kL, b1, kb, b2, T);
    if ((threadIdx.x & 63) == 0) {
        cache_T[pt] = T;
        const bool proven = b2 > T && (unsigned)kb < (unsigned)n;
        bid0[pt] = proven ? kb : -2;  // -2: needs a full scan in the auction kernel
        inc0[pt] = b1 - b2 + eps;
    }
}

// ===========================================================================
// Cache bids: G lanes per bidder, kL/G cached (id, s) entries per lane at
// current prices, a row_shr reduction over the G lanes (G divides the 16-lane
// DPP row); the group's last lane places the bid or lists a full scan.
// ===========================================================================
#ifndef PCM_EMD_FORCE_G
__device__ __forceinline__ int cache_bid_lanes(int nu) {
    // measured per bidder count on MI355X (tools/tune_emd.py, profiles/r01):
    // few bidders are latency-bound (more lanes per bidder), many are
    // VALU-bound (fewer lanes, fewer reduction steps per bidder)
    return nu <= 64 ? 16 : (nu <= 256 ? 8 : 4);
}
#else
__device__ __forceinline__ int cache_bid_lanes(int) { return PCM_EMD_FORCE_G; }
#endif

template <int G>
__device__ __forceinline__ void cache_bids(int nu, float eps, const int *sU, const cid_t *C, const float *CS,
                                           const float *CT, const float *sPrice, int *sBid, float *sInc, int *sMax,
                                           int *sMiss, int *sNm) {
    static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "G lanes inside one DPP row");
    static_assert(kL % G == 0, "entries split evenly");
    constexpr int E = kL / G;
    const int gi = threadIdx.x / G, gl = threadIdx.x % G;
    for (int u0 = 0; u0 < nu; u0 += kEmdThreads / G) {
        const int u = u0 + gi;
        const bool act = u < nu;
        const int j = act ? sU[u] : 0;
        const float tj = CT[j];
        int ke[E];
        float se[E];
#pragma unroll
        for (int e = 0; e < E; ++e) ke[e] = C[(size_t)j * kL + gl + G * e];  // -1: unused slot
#pragma unroll
        for (int e = 0; e < E; ++e) se[e] = CS[(size_t)j * kL + gl + G * e];
        float b1 = -PCM_INF, b2 = -PCM_INF;
        int kb = 0x7fffffff;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            // branch-free: an unused slot (k = -1) evaluates object 0 and is
            // then forced to (-inf, INT_MAX)
            const int k = ke[e];
            const int neg = k >> 31;
            const float v0 = value_from_s(se[e], sPrice[k & ~neg]);
            const float v = __int_as_float((__float_as_int(v0) & ~neg) | (int)(0xff800000u & (unsigned)neg));
            top2_push(b1, kb, b2, v, k & 0x7fffffff);
        }
        if constexpr (G >= 2) dpp_top2_step<kDppRowShr1, 0xf>(b1, kb, b2);
        if constexpr (G >= 4) dpp_top2_step<kDppRowShr2, 0xf>(b1, kb, b2);
        if constexpr (G >= 8) dpp_top2_step<kDppRowShr4, 0xf>(b1, kb, b2);
        if constexpr (G >= 16) dpp_top2_step<kDppRowShr8, 0xf>(b1, kb, b2);
        if (act && gl == G - 1) {
            if (b2 > tj) {
                sBid[j] = kb;
                sInc[j] = b1 - b2 + eps;
                atomicMax(&sMax[kb], f2key(b1 - b2 + eps));
            } else {
                sMiss[atomicAdd(sNm, 1)] = j;
            }
        }
    }
}

// ===========================================================================
// 2. auction kernel: one workgroup per batch element, all iterations
// ===========================================================================

// kStage: both clouds are copied into LDS (LDS-DMA at kernel start) so the
// scans read them with LDS latency instead of L2/HBM latency (the seed kernel
// that last touched them ran on other XCDs, whose L2s this CU does not see).
// (Measured and rejected: the cached ids in LDS with s recomputed from the
// staged clouds -- fewer L2 round trips, more VALU: 287 -> 294 us.)
template <bool kStage>
__global__ __launch_bounds__(kEmdThreads) void emd_auction_kernel(
    const float *__restrict__ xyz1, const float *__restrict__ xyz2, int n, float eps, int iters,
    cid_t *__restrict__ cache_idx, float *__restrict__ cache_s, float *__restrict__ cache_T,
    const int32_t *__restrict__ bid0,
    const float *__restrict__ inc0, float *__restrict__ dist, int32_t *__restrict__ assignment_out,
    float *__restrict__ price_out, int32_t *__restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) int smem[];
    int *sAss = smem;                     // [n] assignment (point -> object)
    int *sInv = sAss + n;                 // [n] owner (object -> point)
    float *sPrice = (float *)(sInv + n);  // [n]
    int *sMax = (int *)(sPrice + n);      // [n] max increment (f2key)
    int *sClaim = sMax + n;               // [n] lowest qualifying bidder
    int *sBid = sClaim + n;               // [n] bid object per point
    float *sInc = (float *)(sBid + n);    // [n] bid increment per point
    int *sU = (int *)(sInc + n);          // [n] unassigned list
    int *sMiss = sU + n;                  // [n] points needing a full scan
    float *sQ = (float *)(sMiss + n);     // [3n] target cloud copy (kStage)
    float *sP = sQ + 3 * n;               // [3n] bidder cloud copy (kStage)
    __shared__ int sNu, sNm;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int batch = blockIdx.x;
    const float *Pg = xyz1 + (size_t)batch * n * 3;
    const float *Qg = xyz2 + (size_t)batch * n * 3;
    if (kStage) {
        pcm_dma_to_lds(sQ, Qg, 12 * n, wave, kEmdThreads / 64);
        pcm_dma_to_lds(sP, Pg, 12 * n, wave, kEmdThreads / 64);
    }
    const float *Qc = kStage ? (const float *)sQ : Qg;
    const float *P = kStage ? (const float *)sP : Pg;
    cid_t *C = cache_idx + (size_t)batch * n * kL;
    float *CS = cache_s + (size_t)batch * n * kL;
    float *CT = cache_T + (size_t)batch * n;

    for (int j = tid; j < n; j += kEmdThreads) {
        sAss[j] = -1;
        sInv[j] = -1;
        sPrice[j] = 0.f;
        sMax[j] = f2key(0.f);  // emd_module.py:49 zero-inits max_increments
        sClaim[j] = 0x7fffffff;
    }
    if (tid == 0) { sNu = 0; sNm = 0; }
    if (kStage) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA has landed
    __syncthreads();

    // diagnostics only (stats != nullptr): per-phase wall time of batch 0
    unsigned long long tprev = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t_start = tprev;
#define PCM_EMD_PHASE(i)                                                               \
    if (stats && tid == 0 && blockIdx.x == 0) {                                        \
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();               \
        atomicAdd(&stats[2 * iters + (i)], (int)(tn - tprev));                         \
        tprev = tn;                                                                    \
    }
    for (int it = 0; it < iters; ++it) {
        const bool last = (it == iters - 1);
        // ---- A: compact the unassigned points (order irrelevant downstream)
        for (int j0 = 0; j0 < n; j0 += kEmdThreads) {
            const int j = j0 + tid;
            const bool un = (j < n) && sAss[j] == -1;
            const unsigned long long bal = __ballot(un);
            int base = 0;
            if (lane == 0 && bal) base = atomicAdd(&sNu, __popcll(bal));
            base = __shfl(base, 0, 64);
            if (un) sU[base + __popcll(bal & ((1ull << lane) - 1ull))] = j;
        }
        __syncthreads();
        PCM_EMD_PHASE(0);
        const int nu = sNu;
        if (nu == 0) break;  // nothing left to bid: later iterations are no-ops

        // ---- B1: bids from the caches (16 lanes per point), misses listed
        if (it == 0) {
            for (int u = tid; u < nu; u += kEmdThreads) {
                const int j = sU[u];
                const int k = bid0[(size_t)batch * n + j];
                if (k >= 0) {
                    const float inc = inc0[(size_t)batch * n + j];
                    sBid[j] = k;
                    sInc[j] = inc;
                    atomicMax(&sMax[k], f2key(inc));
                } else {
                    sMiss[atomicAdd(&sNm, 1)] = j;
                }
            }
        } else {
            const int G = cache_bid_lanes(nu);
            if (G == 16) cache_bids<16>(nu, eps, sU, C, CS, CT, sPrice, sBid, sInc, sMax, sMiss, &sNm);
            else if (G == 8) cache_bids<8>(nu, eps, sU, C, CS, CT, sPrice, sBid, sInc, sMax, sMiss, &sNm);
            else if (G == 4) cache_bids<4>(nu, eps, sU, C, CS, CT, sPrice, sBid, sInc, sMax, sMiss, &sNm);
            else if (G == 2) cache_bids<2>(nu, eps, sU, C, CS, CT, sPrice, sBid, sInc, sMax, sMiss, &sNm);
            else cache_bids<1>(nu, eps, sU, C, CS, CT, sPrice, sBid, sInc, sMax, sMiss, &sNm);
        }
        __syncthreads();
        if (stats && tid == 0 && blockIdx.x == 0)  // per-iteration cache-bid time of batch 0
            stats[2 * iters + 16 + it] = (int)(__builtin_amdgcn_s_memrealtime() - tprev);
        PCM_EMD_PHASE(1);
#ifdef PCM_EMD_DIAG_B2
        const unsigned long long tB2 = tprev;  // diagnostics build: per-iteration full-scan phase time
#endif
        // ---- B2: full scans (one wave per missed point), cache rebuilt
        const int nm = sNm;
        if (stats && tid == 0) {  // diagnostics: [iter] -> (unassigned, full scans), summed over batches
            atomicAdd(&stats[2 * it], nu);
            atomicAdd(&stats[2 * it + 1], nm);
        }
        for (int q = wave; q < nm; q += kEmdThreads / 64) {
            const int j = sMiss[q];
            float b1, b2, T;
            int kb;
            const float x1 = P[3 * j], y1 = P[3 * j + 1], z1 = P[3 * j + 2];
            cid_t *cj = C + (size_t)j * kL;
            float *sj = CS + (size_t)j * kL;
            const unsigned long long ts0 = stats ? __builtin_amdgcn_s_memrealtime() : 0ull;
            const bool fast_ok = scan_fast(x1, y1, z1, Qc, sPrice, n, cj, sj, b1, kb, b2, T);
            const unsigned long long ts1 = stats ? __builtin_amdgcn_s_memrealtime() : 0ull;
            if (!fast_ok) scan_exact(x1, y1, z1, Qc, sPrice, n, cj, sj, b1, kb, b2, T);
            if (stats && lane == 0) {  // diagnostics: fallbacks; wave-0 scan times of batch 0
                if (!fast_ok) atomicAdd(&stats[2 * iters + 6], 1);
                if (blockIdx.x == 0 && wave == 0) {
                    const unsigned long long ts2 = __builtin_amdgcn_s_memrealtime();
                    atomicAdd(&stats[2 * iters + 7], 1);
                    atomicAdd(&stats[2 * iters + 8], (int)(ts1 - ts0));
                    atomicAdd(&stats[2 * iters + 9], (int)(ts2 - ts1));
                }
            }
            if (lane == 0) {
                CT[j] = T;
                const float inc = b1 - b2 + eps;
                const bool valid = (unsigned)kb < (unsigned)n;  // all-NaN values: no bid (oracle: best_i = -1)
                sBid[j] = valid ? kb : -1;
                sInc[j] = inc;
                if (valid) atomicMax(&sMax[kb], f2key(inc));
            }
        }
        __syncthreads();
        PCM_EMD_PHASE(2);
#ifdef PCM_EMD_DIAG_B2
        if (stats && tid == 0 && blockIdx.x == 0) stats[2 * iters + 16 + it] = (int)(tprev - tB2);
#endif

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
        PCM_EMD_PHASE(3);

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
        PCM_EMD_PHASE(4);
        for (int u = tid; u < nu; u += kEmdThreads) {
            const int k = sBid[sU[u]];
            if (k >= 0) sClaim[k] = 0x7fffffff;
        }
        if (tid == 0) { sNu = 0; sNm = 0; }
        __syncthreads();
        PCM_EMD_PHASE(5);
    }

    if (stats && tid == 0)  // diagnostics: whole-auction wall time per batch element
        stats[3 * iters + 16 + blockIdx.x] = (int)(__builtin_amdgcn_s_memrealtime() - t_start);
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

size_t emd_lds_bytes(int n) { return (size_t)9 * 4 * n; }

// workspace layout: cache_idx [b*n*kL] i16 | cache_s [b*n*kL] f32 | cache_T [b*n] f32 |
//                   bid0 [b*n] i32 | inc0 [b*n] f32
size_t ws_bytes(int b, int n) {
    const size_t pts = (size_t)b * n;
    return pts * kL * (sizeof(cid_t) + 4) + pts * 4 * 3;
}

}  // namespace

extern "C" size_t pcm_emd_workspace_bytes(int b, int n) {
    if (b <= 0 || n <= 0) return 0;
    return ws_bytes(b, n);
}

namespace {
int launch_emd(const float *xyz1, const float *xyz2, int b, int n, float eps, int iters, float *dist,
               int32_t *assignment, float *price, void *workspace, size_t workspace_bytes,
               int32_t *stats, void *stream) {
    // emd_cuda.cu:236-249 (n == m is enforced by the single n here)
    if (b < 0 || n < 0 || b > 512 || n % 1024 != 0 || iters < 1) return PCM_ERR_INVALID_ARG;
    if (b == 0 || n == 0) return PCM_OK;
    if (!xyz1 || !xyz2 || !dist || !assignment) return PCM_ERR_INVALID_ARG;
    if (n > kEmdMaxN) return PCM_ERR_UNSUPPORTED;
    if (!workspace || workspace_bytes < ws_bytes(b, n)) return PCM_ERR_WORKSPACE;
    const size_t pts = (size_t)b * n;
    cid_t *cache_idx = (cid_t *)workspace;
    float *cache_s = (float *)(cache_idx + pts * kL);
    float *cache_T = cache_s + pts * kL;
    int32_t *bid0 = (int32_t *)(cache_T + pts);
    float *inc0 = (float *)(bid0 + pts);
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(emd_seed_kernel, dim3((unsigned)(pts / (kSeedThreads / 64))),
                       dim3(kSeedThreads), 0, s, xyz1, xyz2, n, eps, cache_idx, cache_s, cache_T, bid0, inc0);
    const bool stage = n <= kEmdStageMaxN;
    const size_t lds = emd_lds_bytes(n) + (stage ? (size_t)24 * n : 0);
    auto launch = [&](auto kfn) -> int {
        if (lds > 64 * 1024 &&
            hipFuncSetAttribute((const void *)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
                hipSuccess)
            return PCM_ERR_LAUNCH;
        hipLaunchKernelGGL(kfn, dim3(b), dim3(kEmdThreads), lds, s, xyz1, xyz2, n, eps, iters, cache_idx,
                           cache_s, cache_T, bid0, inc0, dist, assignment, price, stats);
        return PCM_OK;
    };
    const int rc = stage ? launch(emd_auction_kernel<true>) : launch(emd_auction_kernel<false>);
    if (rc != PCM_OK) return rc;
    return pcm_launch_status();
}
}  // namespace

extern "C" int pcm_emd_forward(const float *xyz1, const float *xyz2, int b, int n, float eps,
                               int iters, float *dist, int32_t *assignment, float *price,
                               void *workspace, size_t workspace_bytes, void *stream) {
    return launch_emd(xyz1, xyz2, b, n, eps, iters, dist, assignment, price, workspace, workspace_bytes,
                      nullptr, stream);
}

// diagnostics: stats[2*it] += unassigned points, stats[2*it+1] += full scans
// (summed over the batch; caller zero-fills int32[2*iters])
extern "C" int pcm_tune_emd_forward_stats(const float *xyz1, const float *xyz2, int b, int n, float eps,
                                          int iters, float *dist, int32_t *assignment,
                                          void *workspace, size_t workspace_bytes, int32_t *stats,
                                          void *stream) {
    return launch_emd(xyz1, xyz2, b, n, eps, iters, dist, assignment, nullptr, workspace,
                      workspace_bytes, stats, stream);
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
