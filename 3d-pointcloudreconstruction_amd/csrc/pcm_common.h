// pcm_common.h -- shared device helpers for the gfx950 point-set metric kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pcm.h"

#define PCM_INF __builtin_huge_valf()

typedef float pcm_f2 __attribute__((ext_vector_type(2)));
typedef float pcm_f4 __attribute__((ext_vector_type(4)));

// Squared distance in the pinned evaluation order shared with the oracle
// (oracle/pcm_oracle.c: sqd_pinned) -- NVCC's contraction of the reference
// expression x2*x2+y2*y2+z2*z2 (chamfer3D.cu:35).  Explicit fmas, so the
// result does not depend on -ffp-contract.
__device__ __forceinline__ float pcm_sqd(float dx, float dy, float dz) {
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

__device__ __forceinline__ pcm_f2 pcm_sqd2(pcm_f2 dx, pcm_f2 dy, pcm_f2 dz) {
    return __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
}

// (d, k) <- lexicographic min of (d, k) and (dv, kv), branch-free: bitwise
// ops instead of || / && keep hipcc from turning the update into exec-mask
// branches that serialise the surrounding loads
__device__ __forceinline__ void pcm_lexmin(float &d, int &k, float dv, int kv) {
    const bool take = (dv < d) | ((dv == d) & (kv < k));
    d = take ? dv : d;
    k = take ? kv : k;
}

// Wave-wide lexicographic (d, k) minimum by DPP row_shr 1/2/4/8 then
// row_bcast 15/31 (VALU operand modifiers, no LDS round trip); the result is
// returned wave-uniform from lane 63.  Lanes a pattern does not feed keep
// their own pair (old = self), and a lexmin with itself is a no-op.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void pcm_lexmin_dpp_step(float &d, int &k) {
    const float dv = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(d), __float_as_int(d), CTRL, ROWMASK,
                                                                0xf, false));
    const int kv = __builtin_amdgcn_update_dpp(k, k, CTRL, ROWMASK, 0xf, false);
    pcm_lexmin(d, k, dv, kv);
}
__device__ __forceinline__ void pcm_wave_lexmin(float &d, int &k) {
    pcm_lexmin_dpp_step<0x111, 0xf>(d, k);  // row_shr:1
    pcm_lexmin_dpp_step<0x112, 0xf>(d, k);  // row_shr:2
    pcm_lexmin_dpp_step<0x114, 0xf>(d, k);  // row_shr:4
    pcm_lexmin_dpp_step<0x118, 0xf>(d, k);  // row_shr:8
    pcm_lexmin_dpp_step<0x142, 0xa>(d, k);  // row_bcast:15
    pcm_lexmin_dpp_step<0x143, 0xc>(d, k);  // row_bcast:31
    d = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), 63));
    k = __builtin_amdgcn_readlane(k, 63);
}

// Full-wave inclusive steps by DPP (row_shr 1, 2, 4, 8, then row_bcast 15 and
// 31; lane 63 holds the wave's result): VALU operand modifiers, where
// __shfl_xor lowers to six dependent ds_bpermute LDS round trips.  A lane the
// pattern does not feed keeps its value (an idempotent or summing no-op);
// s_nop 1: two wait states before a DPP read of the previous instruction's
// result (asm is not hazard-checked).  Full wave, uniform control flow.
#define PCM_DPP_WAVE_STEPS(OP)                                                   \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"      \
    "s_nop 1\n\t" OP " %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"   \
    "s_nop 1\n\t" OP " %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
// max over the wave of values that are not NaN, returned wave-uniform
__device__ __forceinline__ float pcm_wave_max_f32(float v) {
    asm volatile(PCM_DPP_WAVE_STEPS("v_max_f32_dpp") : "+v"(v));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Inclusive prefix sum over a full wave by DPP (row_shr 1, 2, 4, 8 with
// shifted-in lanes reading 0, then row_bcast 15 and 31 into the later rows):
// six VALU steps, where a __shfl_up loop is six dependent ds_bpermute round
// trips.  Full wave, uniform control flow.
__device__ __forceinline__ int pcm_wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
    return x;
}

// Workgroup-wide OR with ONE barrier, for a full workgroup in uniform control
// flow.  HIP's __syncthreads_or re-reads the workgroup size from the dispatch
// packet (an s_load that the next LDS wait also waits for) and takes three
// barriers around an LDS atomic.  Here lane 0 of each wave writes the wave's
// ballot to its own slot of `flags` (nwaves ints in LDS), one barrier, and
// every thread ORs the slots.  A caller must not write `flags` again before
// one more barrier has passed (a loop alternates two arrays by parity), so a
// fast wave's next write never races a slow wave's read.
__device__ __forceinline__ int pcm_wg_or(bool p, int *flags, int nwaves) {
    const bool any = __ballot(p) != 0ull;
    if ((threadIdx.x & 63) == 0) flags[threadIdx.x >> 6] = any ? 1 : 0;
    __syncthreads();
    int r = 0;
    for (int w = 0; w < nwaves; ++w) r |= flags[w];
    return r;
}

__device__ __forceinline__ bool pcm_finite(float v) {
    return __builtin_isfinite(v);
}

// Input element types: fp32, or IEEE binary16 (BASELINE config 5) widened to
// fp32 on load -- exact, so every fp16 result equals the fp32 result on the
// widened cloud.
typedef _Float16 pcm_h;
__device__ __forceinline__ float pcm_ld(const float *p) { return *p; }
__device__ __forceinline__ float pcm_ld(const pcm_h *p) { return (float)*p; }
__device__ __forceinline__ void pcm_st(float *p, float v) { *p = v; }
__device__ __forceinline__ void pcm_st(pcm_h *p, float v) { *p = (pcm_h)v; }  // round to nearest even

// Layout of one batch element's cloud in global memory: coordinate d of point
// k at base[k * ps + d * ds].  Rows [n, 3] (ps 3, ds 1) are what the
// reference's wrapper hands over (dist_chamfer_3D.py:79-80 .contiguous());
// planes [3, n] (ps 1, ds n) are the generator's B x 3 x N output that
// train.py:163 passes as a transposed view (extension: no copy).  The batch
// stride is 3 n in both.
struct PcmLay {
    int ps, ds;
};
__device__ __forceinline__ PcmLay pcm_lay(int planes, int np) { return planes ? PcmLay{1, np} : PcmLay{3, 1}; }
__device__ __forceinline__ size_t pcm_at(PcmLay L, int k, int d) { return (size_t)k * L.ps + (size_t)d * L.ds; }

// Reference-exact single-query scan (NmDistanceKernel, chamfer3D.cu:12-134):
// 512-point tiles, best = d(first) per tile, strict '<' inside, strict '>'
// across tiles.  Used only when non-finite coordinates are present, where the
// tile boundaries decide which NaN wins.  `t` = target cloud [m,3] in global
// (layout L).
template <typename TIn>
__device__ inline void pcm_ref_nn_scan(float x1, float y1, float z1, const TIn *__restrict__ t,
                                       int m, float &out_d, int &out_i, PcmLay L = PcmLay{3, 1}) {
    float res = 0.f;
    int res_i = 0;
    for (int k2 = 0; k2 < m; k2 += 512) {
        const int end_k = min(m, k2 + 512) - k2;
        float best = 0.f;
        int best_i = 0;
        for (int k = 0; k < end_k; ++k) {
            const TIn *q = t + (size_t)(k2 + k) * L.ps;
            const float d = pcm_sqd(pcm_ld(q) - x1, pcm_ld(q + L.ds) - y1, pcm_ld(q + 2 * (size_t)L.ds) - z1);
            if (k == 0 || d < best) { best = d; best_i = k + k2; }
        }
        if (k2 == 0 || res > best) { res = best; res_i = best_i; }
    }
    out_d = res;
    out_i = res_i;
}

typedef __attribute__((address_space(3))) void pcm_lds_void;

// Asynchronous global -> LDS copy of `nbytes` (multiple of 4) by the W waves of
// a workgroup using LDS-DMA (global_load_lds_*): no VGPRs, no LDS-write
// instructions; the caller waits with `s_waitcnt vmcnt(0)` + a barrier before
// reading.  16 B per lane (1 KiB per wave-instruction) when both ends are
// 16-byte aligned and nbytes % 16 == 0, else 4 B per lane.
__device__ __forceinline__ void pcm_dma_to_lds(void *lds_dst, const void *src, int nbytes, int wave,
                                               int nwaves) {
    const int lane = threadIdx.x & 63;
    const char *g = (const char *)src;
    char *l = (char *)lds_dst;
    if (((((uintptr_t)g) | ((uintptr_t)l) | (uintptr_t)nbytes) & 15) == 0) {
        for (int k = wave; k * 1024 < nbytes; k += nwaves) {
            const int off = k * 1024 + lane * 16;
            if (off < nbytes)
                __builtin_amdgcn_global_load_lds((const void *)(g + off), (pcm_lds_void *)(l + k * 1024), 16,
                                                 0, 0);
        }
    } else {
        for (int k = wave; k * 256 < nbytes; k += nwaves) {
            const int off = k * 256 + lane * 4;
            if (off < nbytes)
                __builtin_amdgcn_global_load_lds((const void *)(g + off), (pcm_lds_void *)(l + k * 256), 4, 0,
                                                 0);
        }
    }
}

// 16-byte vector store with the sc1 (agent-scope, write-through) policy: the
// wide form of a relaxed agent-scope atomic store, for data-tagged granules
typedef unsigned pcm_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void pcm_st_sc1_x4(void *p, pcm_u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

// XCD-aware workgroup numbering.  The dispatcher places workgroup i on XCD
// i % 8 (MI355X: 8 XCDs, each with its own 4 MB L2).  Giving every XCD a
// contiguous range of logical ids keeps the workgroups of one batch element --
// which all read the same clouds -- on one L2 instead of fetching those clouds
// into all eight.  A bijection for any grid size; placement is only a speed
// assumption (nothing depends on it for correctness).
__device__ __forceinline__ int pcm_xcd_remap(int i, int g) {
    constexpr int kXcd = 8;
    const int per = g / kXcd, rem = g % kXcd;
    const int x = i % kXcd, s = i / kXcd;
    return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + s;
}

// Chamfer backward graddist element strides per direction (batch, point),
// read in place: an expanded scalar (stride 0, what torch.mean's backward can
// hand over) needs no materialising copy.  bs < 0: contiguous [b, n].
struct PcmGdStr {
    int bs1 = -1, ps1 = 1, bs2 = -1, ps2 = 1;
};

// Batch-major split of a two-direction grid (b elements, nblk1 direction-1
// and nblk2 direction-2 workgroups each): logical id -> (batch, direction,
// block).  With pcm_xcd_remap's contiguous ranges, both directions of one
// element -- which read the same two clouds -- share an XCD and its L2.
__device__ __forceinline__ void pcm_split_bm(int bid, int nblk1, int nblk2, int &batch, bool &first, int &blk) {
    const int per = nblk1 + nblk2;
    batch = bid / per;
    const int r = bid - batch * per;
    first = r < nblk1;
    blk = first ? r : r - nblk1;
}

// Compute units of the current device (256 on a whole MI355X; fewer on a
// compute partition).  Grids whose workgroups wait on each other are sized
// from it; 256 if the query fails.
static inline int pcm_device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 256;
    return cus;
}

static inline int pcm_launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? PCM_OK : PCM_ERR_LAUNCH;
}
