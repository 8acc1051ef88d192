// chamfer_loss.h -- in-kernel loss hand-off shared by the Chamfer forward kernels
// (mean(dist1), mean(dist2) of loss/loss.py:36, reduced deterministically).
// Included inside an anonymous namespace by each kernel source.
#pragma once
#include "pcm_common.h"

namespace pcm_loss {

// Sum over a full wave, returned wave-uniform, by DPP steps (pcm_common.h):
// no LDS round trips on the way to the partial's publication.
__device__ __forceinline__ float wave_sum(float v) {
    asm volatile(PCM_DPP_WAVE_STEPS("v_add_f32_dpp") : "+v"(v));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}


// Arrival tickets are sharded two-level: one arrival counter per 128-byte line
// for each of kShards shards (block id mod kShards), and a top counter that
// only each shard's last arriver increments.  512 arrivals on ONE counter
// serialise at ~12 ns each (MI355X_MICROARCH.md price list, row "fanin");
// sharded, the tail sees ~16 + 32 arrivals.
constexpr int kShards = 32;
constexpr int kShardStride = 32;  // unsigned words = 128 B per counter line
constexpr size_t kTicketBytes = (size_t)(kShards + 1) * kShardStride * 4;  // then the partials

// Returns 1 in thread 0 of the overall last-arriving workgroup, else 0.  The
// caller tests it only after its remaining work, so the atomics' round trips
// overlap that work instead of stalling the workgroup at the next barrier.
template <int kMode = 1>
__device__ __forceinline__ unsigned publish_partial(float v, int slot, float *partials, unsigned *ticket,
                                                    float (*sRed)[16], unsigned epoch = 0) {
    // deterministic workgroup sum, then (tid 0) write-through store, drain,
    // agent atomic ticket (MI355X_MICROARCH.md visibility table, row 1)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float ws = wave_sum(v);
    if (lane == 0) sRed[0][wave] = ws;
    __syncthreads();
    unsigned last = 0;
    if (threadIdx.x == 0) {
        float s = 0.f;
        const int nw = blockDim.x >> 6;
        for (int w = 0; w < nw; ++w) s += sRed[0][w];
        if constexpr (kMode == 2) {  // reduced by chamfer_loss_finalize_kernel after the kernel boundary
            partials[slot] = s;
            return 0;
        }
        if constexpr (kMode == 3) {  // one {epoch, value} granule, swept by poll_loss
            __hip_atomic_store(reinterpret_cast<unsigned long long *>(partials) + slot,
                               ((unsigned long long)epoch << 32) | __float_as_uint(s), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            return 0;
        }
        __hip_atomic_store(&partials[slot], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned nb = gridDim.x;
        const unsigned sh = blockIdx.x % kShards;
        const unsigned in_shard = (nb - sh + kShards - 1) / kShards;
        const unsigned active = nb < kShards ? nb : kShards;
        const unsigned t = __hip_atomic_fetch_add(ticket + kShardStride * (1 + sh), 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        if (t == in_shard - 1) {
            const unsigned u = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = (u == active - 1);
        }
    }
    return last;
}

__device__ __forceinline__ void finish_loss(int nb1, int b, int n, int m, const float *partials,
                                            unsigned *ticket, float *mean_out, float (*sRed)[16]) {
    // the last-arriving workgroup: fixed-order reduction of every partial
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nbt = (int)gridDim.x;
    float s1 = 0.f, s2 = 0.f;
    for (int i = threadIdx.x; i < nbt; i += blockDim.x) {
        const float v = __hip_atomic_load(&partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
        // every arrival is in: re-arm the counters for the next stream-ordered call
        for (int s = 0; s <= kShards; ++s)
            __hip_atomic_store(ticket + kShardStride * s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Loss mode 3: the data is the flag.  Every producer workgroup stores its
// partial as ONE 8-byte {tag = epoch, value} granule (agent-scope relaxed
// store = sc1 write-through; MI355X_MICROARCH.md visibility, R2: no drain, no
// fence, no counter), and one extra workgroup -- the grid's last -- sweeps the
// granules with sc1 loads until every tag carries this call's epoch, then sums
// them in a fixed order.  The epoch lives in the workspace (word kEpochWord of
// the ticket line): producers and poller read it at start, the poller
// advances it at the end, so stream-ordered calls (and graph replays) never
// match a previous call's granules and nothing needs re-zeroing.  The poll is
// bounded: after kPollMaxSpins sweeps it writes NaN means, advances the epoch
// and sets the sticky error word kErrWord; every later call on the workspace
// then reports NaN means until the caller re-zeroes it (a producer that ran
// late could otherwise tag a granule with a later call's epoch).
// pcm_chamfer_workspace_status reads the word.
constexpr int kEpochWord = 1;
constexpr int kErrWord = 2;
constexpr unsigned kPollMaxSpins = 1u << 22;

__device__ __forceinline__ void poll_loss(int nb1, int nbt, int b, int n, int m,
                                          const unsigned long long *__restrict__ gran, unsigned *ticket,
                                          float *__restrict__ mean_out, unsigned max_spins = kPollMaxSpins) {
    if (threadIdx.x >= 64) return;  // one polling wave
    const int lane = threadIdx.x;
    const unsigned epoch = ticket[kEpochWord] + 1u;
    float s1 = 0.f, s2 = 0.f;
    bool ok = true;
    constexpr int R = 8;  // granules per lane per sweep
    for (int base = 0; base < nbt && ok; base += 64 * R) {
        unsigned long long x[R];
        for (unsigned spins = 0;; ++spins) {
            bool ready = true;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int i = base + r * 64 + lane;
                x[r] = i < nbt ? __hip_atomic_load(gran + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : ((unsigned long long)epoch << 32);
                ready &= (unsigned)(x[r] >> 32) == epoch;
            }
            if (__all(ready)) break;
            if (spins >= max_spins) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = base + r * 64 + lane;
            const float v = __uint_as_float((unsigned)x[r]);
            if (i < nb1) s1 += v;
            else if (i < nbt) s2 += v;
        }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
        if (!ok) __hip_atomic_store(ticket + kErrWord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = ok && ticket[kErrWord] == 0u;
        mean_out[0] = ok ? s1 / ((float)b * (float)n) : __builtin_nanf("");
        mean_out[1] = ok ? s2 / ((float)b * (float)m) : __builtin_nanf("");
        ticket[kEpochWord] = epoch;
    }
}

}  // namespace pcm_loss

// Forward kernel signature shared by every variant (both source files), and
// one row of the variant table (tools/tune_chamfer.py A/Bs them by index).
typedef void (*pcm_fwd_kernel_t)(const float *, const float *, int, int, int, float *, float *, int32_t *,
                                 int32_t *, int, int, float *, unsigned *, float *);
struct PcmFwdVariant {
    pcm_fwd_kernel_t plain, loss, loss2, loss3;  // loss: in-kernel ticket; loss2: partials + finalize
                                                 // kernel; loss3: granules + polling workgroup
    int waves, qpt;
    bool sgpr;  // SGPR-stream form (else LDS-staged)
};
// filtered-scan variants (chamfer_filt.hip), appended to chamfer.hip's table
extern const PcmFwdVariant kPcmFiltVariants[];
// chamfer_filt.hip: the slot-bucket backward (per-point graddists at strides GS)
bool pcm_bwd_slots_fits(int n, int m);
int pcm_launch_bwd_slots(const float *xyz1, const float *xyz2, int b, int n, int m, const float *gd1, const float *gd2,
                         const int32_t *idx1, const int32_t *idx2, float *grad1, float *grad2, int lay1, int lay2,
                         PcmGdStr GS, hipStream_t stream);
extern const int kPcmNumFiltVariants;

// fp16-cloud forward kernels (same signature on binary16 clouds)
typedef void (*pcm_fwd16_kernel_t)(const _Float16 *, const _Float16 *, int, int, int, float *, float *, int32_t *,
                                   int32_t *, int, int, float *, unsigned *, float *);
struct PcmFwd16Variant {
    pcm_fwd16_kernel_t k;
    int waves, qpt;
};
extern const PcmFwd16Variant kPcmFilt16Variants[];
extern const int kPcmNumFilt16Variants;

// One zero-filled workspace serves pcm_chamfer_forward_loss (its bytes first,
// chamfer.hip) and pcm_chamfer_loss_grad (the bytes after that offset,
// chamfer_filt.hip).
size_t pcm_chamfer_loss_ws_offset(int b, int n, int m);
size_t pcm_chamfer_grad_ws_bytes(int b, int n, int m);
int pcm_chamfer_grad_err_word(void);  // word index of the fused kernel's sticky error (its region)
