// dispatch_probe.hip -- how fast does the dispatcher start the workgroups of
// a one-wave-of-workgroups grid (the one-launch Chamfer step's shape: 257
// workgroups of 512 threads, 75 KB of LDS each)?  Every workgroup's thread 0
// stamps s_memrealtime (100 MHz) at entry; the body then spins for a fixed
// number of cycles so that all workgroups are resident together.  Prints, per
// shape, the spread of the start stamps (first -> last) and its quartiles.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/dispatch_probe tools/dispatch_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

template <int kThreads, int kLds>
__global__ __launch_bounds__(kThreads) void probe(unsigned long long *st, int spin, const float *big) {
    __shared__ float lds[kLds > 0 ? kLds / 4 : 1];
    if (threadIdx.x == 0) st[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    float acc = big ? big[0] : 0.f;
    if constexpr (kLds > 0) {
        lds[threadIdx.x] = acc;
        __syncthreads();
        acc += lds[(threadIdx.x + 1) % kThreads];
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < (unsigned long long)spin) acc = acc * 1.0001f + 1.f;
    if (threadIdx.x == 0) st[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() + (acc == 12345.f);
}

template <int kThreads, int kLds>
void run(const char *name, int blocks, int spin, unsigned long long *d, const float *big) {
    std::vector<double> spreads;
    std::vector<unsigned long long> h(2 * blocks);
    for (int rep = 0; rep < 20; ++rep) {
        probe<kThreads, kLds><<<blocks, kThreads>>>(d, spin, big);
        hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
        if (rep < 5) continue;
        unsigned long long lo = ~0ull, hi = 0;
        std::vector<unsigned long long> s(blocks);
        for (int b = 0; b < blocks; ++b) {
            s[b] = h[2 * b];
            lo = std::min(lo, s[b]);
            hi = std::max(hi, s[b]);
        }
        spreads.push_back((hi - lo) * 0.01);
    }
    std::sort(spreads.begin(), spreads.end());
    printf("%-40s blocks %4d threads %4d lds %6d B: start spread median %.2f us (min %.2f max %.2f)\n", name, blocks,
           kThreads, kLds, spreads[spreads.size() / 2], spreads.front(), spreads.back());
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 2 * 4096 * 8);
    float *big;
    hipMalloc(&big, 4096);
    hipMemset(big, 0, 4096);
    const int spin = 20000;  // ~10 us of s_memtime cycles at ~2 GHz
    run<512, 75464>("512 thr, 75 KB LDS (the fused step)", 257, spin, d, big);
    run<512, 75464>("512 thr, 75 KB LDS, 256 WGs", 256, spin, d, big);
    run<512, 16384>("512 thr, 16 KB LDS", 257, spin, d, big);
    run<512, 0>("512 thr, no LDS", 257, spin, d, big);
    run<256, 75464>("256 thr, 75 KB LDS", 257, spin, d, big);
    run<256, 36864>("256 thr, 36 KB LDS", 514, spin, d, big);
    run<1024, 75464>("1024 thr, 75 KB LDS", 129, spin, d, big);
    run<1024, 150000>("1024 thr, 150 KB LDS", 129, spin, d, big);
    run<256, 0>("256 thr, no LDS, 1024 WGs", 1024, spin, d, big);
    hipFree(d);
    hipFree(big);
    return 0;
}
