// MT19937 twist-only microbenchmark: how fast can one workgroup run the word recurrence
//   x[n] = x[n-681] ^ g(n-624) ^ g(n-851) ^ g(n-1078)        (623 independent words per round)
// as a function of the workgroup width, words per thread, LDS ring size and whether every word
// is also stored to HBM (the split sampler's k_mt).  Each variant is checked word for word
// against a host MT19937 of the same key.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mt_bench.hip -o tools/mt_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t mt_g(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000U) | (b & 0x7fffffffU);
    return (y >> 1) ^ ((0U - (y & 1U)) & 0x9908b0dfU);
}

// LDS-only barrier: waits for this wave's LDS traffic, not for its HBM stores
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// NT threads, RUN consecutive words per thread, LDS ring of RW words (+ 1080 mirrored), STORE:
// every word to out[n - 624]; LB: lds-only barriers.  Words [624, 624 + nwords) of the stream
// whose first block is key.
template <int NT, int RUN, int RW, bool STORE, bool LB, bool LIN = false>
__global__ __launch_bounds__(NT) void k_tw(const uint32_t* __restrict__ key, uint32_t* __restrict__ out, int nwords) {
    constexpr int MIR = 1080;
    __shared__ uint32_t ring[RW + MIR];
    const int t = threadIdx.x;
    auto put = [&](int q, uint32_t v) {
        const unsigned p = (unsigned)q & (RW - 1u);
        ring[p] = v;
        if (p < MIR) ring[RW + p] = v;
    };
    auto at = [&](int q) { return ring[(unsigned)q & (RW - 1u)]; };
    for (int i = t; i < 624; i += NT) put(i, key[i]);
    __syncthreads();
    const int w1 = 624 + nwords;
    int n0 = 624;
    while (n0 < 1078) {
        const int n1 = min(1078, n0 + 227);
        for (int n = n0 + t; n < n1; n += NT) {
            const uint32_t v = at(n - 227) ^ mt_g(at(n - 624), at(n - 623));
            put(n, v);
            if (STORE) out[n - 624] = v;
        }
        __syncthreads();
        n0 = n1;
    }
    constexpr int STEP = RUN * (623 / RUN);
    while (n0 < w1) {
        const int n1 = min(w1, n0 + STEP);
        const int n = n0 + RUN * t;
        if (n < n1) {
            const unsigned p = (unsigned)n & (RW - 1u);
            const uint32_t* b = ring + (p >= 1078u ? p : p + RW) - 1078u;
            uint32_t a[RUN + 1], c[RUN + 1], e[RUN], f[RUN + 1];
#pragma unroll
            for (int i = 0; i <= RUN; ++i) {
                a[i] = b[i];
                c[i] = b[227 + i];
                f[i] = b[454 + i];
                if (i < RUN) e[i] = b[397 + i];
            }
#pragma unroll
            for (int i = 0; i < RUN; ++i)
                if (RUN == 1 || n + i < n1) {
                    uint32_t v;
                    if (LIN) {   // g is GF(2)-linear in its two operands: one g of the xors
                        v = e[i] ^ mt_g(f[i] ^ c[i] ^ a[i], f[i + 1] ^ c[i + 1] ^ a[i + 1]);
                    } else {
                        v = e[i] ^ mt_g(f[i], f[i + 1]) ^ mt_g(c[i], c[i + 1]) ^ mt_g(a[i], a[i + 1]);
                    }
                    put(n + i, v);
                    if (STORE) out[n + i - 624] = v;
                }
        }
        if (LB) lds_barrier(); else __syncthreads();
        n0 = n1;
    }
    if (!STORE) {   // the last 624 words, for the check
        __syncthreads();
        for (int i = t; i < 624; i += NT) out[nwords - 624 + i] = at(w1 - 624 + i);
    }
}

struct HostMT {
    uint32_t mt[624];
    int idx = 624;
    void seed(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253U * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    }
};

template <int NT, int RUN, int RW, bool STORE, bool LB, bool LIN = false>
int run(const char* name, const uint32_t* dkey, uint32_t* dout, const std::vector<uint32_t>& ref, int nwords, hipStream_t s) {
    CK(hipMemsetAsync(dout, 0, (size_t)nwords * 4, s));
    hipLaunchKernelGGL((k_tw<NT, RUN, RW, STORE, LB, LIN>), dim3(1), dim3(NT), 0, s, dkey, dout, nwords);
    CK(hipStreamSynchronize(s));
    std::vector<uint32_t> got(nwords);
    CK(hipMemcpy(got.data(), dout, (size_t)nwords * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    const int from = STORE ? 0 : nwords - 624;
    for (int i = from; i < nwords; ++i) bad += got[i] != ref[624 + i];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_tw<NT, RUN, RW, STORE, LB, LIN>), dim3(1), dim3(NT), 0, s, dkey, dout, nwords);
    const int reps = 20;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_tw<NT, RUN, RW, STORE, LB, LIN>), dim3(1), dim3(NT), 0, s, dkey, dout, nwords);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = 1000.0 * ms / reps;
    const double rounds = (nwords - 454) / (double)(RUN * (623 / RUN));
    printf("%-34s %s  %8.2f us per launch  %6.1f ns/round  %6.2f us per 134k words\n", name, bad ? "MISMATCH" : "ok      ",
           us, 1000.0 * us / rounds, us * 134000.0 / nwords);
    return bad ? 1 : 0;
}

int main() {
    const int nwords = 4 * 134000;   // one Humanoid batch of 4 updates
    HostMT h;
    h.seed(12345);
    std::vector<uint32_t> ref(624 + nwords);
    for (int i = 0; i < 624; ++i) ref[i] = h.mt[i];
    for (int n = 624; n < 624 + nwords; ++n) {
        const uint32_t y = (ref[n - 624] & 0x80000000U) | (ref[n - 623] & 0x7fffffffU);
        ref[n] = ref[n - 227] ^ (y >> 1) ^ ((y & 1U) ? 0x9908b0dfU : 0U);
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *dkey, *dout;
    CK(hipMalloc(&dkey, 624 * 4));
    CK(hipMalloc(&dout, (size_t)nwords * 4));
    CK(hipMemcpy(dkey, ref.data(), 624 * 4, hipMemcpyHostToDevice));
    int bad = 0;
    bad += run<1024, 1, 32768, false, false>("1024 thr, 1 w/thr, 32K ring", dkey, dout, ref, nwords, s);
    bad += run<1024, 1, 32768, false, false, true>("linear g, 1024 thr, 32K ring", dkey, dout, ref, nwords, s);
    bad += run<640, 1, 2048, false, false, true>("linear g, 640 thr, 2K ring", dkey, dout, ref, nwords, s);
    bad += run<320, 2, 2048, false, true, true>("linear g, 320 thr, 2 w/thr, ldsbar", dkey, dout, ref, nwords, s);
    bad += run<640, 1, 2048, true, true, true>("linear g, 640 thr, 2K, store, ldsbar", dkey, dout, ref, nwords, s);
    bad += run<640, 1, 32768, false, false>("640 thr, 1 w/thr, 32K ring", dkey, dout, ref, nwords, s);
    bad += run<640, 1, 2048, false, false>("640 thr, 1 w/thr, 2K ring", dkey, dout, ref, nwords, s);
    bad += run<640, 1, 2048, false, true>("640 thr, 1 w/thr, 2K ring, ldsbar", dkey, dout, ref, nwords, s);
    bad += run<320, 2, 2048, false, true>("320 thr, 2 w/thr, 2K ring, ldsbar", dkey, dout, ref, nwords, s);
    bad += run<192, 4, 2048, false, true>("192 thr, 4 w/thr, 2K ring, ldsbar", dkey, dout, ref, nwords, s);
    bad += run<1024, 1, 32768, true, false>("1024 thr, 1 w/thr, 32K, store", dkey, dout, ref, nwords, s);
    bad += run<640, 1, 2048, true, false>("640 thr, 1 w/thr, 2K, store", dkey, dout, ref, nwords, s);
    bad += run<640, 1, 2048, true, true>("640 thr, 1 w/thr, 2K, store, ldsbar", dkey, dout, ref, nwords, s);
    bad += run<320, 2, 2048, true, true>("320 thr, 2 w/thr, 2K, store, ldsbar", dkey, dout, ref, nwords, s);
    bad += run<192, 4, 2048, true, true>("192 thr, 4 w/thr, 2K, store, ldsbar", dkey, dout, ref, nwords, s);
    printf("%s\n", bad ? "FAIL" : "all variants match the host stream");
    return bad ? 1 : 0;
}
