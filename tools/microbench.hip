// Calibration microbenchmark: fixed per-launch cost, dependent-load latency and
// the clock the chip holds, in the launch shapes the SAC step uses.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <chrono>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_empty(int* p) { if (threadIdx.x == 1234567) p[0] = 1; }
__global__ void k_load(const float* __restrict__ a, float* __restrict__ b) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    b[i] = a[i] + 1.f;
}
__global__ void k_chain(const int* __restrict__ nxt, int* out, int hops) {
    int j = (blockIdx.x * blockDim.x + threadIdx.x) & 1023;
    for (int h = 0; h < hops; ++h) j = nxt[j];
    if (j == -1) out[0] = j;
}
__global__ void k_clock(unsigned long long* o) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x = threadIdx.x;
    for (int i = 0; i < 200000; ++i) x = x * 1.0000001f + 0.5f;
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { o[0] = t1 - t0; o[1] = r1 - r0; o[2] = (unsigned long long)x; }
}

struct BigArgs { int v[256]; };
__global__ void k_karg_chain(BigArgs a, int* out, int hops) {
    int j = threadIdx.x & 255;
    for (int h = 0; h < hops; ++h) j = a.v[j];
    if (j == -1) out[0] = j;
}
__global__ void k_gchain_uniform(const int* __restrict__ nxt, int* out, int hops) {
    int j = 0;                       // wave-uniform chain -> scalar loads from global
    for (int h = 0; h < hops; ++h) j = nxt[j];
    if (j == -1) out[0] = j;
}

template <class F>
double time_graph(hipStream_t s, int n, F launch) {
    hipGraph_t g; hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; ++i) launch();
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiateWithFlags(&ge, g, 0);
    (void)hipGraphLaunch(ge, s); (void)hipStreamSynchronize(s);
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    auto t1 = std::chrono::high_resolution_clock::now();
    (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / (5.0 * n);
}

int main() {
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int* pi; float *a, *b; int* nxt; unsigned long long* clk;
    CK(hipMalloc(&pi, 4096)); CK(hipMalloc(&a, 64 << 20)); CK(hipMalloc(&b, 64 << 20));
    CK(hipMalloc(&nxt, 1024 * 4)); CK(hipMalloc(&clk, 64));
    std::vector<int> h(1024); for (int i = 0; i < 1024; ++i) h[i] = (i * 97 + 13) & 1023;
    CK(hipMemcpy(nxt, h.data(), 4096, hipMemcpyHostToDevice));
    const int N = 200;
    printf("empty 1x64     : %.2f us/launch\n", time_graph(s, N, [&] { k_empty<<<1, 64, 0, s>>>(pi); }));
    printf("empty 512x256  : %.2f us/launch\n", time_graph(s, N, [&] { k_empty<<<512, 256, 0, s>>>(pi); }));
    printf("empty 1024x256 : %.2f us/launch\n", time_graph(s, N, [&] { k_empty<<<1024, 256, 0, s>>>(pi); }));
    printf("load 512x256   : %.2f us/launch\n", time_graph(s, N, [&] { k_load<<<512, 256, 0, s>>>(a, b); }));
    printf("pingpong 512x256: %.2f us/launch\n", time_graph(s, N, [&] { static int f = 0; if (f ^= 1) k_load<<<512, 256, 0, s>>>(a, b); else k_load<<<512, 256, 0, s>>>(b, a); }));
    for (int hops : {1, 2, 4, 8, 16})
        printf("chain %2d hops 512x256: %.2f us/launch\n", hops, time_graph(s, N, [&] { k_chain<<<512, 256, 0, s>>>(nxt, pi, hops); }));
    BigArgs ba; for (int i = 0; i < 256; ++i) ba.v[i] = (i * 37 + 11) & 255;
    for (int hops : {1, 4, 16})
        printf("karg chain %2d hops 512x256: %.2f us/launch\n", hops, time_graph(s, N, [&] { k_karg_chain<<<512, 256, 0, s>>>(ba, pi, hops); }));
    for (int hops : {1, 4, 16})
        printf("global uniform chain %2d hops 512x256: %.2f us/launch\n", hops, time_graph(s, N, [&] { k_gchain_uniform<<<512, 256, 0, s>>>(nxt, pi, hops); }));
    k_clock<<<256, 64, 0, s>>>(clk); CK(hipStreamSynchronize(s));
    unsigned long long hc[3]; CK(hipMemcpy(hc, clk, 24, hipMemcpyDeviceToHost));
    printf("clock (1 wave/CU busy loop): %.0f MHz (memtime %llu / realtime %llu @100MHz)\n", 100.0 * hc[0] / hc[1], hc[0], hc[1]);
    return 0;
}
