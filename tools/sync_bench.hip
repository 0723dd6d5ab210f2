// Microbenchmark: can two dependent GEMM stages share ONE launch with row-block counters
// instead of a kernel boundary?  Stage 0 (X0 -> X1) and stage 1 (X1 -> X2) are both
// M x 256 x K forward GEMMs (k_gemm's 16x16 tiles).  Stage-1 tile (rb, cb) needs all of
// stage 0's row block rb.  Fused launch: stage-0 tiles are workgroups [0, T0) (dispatched
// first), each signals cnt[rb] after its stores (release: workgroup barrier + agent fence);
// stage-1 workgroups poll cnt[rb] (bounded spin, error flag on time-out), then acquire.
// The last stage-1 tile of a row block resets the counters for the next launch.
// Compared against the same two stages as two launches, in a replayed graph of N pairs.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I sac-expert_amd/csrc tools/sync_bench.hip -o tools/sync_bench
#include "../sac-expert_amd/csrc/k_sac.hip"
#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>
using namespace sacx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// a per-lane (VGPR) address: the atomics and polls below must be vector memory operations
__device__ __forceinline__ int* vaddr(int* p) {
    uint64_t a = reinterpret_cast<uint64_t>(p);
    asm volatile("" : "+v"(a));
    return reinterpret_cast<int*>(a);
}

__global__ __launch_bounds__(256) void k_pair(GemmArgs ga, int t0, int tn0, int tn1, int* cnt, int* cnt2, int* err) {
    const int t = blockIdx.x;
    const bool consumer = t >= t0;
    const int rb = consumer ? (t - t0) / tn1 : t / tn0;
    if (consumer) {
        if (threadIdx.x == 0) {
            int* p = vaddr(cnt + rb);
            int spins = 0;
            while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < tn0) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1 << 22)) { __hip_atomic_store(vaddr(err), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        __syncthreads();
    }
    gemm_core<GM_FWD, 1, 0, 4, false, false, false>(ga);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (!consumer) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_fetch_add(vaddr(cnt + rb), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (__hip_atomic_fetch_add(vaddr(cnt2 + rb), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tn1 - 1) {
            __hip_atomic_store(vaddr(cnt + rb), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(vaddr(cnt2 + rb), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

static double tgraph(hipStream_t s, int n, std::function<void(int)> launch) {
    hipGraph_t g; hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; ++i) launch(i);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiateWithFlags(&ge, g, 0);
    (void)hipGraphLaunch(ge, s); (void)hipStreamSynchronize(s);
    auto c0 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    auto c1 = std::chrono::high_resolution_clock::now();
    (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
    return std::chrono::duration<double, std::micro>(c1 - c0).count() / (5.0 * n);
}

int main() {
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t NF = 4 << 20;
    float *X0, *X1, *X2, *W;
    Ctl* ctl;
    int *cnt, *cnt2, *err;
    CK(hipMalloc(&X0, NF * 4)); CK(hipMalloc(&X1, NF * 4)); CK(hipMalloc(&X2, NF * 4)); CK(hipMalloc(&W, NF * 4));
    CK(hipMalloc(&ctl, sizeof(Ctl))); CK(hipMalloc(&cnt, 4096)); CK(hipMalloc(&cnt2, 4096)); CK(hipMalloc(&err, 4));
    CK(hipMemset(ctl, 0, sizeof(Ctl))); CK(hipMemset(cnt, 0, 4096)); CK(hipMemset(cnt2, 0, 4096)); CK(hipMemset(err, 0, 4));
    std::vector<float> h(NF);
    for (size_t i = 0; i < NF; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
    CK(hipMemcpy(X0, h.data(), NF * 4, hipMemcpyHostToDevice));
    for (size_t i = 0; i < NF; ++i) h[i] *= 0.05f;
    CK(hipMemcpy(W, h.data(), NF * 4, hipMemcpyHostToDevice));
    auto prob = [&](const float* A, float* C, int M, int N, int K, const float* Wp) {
        GemmProb p{};
        p.A = A; p.lda = K; p.a_kc = 1; p.ones_row = -1; p.B = Wp; p.ldb = N; p.b_kc = 0; p.M = M; p.N = N; p.K = K;
        p.bias = Wp + (size_t)K * N; p.C = C; p.ldc = N; p.epi = EPI_FWD; p.act = ACT_TANH;
        p.tiles_n = (N + 15) / 16; p.tile_begin = 0; p.vec = 1;
        return p;
    };
    auto args = [&](std::vector<GemmProb> ps) {
        GemmArgs ga{};
        int tiles = 0;
        for (size_t i = 0; i < ps.size(); ++i) {
            ps[i].tile_begin = tiles;
            tiles += ((ps[i].M + 15) / 16) * ps[i].tiles_n;
            ga.probs[i] = ps[i];
        }
        ga.nprob = (int)ps.size(); ga.total_tiles = tiles; ga.p_stride = NF; ga.ctl = ctl; ga.mode = GM_FWD; ga.vec = 1;
        ga.xcd_map = 0;          // the fused launch relies on stage-0 tiles taking the low workgroup ids
        return ga;
    };
    for (int M : {256, 512, 1024}) {
        const int K = 256, N = 256, tn = N / 16, T0 = (M / 16) * tn;
        GemmProb p0 = prob(X0, X1, M, N, K, W), p1 = prob(X1, X2, M, N, K, W + 200000);
        GemmArgs s0 = args({p0}), s1 = args({p1}), f = args({p0, p1});
        const int n = 50;
        const double two = tgraph(s, n, [&](int) { launch_gemm(s0, s); launch_gemm(s1, s); });
        std::vector<float> ref((size_t)M * N), got((size_t)M * N);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(ref.data(), X2, ref.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemset(X1, 0, NF * 4)); CK(hipMemset(X2, 0, NF * 4));
        const double one = tgraph(s, n, [&](int) {
            hipLaunchKernelGGL(k_pair, dim3(f.total_tiles), dim3(256), 0, s, f, T0, tn, tn, cnt, cnt2, err);
        });
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(got.data(), X2, got.size() * 4, hipMemcpyDeviceToHost));
        int e = 0, c = 0;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&c, cnt, 4, hipMemcpyDeviceToHost));
        size_t diff = 0;
        for (size_t i = 0; i < ref.size(); ++i) diff += ref[i] != got[i];
        printf("M=%4d: two launches %.2f us/pair, fused %.2f us/pair | mismatches %zu, timeout flag %d, cnt[0] after %d\n",
               M, two, one, diff, e, c);
        if (e) return 2;
    }
    return 0;
}
