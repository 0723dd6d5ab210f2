// Ablation harness for k_gemm: per-launch time (graph replay) by shape/epilogue, and the
// per-workgroup phase split of a dependent chain (SACX_GEMM_PHASES build).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I sac-expert_amd/csrc tools/gemm_bench.hip -o tools/gemm_bench
#define SACX_GEMM_PHASES 1
#include "../sac-expert_amd/csrc/k_sac.hip"
#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>
using namespace sacx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

static double tgraph(hipStream_t s, int n, std::function<void(int)> launch) {
    hipGraph_t g; hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; ++i) launch(i);
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
    const size_t NF = 8 << 20;
    float *X0, *X1, *W, *P; Ctl* ctl;
    CK(hipMalloc(&X0, NF * 4)); CK(hipMalloc(&X1, NF * 4)); CK(hipMalloc(&W, NF * 4)); CK(hipMalloc(&P, 3 * NF * 4));
    CK(hipMalloc(&ctl, sizeof(Ctl)));
    CK(hipMemset(X0, 0, NF * 4)); CK(hipMemset(X1, 0, NF * 4)); CK(hipMemset(W, 0, NF * 4)); CK(hipMemset(P, 0, 3 * NF * 4));
    CK(hipMemset(ctl, 0, sizeof(Ctl)));
    auto fwd = [&](const float* A, float* C, int M, int N, int K) {
        GemmArgs ga{}; GemmProb p{};
        p.A = A; p.lda = K; p.a_kc = 1; p.ones_row = -1; p.B = W; p.ldb = N; p.b_kc = 0; p.M = M; p.N = N; p.K = K;
        p.bias = W + (size_t)K * N; p.C = C; p.ldc = N; p.epi = EPI_FWD; p.act = ACT_RELU;
        p.tiles_n = (N + 15) / 16; p.tile_begin = 0; p.vec = (K % 4 == 0);
        ga.probs[0] = p; ga.nprob = 1; ga.total_tiles = ((M + 15) / 16) * p.tiles_n; ga.p_stride = NF; ga.ctl = ctl;
        ga.mode = GM_FWD; ga.vec = (K % 4 == 0);
        ga.adam.lr[0] = ga.adam.lr[1] = ga.adam.lr[2] = ga.adam.lr[3] = 1e-4f;
        return ga;
    };
    const int n = 100;
    // phase split: dependent chain of FWD launches (512x256; Humanoid's 1024x256 at K = 393),
    // stamps of the last launch
    // (lda = round4(K): the padded staging stride that lets K = 393 take float4 loads)
    struct PV { int M, K, vec; } pvs[] = {{512, 24, 1}, {512, 256, 1}, {1024, 393, 0}, {1024, 393, 1}, {4096, 393, 1}};
    for (auto pv : pvs) {
        const int K = pv.K;
        GemmArgs a0 = fwd(X0, X1, pv.M, 256, K), a1 = fwd(X1, X0, pv.M, 256, K);
        a0.probs[0].lda = a1.probs[0].lda = (K + 3) & ~3;
        a0.vec = a1.vec = a0.probs[0].vec = a1.probs[0].vec = pv.vec;
        const double us = tgraph(s, n, [&](int i) { launch_gemm((i & 1) ? a1 : a0, s); });
        static unsigned long long ph[8192][5];
        CK(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_gemm_ph), sizeof(ph)));
        const int T = a0.total_tiles;
        unsigned long long lo = ~0ull, hi = 0;
        double d[4] = {0, 0, 0, 0};
        for (int b = 0; b < T; ++b) {
            lo = std::min(lo, ph[b][0]);
            hi = std::max(hi, ph[b][4]);
            for (int j = 0; j < 4; ++j) d[j] += (double)(ph[b][j + 1] - ph[b][j]);
        }
        printf("phases fwd %dx256 K=%-3d vec=%d %.2f us/launch | span %.2f us | mean per WG: select %.2f  loads+mfma %.2f  "
               "reduce %.2f  epilogue %.2f us\n", pv.M, K, pv.vec, us, (hi - lo) * 0.01, d[0] * 0.01 / T, d[1] * 0.01 / T,
               d[2] * 0.01 / T, d[3] * 0.01 / T);
    }
    struct V { const char* name; int M, N, K; bool dep; };
    V vs[] = {{"fwd 512x256 K=256 warm", 512, 256, 256, false}, {"fwd 512x256 K=256 dep", 512, 256, 256, true},
              {"fwd 512x256 K=16 warm", 512, 256, 16, false},   {"fwd 512x256 K=16 dep", 512, 256, 16, true},
              {"fwd 64x64 K=16 warm", 64, 64, 16, false},       {"fwd 16x16 K=16 warm", 16, 16, 16, false},
              {"fwd 1024x256 K=256 dep", 1024, 256, 256, true}};
    for (auto& v : vs) {
        GemmArgs a0 = fwd(X0, X1, v.M, v.N, v.K), a1 = fwd(X1, X0, v.M, v.N, v.K);
        double us = tgraph(s, n, [&](int i) { launch_gemm(v.dep ? ((i & 1) ? a1 : a0) : a0, s); });
        printf("%-28s %4d tiles: %.2f us/launch\n", v.name, a0.total_tiles, us);
    }
    // K sweep at 512x256 (dependent chain): launch cost vs operand bytes read per launch
    for (int xm : {0, 1})
        for (int K : {16, 64, 128, 256, 512}) {
            GemmArgs a0 = fwd(X0, X1, 512, 256, K), a1 = fwd(X1, X0, 512, 256, K);
            a0.xcd_map = a1.xcd_map = xm;
            const double mb = 512.0 * 256 * K * 4 * (1.0 / 16 + 1.0 / 16) / 1e6;
            double us = tgraph(s, n, [&](int i) { launch_gemm((i & 1) ? a1 : a0, s); });
            printf("sweep xcd=%d 512x256 K=%-4d L2 reads %5.1f MB: %.2f us/launch\n", xm, K, mb, us);
        }
    // Adam epilogue on a 257x256 grad tile set (dW of a 256x256 layer, K = batch 256)
    {
        GemmArgs ga{}; GemmProb p{};
        p.A = X0; p.lda = 256; p.a_kc = 0; p.ones_row = 256; p.B = X1; p.ldb = 256; p.b_kc = 0;
        p.M = 257; p.N = 256; p.K = 256; p.P = P; p.T = nullptr; p.ldp = 256; p.epi = EPI_ADAM; p.group = 0; p.grad_scale = 1.f;
        {
            static float* ones = nullptr;
            std::vector<float> h1(4096, 1.f);
            CK(hipMalloc(&ones, 4096 * 4));
            CK(hipMemcpy(ones, h1.data(), 4096 * 4, hipMemcpyHostToDevice));
            p.bscale = ones;
        }
        p.tiles_n = 16; p.tile_begin = 0;
        ga.probs[0] = p; ga.nprob = 1; ga.total_tiles = 17 * 16; ga.p_stride = NF; ga.ctl = ctl; ga.mode = GM_DW; ga.vec = 0;
        ga.adam.lr[0] = 3e-4f; ga.adam.tau_keep = 0.995f; ga.adam.tau_take = 0.005f; ga.adam.target_update_int = 1;
        printf("%-28s %4d tiles: %.2f us/launch\n", "dW+adam 257x256 K=256", ga.total_tiles, tgraph(s, n, [&](int) { launch_gemm(ga, s); }));
        // dX (k-contig A and B^T), the critic backward shape: 512x256, K=256
        GemmArgs gx{}; GemmProb q{};
        q.A = X0; q.lda = 256; q.a_kc = 1; q.ones_row = -1; q.B = W; q.ldb = 257 * 0 + 256; q.b_kc = 1; q.M = 512; q.N = 256; q.K = 256;
        q.H = X1; q.ldh = 256; q.C = X1 + 2000000; q.ldc = 256; q.epi = EPI_DACT; q.act = ACT_RELU; q.tiles_n = 16; q.tile_begin = 0; q.vec = 1;
        gx.probs[0] = q; gx.nprob = 1; gx.total_tiles = 32 * 16; gx.p_stride = NF; gx.ctl = ctl; gx.mode = GM_DX; gx.vec = 1;
        printf("%-28s %4d tiles: %.2f us/launch\n", "dX 512x256 K=256", gx.total_tiles, tgraph(s, n, [&](int) { launch_gemm(gx, s); }));
    }
    return 0;
}
