// dW + Adam launch variants on the Humanoid shapes (B = 1,024): the 16x16 k_gemm tiles, the
// 32x32 gemm_tile32 tiles and k_dwl (LDS-DMA staged rows).  Each variant runs from the same
// parameter state; outputs (P, m, v, target) must be bit-identical.  Then each is timed as a
// graph of back-to-back launches.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I sac-expert_amd/csrc tools/dw_bench.hip -o tools/dw_bench
#include "../sac-expert_amd/csrc/k_sac.hip"
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>
using namespace sacx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

static double tgraph(hipStream_t s, int n, std::function<void()> launch) {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; ++i) launch();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiateWithFlags(&ge, g, 0));
    CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    auto t1 = std::chrono::high_resolution_clock::now();
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / (5.0 * n);
}

struct Op { const float* X; int ldx, Kin; const float* D; int N, ldd; const float* bs; size_t poff; int ones; };

static uint32_t lcg = 12345u;
static float frand() { lcg = lcg * 1664525u + 1013904223u; return ((lcg >> 8) * (1.f / 16777216.f)) * 2.f - 1.f; }

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1024;
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t PS = 1 << 20;                     // p_stride (floats)
    float *buf, *P, *P0; Ctl* ctl;
    const size_t NB = 16u << 20;
    CK(hipMalloc(&buf, NB * 4)); CK(hipMalloc(&P, 4 * PS * 4)); CK(hipMalloc(&P0, 4 * PS * 4));
    CK(hipMalloc(&ctl, sizeof(Ctl))); CK(hipMemset(ctl, 0, sizeof(Ctl)));
    {
        std::vector<float> h(NB);
        for (auto& v : h) v = frand();
        CK(hipMemcpy(buf, h.data(), NB * 4, hipMemcpyHostToDevice));
        std::vector<float> p(4 * PS);
        for (size_t i = 0; i < p.size(); ++i) p[i] = (i / PS == 2) ? 0.5f * (frand() + 1.f) : frand();
        CK(hipMemcpy(P0, p.data(), p.size() * 4, hipMemcpyHostToDevice));
    }
    // operand slabs carved from buf (Humanoid: S + A = 393 -> ldQ 396, S = 376 -> ldS 380, H 256, Aout 34, A 17)
    size_t cur = 0;
    auto take = [&](size_t n) { const float* p = buf + cur; cur += (n + 63) & ~size_t(63); return p; };
    const float* Xq = take((size_t)B * 396);
    const float* Dq1[2] = {take((size_t)B * 256), take((size_t)B * 256)};
    const float* Hq1[2] = {take((size_t)B * 256), take((size_t)B * 256)};
    const float* Dq2[2] = {take((size_t)B * 256), take((size_t)B * 256)};
    const float* Hq2[2] = {take((size_t)B * 256), take((size_t)B * 256)};
    const float* gq = take((size_t)2 * B);
    const float* Xa = take((size_t)B * 380);
    const float* Da1 = take((size_t)B * 256);
    const float* Ha1 = take((size_t)B * 256);
    const float* Da2 = take((size_t)B * 256);
    const float* Ha2 = take((size_t)B * 256);
    const float* Da3 = take((size_t)B * 34);
    const float* E = take((size_t)B * 17);
    float* ones = const_cast<float*>(take(B));
    { std::vector<float> o(B, 1.f); CK(hipMemcpy(ones, o.data(), B * 4, hipMemcpyHostToDevice)); }

    auto prob = [&](const Op& o) {
        GemmProb p{};
        p.A = o.X; p.lda = o.ldx; p.a_kc = 0; p.ones_row = o.ones;
        p.B = o.D; p.ldb = o.ldd; p.b_kc = 0;
        p.M = o.Kin + 1; p.N = o.N; p.K = B;
        p.P = P + o.poff; p.T = P + 3 * PS + o.poff; p.ldp = o.N;
        p.epi = EPI_ADAM; p.group = 0; p.grad_scale = 1.f; p.bscale = o.bs;
        return p;
    };
    std::vector<Op> critic, actor;
    size_t po = 0;
    for (int k = 0; k < 2; ++k) {
        critic.push_back({Xq, 396, 393, Dq1[k], 256, 256, gq + (size_t)k * B, po, 393}); po += 394 * 256;
        critic.push_back({Hq1[k], 256, 256, Dq2[k], 256, 256, ones, po, 256}); po += 257 * 256;
        critic.push_back({Hq2[k], 256, 256, gq + (size_t)k * B, 1, 1, ones, po, 256}); po += 257;
    }
    po = (po + 63) & ~size_t(63);
    actor.push_back({Xa, 380, 376, Da1, 256, 256, ones, po, 376}); po += 377 * 256;
    actor.push_back({Ha1, 256, 256, Da2, 256, 256, ones, po, 256}); po += 257 * 256;
    actor.push_back({Ha2, 256, 256, Da3, 34, 34, ones, po, 256}); po += 257 * 34;
    actor.push_back({E, 1, 0, E, 17, 17, ones, po, 0}); po += 17;
    auto args = [&](const std::vector<Op>& ops, int variant, bool bf) {   // 0: 16x16, 1: T32, 2: dwl 32x32, 3: dwl 32x16
        GemmArgs ga{};
        const int ts = variant ? 32 : 16, tsn = variant == 3 ? 16 : ts;
        int tiles = 0;
        for (size_t i = 0; i < ops.size(); ++i) {
            GemmProb p = prob(ops[i]);
            p.tiles_n = (p.N + tsn - 1) / tsn; p.tile_begin = tiles;
            tiles += ((p.M + ts - 1) / ts) * p.tiles_n;
            if (variant >= 2) {
                const bool a4 = p.lda >= 4 && p.lda % 4 == 0 && (((uintptr_t)p.A) & 15) == 0;
                const bool b4 = p.ldb >= 4 && p.ldb % 4 == 0 && (((uintptr_t)p.B) & 15) == 0;
                p.vec = (a4 ? 1 : 0) | (b4 ? 2 : 0);
            }
            ga.probs[i] = p;
        }
        ga.nprob = (int)ops.size(); ga.mode = GM_DW; ga.total_tiles = tiles; ga.xcd_map = 1;
        ga.t32 = variant == 1; ga.dwl = variant == 2 ? 1 : variant == 3 ? 2 : 0; ga.bf16 = bf; ga.p_stride = PS; ga.ctl = ctl;
        ga.adam.lr[0] = 3e-4f; ga.adam.tau_keep = 0.995f; ga.adam.tau_take = 0.005f; ga.adam.target_update_int = 1;
        return ga;
    };
    const char* vn[4] = {"16x16", "t32  ", "dwl  ", "dwl16"};
    for (int bf = 0; bf < 2; ++bf)
        for (int set = 0; set < 2; ++set) {
            const auto& ops = set ? actor : critic;
            std::vector<float> out[6];
            for (int v = 0; v < 6; ++v) {      // 3: 16x16 again, 4: 16x16 without the XCD map, 5: dwl 32x16
                CK(hipMemcpy(P, P0, 4 * PS * 4, hipMemcpyDeviceToDevice));
                CK(hipDeviceSynchronize());
                GemmArgs ga = args(ops, v < 3 ? v : v == 5 ? 3 : 0, bf);
                if (v == 4) ga.xcd_map = 0;
                launch_gemm(ga, s);
                CK(hipStreamSynchronize(s));
                out[v].resize(4 * PS);
                CK(hipMemcpy(out[v].data(), P, 4 * PS * 4, hipMemcpyDeviceToHost));
            }
            const int pairs[6][2] = {{0, 1}, {0, 2}, {1, 2}, {0, 3}, {0, 4}, {0, 5}};
            const char* pn[6] = {"16x16 vs t32", "16x16 vs dwl", "t32 vs dwl", "16x16 vs 16x16 again", "16x16 vs 16x16 no xcd",
                                 "16x16 vs dwl 32x16"};
            for (int q = 0; q < 6; ++q) {
                const auto& x = out[pairs[q][0]];
                const auto& y = out[pairs[q][1]];
                size_t diff = 0, first = 0;
                for (size_t i = 0; i < x.size(); ++i)
                    if (memcmp(&x[i], &y[i], 4) != 0) { if (!diff) first = i; ++diff; }
                printf("%s bf16=%d %-24s: %zu elements differ%s", set ? "actor.adam " : "critic.adam", bf, pn[q], diff,
                       diff ? "" : " (bit-identical)\n");
                if (diff) printf(" first at %zu: %a vs %a (P0 %s)\n", first, x[first], y[first], "");
            }
            for (int v = 0; v < 4; ++v) {
                GemmArgs ga = args(ops, v, bf);
                {   // per-workgroup start / end stamps (100 MHz) of one launch
                    static uint64_t* kt = nullptr;
                    if (!kt) CK(hipMalloc(&kt, 2 * 8192 * 8));
                    GemmArgs gk = ga;
                    gk.ktime = kt;
                    for (int rep = 0; rep < 3; ++rep) launch_gemm(gk, s);
                    CK(hipStreamSynchronize(s));
                    std::vector<uint64_t> h(2 * gk.total_tiles);
                    CK(hipMemcpy(h.data(), kt, h.size() * 8, hipMemcpyDeviceToHost));
                    uint64_t lo = ~0ull, hi = 0, smax = 0; double sum = 0, dmax = 0;
                    for (int b = 0; b < gk.total_tiles; ++b) {
                        lo = std::min(lo, h[2 * b]); hi = std::max(hi, h[2 * b + 1]);
                        sum += (double)(h[2 * b + 1] - h[2 * b]); dmax = std::max(dmax, (double)(h[2 * b + 1] - h[2 * b]));
                        smax = std::max(smax, h[2 * b]);
                    }
#ifdef SACX_GEMM_PHASES
                    if (v >= 2) {
                        static unsigned long long ph[8192][5];
                        CK(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_gemm_ph), sizeof(ph)));
                        double d[4] = {0, 0, 0, 0};
                        for (int b = 0; b < gk.total_tiles; ++b)
                            for (int q = 0; q < 4; ++q) d[q] += (double)(ph[b][q + 1] - ph[b][q]);
                        printf("   phases dwl (wave 0): prologue %.2f  slab loop %.2f  reduce %.2f  epilogue %.2f us\n",
                               d[0] * 0.01 / gk.total_tiles, d[1] * 0.01 / gk.total_tiles, d[2] * 0.01 / gk.total_tiles,
                               d[3] * 0.01 / gk.total_tiles);
                    }
#endif
                    printf("   stamps %s: span %.2f us, WG mean %.2f max %.2f, last start %.2f us\n", vn[v], (hi - lo) * 0.01,
                           sum * 0.01 / gk.total_tiles, dmax * 0.01, (smax - lo) * 0.01);
                }
                const double us = tgraph(s, 200, [&]() { launch_gemm(ga, s); });
                printf("%s %s bf16=%d B=%d: %5d tiles %7.2f us/launch\n", set ? "actor.adam " : "critic.adam", vn[v], bf, B,
                       ga.total_tiles, us);
            }
        }
    return 0;
}
