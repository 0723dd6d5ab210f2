// Sampler microbenchmark: launch_rng batches at HC / Humanoid shapes -- the one-workgroup k_rng
// (with the per-phase tick split of the SACX_RNG_PROF build: twist bursts, randint chunks, gauss
// chunks), the split k_rng + k_polar, and the segmented k_mtj_* pipeline (plus its forced
// fallback).  Every path is first checked word for word against the one-kernel path over three
// chained batches after an odd-count draw (outputs and the final MT state).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I sac-expert_amd/csrc tools/rng_bench.hip \
//            sac-expert_amd/csrc/mt_jump.cpp -o tools/rng_bench
#define SACX_RNG_PROF 1
#include "../sac-expert_amd/csrc/k_sac.hip"
#include "../sac-expert_amd/csrc/mt_jump.h"
#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
using namespace sacx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {   // argv[1]: run only the configurations whose name contains it
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    RngState* st; Ctl* ctl; int32_t* idx; float* nz;
    CK(hipMalloc(&st, sizeof(RngState))); CK(hipMalloc(&ctl, sizeof(Ctl)));
    CK(hipMalloc(&idx, 32 << 20)); CK(hipMalloc(&nz, 32 << 20));   // 4 slots x 4 MiB apart
    RngState h{};
    uint32_t seed = 12345;
    for (int i = 0; i < 624; ++i) { h.key[i] = seed; seed = 1812433253U * (seed ^ (seed >> 30)) + (uint32_t)i + 1U; }
    h.pos = 624;
    CK(hipMemcpy(st, &h, sizeof(h), hipMemcpyHostToDevice));
    Ctl c{}; c.cur_size = 1000000;
    CK(hipMemcpy(ctl, &c, sizeof(c), hipMemcpyHostToDevice));
    uint32_t* pairs; int32_t* poi; float* nz2; int32_t* idx2;
    CK(hipMalloc(&pairs, 8 << 20)); CK(hipMalloc(&poi, 64)); CK(hipMalloc(&nz2, 32 << 20)); CK(hipMalloc(&idx2, 32 << 20));
    struct Cfg { const char* name; int B, A, nupd, mode; } cfgs[] = {   // mode: 0 k_rng, 1 split, 2 segmented, 3 forced fallback
        {"hc B=256 A=6", 256, 6, 8, 0}, {"hc split", 256, 6, 8, 1}, {"hc segmented", 256, 6, 8, 2},
        {"humanoid B=1024 A=17", 1024, 17, 4, 0}, {"humanoid split", 1024, 17, 4, 1},
        {"humanoid segmented", 1024, 17, 4, 2}, {"humanoid seg nupd=1", 1024, 17, 1, 2},
        {"humanoid seg fallback", 1024, 17, 4, 3}};
    int fails = 0;
    for (auto& cf : cfgs) {
        if (argc > 1 && !strstr(cf.name, argv[1])) continue;
        RngArgs a{};
        a.st = st; a.ctl = ctl; a.n_int = cf.B; a.n_norm = 3 * cf.B * cf.A; a.out_idx = idx; a.out_norm = nz;
        a.slot = -1; a.nupd = cf.nupd; a.slot_bytes = (int64_t)2 << 20;
        if (cf.mode == 1) { a.pairs = pairs; a.pairs_oi = poi; a.pcap = (a.n_norm + 1) / 2; }
        uint32_t* jw = nullptr; uint32_t* jc = nullptr;
        if (cf.mode >= 2) {   // the plan's rule (sacx.cpp build_layout)
            const double per = 2.0 * a.n_int + (double)((a.n_norm + 1) >> 1) * (4.0 / 0.78539816339744831);
            int64_t L = ((int64_t)std::ceil(per * 1.02 / 4.0) + 63) / 64 * 64;
            if (const char* e = std::getenv("SACX_MTJ_L")) L = std::atoll(e);
            L = std::max<int64_t>(MTJ_HEAD, L);
            const double words = NBATCH_MAX * per;
            const int smax = (int)std::ceil((624.0 + 1.02 * words + 8.0 * std::sqrt(words) + 64.0 * NBATCH_MAX + 1024.0 + MTJ_HEAD) / L) + 1;
            const MtjLayout y = mtj_layout(L, smax);
            std::vector<int32_t> hj((size_t)sacx::mt_jump_lists_words(smax - 1, MTJ_CH));
            const int64_t used = sacx::mt_jump_lists(L, smax - 1, MTJ_CH, hj.data());
            CK(hipMalloc(&jw, y.total * 4)); CK(hipMalloc(&jc, used * 4));
            CK(hipMemcpy(jc, hj.data(), used * 4, hipMemcpyHostToDevice));
            a.jw = jw; a.jc = jc; a.jL = (int32_t)L; a.jsmax = smax;
            printf("%-22s L = %lld, %d segments per launch (max %d)\n", cf.name, (long long)L, mtj_segments(a), smax);
        }
        if (cf.mode == 3) setenv("SACX_MTJ_UNDER", "1", 1);
        {   // bit-identity with the one-kernel path from the same state: an odd-count draw first
            // (cached gauss), then three chained batches; outputs of the last and the final state
            RngArgs b = a;
            b.pairs = nullptr; b.jw = nullptr; b.out_idx = idx2; b.out_norm = nz2;
            RngArgs o = a; o.n_int = 0; o.n_norm = 7; o.nupd = 1; o.pairs = nullptr; o.jw = nullptr;
            o.out_norm = nz + (24 << 20) / 4;   // away from the compared slots
            RngState sa, sb;
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(st, &h, sizeof(h), hipMemcpyHostToDevice));
            launch_rng(o, s); for (int r = 0; r < 3; ++r) launch_rng(a, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(&sa, st, sizeof(sa), hipMemcpyDeviceToHost));
            CK(hipMemcpy(st, &h, sizeof(h), hipMemcpyHostToDevice));
            launch_rng(o, s); for (int r = 0; r < 3; ++r) launch_rng(b, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(&sb, st, sizeof(sb), hipMemcpyDeviceToHost));
            size_t bad = memcmp(&sa, &sb, sizeof(sa)) != 0;
            std::vector<float> x(a.n_norm), y(a.n_norm);
            std::vector<int32_t> ix(a.n_int), iy(a.n_int);
            for (int u = 0; u < a.nupd; ++u) {
                CK(hipMemcpy(x.data(), (char*)nz + u * a.slot_bytes, 4 * a.n_norm, hipMemcpyDeviceToHost));
                CK(hipMemcpy(y.data(), (char*)nz2 + u * a.slot_bytes, 4 * a.n_norm, hipMemcpyDeviceToHost));
                CK(hipMemcpy(ix.data(), (char*)idx + u * a.slot_bytes, 4 * a.n_int, hipMemcpyDeviceToHost));
                CK(hipMemcpy(iy.data(), (char*)idx2 + u * a.slot_bytes, 4 * a.n_int, hipMemcpyDeviceToHost));
                for (int i = 0; i < a.n_norm; ++i) bad += memcmp(&x[i], &y[i], 4) != 0;
                for (int i = 0; i < a.n_int; ++i) bad += ix[i] != iy[i];
            }
            printf("%-22s == one-kernel: %s (%zu mismatches, state %s)\n", cf.name, bad ? "NO" : "yes", bad,
                   memcmp(&sa, &sb, sizeof(sa)) ? "differs" : "equal");
            fails += bad != 0;
        }
        for (int w = 0; w < 3; ++w) launch_rng(a, s);
        CK(hipStreamSynchronize(s));
        unsigned long long z[16] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_rng_prof), z, sizeof(z)));
        const int n = 20;
        auto t0 = std::chrono::high_resolution_clock::now();
        for (int i = 0; i < n; ++i) launch_rng(a, s);
        CK(hipStreamSynchronize(s));
        auto t1 = std::chrono::high_resolution_clock::now();
        CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(g_rng_prof), sizeof(z)));
        const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / (n * cf.nupd);
        const double upd = (double)n * cf.nupd;
        if (cf.mode == 3) unsetenv("SACX_MTJ_UNDER");
        if (cf.mode >= 2) {
            printf("%-22s %8.2f us/update (%d updates per launch) | resolve: prefixes %.2f walk %.2f state %.2f us per launch\n",
                   cf.name, us, cf.nupd, z[8] * 0.01 / z[11], z[9] * 0.01 / z[11], z[10] * 0.01 / z[11]);
            printf("%-22s emit per workgroup: loads %.2f ranks %.2f transforms %.2f us\n", cf.name,
                   z[12] * 0.01 / z[15], z[13] * 0.01 / z[15], z[14] * 0.01 / z[15]);
            CK(hipFree(jw)); CK(hipFree(jc));
        } else {
            printf("%-22s %8.2f us/update | twist %7.2f  randint %6.2f  gauss %7.2f  kernel %7.2f us/update | "
                   "bursts %.1f chunks %.1f per update\n", cf.name, us, z[0] * 0.01 / upd, z[1] * 0.01 / upd,
                   z[2] * 0.01 / upd, z[3] * 0.01 / upd, z[4] / upd, z[5] / upd);
        }
    }
    printf("%s\n", fails ? "FAIL: a path differs from the one-kernel draws" : "all paths equal the one-kernel draws");
    return fails ? 1 : 0;
}

