// Sampler microbenchmark: one k_rng launch per update at HC / Humanoid shapes, with the
// per-phase tick split of the SACX_RNG_PROF build (twist bursts, randint chunks, gauss chunks).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I sac-expert_amd/csrc tools/rng_bench.hip -o tools/rng_bench
#define SACX_RNG_PROF 1
#include "../sac-expert_amd/csrc/k_sac.hip"
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
using namespace sacx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
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
    struct Cfg { const char* name; int B, A, nupd; bool split; } cfgs[] = {
        {"hc B=256 A=6", 256, 6, 4, false}, {"hc B=256 A=6 split", 256, 6, 4, true},
        {"humanoid B=1024 A=17", 1024, 17, 4, false}, {"humanoid split", 1024, 17, 4, true}};
    for (auto& cf : cfgs) {
        RngArgs a{};
        a.st = st; a.ctl = ctl; a.n_int = cf.B; a.n_norm = 3 * cf.B * cf.A; a.out_idx = idx; a.out_norm = nz;
        a.slot = -1; a.nupd = cf.nupd; a.slot_bytes = (int64_t)4 << 20;
        if (cf.split) { a.pairs = pairs; a.pairs_oi = poi; a.pcap = (a.n_norm + 1) / 2; }
        {   // bit-identity of the two paths from the same state (one odd-count draw first: cached gauss)
            RngArgs b = a;
            b.pairs = nullptr; b.out_idx = idx2; b.out_norm = nz2;
            RngArgs o = a; o.n_int = 0; o.n_norm = 7; o.nupd = 1; o.pairs = nullptr;
            o.out_norm = nz + (24 << 20) / 4;   // away from the compared slots
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(st, &h, sizeof(h), hipMemcpyHostToDevice));
            launch_rng(o, s); launch_rng(a, s);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(st, &h, sizeof(h), hipMemcpyHostToDevice));
            launch_rng(o, s); launch_rng(b, s);
            CK(hipStreamSynchronize(s));
            size_t bad = 0;
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
            printf("%-22s split == one-kernel: %s (%zu mismatches)\n", cf.name, bad ? "NO" : "yes", bad);
        }
        for (int w = 0; w < 3; ++w) launch_rng(a, s);
        CK(hipStreamSynchronize(s));
        unsigned long long z[8] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_rng_prof), z, sizeof(z)));
        const int n = 20;
        auto t0 = std::chrono::high_resolution_clock::now();
        for (int i = 0; i < n; ++i) launch_rng(a, s);
        CK(hipStreamSynchronize(s));
        auto t1 = std::chrono::high_resolution_clock::now();
        CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(g_rng_prof), sizeof(z)));
        const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / (n * cf.nupd);
        const double upd = (double)n * cf.nupd;
        printf("%-22s %8.2f us/update | twist %7.2f  randint %6.2f  gauss %7.2f  kernel %7.2f us/update | "
               "bursts %.1f chunks %.1f per update\n", cf.name, us, z[0] * 0.01 / upd, z[1] * 0.01 / upd,
               z[2] * 0.01 / upd, z[3] * 0.01 / upd, z[4] / upd, z[5] / upd);
    }
    return 0;
}
