// Isolated timing of the row kernels with random data (graph replay).
#include "../sac-expert_amd/csrc/k_sac.hip"
#include <chrono>
#include <cstdio>
#include <functional>
#include <vector>
#include <random>
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
    const size_t NF = 16 << 20;
    float* buf; CK(hipMalloc(&buf, NF * 4));
    std::vector<float> h(NF); std::mt19937 g(1); std::uniform_real_distribution<float> U(-0.5f, 0.5f);
    for (auto& x : h) x = U(g);
    CK(hipMemcpy(buf, h.data(), NF * 4, hipMemcpyHostToDevice));
    Ctl* ctl; CK(hipMalloc(&ctl, sizeof(Ctl))); CK(hipMemset(ctl, 0, sizeof(Ctl)));
    size_t off = 0; auto take = [&](size_t n) { float* p = buf + off; off += (n + 63) & ~size_t(63); return p; };
    const int B = 256, S = 17, A = 6, H = 256, ldQ = 24;
    const int n = 100;
    // ---- actor head (actor.head shape: 512 rows, 2 evaluate segments)
    {
        HeadArgs a{}; FinalArgs f{};
        a.H2 = take(2 * B * H); a.ldh = H; a.W3 = take((H + 1) * A); a.logstd = take(A);
        a.H1 = H; a.A = A; a.Aout = A; a.S = S; a.ldQ = ldQ; a.lim = 1.f;
        a.a_mean = take(A); a.a_den = take(A);
        CK(hipMemset((void*)a.a_den, 0, 4)); // den must be non-zero: fill below
        std::vector<float> one(A, 1.f); CK(hipMemcpy((void*)a.a_den, one.data(), 4 * A, hipMemcpyHostToDevice));
        a.nseg = 2;
        a.seg[0] = {0, B, 0, 0, take(B * A), take(B * ldQ), take(B)};
        a.seg[1] = {B, 2 * B, 0, 0, take(B * A), take(B * ldQ), take(B)};
        a.total_rows = 2 * B; a.cache_row0 = B;
        a.c_t = take(B * A); a.c_std = take(B * A); a.c_u = take(B * A); a.c_mask = take(B * A);
        printf("actor_head 512 rows          : %.2f us\n", tgraph(s, n, [&](int) { launch_actor_head(a, f, s); }));
        HeadArgs b = a; b.nseg = 1; b.seg[0].r1 = B; b.total_rows = B; b.cache_row0 = 1 << 30; b.c_t = nullptr;
        printf("actor_head 256 rows no cache : %.2f us\n", tgraph(s, n, [&](int) { launch_actor_head(b, f, s); }));
        // alpha mode with finalize
        f.alpha = take(1); f.alpha_m = take(1); f.alpha_v = take(1); f.ctl = ctl; f.target_entropy = -6.f;
        f.B = B; f.lq = take(2 * B); f.lp = take(B); f.mse_rows = take(32); f.red = take(1024); f.stats = take(4096 * 8);
        f.stats_cap = 4096; f.adam.lr[2] = 1e-4f;
        HeadArgs c = b; c.alpha_mode = 1;
        printf("alpha head + finalize        : %.2f us\n", tgraph(s, n, [&](int) { launch_actor_head(c, f, s); }));
    }
    // ---- qhead mode 0 and 1
    {
        QHeadArgs q{};
        q.mode = 0; q.B = B; q.H1 = H; q.H2 = take(4 * B * H);
        for (int k = 0; k < 4; ++k) q.W3[k] = take(H + 1);
        q.act = ACT_RELU; q.D2 = take(2 * B * H); q.g = take(2 * B); q.loss_rows = take(2 * B);
        q.alpha = take(1); q.nlp = take(B); q.r = take(B); q.d = take(B); q.gamma = 0.995f; q.ret_den = take(1);
        q.w_sac = 1.f; q.ctl = ctl;
        printf("qhead mode 0                 : %.2f us\n", tgraph(s, n, [&](int) { launch_qhead(q, s); }));
        QHeadArgs q1 = q; q1.mode = 1;
        printf("qhead mode 1                 : %.2f us\n", tgraph(s, n, [&](int) { launch_qhead(q1, s); }));
    }
    // ---- actor bwd
    {
        ActorBwdArgs b{};
        b.B = B; b.ne = 0; b.S = S; b.A = A; b.Aout = A; b.H0 = H; b.H1 = H; b.Hm0 = 1; b.lim = 1.f;
        b.Dp1 = take(2 * B * H); b.Wq1[0] = take((S + A + 1) * H); b.Wq1[1] = take((S + A + 1) * H);
        b.a_den = take(A); std::vector<float> one(A, 1.f); CK(hipMemcpy((void*)b.a_den, one.data(), 4 * A, hipMemcpyHostToDevice));
        b.alpha = take(1); b.ctl = ctl; b.c_t = take(B * A); b.c_std = take(B * A); b.c_u = take(B * A); b.c_mask = take(B * A);
        b.W3a = take((H + 1) * A); b.Ha2 = take(B * H); b.act = ACT_RELU; b.Da3 = take(B * A); b.Da2 = take(B * H); b.E = take(B * A);
        printf("actor_bwd 256 rows           : %.2f us\n", tgraph(s, n, [&](int) { launch_actor_bwd(b, s); }));
    }
    {
        GatherArgs g{};
        int* idx; CK(hipMalloc(&idx, 4 * B)); std::vector<int> hi(B); for (int i = 0; i < B; ++i) hi[i] = (i * 7919) % 100000;
        CK(hipMemcpy(idx, hi.data(), 4 * B, hipMemcpyHostToDevice));
        Ctl hc{}; hc.cur_size = 100000; CK(hipMemcpy(ctl, &hc, sizeof(hc), hipMemcpyHostToDevice));
        g.replay = take(100000 * 44); g.cap = 100000; g.stride = 44; g.S = S; g.A = A; g.B = B; g.ne = 0; g.idx = idx; g.ctl = ctl;
        g.s_mean = take(S); g.s_den = take(S); g.a_mean = take(A); g.a_den = take(A);
        g.Xa = take(2 * B * 20); g.ldS = 20; g.Xq = take(B * ldQ); g.Xt = take(B * ldQ); g.Xp = take(B * ldQ); g.Xm = take(ldQ); g.ldQ = ldQ;
        g.r = take(B); g.d = take(B);
        printf("gather 256 rows              : %.2f us\n", tgraph(s, n, [&](int) { launch_gather(g, s); }));
    }
    return 0;
}
