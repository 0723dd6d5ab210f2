// gfx950 (MI355X / CDNA4) kernels of the SAC / SAC-EO update.
//
// One gradient step (SAC_expert.py:463-477) is a fixed DAG of ~20 launches,
// captured once into a hipGraph by sacx.cpp:
//   k_rng          NumPy-legacy MT19937 sampler: randint + polar normals (1 WG)
//   k_gather       replay ring -> normalised batch staging (coalesced rows)
//   k_gemm         grouped fp32-MFMA GEMM, 16x16 tiles, K split over 4 waves,
//                  fused epilogues: bias+activation / activation-derivative /
//                  Keras-Adam (+ Polyak target sync)
//   k_actor_head   Dense(H->A) + squashed-Gaussian evaluate/sample (+ alpha
//                  update & per-step statistics by the last-arriving workgroup)
//   k_qhead        Dense(H->1) of the twin Q / targets + min + TD target + loss
//                  gradients (+ world-model expert-MSE rows for SAC-EO)
//   k_actor_bwd    action gradient through Q / model input columns + tanh-
//                  Gaussian backward + Dense(H->A) backward
//
// Elementwise arithmetic is compiled without FP contraction so every op
// rounds like the reference's separate TF ops (dot products use explicit
// fmaf).  GEMM accumulation is the exact-f32 MFMA (k-ordered fmaf chain).
#include <hip/hip_runtime.h>
#include <math.h>
#include "sacx_internal.h"

#pragma clang fp contract(off)

namespace sacx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define LOG2PI_F 0x1.d67f1ep+0f     // f32 log(f32(2*pi))  (continuous_actors.py:360)
#define LN2_F 0x1.62e430p-1f        // f32(np.log(2.))     (continuous_actors.py:366)
#define SOFTPLUS_THR -0x1.be2804p+3f  // log(FLT_EPSILON) + 2 (TF softplus_op.h)

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ float act_f(float z, int act) {
    switch (act) {
        case ACT_RELU: return z > 0.f ? z : 0.f;
        case ACT_TANH: return tanhf(z);
        case ACT_ELU: return z < 0.f ? expf(z) - 1.f : z;
        default: return z;
    }
}

// derivative through the layer OUTPUT h (TF ReluGrad / TanhGrad / EluGrad)
__device__ __forceinline__ float dact_f(float h, int act) {
    switch (act) {
        case ACT_RELU: return h > 0.f ? 1.f : 0.f;
        case ACT_TANH: return 1.f - h * h;
        case ACT_ELU: return h < 0.f ? h + 1.f : 1.f;
        default: return 1.f;
    }
}

__device__ __forceinline__ float softplus_f(float x) {
    if (x > -SOFTPLUS_THR) return x;
    if (x < SOFTPLUS_THR) return expf(x);
    return log1pf(expf(x));
}

// butterfly sum over the 64 lanes; lane 0's value is broadcast so every lane
// holds the bit-identical result
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// quad xor-1, xor-2, then row rotate 4 and 8 (DPP, full-rate VALU): every lane of
// a 16-lane row holds the row sum; the four row sums are read from lanes
// 0/16/32/48 and added in a fixed order, so the result is wave-uniform and
// bit-identical on every lane.
__device__ __forceinline__ float wave_sum(float v) {
    v = v + dpp<0xB1>(v);
    v = v + dpp<0x4E>(v);
    v = v + dpp<0x124>(v);
    v = v + dpp<0x128>(v);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}

__device__ __forceinline__ float adam_lr(const AdamConsts& c, int group, int64_t t) {
    const float b1 = 0.9f, b2 = 0.999f;
    const float tt = (float)t;
    const float b1p = powf(b1, tt), b2p = powf(b2, tt);
    return c.lr[group] * sqrtf(1.f - b2p) / (1.f - b1p);
}

// Keras Adam (ResourceApplyAdam): m += (g-m)(1-b1); v += (g^2-v)(1-b2);
// var -= (m*lr_t)/(sqrt(v)+eps)
__device__ __forceinline__ float adam_update(float* p, float* m, float* v, float g, float lr_t) {
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
    float mm = *m, vv = *v;
    mm = mm + (g - mm) * (1.f - b1);
    vv = vv + (g * g - vv) * (1.f - b2);
    const float pn = *p - (mm * lr_t) / (sqrtf(vv) + eps);
    *m = mm;
    *v = vv;
    *p = pn;
    return pn;
}

// ---------------------------------------------------------------- row helpers
// A row of a hidden layer (width H <= 64*MAXQ) is held as hv[q] = h[lane + 64 q];
// all loads of a row are issued before any reduction so the wave's memory
// latency overlaps instead of serialising behind each butterfly.
#define MAXQ 8
__device__ __forceinline__ void load_row(const float* __restrict__ h, int H, float (&hv)[MAXQ]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
        const int k = lane + 64 * q;
        hv[q] = (k < H) ? h[k] : 0.f;
    }
}

// out[u] = sum_k hv(k) * W[k*ldw + o0 + u] for u < 8 (o0+u < O); broadcast to all lanes
__device__ __forceinline__ void rowdot8(const float (&hv)[MAXQ], const float* __restrict__ W, int H, int ldw,
                                        int o0, int O, float (&out)[8]) {
    const int lane = threadIdx.x & 63;
    float p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = 0.f;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
        const int k = lane + 64 * q;
        if (k < H) {
            const float* wr = W + (size_t)k * ldw + o0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (o0 + u < O) p[u] = fmaf(hv[q], wr[u], p[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) out[u] = wave_sum(p[u]);
}

// ==================================================================== k_gemm
__device__ __forceinline__ void load_a(const GemmProb& g, int m, bool mok, int k0, bool vec, float (&a)[4]) {
    if (g.a_kc) {
        if (mok) {
            const float* src = g.A + (size_t)m * g.lda + k0;
            if (vec && k0 + 3 < g.K) {
                const float4 v = *reinterpret_cast<const float4*>(src);
                a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) a[j] = (k0 + j < g.K) ? src[j] : 0.f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = 0.f;
        }
    } else {
        const bool ones = (m == g.ones_row);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + j;
            float x = 0.f;
            if (mok && k < g.K) x = ones ? 1.f : g.A[(size_t)k * g.lda + m];
            a[j] = x;
        }
    }
}

__device__ __forceinline__ void load_b(const GemmProb& g, int n, bool nok, int k0, bool vec, float (&b)[4]) {
    if (g.b_kc) {
        if (nok) {
            const float* src = g.B + (size_t)n * g.ldb + k0;
            if (vec && k0 + 3 < g.K) {
                const float4 v = *reinterpret_cast<const float4*>(src);
                b[0] = v.x; b[1] = v.y; b[2] = v.z; b[3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) b[j] = (k0 + j < g.K) ? src[j] : 0.f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = 0.f;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + j;
            b[j] = (nok && k < g.K) ? g.B[(size_t)k * g.ldb + n] : 0.f;
        }
    }
}

__global__ __launch_bounds__(256) void k_gemm(GemmArgs ga) {
    __shared__ float red[4][4][64];
    const int tile = blockIdx.x;
    int p = 0;
#pragma unroll
    for (int i = 1; i < GEMM_MAXP; ++i)
        if (i < ga.nprob && tile >= ga.probs[i].tile_begin) p = i;
    const GemmProb& g = ga.probs[p];
    const int lt = tile - g.tile_begin;
    const int tm = lt / g.tiles_n;
    const int tn = lt - tm * g.tiles_n;
    const int m0 = tm * 16, n0 = tn * 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, grp = lane >> 4;

    // ---- epilogue operands first: this thread's output element is known now,
    //      so its loads overlap the operand loads instead of following the MFMAs
    const int t = threadIdx.x;
    const int row = t >> 4, col = t & 15;
    const int mm = m0 + row, nn = n0 + col;
    const bool out_ok = (mm < g.M) && (nn < g.N);
    const int epi = g.epi;
    float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;
    size_t pidx = 0;
    if (out_ok) {
        if (epi == EPI_FWD) {
            e0 = g.bias[nn];
        } else if (epi == EPI_DACT) {
            e0 = g.H[(size_t)mm * g.ldh + nn];
        } else if (epi == EPI_ADAM) {
            pidx = (size_t)mm * g.ldp + nn;
            e0 = g.P[pidx];
            e1 = g.P[pidx + ga.p_stride];
            e2 = g.P[pidx + 2 * ga.p_stride];
            if (g.T != nullptr) e3 = g.T[pidx];
        }
    }

    const int nIt = (g.K + 15) >> 4;
    const int per = (nIt + 3) >> 2;
    const int it0 = wave * per;
    const int it1 = min(nIt, it0 + per);
    const int m = m0 + r, n = n0 + r;
    const bool mok = m < g.M, nok = n < g.N;
    const bool avec = g.a_kc && ((g.lda & 3) == 0) && ((((uintptr_t)g.A) & 15) == 0);
    const bool bvec = g.b_kc && ((g.ldb & 3) == 0) && ((((uintptr_t)g.B) & 15) == 0);

    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f};
    floatx4 acc1 = {0.f, 0.f, 0.f, 0.f};
    for (int it = it0; it < it1; it += 4) {
        float a[4][4], b[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (it + u < it1) {
                const int k0 = (it + u) * 16 + grp * 4;
                load_a(g, m, mok, k0, avec, a[u]);
                load_b(g, n, nok, k0, bvec, b[u]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) { a[u][j] = 0.f; b[u][j] = 0.f; }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0], b[u][0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1], b[u][1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][2], b[u][2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][3], b[u][3], acc1, 0, 0, 0);
        }
    }
    const floatx4 acc = acc0 + acc1;
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][q][lane] = acc[q];
    __syncthreads();

    // (row, col) lives in lane (row>>2)*16+col, register row&3 of each wave's tile
    const int L = ((row >> 2) << 4) | col, R = row & 3;
    float v = red[0][R][L] + red[1][R][L];
    v = v + red[2][R][L];
    v = v + red[3][R][L];
    if (!out_ok) return;
    switch (epi) {
        case EPI_FWD:
            g.C[(size_t)mm * g.ldc + nn] = act_f(v + e0, g.act);
            break;
        case EPI_DACT:
            g.C[(size_t)mm * g.ldc + nn] = v * dact_f(e0, g.act);
            break;
        case EPI_STORE:
            g.C[(size_t)mm * g.ldc + nn] = v;
            break;
        case EPI_ADAM: {
            const Ctl* ctl = ga.ctl;
            const int64_t tstep = (g.group == GRP_MODEL ? ctl->t_model : ctl->t_sac) + 1;
            const float lr_t = adam_lr(ga.adam, g.group, tstep);
            const float gr = v * g.grad_scale;
            const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
            const float mm1 = e1 + (gr - e1) * (1.f - b1);
            const float vv1 = e2 + (gr * gr - e2) * (1.f - b2);
            const float pn = e0 - (mm1 * lr_t) / (sqrtf(vv1) + eps);
            g.P[pidx] = pn;
            g.P[pidx + ga.p_stride] = mm1;
            g.P[pidx + 2 * ga.p_stride] = vv1;
            if (g.T != nullptr) {
                const int64_t tui = ga.adam.target_update_int > 0 ? ga.adam.target_update_int : 1;
                if (ctl->num_timesteps % tui == 0) g.T[pidx] = e3 * ga.adam.tau_keep + pn * ga.adam.tau_take;
            }
            break;
        }
    }
}

void launch_gemm(const GemmArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gemm, dim3(a.total_tiles), dim3(256), 0, s, a);
}

// ==================================================================== k_rng
// NumPy legacy RandomState stream, one workgroup:
//   phase 1: randint(cur_size, n_int)  masked rejection on 32-bit words
//   phase 2: n_norm x legacy_gauss     polar method, cached second value
// Words are consumed straight from the current MT block; items are accepted in
// parallel and ranked with a block-wide ballot prefix count.  A twist happens
// only once the block is exhausted (a <4-word gauss remainder is carried), so
// the state written back is always (current block, position).
#define RNG_THREADS 1024

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_tw(uint32_t cur, uint32_t nxt, uint32_t far) {
    const uint32_t y = (cur & 0x80000000U) | (nxt & 0x7fffffffU);
    return far ^ (y >> 1) ^ ((0U - (y & 1U)) & 0x9908b0dfU);
}

__device__ void mt_twist(uint32_t* mt) {
    const int t = threadIdx.x;
    uint32_t v = 0;
    if (t < 227) v = mt_tw(mt[t], mt[t + 1], mt[t + 397]);
    __syncthreads();
    if (t < 227) mt[t] = v;
    __syncthreads();
    if (t < 227) v = mt_tw(mt[227 + t], mt[228 + t], mt[t]);
    __syncthreads();
    if (t < 227) mt[227 + t] = v;
    __syncthreads();
    if (t < 170) {
        const int i = 454 + t;
        v = (i < 623) ? mt_tw(mt[i], mt[i + 1], mt[i - 227]) : mt_tw(mt[623], mt[0], mt[396]);
    }
    __syncthreads();
    if (t < 170) mt[454 + t] = v;
    __syncthreads();
}

// exclusive rank of `flag` among flagged threads, and the block total
__device__ __forceinline__ int block_rank(bool flag, int* wtot, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long bal = __ballot(flag);
    const int below = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wtot[w] = __popcll(bal);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < RNG_THREADS / 64; ++i) {
        const int c = wtot[i];
        off += (i < w) ? c : 0;
        tot += c;
    }
    total = tot;
    __syncthreads();
    return off + below;
}

__global__ __launch_bounds__(RNG_THREADS) void k_rng(RngArgs a) {
    __shared__ uint32_t mt[624];
    __shared__ uint32_t win[628];
    __shared__ int wtot[RNG_THREADS / 64];
    __shared__ int sh_last;
    __shared__ double sh_gauss;
    __shared__ int sh_has;
    const int t = threadIdx.x;
    for (int i = t; i < 624; i += RNG_THREADS) mt[i] = a.st->key[i];
    int pos = a.st->pos;
    if (t == 0) {
        sh_has = a.st->has_gauss;
        sh_gauss = a.st->gauss;
    }
    __syncthreads();

    // ---------------- randint(high, n_int)
    if (a.n_int > 0) {
        const uint64_t high = (uint64_t)a.ctl->cur_size;
        const uint64_t rng = high > 0 ? high - 1 : 0;
        uint64_t mask = rng;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
        mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
        int done = 0;
        while (done < a.n_int) {
            if (rng == 0) {
                for (int i = t; i < a.n_int; i += RNG_THREADS) a.out_idx[i] = 0;
                break;
            }
            if (pos == 624) {
                mt_twist(mt);
                pos = 0;
            }
            const int L = 624 - pos;
            bool acc = false;
            uint32_t v = 0;
            if (t < L) {
                const uint32_t w = mt_temper(mt[pos + t]);
                if (rng == 0xFFFFFFFFULL) {
                    v = w;
                    acc = true;
                } else {
                    v = w & (uint32_t)mask;
                    acc = (uint64_t)v <= rng;
                }
            }
            int total;
            const int rank = block_rank(acc, wtot, total);
            const int need = a.n_int - done;
            if (acc && rank < need) a.out_idx[done + rank] = (int32_t)v;
            if (acc && rank == need - 1) sh_last = t;
            __syncthreads();
            if (total >= need) {
                pos += sh_last + 1;
                done = a.n_int;
            } else {
                pos += L;
                done += total;
            }
            __syncthreads();
        }
    }

    // ---------------- n_norm x gauss
    int oi = 0;
    if (a.n_norm > 0 && sh_has) {
        if (t == 0) a.out_norm[0] = (float)sh_gauss;
        oi = 1;
        __syncthreads();
        if (t == 0) { sh_has = 0; sh_gauss = 0.0; }
    }
    int cl = 0;  // carried words at win[0..cl)
    while (oi < a.n_norm) {
        if (pos == 624) {          // only reachable when the previous phase ended exactly on a block edge
            mt_twist(mt);
            pos = 0;
        }
        const int fresh = 624 - pos;
        const int L = cl + fresh;
        if (t < fresh) win[cl + t] = mt_temper(mt[pos + t]);
        __syncthreads();
        const int items = L >> 2;
        bool acc = false;
        double f = 0.0, x1 = 0.0, x2 = 0.0;
        if (t < items) {
            const uint32_t w0 = win[4 * t], w1 = win[4 * t + 1], w2 = win[4 * t + 2], w3 = win[4 * t + 3];
            const double u1 = ((double)(int32_t)(w0 >> 5) * 67108864.0 + (double)(int32_t)(w1 >> 6)) / 9007199254740992.0;
            const double u2 = ((double)(int32_t)(w2 >> 5) * 67108864.0 + (double)(int32_t)(w3 >> 6)) / 9007199254740992.0;
            x1 = 2.0 * u1 - 1.0;
            x2 = 2.0 * u2 - 1.0;
            const double r2 = x1 * x1 + x2 * x2;
            acc = (r2 < 1.0) && (r2 != 0.0);
            if (acc) f = sqrt(-2.0 * log(r2) / r2);
        }
        int total;
        const int rank = block_rank(acc, wtot, total);
        const int need_vals = a.n_norm - oi;
        const int need_pairs = (need_vals + 1) >> 1;
        if (acc && rank < need_pairs) {
            const int o = oi + 2 * rank;
            a.out_norm[o] = (float)(f * x2);
            if (o + 1 < a.n_norm) {
                a.out_norm[o + 1] = (float)(f * x1);
            } else {
                sh_gauss = f * x1;
                sh_has = 1;
            }
        }
        if (acc && rank == need_pairs - 1) sh_last = t;
        __syncthreads();
        if (total >= need_pairs) {
            pos = pos + 4 * (sh_last + 1) - cl;
            cl = 0;
            oi = a.n_norm;
        } else {
            oi += 2 * total;
            const int used = 4 * items;
            const int left = L - used;
            uint32_t keep = 0;
            if (t < left) keep = win[used + t];
            __syncthreads();
            if (t < left) win[t] = keep;
            cl = left;
            mt_twist(mt);
            pos = 0;
        }
        __syncthreads();
    }

    for (int i = t; i < 624; i += RNG_THREADS) a.st->key[i] = mt[i];
    if (t == 0) {
        a.st->pos = pos;
        a.st->has_gauss = sh_has;
        a.st->gauss = sh_gauss;
    }
}

void launch_rng(const RngArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_rng, dim3(1), dim3(RNG_THREADS), 0, s, a);
}

// ==================================================================== k_gather
// one wave per sampled row (then per expert row); rows are [s | a | sp | r | d]
__global__ __launch_bounds__(256) void k_gather(GatherArgs g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    const int S = g.S, A = g.A;
    if (row < g.B) {
        const int64_t li = g.idx[row];
        const int64_t phys = (g.ctl->start + li) % g.cap;
        const float* rec = g.replay + phys * (int64_t)g.stride;
        for (int c = lane; c < g.ldQ; c += 64) {
            float sn = 0.f, spn = 0.f, an = 0.f;
            if (c < S) {
                sn = (rec[c] - g.s_mean[c]) / g.s_den[c];
                spn = (rec[S + A + c] - g.s_mean[c]) / g.s_den[c];
            } else if (c < S + A) {
                an = (rec[c] - g.a_mean[c - S]) / g.a_den[c - S];
            }
            if (c < g.ldS) {
                g.Xa[(size_t)row * g.ldS + c] = spn;
                g.Xa[(size_t)(g.B + row) * g.ldS + c] = sn;
            }
            g.Xq[(size_t)row * g.ldQ + c] = (c < S) ? sn : an;
            if (c < S) {
                g.Xt[(size_t)row * g.ldQ + c] = spn;
                g.Xp[(size_t)row * g.ldQ + c] = sn;
            } else if (c >= S + A) {
                g.Xt[(size_t)row * g.ldQ + c] = 0.f;
                g.Xp[(size_t)row * g.ldQ + c] = 0.f;
            }
        }
        if (lane == 0) {
            g.r[row] = rec[2 * S + A];
            g.d[row] = rec[2 * S + A + 1];
        }
    } else if (row < g.B + g.ne) {
        const int e = row - g.B;
        const int64_t slot = g.ctl->step_seq % g.perm_cap;
        const int src = g.perm_ring[slot * g.ne + e];
        const float* s_e = g.exp_s + (size_t)src * S;
        const float* sp_e = g.exp_sp + (size_t)src * S;
        for (int c = lane; c < g.ldQ; c += 64) {
            float sn = 0.f;
            if (c < S) {
                sn = (s_e[c] - g.s_mean[c]) / g.s_den[c];
                g.se_raw[(size_t)e * S + c] = s_e[c];
                g.spe_raw[(size_t)e * S + c] = sp_e[c];
            }
            if (c < g.ldS) g.Xa[(size_t)(2 * g.B + e) * g.ldS + c] = sn;
            if (c < S) g.Xm[(size_t)e * g.ldQ + c] = sn;
            else if (c >= S + A) g.Xm[(size_t)e * g.ldQ + c] = 0.f;
        }
    }
}

void launch_gather(const GatherArgs& a, hipStream_t s) {
    const int rows = a.B + a.ne;
    hipLaunchKernelGGL(k_gather, dim3((rows + 3) / 4), dim3(256), 0, s, a);
}

// ==================================================================== finalize
// alpha Adam + clamp and the per-update statistics (last-arriving workgroup).
__device__ float mean_rows(const float* x, int n) {
    // deterministic: lane-strided partials then butterfly (wave 0 only)
    const int lane = threadIdx.x & 63;
    float s = 0.f;
    for (int i = lane; i < n; i += 64) s += x[i];
    return wave_sum(s) / (float)n;
}

__device__ void finalize_update(const FinalArgs& f, int nred, float nlp_sum_total_unused) {
    (void)nlp_sum_total_unused;
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x & 63;
    float s = 0.f;
    for (int i = lane; i < nred; i += 64) s += f.red[i];
    const float ent_sum = wave_sum(s);          // sum_i (-nlp_i + H)
    const float m_ent = ent_sum / (float)f.B;   // reduce_mean
    const float q1 = mean_rows(f.lq, f.B);
    const float q2 = mean_rows(f.lq + f.B, f.B);
    float pl = mean_rows(f.lp, f.B);
    float mse = 0.f;
    if (f.use_expert && f.ne > 0) {
        const int h = f.ne / 2;
        float sm = 0.f;
        for (int i = lane; i < h; i += 64) sm += 0.5f * (f.mse_rows[i] + f.mse_rows[i + h]);
        mse = wave_sum(sm) / (float)h;
        const float eps = f.ctl->epsilon;
        pl = (1.f - eps) * pl + eps * mse;
    }
    if (lane == 0) {
        Ctl* ctl = f.ctl;
        const int64_t tnew = ctl->t_sac + 1;
        const float alpha_old = *f.alpha;
        const float g = -m_ent;                 // d(-alpha*m)/d alpha
        const float lr_t = adam_lr(f.adam, GRP_ALPHA, tnew);
        float an = adam_update(f.alpha, f.alpha_m, f.alpha_v, g, lr_t);
        an = fmaxf(an, 1e-5f);                  // SAC_expert.py:348
        *f.alpha = an;
        const int64_t seq = ctl->step_seq;
        float* st = f.stats + (size_t)(seq % f.stats_cap) * 8;
        st[0] = q1;
        st[1] = q2;
        st[2] = pl;
        st[3] = -alpha_old * m_ent;
        st[4] = an;
        st[5] = mse;
        st[6] = -(m_ent - f.target_entropy);    // mean neglogp (diagnostic)
        st[7] = (float)seq;
        ctl->t_sac = tnew;
        ctl->num_timesteps += ctl->ts_increment;
        ctl->step_seq = seq + 1;
    }
}

// ==================================================================== k_actor_head
// one wave per actor row: mu = h2 . W3 + b, then evaluate()/sample() per column.
// The wave sums are broadcast, so lane j keeps output j in a register.
__global__ __launch_bounds__(256) void k_actor_head(HeadArgs h, FinalArgs f) {
    __shared__ float red_s[4];
    __shared__ int last_s;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    float row_ent = 0.f;
    if (row < h.total_rows) {
        int sidx = 0;
        for (int i = 1; i < h.nseg; ++i)
            if (row >= h.seg[i].r0) sidx = i;
        const HeadSeg sg = h.seg[sidx];
        float hv[MAXQ];
        load_row(h.H2 + (size_t)row * h.ldh, h.H1, hv);
        float u_pf = 0.f, ls_pf = 0.f, am_pf = 0.f, ad_pf = 1.f;
        if (lane < h.A) {
            u_pf = sg.noise[(size_t)(row - sg.r0) * h.A + lane];
            if (!h.per_state_std) ls_pf = h.logstd[lane];
            am_pf = h.a_mean[lane];
            ad_pf = h.a_den[lane];
        }
        const float* bias = h.W3 + (size_t)h.H1 * h.Aout;
        float mu = 0.f, lraw = 0.f;
        for (int o0 = 0; o0 < h.Aout; o0 += 8) {
            float s8[8];
            rowdot8(hv, h.W3, h.H1, h.Aout, o0, h.Aout, s8);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int o = o0 + u;
                if (o < h.Aout) {
                    const float sv = s8[u] + bias[o];
                    if (lane == o) mu = sv;
                    if (h.per_state_std && lane + h.A == o) lraw = sv;
                }
            }
        }
        float nlp_vec = 0.f, nlp_corr = 0.f;
        if (lane < h.A) {
            const int j = lane;
            if (!h.per_state_std) lraw = ls_pf;
            const float l = fminf(fmaxf(lraw, -5.f), 2.f);
            const float sd = expf(l);
            const float u = u_pf;
            const float x = mu + sd * u;
            const float t = tanhf(x);
            const float pi = h.lim * t;
            if (sg.mode == 0) {
                const float z = (x - mu) / expf(l);
                nlp_vec = z * z + 2.f * l + LOG2PI_F;
                nlp_corr = 2.f * ((LN2_F - x) - softplus_f(-2.f * x));
            }
            if (sg.xq_out != nullptr)
                sg.xq_out[(size_t)(sg.xq_row0 + row - sg.r0) * h.ldQ + h.S + j] = (pi - am_pf) / ad_pf;
            if (row >= h.cache_row0 && h.c_t != nullptr) {
                const size_t ci = (size_t)(row - h.cache_row0) * h.A + j;
                h.c_t[ci] = t;
                h.c_std[ci] = sd;
                h.c_u[ci] = u;
                h.c_mask[ci] = (lraw >= -5.f && lraw <= 2.f) ? 1.f : 0.f;
            }
        }
        if (sg.mode == 0) {
            const float nlp = 0.5f * wave_sum(nlp_vec) + wave_sum(nlp_corr);
            if (lane == 0 && sg.nlp_out != nullptr) sg.nlp_out[row - sg.r0] = nlp;
            row_ent = -nlp + f.target_entropy;
        }
    }
    if (!h.alpha_mode) return;
    // ---- alpha: block partial of sum(-nlp + H), then the last arriver finalises
    if (lane == 0) red_s[wave] = row_ent;
    __syncthreads();
    if (threadIdx.x == 0) {
        float part = red_s[0] + red_s[1];
        part = part + red_s[2];
        part = part + red_s[3];
        f.red[blockIdx.x] = part;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int tk = __hip_atomic_fetch_add(&f.ctl->red_counter[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int is_last = (tk == (int)gridDim.x - 1);
        if (is_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&f.ctl->red_counter[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        last_s = is_last;
    }
    __syncthreads();
    if (!last_s) return;
    finalize_update(f, (int)gridDim.x, 0.f);
}

void launch_actor_head(const HeadArgs& a, const FinalArgs& f, hipStream_t s) {
    hipLaunchKernelGGL(k_actor_head, dim3((a.total_rows + 3) / 4), dim3(256), 0, s, a, f);
}

// ==================================================================== k_qhead
template <int MODE>
__global__ __launch_bounds__(256) void k_qhead(QHeadArgs q) {
    __shared__ float buf[4][512];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    const int B = q.B, H1 = q.H1;
    if (row < B) {
        constexpr int nnet = (MODE == 0) ? 4 : 2;
        const float alpha = *q.alpha;
        const float nlp_r = q.nlp[row];
        float r_r = 0.f, d_r = 0.f, rd = 1.f;
        if (MODE == 0) {
            r_r = q.r[row];
            d_r = q.d[row];
            rd = *q.ret_den;
        }
        float hv[4][MAXQ];
        float wv[4][MAXQ];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < nnet) {
                load_row(q.H2 + ((size_t)k * B + row) * H1, H1, hv[k]);
                load_row(q.W3[k], H1, wv[k]);
            }
        }
        float out[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float p = 0.f;
            if (k < nnet) {
#pragma unroll
                for (int i = 0; i < MAXQ; ++i) p = fmaf(hv[k][i], wv[k][i], p);
            }
            out[k] = wave_sum(p);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < nnet) out[k] = out[k] + q.W3[k][H1];
        float g0, g1;
        if (MODE == 0) {
            const float v0 = out[0] * rd, v1 = out[1] * rd;
            const float nv = fminf(v0, v1) + alpha * nlp_r;
            const float y = r_r + q.gamma * ((1.f - d_r) * nv);
            const float e0 = out[2] - y, e1 = out[3] - y;
            const float invB = 1.f / (float)B;
            g0 = e0 * invB;
            g1 = e1 * invB;
            if (lane == 0) {
                q.loss_rows[row] = 0.5f * (e0 * e0);
                q.loss_rows[B + row] = 0.5f * (e1 * e1);
                q.g[row] = g0;
                q.g[B + row] = g1;
            }
        } else {
            const float q0 = out[0], q1 = out[1];
            const float minq = fminf(q0, q1);
            if (lane == 0) q.loss_rows[row] = (-alpha) * nlp_r - minq;
            const float gmin = -q.w_sac * (1.f / (float)B);
            const float s0 = q0 < q1 ? 1.f : (q0 == q1 ? 0.5f : 0.f);
            const float s1 = q1 < q0 ? 1.f : (q0 == q1 ? 0.5f : 0.f);
            g0 = gmin * s0;
            g1 = gmin * s1;
        }
        // differentiated nets: slabs 2,3 (mode 0) or 0,1 (mode 1)
        constexpr int dn0 = MODE == 0 ? 2 : 0;
        float* d0 = q.D2 + (size_t)row * H1;
        float* d1 = q.D2 + ((size_t)B + row) * H1;
#pragma unroll
        for (int i = 0; i < MAXQ; ++i) {
            const int k = lane + 64 * i;
            if (k < H1) {
                const float a0 = dn0 == 2 ? hv[2][i] : hv[0][i];
                const float a1 = dn0 == 2 ? hv[3][i] : hv[1][i];
                const float w0 = dn0 == 2 ? wv[2][i] : wv[0][i];
                const float w1 = dn0 == 2 ? wv[3][i] : wv[1][i];
                d0[k] = (g0 * w0) * dact_f(a0, q.act);
                d1[k] = (g1 * w1) * dact_f(a1, q.act);
            }
        }
        return;
    }
    // ---- SAC-EO: world-model L3 on the expert rows + MSE and its gradient
    if (MODE != 0 || row >= B + q.ne) return;
    const int e = row - B;
    const int half = q.ne / 2;
    const int k = e < half ? 0 : 1;
    const int S = q.S, Hm = q.Hm1, O = S + 1;
    const float* hr = q.Hm2 + (size_t)e * Hm;
    const float* W = k ? q.Wm3[1] : q.Wm3[0];
    float* ob = buf[wave];
    for (int j = 0; j < S; ++j) {
        float p = 0.f;
        for (int i = lane; i < Hm; i += 64) p = fmaf(hr[i], W[(size_t)i * O + j], p);
        const float s = wave_sum(p);
        if (lane == 0) ob[j] = s + W[(size_t)Hm * O + j];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const float eps = q.ctl->epsilon;
    const float gscale = -eps * (1.f / (float)half);
    float sq = 0.f;
    for (int j = lane; j < S; j += 64) {
        const float sp_hat = q.se_raw[(size_t)e * S + j] + (ob[j] * q.d_den[j] + q.d_mean[j]);
        const float diff = q.spe_raw[(size_t)e * S + j] - sp_hat;
        sq = sq + diff * diff;
        ob[j] = (gscale * diff) * q.d_den[j];   // d loss / d out_j
    }
    const float tot = wave_sum(sq);
    if (lane == 0) q.mse_rows[e] = tot;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int i = lane; i < Hm; i += 64) {
        float p = 0.f;
        for (int j = 0; j < S; ++j) p = fmaf(ob[j], W[(size_t)i * O + j], p);
        q.Dm2[(size_t)e * Hm + i] = p * dact_f(hr[i], q.mact);
    }
}

void launch_qhead(const QHeadArgs& a, hipStream_t s) {
    const int rows = a.B + (a.mode == 0 ? a.ne : 0);
    if (a.mode == 0) hipLaunchKernelGGL(k_qhead<0>, dim3((rows + 3) / 4), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_qhead<1>, dim3((rows + 3) / 4), dim3(256), 0, s, a);
}

// ==================================================================== k_actor_bwd
// one wave per actor row of the loss: action gradient through the Q (policy
// rows) or world-model (expert rows) input columns, tanh-Gaussian backward
// (SURVEY.md §8a A5), then the Dense(H1 -> Aout) backward with the activation
// derivative.  Per-column values live in lane j and are broadcast by shuffles.
__global__ __launch_bounds__(256) void k_actor_bwd(ActorBwdArgs b) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    const int B = b.B, S = b.S, A = b.A;
    if (row >= B + b.ne) return;
    const bool pol = row < B;
    const float eps = b.use_expert ? b.ctl->epsilon : 0.f;
    const float alpha = *b.alpha;
    float t_pf = 0.f, sd_pf = 0.f, u_pf = 0.f, mk_pf = 0.f;
    if (lane < A) {
        const size_t ci = (size_t)row * A + lane;
        t_pf = b.c_t[ci];
        sd_pf = b.c_std[ci];
        u_pf = b.c_u[ci];
        mk_pf = b.c_mask[ci];
    }
    float h2v[MAXQ];
    load_row(b.Ha2 + (size_t)row * b.H1, b.H1, h2v);
    const float w_sac = 1.f - eps;
    const float c = -w_sac * alpha * (1.f / (float)B);
    // action gradient: ga_j = sum over the input rows S+j of W1 of the row's layer-1 delta
    float ga = 0.f;
    float dv0[MAXQ], dv1[MAXQ];
    const float* Wa;
    const float* Wb;
    int Hd;
    if (pol) {
        Hd = b.H0;
        load_row(b.Dp1 + (size_t)row * b.H0, Hd, dv0);
        load_row(b.Dp1 + ((size_t)B + row) * b.H0, Hd, dv1);
        Wa = b.Wq1[0];
        Wb = b.Wq1[1];
    } else {
        const int e = row - B;
        const int k = e < b.ne / 2 ? 0 : 1;
        Hd = b.Hm0;
        load_row(b.Dm1 + (size_t)e * b.Hm0, Hd, dv0);
#pragma unroll
        for (int i = 0; i < MAXQ; ++i) dv1[i] = 0.f;
        Wa = b.Wm1[k];
        Wb = b.Wm1[k];
    }
    for (int j0 = 0; j0 < A; j0 += 8) {
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            p[u] = 0.f;
            if (j0 + u < A) {
                const float* wa = Wa + (size_t)(S + j0 + u) * Hd;
                const float* wb = Wb + (size_t)(S + j0 + u) * Hd;
#pragma unroll
                for (int i = 0; i < MAXQ; ++i) {
                    const int k = lane + 64 * i;
                    if (k < Hd) {
                        p[u] = fmaf(dv0[i], wa[k], p[u]);
                        if (pol) p[u] = fmaf(dv1[i], wb[k], p[u]);
                    }
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float sj = wave_sum(p[u]);
            if (j0 + u < A && lane == j0 + u) ga = sj / b.a_den[j0 + u];
        }
    }
    float gx = 0.f, dl = 0.f;
    if (lane < A) {
        const size_t ci = (size_t)row * A + lane;
        const float t = t_pf, sd = sd_pf, u = u_pf, mask = mk_pf;
        gx = ga * b.lim * (1.f - t * t);
        if (pol) gx = gx - (2.f * c) * t;
        dl = (gx * sd) * u;
        if (pol) dl = dl + c;
        dl = dl * mask;
        b.Da3[(size_t)row * b.Aout + lane] = gx;
        if (b.per_state_std) b.Da3[(size_t)row * b.Aout + A + lane] = dl;
        else b.E[ci] = dl;
    }
#pragma unroll
    for (int qq = 0; qq < MAXQ; ++qq) {
        const int i0 = qq * 64;
        const int i = i0 + lane;
        if (i0 >= b.H1) break;
        float p = 0.f;
        for (int o = 0; o < A; ++o) {
            const float d3 = __shfl(gx, o, 64);
            if (i < b.H1) p = fmaf(d3, b.W3a[(size_t)i * b.Aout + o], p);
        }
        if (b.per_state_std) {
            for (int o = 0; o < A; ++o) {
                const float d3 = __shfl(dl, o, 64);
                if (i < b.H1) p = fmaf(d3, b.W3a[(size_t)i * b.Aout + A + o], p);
            }
        }
        if (i < b.H1) b.Da2[(size_t)row * b.H1 + i] = p * dact_f(h2v[qq], b.act);
    }
}

void launch_actor_bwd(const ActorBwdArgs& a, hipStream_t s) {
    const int rows = a.B + a.ne;
    hipLaunchKernelGGL(k_actor_bwd, dim3((rows + 3) / 4), dim3(256), 0, s, a);
}

// ==================================================================== k_append
// TrajectoryBuffer.add (buffers.py:41-71) as a device ring: one workgroup so the
// control-block update is ordered after every row write.
__global__ __launch_bounds__(256) void k_append(AppendArgs a) {
    __shared__ int64_t cur_s, start_s;
    if (threadIdx.x == 0) {
        cur_s = a.ctl->cur_size;
        start_s = a.ctl->start;
    }
    __syncthreads();
    const int64_t cur = cur_s, start = start_s, cap = a.cap, n = a.n;
    const int64_t first = n > cap ? n - cap : 0;   // rows that survive truncation
    const int S = a.S, A = a.A, W = 2 * S + A + 2;
    for (int64_t e = (int64_t)threadIdx.x + first * W; e < n * W; e += blockDim.x) {
        const int64_t i = e / W;
        const int c = (int)(e - i * W);
        const int64_t phys = (start + cur + i) % cap;
        float v;
        if (c < S) v = a.s[i * S + c];
        else if (c < S + A) v = a.a[i * A + (c - S)];
        else if (c < 2 * S + A) v = a.sp[i * S + (c - S - A)];
        else if (c == 2 * S + A) v = a.r[i];
        else v = a.d[i];
        a.replay[phys * a.stride + c] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int64_t tot = cur + n;
        const int64_t drop = tot > cap ? tot - cap : 0;
        a.ctl->start = (start + drop) % cap;
        a.ctl->cur_size = tot - drop;
    }
}

void launch_append(const AppendArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_append, dim3(1), dim3(256), 0, s, a);
}

}  // namespace sacx

namespace sacx {
// per-call control values as kernel arguments (graph/stream ordered, no host buffer lifetime issues)
__global__ void k_set_ctl(Ctl* ctl, int64_t num_timesteps, int64_t ts_increment) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        ctl->num_timesteps = num_timesteps;
        ctl->ts_increment = ts_increment;
    }
}
void launch_set_ctl(Ctl* ctl, int64_t num_timesteps, int64_t ts_increment, hipStream_t s) {
    hipLaunchKernelGGL(k_set_ctl, dim3(1), dim3(64), 0, s, ctl, num_timesteps, ts_increment);
}
}  // namespace sacx

namespace sacx {
// ==================================================================== world-model fitting
// MSEModel.get_loss (continuous_models.py:280-302) summed over the two models
// and one Keras Adam over all their variables (mbrl_onpolicy_alg.py:301-319).
__global__ __launch_bounds__(256) void k_mgather(MGatherArgs g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= 2 * g.mb) return;
    const int S = g.S, A = g.A;
    const int64_t slot = g.ctl->mfit_seq % g.idx_cap;
    const int64_t li = g.idx_ring[slot * 2 * g.mb + row];
    const int64_t phys = (g.ctl->start + li) % g.cap;
    const float* rec = g.replay + phys * (int64_t)g.stride;
    for (int c = lane; c < g.ldQ; c += 64) {
        float x = 0.f;
        if (c < S) x = (rec[c] - g.s_mean[c]) / g.s_den[c];
        else if (c < S + A) x = (rec[c] - g.a_mean[c - S]) / g.a_den[c - S];
        g.X[(size_t)row * g.ldQ + c] = x;
    }
    for (int c = lane; c <= S; c += 64) {
        float y;
        if (c < S) y = ((rec[S + A + c] - rec[c]) - g.d_mean[c]) / g.d_den[c];
        else y = (rec[2 * S + A] - g.r_norm[0]) / g.r_norm[1];
        g.T[(size_t)row * (S + 1) + c] = y;
    }
}

__global__ __launch_bounds__(256) void k_mloss(MLossArgs g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= 2 * g.mb) return;
    const int S = g.S, O = S + 1;
    const float inv = 1.f / (float)g.mb;
    float sq = 0.f, er = 0.f;
    for (int c = lane; c <= S; c += 64) {
        const float e = g.T[(size_t)row * O + c] - g.O[(size_t)row * O + c];
        if (c < S) {
            sq = sq + e * e;
            g.D3[(size_t)row * O + c] = -e * inv;
        } else {
            er = e;
            g.D3[(size_t)row * O + c] = -e * (g.reward_coef * inv);
        }
    }
    const float tot = wave_sum(sq);
    const float e_r = wave_sum(er);
    if (lane == 0) g.loss_rows[row] = 0.5f * tot + g.reward_coef * (0.5f * (e_r * e_r));
}

__global__ __launch_bounds__(64) void k_mfinal(MFinalArgs f) {
    const int lane = threadIdx.x & 63;
    float s0 = 0.f, s1 = 0.f;
    for (int i = lane; i < f.mb; i += 64) {
        s0 += f.loss_rows[i];
        s1 += f.loss_rows[f.mb + i];
    }
    const float l0 = wave_sum(s0) / (float)f.mb, l1 = wave_sum(s1) / (float)f.mb;
    if (lane == 0) {
        const int64_t seq = f.ctl->mfit_seq;
        f.mstats[(size_t)(seq % f.mstats_cap) * 2] = l0 + l1;
        f.mstats[(size_t)(seq % f.mstats_cap) * 2 + 1] = (float)seq;
        f.ctl->t_model += 1;
        f.ctl->mfit_seq = seq + 1;
    }
}

void launch_mgather(const MGatherArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_mgather, dim3((2 * a.mb + 3) / 4), dim3(256), 0, s, a);
}
void launch_mloss(const MLossArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_mloss, dim3((2 * a.mb + 3) / 4), dim3(256), 0, s, a);
}
void launch_mfinal(const MFinalArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_mfinal, dim3(1), dim3(64), 0, s, a);
}
}  // namespace sacx
