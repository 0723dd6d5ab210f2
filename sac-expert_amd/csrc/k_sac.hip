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
#include <cstddef>
#include <cstdlib>
#include <type_traits>
#include <math.h>
#include "sacx_internal.h"

#pragma clang fp contract(off)

namespace sacx {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// fp32 -> bf16 (__bf16 conversion): round to nearest even (v_cvt_pk_bf16_f32 on gfx950)

// One gfx950 v_mfma_f32_16x16x32_bf16 over TWO 16-wide k slabs held the f32 way: lane (r, grp)
// has k = 4 grp + 0..3 of slab 0 in a0 / b0 and of slab 1 in a1 / b1.  The instruction wants k =
// 8 grp + j in element j; A and B carry the same k permutation (element j <-> slab j >> 2, k
// 4 grp + (j & 3)), and a permutation of k common to both operands leaves the sum over k as is.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ floatx4 mfma_bf16_2slab(const float (&a0)[4], const float (&a1)[4], const float (&b0)[4],
                                                   const float (&b1)[4], floatx4 c) {
    const bf16x8_t av = {(__bf16)a0[0], (__bf16)a0[1], (__bf16)a0[2], (__bf16)a0[3],
                         (__bf16)a1[0], (__bf16)a1[1], (__bf16)a1[2], (__bf16)a1[3]};
    const bf16x8_t bv = {(__bf16)b0[0], (__bf16)b0[1], (__bf16)b0[2], (__bf16)b0[3],
                         (__bf16)b1[0], (__bf16)b1[1], (__bf16)b1[2], (__bf16)b1[3]};
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c, 0, 0, 0);
}

#define LOG2PI_F 0x1.d67f1ep+0f     // f32 log(f32(2*pi))  (continuous_actors.py:360)
#define LN2_F 0x1.62e430p-1f        // f32(np.log(2.))     (continuous_actors.py:366)
#define SOFTPLUS_THR -0x1.be2804p+3f  // log(FLT_EPSILON) + 2 (TF softplus_op.h)

// ------------------------------------------------------------------ helpers
template <int ACT>
__device__ __forceinline__ float act_t(float z) {
    if constexpr (ACT == ACT_RELU) return z > 0.f ? z : 0.f;
    else if constexpr (ACT == ACT_TANH) return tanhf(z);
    else if constexpr (ACT == ACT_ELU) return z < 0.f ? expf(z) - 1.f : z;
    else return z;
}

__device__ __forceinline__ float act_f(float z, int act) {
    switch (act) {
        case ACT_RELU: return act_t<ACT_RELU>(z);
        case ACT_TANH: return act_t<ACT_TANH>(z);
        case ACT_ELU: return act_t<ACT_ELU>(z);
        default: return z;
    }
}

// act over a whole register block under ONE wave-uniform branch
template <int N>
__device__ __forceinline__ void act_block(float (&h)[N], int act) {
    switch (act) {
        case ACT_RELU:
#pragma unroll
            for (int i = 0; i < N; ++i) h[i] = act_t<ACT_RELU>(h[i]);
            break;
        case ACT_TANH:
#pragma unroll
            for (int i = 0; i < N; ++i) h[i] = act_t<ACT_TANH>(h[i]);
            break;
        case ACT_ELU:
#pragma unroll
            for (int i = 0; i < N; ++i) h[i] = act_t<ACT_ELU>(h[i]);
            break;
        default: break;
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

// dact_f without a branch on the (launch-uniform) activation: every form, then a select
__device__ __forceinline__ float dact_sel(float h, int act) {
    const float dr = h > 0.f ? 1.f : 0.f;
    const float dt = 1.f - h * h;
    const float de = h < 0.f ? h + 1.f : 1.f;
    return act == ACT_RELU ? dr : (act == ACT_TANH ? dt : (act == ACT_ELU ? de : 1.f));
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
    // c.lr[group], not a chain of selects: the selects made the compiler copy the whole kernarg
    // block into scratch in the 32x32 dW variants
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

// Epilogue stores of the update chain.  Every output is read by the next launch on other
// XCDs; with SACX_WT_STORES the stores are agent-scope (sc1: written through, the line is
// dropped from this XCD's L2), so the end-of-kernel release has no dirty lines to write back.
#ifndef SACX_WT_STORES
#define SACX_WT_STORES 0
#endif
__device__ __forceinline__ void st_out(float* p, float v) {
#if SACX_WT_STORES
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p = v;
#endif
}

// The Adam moments: read again only by the next update's same epilogue, so SACX_NT_MOMENTS stores
// them non-temporal (they need not sit dirty in the XCD L2 that the launch boundary writes back)
#ifndef SACX_NT_MOMENTS
#define SACX_NT_MOMENTS 0
#endif
__device__ __forceinline__ void st_mom(float* p, float v) {
#if SACX_NT_MOMENTS
    __builtin_nontemporal_store(v, p);
#else
    st_out(p, v);
#endif
}

// Raw buffer loads.  Out-of-range elements get an offset past the resource's
// num_records and the hardware returns 0, so every load is unconditional and no
// select follows it (a select on a load result is turned back into a branch
// around the load by the compiler, and a load under a branch ends in vmcnt(0)
// at the block boundary).  Offsets are 32-bit: every tensor read this way is
// < 2 GiB (the replay ring is read with global loads).
#define SACX_BUF_OOB 0x80000000u
#define SACX_RSRC_WORD3 0x00020000

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, SACX_RSRC_WORD3);
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const float* p) { return make_rsrc(p, p ? 0x7fffffffu : 0u); }
// The empty asm hides the select from the optimiser, which would otherwise
// split load(select(ok, off, OOB)) back into two loads under branches.
__device__ __forceinline__ uint32_t boff(bool ok, int elem) {
    uint32_t o = ok ? (uint32_t)elem * 4u : SACX_BUF_OOB;
    asm("" : "+v"(o));
    return o;
}

// a converted slab pair as one bf16x8 operand (k = s0 + 4 grp + j, then s1 + 4 grp + j)
__device__ __forceinline__ bf16x8_t pack_bf16(const float (&x0)[4], const float (&x1)[4]) {
    return bf16x8_t{(__bf16)x0[0], (__bf16)x0[1], (__bf16)x0[2], (__bf16)x0[3],
                    (__bf16)x1[0], (__bf16)x1[1], (__bf16)x1[2], (__bf16)x1[3]};
}
__device__ __forceinline__ bf16x8_t wbf_load(__amdgpu_buffer_rsrc_t r, bool ok, int elem) {
    uint32_t o = ok ? (uint32_t)elem * 2u : SACX_BUF_OOB;
    asm("" : "+v"(o));
    return __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 0));
}
// bf16 image of a float as raw bits (round to nearest even, as the converting loads)
__device__ __forceinline__ uint32_t bf16_bits(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }
// a weight's bf16 shadow element (the Adam epilogues: one 2-B store per updated weight; the
// lane-gathered 8-B form measured slower there -- 3 cross-lane reads per piece, 22.1 vs 17.9 us
// for Humanoid's critic.adam)
__device__ __forceinline__ void wbf_store(uint16_t* S, const GemmProb& g, int k, int n, float v) {
    if (S != nullptr && k < g.wbf_k) S[(size_t)n * g.wbf_ld + wbf_pos(k, g.wbf_per)] = (uint16_t)bf16_bits(v);
}
// An activation shadow's 4 consecutive columns n of row m (lanes l .. l + 3 of a row's 16):
// lane l % 4 == 0 stores them as one 8-B piece (N % 128 == 0: no partial group).  Every lane calls it.
__device__ __forceinline__ void abf_store4(uint16_t* S, int N, int m, bool mok, int n, float v) {
    const int lane = threadIdx.x & 63;
    const float v1 = __shfl_down(v, 1, 64), v2 = __shfl_down(v, 2, 64), v3 = __shfl_down(v, 3, 64);
    if ((lane & 3) != 0 || !mok || n >= N) return;
    uint2 o;
    o.x = bf16_bits(v) | (bf16_bits(v1) << 16);
    o.y = bf16_bits(v2) | (bf16_bits(v3) << 16);
    *reinterpret_cast<uint2*>(S + (size_t)m * N + wbf_pos(n, wbf_per_of(N))) = o;
}
// A transposed image's 4 consecutive rows m .. m + 3 (m % 4 == 0) of column n: a 32x32 tile's lanes
// l, l + 16, l + 32, l + 48 hold them (rows 4 wave + 0 .. 3 of a 16-row sub-tile); lane l < 16
// stores them as one 8-B piece of row n (wbf_pos positions of K = M, the consumer's reduction).
// Every lane calls it.
__device__ __forceinline__ void tbf_store4(uint16_t* S, int M, int m, int n, bool nok, float v) {
    const int lane = threadIdx.x & 63;
    const float v1 = __shfl_down(v, 16, 64), v2 = __shfl_down(v, 32, 64), v3 = __shfl_down(v, 48, 64);
    if (lane >= 16 || !nok || m >= M) return;
    uint2 o;
    o.x = bf16_bits(v) | (bf16_bits(v1) << 16);
    o.y = bf16_bits(v2) | (bf16_bits(v3) << 16);
    *reinterpret_cast<uint2*>(S + (size_t)n * wbf_ld_of(M) + wbf_pos(m, wbf_per_of(M))) = o;
}
// The control-block scalars a GEMM epilogue needs (the optimiser step, the Polyak gate, the
// expert weight), requested with the epilogue operands before the main loop: read after the
// tile reduction they were two more dependent memory round trips (the kernarg ctl pointer,
// then the field) on every dW + Adam workgroup.
struct EpiScalars {
    int64_t t, nts;
    float eps;
};
__device__ __forceinline__ EpiScalars epi_scalars(const Ctl* ctl, int group) {
    // per-lane buffer loads (boff hides the uniform offsets): the values stay in VGPRs, where a
    // uniform load would be moved to SGPRs right away and stall the main loop's loads behind it
    const __amdgpu_buffer_rsrc_t r = make_rsrc(reinterpret_cast<const float*>(ctl), (uint32_t)sizeof(Ctl));
    const int ot = (int)((group == GRP_MODEL ? offsetof(Ctl, t_model) : offsetof(Ctl, t_sac)) / 4);
    const int on = (int)(offsetof(Ctl, num_timesteps) / 4), oe = (int)(offsetof(Ctl, epsilon) / 4);
    const uint32_t t_lo = __float_as_uint(bload(r, boff(true, ot))), t_hi = __float_as_uint(bload(r, boff(true, ot + 1)));
    const uint32_t n_lo = __float_as_uint(bload(r, boff(true, on))), n_hi = __float_as_uint(bload(r, boff(true, on + 1)));
    EpiScalars e;
    e.t = (int64_t)(((uint64_t)t_hi << 32) | t_lo);
    e.nts = (int64_t)(((uint64_t)n_hi << 32) | n_lo);
    e.eps = bload(r, boff(true, oe));
    return e;
}

// wave index as a scalar (lets per-row pointers and branches stay in SGPRs)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// ---------------------------------------------------------------- packed seeds
// A handle created with cfg.seeds = K holds K independent learners (the reference's --runs)
// in K equal arena blocks sstride bytes apart.  Every launch of the update graph runs all of
// them: grid z is the seed, and each arena pointer of the (seed-0) launch arguments moves by
// blockIdx.z * sstride (a scalar add; null pointers stay null).
__device__ __forceinline__ int64_t seed_off(int64_t sstride) { return (int64_t)blockIdx.z * sstride; }
template <class T>
__device__ __forceinline__ T* sr(T* p, int64_t so) {
    return p ? reinterpret_cast<T*>(reinterpret_cast<unsigned long long>(p) + (unsigned long long)so) : p;
}
__device__ __forceinline__ void reloc(GemmProb& g, int64_t so) {
    g.A = sr(g.A, so); g.B = sr(g.B, so); g.C = sr(g.C, so); g.bias = sr(g.bias, so); g.H = sr(g.H, so);
    g.P = sr(g.P, so); g.T = sr(g.T, so); g.wgen = sr(g.wgen, so);
    g.bscale = sr(g.bscale, so); g.se_raw = sr(g.se_raw, so); g.spe_raw = sr(g.spe_raw, so);
    g.dmean = sr(g.dmean, so); g.dden = sr(g.dden, so); g.part = sr(g.part, so);
    g.pw = sr(g.pw, so); g.ppart = sr(g.ppart, so);
    g.wbf = sr(g.wbf, so); g.obf = sr(g.obf, so); g.abf = sr(g.abf, so);
}
__device__ __forceinline__ void reloc(HeadBwdArgs& b, int64_t so) {
    b.part = sr(b.part, so); b.gpol = sr(b.gpol, so); b.a_den = sr(b.a_den, so); b.alpha = sr(b.alpha, so);
    b.c_t = sr(b.c_t, so); b.c_std = sr(b.c_std, so); b.c_u = sr(b.c_u, so); b.c_mask = sr(b.c_mask, so);
    b.Da3 = sr(b.Da3, so); b.E = sr(b.E, so); b.Da2 = sr(b.Da2, so);
    b.mpart = sr(b.mpart, so); b.ctl = sr(b.ctl, so); b.ma_den = sr(b.ma_den, so);
}
__device__ __forceinline__ void reloc(FinalArgs& f, int64_t so) {
    f.alpha = sr(f.alpha, so); f.alpha_m = sr(f.alpha_m, so); f.alpha_v = sr(f.alpha_v, so); f.ctl = sr(f.ctl, so);
    f.lq = sr(f.lq, so); f.lp = sr(f.lp, so); f.mse_rows = sr(f.mse_rows, so); f.red = sr(f.red, so);
    f.stats = sr(f.stats, so); f.alpha_g = sr(f.alpha_g, so);
}
__device__ __forceinline__ void reloc(HeadSeg& g, int64_t so) {
    g.noise = sr(g.noise, so); g.xq_out = sr(g.xq_out, so); g.nlp_out = sr(g.nlp_out, so); g.pi_out = sr(g.pi_out, so);
}
__device__ __forceinline__ void reloc(QHeadArgs& q, int64_t so) {
    q.H2 = sr(q.H2, so);
#pragma unroll
    for (int k = 0; k < 4; ++k) q.W3[k] = sr(q.W3[k], so);
    q.D2 = sr(q.D2, so); q.g = sr(q.g, so); q.loss_rows = sr(q.loss_rows, so); q.alpha = sr(q.alpha, so);
    q.nlp = sr(q.nlp, so); q.r = sr(q.r, so); q.d = sr(q.d, so); q.ret_den = sr(q.ret_den, so);
    q.Hm2 = sr(q.Hm2, so);
#pragma unroll
    for (int k = 0; k < 2; ++k) q.Wm3[k] = sr(q.Wm3[k], so);
    q.se_raw = sr(q.se_raw, so); q.spe_raw = sr(q.spe_raw, so); q.d_mean = sr(q.d_mean, so);
    q.d_den = sr(q.d_den, so); q.ctl = sr(q.ctl, so); q.Dm2 = sr(q.Dm2, so); q.mse_rows = sr(q.mse_rows, so);
}
__device__ __forceinline__ void reloc(ActorBwdArgs& b, int64_t so) {
    b.Dp1 = sr(b.Dp1, so);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        b.Wq1[k] = sr(b.Wq1[k], so);
        b.Wm1[k] = sr(b.Wm1[k], so);
    }
    b.Dm1 = sr(b.Dm1, so); b.a_den = sr(b.a_den, so); b.ma_den = sr(b.ma_den, so); b.alpha = sr(b.alpha, so);
    b.ctl = sr(b.ctl, so);
    b.c_t = sr(b.c_t, so); b.c_std = sr(b.c_std, so); b.c_u = sr(b.c_u, so); b.c_mask = sr(b.c_mask, so);
    b.W3a = sr(b.W3a, so); b.Ha2 = sr(b.Ha2, so); b.Da3 = sr(b.Da3, so); b.Da2 = sr(b.Da2, so); b.E = sr(b.E, so);
    b.gpol = sr(b.gpol, so);
}
// tools/gemm_bench.hip builds with SACX_GEMM_PHASES: wave 0 of each 16x16 tile workgroup
// stores s_memrealtime at kernel start [0], problem selected [1], main loop done [2], tile
// reduced [3] and kernel end [4] (the last launch's workgroups, by blockIdx.x)
#ifdef SACX_GEMM_PHASES
__device__ unsigned long long g_gemm_ph[8192][5];
#define GEMM_PH(i) do { if (threadIdx.x == 0) g_gemm_ph[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define GEMM_PH(i) do { } while (0)
#endif

// forces a kernarg value into an SGPR at this point: values pinned together load as one batch
template <class T>
__device__ __forceinline__ void pin_s(const T& v) { asm volatile("" ::"s"(v)); }

// the grid z extent of a launch (1 for the single-seed eager calls, whose nseeds is 0)
inline unsigned seeds_z(int n) { return n > 1 ? (unsigned)n : 1u; }
// per-workgroup measurement slot (ktime): workgroups of seed z follow those of seed z-1
__device__ __forceinline__ int ktime_wg() { return (int)(blockIdx.z * gridDim.x + blockIdx.x); }

// ---------------------------------------------------------------- row helpers
// A row of a hidden layer (width H <= 64*NQ) is held as hv[q] = h[lane + 64 q];
// all loads of a row are issued before any reduction so the wave's memory
// latency overlaps instead of serialising behind each butterfly.
#define MAXQ 8
// hv[q] = h[base + lane + 64 q] (0 beyond H)
template <int NQ>
__device__ __forceinline__ void load_row(__amdgpu_buffer_rsrc_t r, int base, int H, float (&hv)[NQ]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int k = lane + 64 * q;
        hv[q] = bload(r, boff(k < H, base + k));
    }
}

// out[u] = sum_k hv(k) * W[k*ldw + o0 + u] for u < 8 (0 for o0+u >= O); broadcast to all lanes.
template <int NQ>
__device__ __forceinline__ void rowdot8(const float (&hv)[NQ], __amdgpu_buffer_rsrc_t rW, int H, int ldw,
                                        int o0, int O, float (&out)[8]) {
    const int lane = threadIdx.x & 63;
    float w[NQ][8];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int k = lane + 64 * q;
#pragma unroll
        for (int u = 0; u < 8; ++u) w[q][u] = bload(rW, boff(k < H && o0 + u < O, k * ldw + o0 + u));
    }
    float p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        p[u] = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q) p[u] = fmaf(hv[q], w[q][u], p[u]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) out[u] = wave_sum(p[u]);
}

// rowdot8 over the whole output row [0, OW) at once, W (H x O, dense) staged in LDS by the
// workgroup.  Read from memory, lane k's W[k][u] for all u is OW single-dword loads 4*O bytes
// apart -- 64 cache lines per instruction, which made the per-CU L1 the bottleneck of
// Humanoid's actor.head (O = 17: 96 scattered loads per row).  Per output the same fmaf
// order and wave_sum as rowdot8, so the sums are identical.
template <int NQ, int OW>
__device__ __forceinline__ void rowdot_lds(const float (&hv)[NQ], const float* Ws, int H, int O, float (&out)[OW]) {
    const int lane = threadIdx.x & 63;
    float w[NQ][OW];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int k = lane + 64 * q;
#pragma unroll
        for (int u = 0; u < OW; ++u) w[q][u] = (k < H && u < O) ? Ws[k * O + u] : 0.f;   // stride O: odd O conflict-free
    }
#pragma unroll
    for (int u = 0; u < OW; ++u) {
        float p = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q) p = fmaf(hv[q], w[q][u], p);
        out[u] = wave_sum(p);
    }
}

// ==================================================================== finalize
// alpha Adam + clamp and the per-update statistics.
__device__ float mean_rows(const float* x, int n) {
    // deterministic: lane-strided partials then butterfly (wave 0 only)
    const int lane = threadIdx.x & 63;
    float s = 0.f;
    for (int i = lane; i < n; i += 64) s += x[i];
    return wave_sum(s) / (float)n;
}

// Lane-strided partial sums of four row arrays at once, each in increasing i -- the order of
// mean_rows, so the results are bit-identical -- in rounds of 4 chunks of 64 rows per array:
// 16 loads in flight per round, one round for B <= 256 and four for Humanoid's B = 1,024.
// (One array after the other, the dependent chunk loads made the folded alpha.final the
// longest workgroup of its Humanoid launch.)
template <int NA>
__device__ __forceinline__ void strided_sums(const float* const (&x)[NA], const int (&n)[NA], float (&s)[NA]) {
    const int lane = threadIdx.x & 63;
    __amdgpu_buffer_rsrc_t r[NA];
    int nmax = 0;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        r[a] = rs(x[a]);
        s[a] = 0.f;
        nmax = max(nmax, n[a]);
    }
    for (int base = 0; base < nmax; base += 256) {
        float v[NA][4];
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = base + lane + 64 * u;
                v[a][u] = bload(r[a], boff(i < n[a], i));
            }
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int u = 0; u < 4; ++u) s[a] += v[a][u];
    }
}

// The finalisation's operands that are final before the alpha rows run (the critic and policy
// loss rows of the update, alpha and its moments, the counters): the ticketed path (k_fwd2's
// fused q launch) loads them before its blocks take their tickets, so the last block's critical
// path after the ticket is the alpha partials' load alone.  Same sums, same order.
#ifndef SACX_FIN_PRE
#define SACX_FIN_PRE 1
#endif
struct FinPre {
    float ps[3];
    float a_old, a_m, a_v;
    int64_t t_sac, seq0, nts, tsi;
};

__device__ __forceinline__ void fin_prefetch(const FinalArgs& f, FinPre& p) {
    const float* const xs[3] = {f.lq, f.lq + f.B, f.lp};
    const int ns[3] = {f.B, f.B, f.B};
    p.a_old = p.a_m = p.a_v = 0.f;
    p.t_sac = p.seq0 = p.nts = p.tsi = 0;
    if ((threadIdx.x & 63) == 0) {
        p.a_old = *f.alpha; p.a_m = *f.alpha_m; p.a_v = *f.alpha_v;
        p.t_sac = f.ctl->t_sac; p.seq0 = f.ctl->step_seq;
        p.nts = f.ctl->num_timesteps; p.tsi = f.ctl->ts_increment;
    }
    strided_sums<3>(xs, ns, p.ps);
}

template <bool PRE = false>
__device__ void finalize_update(const FinalArgs& f, int nred, const FinPre* pre = nullptr) {
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x & 63;
    // every operand of the common case (B <= 256, nred <= 256) is requested before the first
    // use: one memory round trip instead of one per reduction (PRE: all but the alpha partials
    // were loaded before the ticket, by fin_prefetch)
    float ps[4];
    float a_old = 0.f, a_m = 0.f, a_v = 0.f;
    int64_t t_sac = 0, seq0 = 0, nts = 0, tsi = 0;
    if constexpr (PRE) {
        const float* const xs[1] = {f.red};
        const int ns[1] = {nred};
        float p0[1];
        strided_sums<1>(xs, ns, p0);
        ps[0] = p0[0]; ps[1] = pre->ps[0]; ps[2] = pre->ps[1]; ps[3] = pre->ps[2];
        a_old = pre->a_old; a_m = pre->a_m; a_v = pre->a_v;
        t_sac = pre->t_sac; seq0 = pre->seq0; nts = pre->nts; tsi = pre->tsi;
    } else {
        const float* const xs[4] = {f.red, f.lq, f.lq + f.B, f.lp};
        const int ns[4] = {nred, f.B, f.B, f.B};
        strided_sums<4>(xs, ns, ps);
        if (lane == 0) {
            a_old = *f.alpha; a_m = *f.alpha_m; a_v = *f.alpha_v;
            t_sac = f.ctl->t_sac; seq0 = f.ctl->step_seq;
            nts = f.ctl->num_timesteps; tsi = f.ctl->ts_increment;
        }
    }
    const float ent_sum = wave_sum(ps[0]);   // sum_i (-nlp_i + H)
    const float m_ent = ent_sum / (float)f.B;   // reduce_mean
    const float q1 = wave_sum(ps[1]) / (float)f.B;
    const float q2 = wave_sum(ps[2]) / (float)f.B;
    float pl = wave_sum(ps[3]) / (float)f.B;
    float mse = 0.f;
    if (f.use_expert && f.ne > 0 && f.nm == 1) {
        // one model (SAC_expert.py:293-295): mean over the n_e rows of 0.5 ||sp_e - sp_pred||^2
        float sm = 0.f;
        const int nt = f.mse_tiles;
        for (int i = lane; i < f.ne; i += 64) {
            float a = 0.f;
            for (int t = 0; t < nt; ++t) a += f.mse_rows[i * nt + t];
            sm += 0.5f * a;
        }
        mse = wave_sum(sm) / (float)f.ne;
        const float eps = f.ctl->epsilon;
        pl = (1.f - eps) * pl + eps * mse;
    } else if (f.use_expert && f.ne > 0) {
        // two models (:329-335): row i pairs half 1 row i with half 2 row i
        const int h = f.ne / 2;
        float sm = 0.f;
        const int nt = f.mse_tiles;
        for (int i = lane; i < h; i += 64) {
            float a = 0.f, b = 0.f;
            for (int t = 0; t < nt; ++t) {
                a += f.mse_rows[i * nt + t];
                b += f.mse_rows[(i + h) * nt + t];
            }
            sm += 0.5f * (a + b);
        }
        mse = wave_sum(sm) / (float)h;
        const float eps = f.ctl->epsilon;
        pl = (1.f - eps) * pl + eps * mse;
    }
    if (lane == 0) {
        Ctl* ctl = f.ctl;
        const int64_t tnew = t_sac + 1;
        const float alpha_old = a_old;
        const float g = -m_ent;                 // d(-alpha*m)/d alpha
        if (f.alpha_g != nullptr) {             // data-parallel: k_alpha_apply finishes after the all-reduce
            *f.alpha_g = g;
            float* st = f.stats + (size_t)(seq0 % f.stats_cap) * 8;
            st[0] = q1;
            st[1] = q2;
            st[2] = pl;
            st[3] = -alpha_old * m_ent;
            st[5] = mse;
            st[6] = -(m_ent - f.target_entropy);
            st[7] = (float)seq0;
            return;
        }
        const float lr_t = adam_lr(f.adam, GRP_ALPHA, tnew);
        // adam_update on the prefetched alpha, m, v (same arithmetic)
        const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
        const float mm = a_m + (g - a_m) * (1.f - b1);
        const float vv = a_v + (g * g - a_v) * (1.f - b2);
        float an = a_old - (mm * lr_t) / (sqrtf(vv) + eps);
        *f.alpha_m = mm;
        *f.alpha_v = vv;
        an = fmaxf(an, 1e-5f);                  // SAC_expert.py:348
        *f.alpha = an;
        const int64_t seq = seq0;
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
        ctl->num_timesteps = nts + tsi;
        ctl->step_seq = seq + 1;
    }
}

// ==================================================================== k_gemm
template <bool KC, bool VEC, bool GEN = false>
__device__ __forceinline__ void load_a(__amdgpu_buffer_rsrc_t ra, const GemmProb& g, int m, bool mok, int k0,
                                       float (&a)[4], __amdgpu_buffer_rsrc_t rw) {
    if constexpr (KC) {
        if constexpr (VEC) {
            const uint32_t off = boff(mok && k0 < g.K, m * g.lda + k0);
            const float4 v = bload4(ra, off);
            a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = k0 + j;
                a[j] = bload(ra, boff(mok && k < g.K, m * g.lda + k));
            }
        }
        if constexpr (GEN) {       // A = wgen[k] * act'(A) for problems with wgen (else unchanged)
            float w[4];
            if constexpr (VEC) {
                const float4 v = bload4(rw, boff(k0 < g.K, k0));
                w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = bload(rw, boff(k0 + j < g.K, k0 + j));
            }
            const bool gen = g.wgen != nullptr;
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = gen ? w[j] * dact_sel(a[j], g.gen_act) : a[j];
        }
    } else {
        // A[m][k] = X[k][m]; logical row ones_row is all ones (bias-gradient row)
        const float one = (m == g.ones_row) ? 1.f : 0.f;
        const bool rd = mok && (m != g.ones_row);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + j;
            const bool kok = k < g.K;
            a[j] = bload(ra, boff(rd && kok, k * g.lda + m)) + (kok ? one : 0.f);
        }
    }
}

template <bool KC, bool VEC, bool SCALE = false>
__device__ __forceinline__ void load_b(__amdgpu_buffer_rsrc_t rb, const GemmProb& g, int n, bool nok, int k0,
                                       float (&b)[4]) {
    if constexpr (KC) {
        if constexpr (VEC) {
            const uint32_t off = boff(nok && k0 < g.K, n * g.ldb + k0);
            const float4 v = bload4(rb, off);
            b[0] = v.x; b[1] = v.y; b[2] = v.z; b[3] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = k0 + j;
                b[j] = bload(rb, boff(nok && k < g.K, n * g.ldb + k));
            }
        }
    } else if constexpr (SCALE) {
        // GM_DW: k is the row of the reduction (a batch row): scale by bscale[k]
        const __amdgpu_buffer_rsrc_t rs_ = rs(g.bscale);   // host always sets it (ones if unscaled)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + j;
            b[j] = bload(rb, boff(nok && k < g.K, k * g.ldb + n)) * bload(rs_, boff(k < g.K, k));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = k0 + j;
            b[j] = bload(rb, boff(nok && k < g.K, k * g.ldb + n));
        }
    }
}

// The end of a world-model fitting step (mbrl_onpolicy_alg.py:305-319): each model's loss
// (reduce_mean over its minibatch) into the stats ring, loss_all = their sum, and the optimiser
// step / fit sequence advanced.  k_mfinal (one wave, per-row losses of k_mloss) or one extra
// workgroup of a later launch of the step (256 threads, the fit-loss epilogue's tile partials).
// block sum of v over all threads (nw waves); every thread gets the result
__device__ __forceinline__ float mfit_block_sum(float v, float* sh, int nw) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    float a = sh[0];
    for (int w = 1; w < nw; ++w) a += sh[w];
    return a;
}

__device__ void mfit_final(const MFinalArgs& f, const AdamConsts* adam = nullptr, int64_t p_stride = 0) {
    __shared__ float mred[MAX_MODELS][4];
    __shared__ float lred[4];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, nw = blockDim.x >> 6;
    const int64_t t_model = f.ctl->t_model;      // read by every thread before thread 0 advances it
    const int n = f.nt > 0 ? f.mb * f.nt : f.mb;
    for (int k = 0; k < f.nm; ++k) {             // model k's loss partials, then its reward head's
        float sk = 0.f;
        for (int i = t; i < n; i += blockDim.x) sk += f.loss_rows[(size_t)k * n + i];
        if (f.nt2 > 0) {                         // the separate reward heads' partials
            const int n2 = f.mb * f.nt2;
            const float* r2 = f.loss_rows + (size_t)f.nm * n;
            for (int i = t; i < n2; i += blockDim.x) sk += r2[(size_t)k * n2 + i];
        }
        sk = wave_sum(sk);
        if (lane == 0) mred[k][wave] = sk;
    }
    __syncthreads();
    if (f.lgpart != nullptr && adam != nullptr) {
        // GaussianModel's logstd (continuous_models.py:101-131): d loss / d l_j = (ds / mb) sum_i
        // (1 - q_ij^2) from the fit epilogue's per-tile partials, then Keras Adam at the step this
        // finalisation advances to (model.adam's t_adv), or the gradient stored for the global-norm clip
        const int S = f.S;
        const float lr_t = adam_lr(*adam, GRP_MODEL, t_model + 1);
        for (int k = 0; k < f.nm; ++k) {
            float* L = f.logstd + (size_t)k * f.lstride;
            float ds = 1.f;
            if (f.lscale) {                      // tf.stop_gradient(reduce_mean(square(exp(logstd))))
                float q = 0.f;
                for (int j = t; j < S; j += blockDim.x) {
                    const float e = expf(L[j]);
                    q += e * e;
                }
                ds = mfit_block_sum(q, lred, nw) / (float)S;
            }
            __syncthreads();                     // every read of L before any update of it
            const float* P = f.lgpart + (size_t)k * f.ntm * S;
            for (int j = t; j < S; j += blockDim.x) {
                float sum = 0.f;
                for (int i = 0; i < f.ntm; ++i) sum += P[(size_t)i * S + j];
                const float gr = sum * (ds / (float)f.mb);
                if (f.gstore) L[j + 3 * p_stride] = gr;
                else adam_update(L + j, L + j + p_stride, L + j + 2 * p_stride, gr, lr_t);
            }
        }
    }
    if (t == 0) {
        float tot = 0.f;
        for (int k = 0; k < f.nm; ++k) {
            float ak = mred[k][0];
            for (int w = 1; w < nw; ++w) ak += mred[k][w];
            if (f.nt > 0) ak = 0.5f * ak;        // partials of e^2: get_loss's 0.5 factor
            const float lk = ak / (float)f.mb;
            tot = k == 0 ? lk : tot + lk;        // loss_all (:305-312), in model order
        }
        const int64_t seq = f.ctl->mfit_seq;
        f.mstats[(size_t)(seq % f.mstats_cap) * 2] = tot;
        f.mstats[(size_t)(seq % f.mstats_cap) * 2 + 1] = (float)seq;
        f.ctl->t_model = t_model + 1;
        f.ctl->mfit_seq = seq + 1;
    }
}

// MODE: GM_FWD (A k-contig, B=W n-contig, bias+act), GM_DX (A k-contig, B=W^T k-contig,
// act'), GM_DW (A=X^T and B=delta both mn-contig, Keras Adam [+Polyak]).  VEC: float4 along k.
template <int MODE, int NQ>
__device__ __forceinline__ void qhead_block(const QHeadArgs& q, int block, int64_t so, const FinalArgs* fin = nullptr);
template <int NQ, int OW = 0, int FIN = 0>
__device__ __forceinline__ void actor_head_body(const HeadArgs& h, const FinalArgs& f, int block, int64_t so,
                                                const FinalArgs& ffin);
template <int NQ, int OW = 0>
__device__ __forceinline__ void actor_head_body(const HeadArgs& h, const FinalArgs& f, int block, int64_t so) {
    actor_head_body<NQ, OW, 0>(h, f, block, so, f);
}

// Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch),
// so blocks b and b+8 share an L2.  xcd_tile gives the blocks of one XCD a contiguous range of
// the row-major tile order: whole row blocks, so each A row block is fetched into one L2
// instead of all eight (B is the small shared operand).  A bijection on [0, T) for any T.
__device__ __forceinline__ int xcd_tile(int b, int T) {
    const int x = b & 7, j = b >> 3, q = T >> 3, r = T & 7;
    return x * q + (x < r ? x : r) + j;
}

// actor.head folded into the target tiles of q.fwd0 (GM_FWD, rowk = 3, problem headp): the
// tile's 16 target rows get evaluate() (continuous_actors.py:327-379) from the actor's
// layer-2 output -- mu / logstd rows = Ha2[m0.., :] W3 (a 16 x Aout MFMA tile, K = H1 split
// over the 4 waves) -- and the A tile [state columns of A | normalised actions] is staged in
// LDS for the main loop.  Column tile 0 stores the rows' neglogp for q.head.  The same
// arithmetic as k_actor_head, with the 16-lane row sums of the MFMA layout.
// The prologue's operands, requested as one batch (head_pre_load) before anything else of the
// launch so its arithmetic (head_pre_finish) can start while the GEMM operands are in flight
struct HeadPre {
    float xs[4], u, ls, am, ad, bias;
    float4 pv[4];      // actor.fwd1's partial dots of the row's output `col` (parts)
};
__device__ __forceinline__ void head_pre_load(const HeadArgs& hd, const GemmProb& g, int m0, int64_t so, bool parts,
                                              HeadPre& p) {
    const int t = threadIdx.x, row = t >> 4, col = t & 15;
    const int A = hd.A, Aout = hd.Aout, H1 = hd.H1, S = g.K - A;
    HeadSeg sg = hd.seg[0];
    reloc(sg, so);
    const bool rok = m0 + row < g.M;
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(g.A, 0x7fffffffu);
#pragma unroll
    for (int q = 0; q < 4; ++q) p.xs[q] = bload(rx, boff(rok && col + 16 * q < S, (m0 + row) * g.lda + col + 16 * q));
    const bool jok = col < A;
    p.u = bload(rs(sg.noise), boff(jok && rok, (m0 + row - sg.r0) * A + col));
    p.ls = bload(rs(sr(hd.logstd, so)), boff(jok && !hd.per_state_std, col));
    p.am = bload(rs(sr(hd.a_mean, so)), boff(jok, col));
    p.ad = bload(rs(sr(hd.a_den, so)), boff(jok, col));
    const __amdgpu_buffer_rsrc_t rw3 = make_rsrc(sr(hd.W3, so), 0x7fffffffu);
    p.bias = bload(rw3, boff(col < Aout, H1 * Aout + col));
    if (parts) {
        // Ha2 . W3 from actor.fwd1's per-column-tile partials: 4 float4 per (row, output)
        const __amdgpu_buffer_rsrc_t rp = rs(sr(hd.part, so));
        const bool pok = rok && col < Aout;
#pragma unroll
        for (int i = 0; i < 4; ++i) p.pv[i] = bload4(rp, boff(pok && 4 * i < hd.tq, ((m0 + row) * Aout + col) * hd.tq + 4 * i));
    }
}
__device__ __forceinline__ float head_pre_mu(const HeadPre& p) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v = v + p.pv[i].x; v = v + p.pv[i].y; v = v + p.pv[i].z; v = v + p.pv[i].w;
    }
    return v + p.bias;
}
// evaluate() of the row's action col from mu, the neglogp store and the A tile in LDS
__device__ __forceinline__ void head_pre_finish(const HeadArgs& hd, const GemmProb& g, int m0, int tn,
                                                float (&As)[16][68], const HeadPre& p, float mu, int64_t so) {
    const int t = threadIdx.x, lane = t & 63;
    const int row = t >> 4, col = t & 15;
    const int A = hd.A, S = g.K - A;
    HeadSeg sg = hd.seg[0];
    reloc(sg, so);
    const bool rok = m0 + row < g.M;
    const bool jok = col < A;
    // per_state_std: logstd_raw of action j sits in column A + j of the same row (same 16 lanes)
    const float lv = __shfl(mu, (lane & ~15) | min(col + A, 15), 64);
    const float lraw = hd.per_state_std ? lv : p.ls;
    float nv = 0.f, nc = 0.f, pin = 0.f;
    if (jok) {
        const float l = fminf(fmaxf(lraw, -5.f), 2.f);
        const float sd = expf(l);
        const float x = mu + sd * p.u;
        const float th = tanhf(x);
        const float pi = hd.lim * th;
        const float z = (x - mu) / expf(l);
        nv = z * z + 2.f * l + LOG2PI_F;
        nc = 2.f * ((LN2_F - x) - softplus_f(-2.f * x));
        pin = (pi - p.am) / p.ad;
    }
    nv += __shfl_xor(nv, 8, 16);
    nv += __shfl_xor(nv, 4, 16);
    nv += __shfl_xor(nv, 2, 16);
    nv += __shfl_xor(nv, 1, 16);
    nc += __shfl_xor(nc, 8, 16);
    nc += __shfl_xor(nc, 4, 16);
    nc += __shfl_xor(nc, 2, 16);
    nc += __shfl_xor(nc, 1, 16);
    if (tn == 0 && col == 0 && rok && sg.nlp_out != nullptr) sg.nlp_out[m0 + row - sg.r0] = 0.5f * nv + nc;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (col + 16 * q < S) As[row][col + 16 * q] = p.xs[q];
    if (jok) As[row][S + col] = pin;
}

template <bool SYNC = true>
__device__ __forceinline__ void head_prologue(const HeadArgs& hd, const GemmProb& g, int m0, int tn,
                                              float (&As)[16][68], float (&red)[4][4][64], int64_t so) {
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 15, grp = lane >> 4;
    const int row = t >> 4, col = t & 15;
    const int Aout = hd.Aout, H1 = hd.H1;
    // everything the prologue reads is requested first
    HeadPre p;
    head_pre_load(hd, g, m0, so, hd.part != nullptr, p);
    float mu;
    if (hd.part != nullptr) {
        mu = head_pre_mu(p);
    } else {
        const __amdgpu_buffer_rsrc_t rw3 = make_rsrc(sr(hd.W3, so), 0x7fffffffu);
        const __amdgpu_buffer_rsrc_t rh = make_rsrc(sr(hd.H2, so), 0x7fffffffu);
        const int nIt = H1 >> 4, per = (nIt + 3) >> 2, i0 = wave * per, i1 = min(nIt, i0 + per);
        const bool hm = m0 + r < g.M, wn = r < Aout;
        floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
        for (int it = i0; it < i1; it += 4) {
            float a[4][4], b[4][4];
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                const bool ok = it + u4 < i1;
                const int k0 = (it + u4) * 16 + grp * 4;
                const float4 v = bload4(rh, boff(ok && hm, (m0 + r) * hd.ldh + k0));
                a[u4][0] = v.x; a[u4][1] = v.y; a[u4][2] = v.z; a[u4][3] = v.w;
#pragma unroll
                for (int j = 0; j < 4; ++j) b[u4][j] = bload(rw3, boff(ok && wn, (k0 + j) * Aout + r));
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u4 = 0; u4 < 4; ++u4) {
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u4][0], b[u4][0], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u4][1], b[u4][1], c1, 0, 0, 0);
                c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u4][2], b[u4][2], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u4][3], b[u4][3], c1, 0, 0, 0);
            }
        }
        const floatx4 acc = c0 + c1;
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave][q][lane] = acc[q];
        __syncthreads();
        const int L = ((row >> 2) << 4) | col, R = row & 3;
        float v = red[0][R][L] + red[1][R][L];
        v = v + red[2][R][L];
        v = v + red[3][R][L];
        mu = v + p.bias;
    }
    head_pre_finish(hd, g, m0, tn, As, p, mu, so);
    if constexpr (SYNC) __syncthreads();
}

// actor.head.bwd folded into actor.bwd1 (rowk 4): the policy-row work of k_actor_bwd for the
// tile's 16 rows (SAC_expert.py:262-296 through continuous_actors.py:327-379).
// Thread (row, col) owns action col of row m0 + row: the action gradient is the sum of the
// critics' partial dots (written by the pi.q.bwd1 tiles) scaled by the rows' output gradients,
// then the tanh-Gaussian backward; d3s[row][o] receives Da3 (o < Aout, zeros past it) for the
// A-operand generation, and column tile 0 stores Da3 / E for actor.adam.
__device__ __forceinline__ void head_bwd_prologue(HeadBwdArgs hb, int m0, int tn, float (&d3s)[16][17], int64_t so) {
    reloc(hb, so);
    const int t = threadIdx.x, lane = t & 63, row = t >> 4, col = t & 15;
    const int B = hb.B, A = hb.A;
    const int m = m0 + row;
    const bool rok = m < B + hb.ne, jok = col < A, ok = rok && jok;
    const bool pol = m < B;                     // policy row (else an expert row, SAC-EO)
    const int ci = m * A + col;
    const float ct = bload(rs(hb.c_t), boff(ok, ci));
    const float sd = bload(rs(hb.c_std), boff(ok, ci));
    const float u = bload(rs(hb.c_u), boff(ok, ci));
    const float mk = bload(rs(hb.c_mask), boff(ok, ci));
    // the action column's normaliser: the critics' for policy rows, the world models' for expert rows
    const float ad = bload(rs(pol ? hb.a_den : hb.ma_den), boff(jok, col));
    const __amdgpu_buffer_rsrc_t rg = rs(hb.gpol);
    const float g0 = bload(rg, boff(rok && pol, m));
    const float g1 = bload(rg, boff(rok && pol, B + m));
    const float alpha = bload(rs(hb.alpha), 0u);
    const float eps = hb.ctl != nullptr ? bload(rs(reinterpret_cast<const float*>(hb.ctl)),
                                               (uint32_t)offsetof(Ctl, epsilon)) : 0.f;
    // partials [critic][row][action][tq] (policy rows, tq <= 16) or [expert row][action][tqm]
    // (expert rows, tqm <= 32), both multiples of 4: float4 loads, all issued together
    const __amdgpu_buffer_rsrc_t rp = rs(hb.part), rm = rs(hb.mpart);
    const int tq = hb.tq, tqm = hb.tqm, e = m - B;
    float4 v0[4], v1[4], vm[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool iok = ok && pol && 4 * i < tq;
        v0[i] = bload4(rp, boff(iok, (m * A + col) * tq + 4 * i));
        v1[i] = bload4(rp, boff(iok, ((B + m) * A + col) * tq + 4 * i));
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) vm[i] = bload4(rm, boff(ok && !pol && 4 * i < tqm, (e * A + col) * tqm + 4 * i));
    float p0 = 0.f, p1 = 0.f, pm = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        p0 = p0 + v0[i].x; p0 = p0 + v0[i].y; p0 = p0 + v0[i].z; p0 = p0 + v0[i].w;
        p1 = p1 + v1[i].x; p1 = p1 + v1[i].y; p1 = p1 + v1[i].z; p1 = p1 + v1[i].w;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        pm = pm + vm[i].x; pm = pm + vm[i].y; pm = pm + vm[i].z; pm = pm + vm[i].w;
    }
    const float c = -(1.f - eps) * alpha * (1.f / (float)B);
    float gx = 0.f, dl = 0.f;
    if (jok) {
        const float ga = (pol ? g0 * p0 + g1 * p1 : pm) / ad;
        gx = ga * hb.lim * (1.f - ct * ct);
        if (pol) gx = gx - (2.f * c) * ct;
        dl = (gx * sd) * u;
        if (pol) dl = dl + c;
        dl = dl * mk;
    }
    // per_state_std: the logstd rows' gradients follow the mean rows (column A + j <- lane j)
    const float dlv = __shfl(dl, (lane & ~15) | max(col - A, 0), 64);
    d3s[row][col] = col < A ? gx : ((hb.per_state_std && col < hb.Aout) ? dlv : 0.f);
    if (tn == 0 && ok) {
        hb.Da3[(size_t)m * hb.Aout + col] = gx;
        if (hb.per_state_std) hb.Da3[(size_t)m * hb.Aout + A + col] = dl;
        else hb.E[ci] = dl;
    }
    __syncthreads();
}

// 32x32 output tiles (T32, launches with many tiles: packed seeds).  A workgroup owns a 2x2
// block of 16x16 MFMA tiles and each wave computes all four over its quarter of K, so a
// workgroup does 4x the MFMA work of a 16x16 one for 2x the operand loads, and a launch has a
// quarter of the workgroups.  Every 16x16 sub-tile accumulates exactly as gemm_core's 16x16
// path does (same k order, same acc0 / acc1 split, same 4-wave reduction order, same
// epilogue), so both tilings give bit-identical results.
#ifndef SACX_T32_NS
#define SACX_T32_NS 1   // k slabs per load group of a 32x32 tile (1: 6 workgroups per CU fit)
#endif
#ifndef SACX_T32_DW_NS
#define SACX_T32_DW_NS 1   // the same for the dW + Adam tiles (uncapped registers)
#endif
// SACX_T32_STAMP (diagnostic builds): a 32x32-tile workgroup's end stamp is taken after phase P
// instead -- 1: its epilogue operands (bias / act' input / P, m, v, T) have arrived, 2: its main-loop
// MFMAs are done, 3: the K-quarter reduction is in LDS (k_gemm skips its own end stamp for these launches)
#ifndef SACX_T32_STAMP
#define SACX_T32_STAMP 0
#endif
#define T32_STAMP(P, ...)                                                                   \
    do {                                                                                     \
        if (SACX_T32_STAMP == (P) && ga.ktime != nullptr) {                                  \
            asm volatile("" ::__VA_ARGS__);                                                  \
            __syncthreads();                                                                 \
            if (threadIdx.x == 0) ga.ktime[2 * ktime_wg() + 1] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                    \
    } while (0)
template <int MODE, int VEC, bool BF, bool PART = false, bool MSE = false>
__device__ __forceinline__ void gemm_tile32(const GemmArgs& ga, const GemmProb& g, int lt, int64_t so,
                                            float (&red)[16][4][64]) {
    constexpr bool AKC = (MODE != GM_DW);
    constexpr bool BKC = (MODE == GM_DX);
    const int tm = lt / g.tiles_n;          // tiles_n counts 32-wide column tiles here
    const int tn = lt - tm * g.tiles_n;
    const int m0 = tm * 32, n0 = tn * 32;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, grp = lane >> 4;
    const int t = threadIdx.x, row = t >> 4, col = t & 15;

    // ---- epilogue operands of this thread's four outputs (sub-tile s = 2 i + j: rows +16 i, cols +16 j)
    float e0[4], e1[4], e2[4], e3[4], e4[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int mm = m0 + 16 * (s >> 1) + row, nn = n0 + 16 * (s & 1) + col;
        const int mmc = min(mm, g.M - 1), nnc = min(nn, g.N - 1);
        const size_t pidx = (size_t)mmc * g.ldp + nnc;
        e0[s] = e1[s] = e2[s] = e3[s] = e4[s] = 0.f;
        if constexpr (MODE == GM_FWD) {
            e0[s] = g.bias[nnc];
            if constexpr (MSE) {   // launches with world-model head rows only (the registers cost occupancy)
                e1[s] = bload(rs(g.se_raw), boff(g.mse != 0, mmc * ((g.mse & MSE_FIT) ? g.ldp : g.N) + nnc));
                e2[s] = bload(rs(g.spe_raw), boff(g.mse != 0, mmc * g.N + nnc));
                e3[s] = bload(rs(g.dmean), boff(g.mse != 0, nnc));
                e4[s] = bload(rs(g.dden), boff(g.mse != 0, nnc));
            }
        } else if constexpr (MODE == GM_DX) {
            e0[s] = g.H[(size_t)mmc * g.ldh + nnc];
        } else {
            e0[s] = g.P[pidx];
            e1[s] = g.P[pidx + ga.p_stride];
            e2[s] = g.P[pidx + 2 * ga.p_stride];
            e3[s] = bload(make_rsrc(g.T, g.T != nullptr ? 0x7fffffffu : 0u), (uint32_t)pidx * 4u);
        }
    }
    EpiScalars es{};
    if constexpr (MODE == GM_DW || MSE) es = epi_scalars(sr(ga.ctl, so), g.group);
    T32_STAMP(1, "v"(e0[0]), "v"(e1[1]), "v"(e2[2]), "v"(e3[3]));

    const int nIt = (g.K + 15) >> 4;
    const int per = (nIt + 3) >> 2;
    const int it0 = wave * per;
    const int it1 = min(nIt, it0 + per);
    const int ma = m0 + r, mb = m0 + 16 + r, na = n0 + r, nb = n0 + 16 + r;
    const bool maok = ma < g.M, mbok = mb < g.M, naok = na < g.N, nbok = nb < g.N;
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.A, 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(g.B, 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rw = rs(g.wgen);
    floatx4 acc0[4], acc1[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        acc0[s] = floatx4{0.f, 0.f, 0.f, 0.f};
        acc1[s] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    // bf16: two k slabs per load group, one 16x16x32 MFMA per sub-tile and slab pair
    constexpr int NS = BF ? 2 : (MODE == GM_DW ? SACX_T32_DW_NS : SACX_T32_NS);
    auto main_loop = [&](auto vt) {   // unswitched on the problem's float4 flag, as gemm_core
    constexpr bool V = decltype(vt)::value;
    auto load_group = [&](int it, float (&a)[NS][2][4], float (&b)[NS][2][4]) {
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const int k0 = (it + u) * 16 + grp * 4;
            const int k0e = (it + u < it1) ? k0 : (1 << 30);
            load_a<AKC, V && AKC, MODE == GM_DX>(ra, g, ma, maok, k0e, a[u][0], rw);
            load_a<AKC, V && AKC, MODE == GM_DX>(ra, g, mb, mbok, k0e, a[u][1], rw);
            load_b<BKC, V && BKC, MODE == GM_DW>(rb, g, na, naok, k0e, b[u][0]);
            load_b<BKC, V && BKC, MODE == GM_DW>(rb, g, nb, nbok, k0e, b[u][1]);
        }
    };
#if SACX_DW_DIAG_XBF   // diagnostic timing builds only: the dW A operand as one bf16x8 per sub-row and
                      // slab pair (reinterpreted fp32 rows: wrong values, the shadow's load shape)
    if constexpr (BF && MODE == GM_DW) {
        const __amdgpu_buffer_rsrc_t rab = make_rsrc(g.A, 0x7fffffffu);
        for (int it = it0; it < it1; it += 2) {
            float b[2][2][4];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int k0 = (it + u) * 16 + grp * 4;
                const int k0e = (it + u < it1) ? k0 : (1 << 30);
                load_b<false, false, true>(rb, g, na, naok, k0e, b[u][0]);
                load_b<false, false, true>(rb, g, nb, nbok, k0e, b[u][1]);
            }
            const int po = (it >> 1) * 32 + grp * 8;
            bf16x8_t aw[2], bw[2];
            aw[0] = wbf_load(rab, maok, (ma * 512 + po) & 0xffff);
            aw[1] = wbf_load(rab, mbok, (mb * 512 + po) & 0xffff);
            bw[0] = pack_bf16(b[0][0], b[1][0]);
            bw[1] = pack_bf16(b[0][1], b[1][1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (((it - it0) >> 1) & 1)
                    acc1[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[s >> 1], bw[s & 1], acc1[s], 0, 0, 0);
                else
                    acc0[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[s >> 1], bw[s & 1], acc0[s], 0, 0, 0);
            }
        }
        return;
    }
#endif
    for (int it = it0; it < it1; it += NS) {
        float a[NS][2][4], b[NS][2][4];
        load_group(it, a, b);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (BF) {
            // slab pairs (it0 + 2i, it0 + 2i + 1), alternately into acc0 / acc1 -- the pairs and
            // accumulators of gemm_core's 16x16 path (groups of 4 from it0), so both tile shapes
            // sum alike
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (((it - it0) >> 1) & 1) acc1[s] = mfma_bf16_2slab(a[0][s >> 1], a[1][s >> 1], b[0][s & 1], b[1][s & 1], acc1[s]);
                else acc0[s] = mfma_bf16_2slab(a[0][s >> 1], a[1][s >> 1], b[0][s & 1], b[1][s & 1], acc0[s]);
            }
            continue;
        }
#pragma unroll
        for (int u = 0; u < NS; ++u) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if (j & 1) acc1[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][s >> 1][j], b[u][s & 1][j], acc1[s], 0, 0, 0);
                    else acc0[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][s >> 1][j], b[u][s & 1][j], acc0[s], 0, 0, 0);
                }
        }
    }
    };
    // bf16 forward with operand shadows: B from the weight's (wbf) and / or A from the layer-0
    // activations' (abf), one bf16x8 per lane, sub-tile row / column and slab pair -- the values and
    // order the converting path packs, so the sums are bit-identical
    auto shadow_loop = [&](auto vt, auto at, auto bt) {
    constexpr bool V = decltype(vt)::value, SA = decltype(at)::value, SB = decltype(bt)::value;
    const __amdgpu_buffer_rsrc_t rwb = make_rsrc(reinterpret_cast<const float*>(g.wbf), 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rab = make_rsrc(reinterpret_cast<const float*>(g.abf), 0x7fffffffu);
    const int pb = wave * ((per + 1) >> 1);     // this wave's first slab pair in a shadow row
    for (int it = it0; it < it1; it += 2) {
        float a[2][2][4], b[2][2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k0 = (it + u) * 16 + grp * 4;
            const int k0e = (it + u < it1) ? k0 : (1 << 30);
            if constexpr (!SA) {
                load_a<true, V, false>(ra, g, ma, maok, k0e, a[u][0], rw);
                load_a<true, V, false>(ra, g, mb, mbok, k0e, a[u][1], rw);
            }
            if constexpr (!SB) {
                load_b<false, false, false>(rb, g, na, naok, k0e, b[u][0]);
                load_b<false, false, false>(rb, g, nb, nbok, k0e, b[u][1]);
            }
        }
        const int po = (pb + ((it - it0) >> 1)) * 32 + grp * 8;
        bf16x8_t aw[2], bw[2];
        if constexpr (SA) {
            aw[0] = wbf_load(rab, maok, ma * g.K + po);
            aw[1] = wbf_load(rab, mbok, mb * g.K + po);
        } else {
            aw[0] = pack_bf16(a[0][0], a[1][0]);
            aw[1] = pack_bf16(a[0][1], a[1][1]);
        }
        if constexpr (SB) {
            bw[0] = wbf_load(rwb, naok, na * g.wbf_ld + po);
            bw[1] = wbf_load(rwb, nbok, nb * g.wbf_ld + po);
        } else {
            bw[0] = pack_bf16(b[0][0], b[1][0]);
            bw[1] = pack_bf16(b[0][1], b[1][1]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (((it - it0) >> 1) & 1)
                acc1[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[s >> 1], bw[s & 1], acc1[s], 0, 0, 0);
            else
                acc0[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[s >> 1], bw[s & 1], acc0[s], 0, 0, 0);
        }
    }
    };
    // bf16 dW + Adam with X^T from its transposed image (abf, wbf_ld_of(K) positions per row m):
    // one bf16x8 per lane, sub-tile row and slab pair; the ones row (bias gradient) generated as
    // the converting path makes it; B converted (its per-row scale is produced in the launch before)
    auto xbf_loop = [&]() {
    const __amdgpu_buffer_rsrc_t rab = make_rsrc(reinterpret_cast<const float*>(g.abf), 0x7fffffffu);
    const int pb = wave * ((per + 1) >> 1);
    const int ld = 4 * ((per + 1) >> 1) * 32;        // wbf_ld_of(K)
    const bool aone = ma == g.ones_row, bone = mb == g.ones_row;
    for (int it = it0; it < it1; it += 2) {
        float b[2][2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k0 = (it + u) * 16 + grp * 4;
            const int k0e = (it + u < it1) ? k0 : (1 << 30);
            load_b<false, false, true>(rb, g, na, naok, k0e, b[u][0]);
            load_b<false, false, true>(rb, g, nb, nbok, k0e, b[u][1]);
        }
        const int po = (pb + ((it - it0) >> 1)) * 32 + grp * 8;
        bf16x8_t aw[2], bw[2];
        aw[0] = wbf_load(rab, maok && !aone, ma * ld + po);
        aw[1] = wbf_load(rab, mbok && !bone, mb * ld + po);
        if (aone || bone) {
            float o0[4], o1[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                o0[j] = it * 16 + grp * 4 + j < g.K ? 1.f : 0.f;
                o1[j] = (it + 1 < it1 && (it + 1) * 16 + grp * 4 + j < g.K) ? 1.f : 0.f;
            }
            const bf16x8_t ones = pack_bf16(o0, o1);
            if (aone) aw[0] = ones;
            if (bone) aw[1] = ones;
        }
        bw[0] = pack_bf16(b[0][0], b[1][0]);
        bw[1] = pack_bf16(b[0][1], b[1][1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (((it - it0) >> 1) & 1)
                acc1[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[s >> 1], bw[s & 1], acc1[s], 0, 0, 0);
            else
                acc0[s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[s >> 1], bw[s & 1], acc0[s], 0, 0, 0);
        }
    }
    };
    bool shadow = false;
    if constexpr (MODE == GM_FWD && BF) shadow = g.wbf != nullptr || g.abf != nullptr;
    if constexpr (MODE == GM_DW && BF) shadow = g.abf != nullptr;
    if (shadow) {
        if constexpr (MODE == GM_DW && BF) xbf_loop();
        if constexpr (MODE == GM_FWD && BF) {
            using T_ = std::true_type;
            using F_ = std::false_type;
            if (g.abf != nullptr) {
                if (g.wbf != nullptr) shadow_loop(F_{}, T_{}, T_{});
                else shadow_loop(F_{}, T_{}, F_{});
            } else if constexpr (VEC == 1) {
                if (g.vec) shadow_loop(T_{}, F_{}, T_{});
                else shadow_loop(F_{}, F_{}, T_{});
            } else {
                shadow_loop(F_{}, F_{}, T_{});
            }
        }
    } else if constexpr (VEC == 1) {
        if (g.vec) main_loop(std::true_type{});
        else main_loop(std::false_type{});
    } else {
        main_loop(std::false_type{});
    }
    T32_STAMP(2, "v"(acc0[0]), "v"(acc1[3]));
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const floatx4 acc = acc0[s] + acc1[s];
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave * 4 + s][q][lane] = acc[q];
    }
    __syncthreads();
    T32_STAMP(3, "v"(red[0][0][lane]));

    const int L = ((row >> 2) << 4) | col, R = row & 3;
    // the Polyak gate once per workgroup, as a scalar (a per-lane 64-bit modulo per sub-tile
    // would be outlined, with a stack frame in scratch)
    bool polyak = false;
    if constexpr (MODE == GM_DW) {
        const int64_t nts = (int64_t)__builtin_amdgcn_readfirstlane((int)(es.nts >> 32)) << 32 |
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)es.nts);
        const int64_t tui = ga.adam.target_update_int > 0 ? ga.adam.target_update_int : 1;
        polyak = nts % tui == 0;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        float v = red[s][R][L] + red[4 + s][R][L];
        v = v + red[8 + s][R][L];
        v = v + red[12 + s][R][L];
        const int mm = m0 + 16 * (s >> 1) + row, nn = n0 + 16 * (s & 1) + col;
        const bool out_ok = (mm < g.M) && (nn < g.N);
        const int mmc = min(mm, g.M - 1), nnc = min(nn, g.N - 1);
        const size_t pidx = (size_t)mmc * g.ldp + nnc;
        if constexpr (PART) {
            if (g.ppart != nullptr) {     // uniform: the partial head dots of gemm_core's 16x16 path,
                                          // per 16-column sub-tile (same values, same order)
                float x;
                if constexpr (MODE == GM_DX) x = nn < g.N ? v * dact_f(e0[s], g.act) : 0.f;
                else x = nn < g.N ? act_f(v + e0[s], g.act) : 0.f;
                if (mm < g.M) {           // whole 16-lane rows
                    const __amdgpu_buffer_rsrc_t rpw = rs(g.pw);
                    float w[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) w[j] = bload(rpw, boff(j < g.pw_n && nn < g.N, j * g.pw_ld + nnc * g.pw_cs));
                    float mine = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float d = x * w[j];
                        d = d + dpp<0xB1>(d);
                        d = d + dpp<0x4E>(d);
                        d = d + dpp<0x124>(d);
                        d = d + dpp<0x128>(d);
                        mine = col == j ? d : mine;
                    }
                    if (col < g.pw_n)
                        st_out(&g.ppart[((size_t)mm * g.pw_n + col) * ((g.N + 15) >> 4) + 2 * tn + (s & 1)], mine);
                }
                if (out_ok && g.C != nullptr) st_out(&g.C[(size_t)mm * g.ldc + nn], x);
                continue;
            }
        }
        if constexpr (MODE == GM_FWD && MSE) {
            if (g.mse) {          // uniform: the expert MSE / fit-loss epilogue (all 256 threads take part)
                const bool fit = (g.mse & MSE_FIT) != 0;
                float pred = v + e0[s];
                // --delta_clip_pred (base_world_model.py:80-82): clip, no gradient outside [-c, c]
                const bool pass = g.dclip <= 0.f || (pred >= -g.dclip && pred <= g.dclip);
                if (g.dclip > 0.f) pred = fminf(fmaxf(pred, -g.dclip), g.dclip);
                const float sp_hat = e1[s] + (pred * e4[s] + e3[s]);
                const float diff = fit ? e1[s] - pred : e2[s] - sp_hat;
                const float gscale = -es.eps * g.grad_scale;
                const float cf = (fit && !(g.mse & MSE_NOREW) && nn == g.N - 1) ? g.fcoef : 1.f;     // the reward column
                float sq = out_ok ? diff * diff * cf : 0.f;
                sq += __shfl_xor(sq, 8, 16);   // the 16 columns of this thread's sub-tile row
                sq += __shfl_xor(sq, 4, 16);
                sq += __shfl_xor(sq, 2, 16);
                sq += __shfl_xor(sq, 1, 16);
                if (out_ok) {
                    st_out(&g.C[(size_t)mm * g.ldc + nn],
                           fit ? -diff * (cf * g.grad_scale) : (pass ? (gscale * diff) * e4[s] : 0.f));
                    if (col == 0) st_out(&g.part[(size_t)mm * ((g.N + 15) >> 4) + 2 * tn + (s & 1)], sq);
                }
                continue;
            }
        }
        if constexpr (MODE == GM_FWD) {
            const float o = act_f(v + e0[s], g.act);
            if (out_ok) st_out(&g.C[(size_t)mm * g.ldc + nn], o);
            if constexpr (BF) {     // the next layer's bf16 A operand (its K = this N)
                if (g.obf != nullptr) abf_store4(g.obf, g.N, mm, mm < g.M, nn, o);
                // and the dW + Adam tiles' (the transposed image: K = this M)
                if (g.tbf != nullptr) tbf_store4(sr(g.tbf, so), g.M, mm, nn, nn < g.N, o);
            }
        } else if constexpr (MODE == GM_DX) {
            if (out_ok) st_out(&g.C[(size_t)mm * g.ldc + nn], v * dact_f(e0[s], g.act));
        } else {
            if (g.epi == EPI_STORE) {    // data-parallel: the local gradient, Adam after the all-reduce
                if (out_ok) st_out(&g.P[pidx + 3 * ga.p_stride], v * g.grad_scale);
                continue;
            }
            // every lane computes (clamped operands) so the shadow stores can gather across lanes
            const float lr_t = adam_lr(ga.adam, g.group, es.t + 1 - ga.t_adv);
            const float gr = v * g.grad_scale;
            const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
            const float mm1 = e1[s] + (gr - e1[s]) * (1.f - b1);
            const float vv1 = e2[s] + (gr * gr - e2[s]) * (1.f - b2);
            const float pn = e0[s] - (mm1 * lr_t) / (sqrtf(vv1) + eps);
            const float tv = e3[s] * ga.adam.tau_keep + pn * ga.adam.tau_take;
            if (out_ok) {
                st_out(&g.P[pidx], pn);
                st_mom(&g.P[pidx + ga.p_stride], mm1);
                st_mom(&g.P[pidx + 2 * ga.p_stride], vv1);
                wbf_store(g.wbf, g, mm, nn, pn);
                if (g.T != nullptr && polyak) {
                    st_out(&g.T[pidx], tv);
                    wbf_store(g.obf, g, mm, nn, tv);
                }
            }
        }
    }
}

template <int MODE, int VEC, int ROWK, int NQ, bool BF = false, bool PK = false, bool T32 = false>
__device__ __forceinline__ void gemm_core(const KHdr kh, const GemmArgs& ga) {
    constexpr bool AKC = (MODE != GM_DW);
    constexpr bool BKC = (MODE == GM_DX);
    __shared__ float red[T32 ? 16 : 4][4][64];
    // PK: packed seeds (nseeds > 1); a one-seed launch compiles the relocation away (so = 0)
    const int64_t so = PK ? seed_off(ga.sstride) : 0;
    // Every scalar that decides this workgroup's role and problem is read in ONE batch of
    // kernarg loads: left alone, the compiler loads each behind its own branch, a chain of
    // dependent scalar round trips in front of the first operand load.
    // With a valid launch header (KHdr) they are already in SGPRs at dispatch.
    int has_final, row_blocks, total_tiles, xcd_map, nprob;
    int tb[GEMM_MAXP];
    static_assert(GEMM_MAXP == 8, "one pin per problem's tile_begin");
    const uint32_t kf = khdr_flags(kh);
    if (kf & 0x80u) {
        total_tiles = (int)khdr_field(kh, 0);
        row_blocks = (int)khdr_field(kh, 1);
        tb[0] = 0;
#pragma unroll
        for (int i = 1; i < GEMM_MAXP; ++i) tb[i] = (int)khdr_field(kh, i + 1);
        nprob = (int)(kf & 15u);
        has_final = (int)((kf >> 4) & 3u);
        xcd_map = (int)((kf >> 6) & 1u);
    } else {
        has_final = ga.has_final; row_blocks = ga.row_blocks; total_tiles = ga.total_tiles;
        xcd_map = ga.xcd_map; nprob = ga.nprob;
#pragma unroll
        for (int i = 0; i < GEMM_MAXP; ++i) tb[i] = ga.probs[i].tile_begin;
        asm volatile("" ::"s"(has_final), "s"(row_blocks), "s"(total_tiles), "s"(xcd_map), "s"(nprob),
                     "s"(tb[1]), "s"(tb[2]), "s"(tb[3]), "s"(tb[4]), "s"(tb[5]), "s"(tb[6]), "s"(tb[7]));
    }
    // the folded alpha.final of the previous update is workgroup 0: dispatched first, its
    // serial reductions overlap the tiles instead of trailing them
    int tile = (int)blockIdx.x - (has_final ? 1 : 0);
    if (tile < 0) {
        FinalArgs f = ga.fin;
        reloc(f, so);
        finalize_update(f, f.nred);
        return;
    }
    if constexpr (ROWK == 3) {
        // actor.head rows beside the tiles: dispatched first, so their serial row work
        // overlaps the tiles instead of trailing the launch
        if (tile < row_blocks) {
            actor_head_body<NQ>(ga.head, ga.hfin, ga.head_block0 + tile, so);
            return;
        }
        tile -= row_blocks;
    }
    if (tile >= total_tiles) {
        if constexpr (ROWK > 0 && ROWK < 3) {   // horizontally fused Q-head rows
            qhead_block<ROWK - 1, NQ>(ga.qh, tile - total_tiles, so, ROWK == 1 ? &ga.fin : nullptr);
        } else if constexpr (ROWK == 0 || ROWK == 7) {
            if (ga.has_mfinal) mfit_final(ga.mfin, &ga.adam, ga.p_stride);   // the world-model fit step's k_mfinal
        }
        return;
    }
    if (xcd_map) tile = xcd_tile(tile, total_tiles);
    int p = 0;
#pragma unroll
    for (int i = 1; i < GEMM_MAXP; ++i)
        if (i < nprob && tile >= tb[i]) p = i;
    GemmProb g = ga.probs[p];   // by value: every field loads once, up front (speculatable)
    // the selected problem's fields of this mode, again in one batch (one asm statement: the
    // loads cannot be split by waits between separate pins)
    if constexpr (MODE == GM_FWD && ROWK == 3) {
        // q.fwd0 with the actor head folded in (plain SAC: never an mse problem): the head
        // prologue's operands ride in the same batch
        const HeadArgs& hd = ga.head;
        const HeadSeg& s0 = hd.seg[0];
        asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                     "s"(g.tile_begin), "s"(g.act), "s"(g.bias), "s"(g.headp), "s"(hd.H2), "s"(hd.W3), "s"(hd.logstd),
                     "s"(hd.a_mean), "s"(hd.a_den), "s"(hd.ldh), "s"(hd.H1), "s"(hd.A), "s"(hd.Aout),
                     "s"(hd.per_state_std), "s"(hd.lim), "s"(s0.r0), "s"(s0.noise), "s"(s0.nlp_out), "s"(g.vec),
                     "s"(hd.part), "s"(hd.tq));
    } else if constexpr (MODE == GM_FWD && ROWK == 5) {
        asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                     "s"(g.tile_begin), "s"(g.act), "s"(g.bias), "s"(g.vec), "s"(g.C), "s"(g.ldc),
                     "s"(g.pw), "s"(g.ppart), "s"(g.pw_ld), "s"(g.pw_cs), "s"(g.pw_n));
    } else if constexpr (MODE == GM_FWD) {
        asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                     "s"(g.tile_begin), "s"(g.act), "s"(g.bias), "s"(g.mse), "s"(g.se_raw), "s"(g.spe_raw),
                     "s"(g.dmean), "s"(g.dden), "s"(g.headp), "s"(g.vec));
    } else if constexpr (MODE == GM_DX && ROWK == 2) {
        asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                     "s"(g.tile_begin), "s"(g.act), "s"(g.wgen), "s"(g.gen_act), "s"(g.H), "s"(g.ldh), "s"(g.vec),
                     "s"(g.pw), "s"(g.ppart), "s"(g.pw_ld), "s"(g.pw_cs), "s"(g.pw_n), "s"(g.C));
    } else if constexpr (MODE == GM_DX && ROWK == 7) {
        asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                     "s"(g.tile_begin), "s"(g.act), "s"(g.wgen), "s"(g.gen_act), "s"(g.H), "s"(g.ldh), "s"(g.vec),
                     "s"(g.gd), "s"(g.gst), "s"(g.gd_ld), "s"(g.g_o), "s"(g.gst_ld));
    } else if constexpr (MODE == GM_DX) {
        asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                     "s"(g.tile_begin), "s"(g.act), "s"(g.wgen), "s"(g.gen_act), "s"(g.H), "s"(g.ldh), "s"(g.vec));
    } else {
        asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                     "s"(g.tile_begin), "s"(g.act), "s"(g.bscale), "s"(g.P), "s"(g.T), "s"(g.ldp), "s"(g.ones_row),
                     "s"(g.group), "s"(g.epi), "s"(g.grad_scale), "s"(ga.adam.lr[0]), "s"(ga.adam.lr[1]),
                     "s"(ga.adam.lr[2]), "s"(ga.adam.lr[3]), "s"(ga.adam.tau_keep), "s"(ga.adam.tau_take),
                     "s"(ga.adam.target_update_int));
    }
    reloc(g, so);
    GEMM_PH(1);
    if constexpr (T32) {
        static_assert(!(MODE == GM_FWD && ROWK == 3), "T32: plain FWD / DX / DW tiles");
        gemm_tile32<MODE, VEC, BF, (MODE == GM_DX && ROWK == 2) || (MODE == GM_FWD && ROWK == 5),
                    MODE == GM_FWD && ROWK == 8>(ga, g, tile - g.tile_begin, so, red);
        return;
    }
    const int lt = tile - g.tile_begin;
    const int tm = lt / g.tiles_n;
    const int tn = lt - tm * g.tiles_n;
    const int m0 = tm * 16, n0 = tn * 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = lane & 15, grp = lane >> 4;

    // ---- epilogue operands first (this thread's output element is known now)
    const int t = threadIdx.x;
    const int row = t >> 4, col = t & 15;
    const int mm = m0 + row, nn = n0 + col;
    const bool out_ok = (mm < g.M) && (nn < g.N);
    const int mmc = min(mm, g.M - 1), nnc = min(nn, g.N - 1);
    float e0 = 0.f, e1 = 0.f, e2 = 0.f, e3 = 0.f;
    const size_t pidx = (size_t)mmc * g.ldp + nnc;
    float e4 = 0.f;
    if constexpr (MODE == GM_FWD) {
        e0 = g.bias[nnc];
        if constexpr (ROWK == 8) {   // launches with world-model head rows (mse problems) only
            // world-model head rows (mse): zero-sized resources when not an mse problem
            e1 = bload(rs(g.se_raw), boff(g.mse != 0, mmc * ((g.mse & MSE_FIT) ? g.ldp : g.N) + nnc));
            // (MSE_GAUSS: the model's logstd of this column; none for the reward column)
            const bool gl = (g.mse & MSE_GAUSS) != 0;
            e2 = bload(rs(g.spe_raw), boff(g.mse != 0 && !(gl && !(g.mse & MSE_NOREW) && nnc == g.N - 1),
                                           gl ? nnc : mmc * g.N + nnc));
            e3 = bload(rs(g.dmean), boff(g.mse != 0, nnc));
            e4 = bload(rs(g.dden), boff(g.mse != 0, nnc));
        }
    } else if constexpr (MODE == GM_DX) {
        e0 = g.H[(size_t)mmc * g.ldh + nnc];
    } else {
        e0 = g.P[pidx];
        e1 = g.P[pidx + ga.p_stride];
        e2 = g.P[pidx + 2 * ga.p_stride];
        // no target: a zero-sized resource reads 0 without a branch
        e3 = bload(make_rsrc(g.T, g.T != nullptr ? 0x7fffffffu : 0u), (uint32_t)pidx * 4u);
    }
    EpiScalars es{};
    if constexpr (MODE == GM_DW || (MODE == GM_FWD && ROWK == 8))
        es = epi_scalars(sr(ga.ctl, so), g.group);
    // partial-dot weights of this thread's output column (zero-sized resource: no partials)
    constexpr bool PART = (MODE == GM_DX && ROWK == 2) || (MODE == GM_FWD && ROWK == 5);
    float pwv[8];
    if constexpr (PART) {
        const __amdgpu_buffer_rsrc_t rpw = rs(g.pw);
#pragma unroll
        for (int j = 0; j < 8; ++j) pwv[j] = bload(rpw, boff(j < g.pw_n && nn < g.N, j * g.pw_ld + nnc * g.pw_cs));
    }

    const int nIt = (g.K + 15) >> 4;
    const int per = (nIt + 3) >> 2;
    const int it0 = wave * per;
    const int it1 = min(nIt, it0 + per);
    const int m = m0 + r, n = n0 + r;
    const bool mok = m < g.M, nok = n < g.N;

    // operand extents in bytes (offsets are 32-bit: every operand < 2 GiB, checked on the host)
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.A, 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(g.B, 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rw = rs(g.wgen);
    floatx4 acc0 = {0.f, 0.f, 0.f, 0.f};
    floatx4 acc1 = {0.f, 0.f, 0.f, 0.f};
    __shared__ float As[16][68];
    bool a_lds = false;
    if constexpr (MODE == GM_FWD && ROWK == 3) {
        if (g.headp) {
            // K <= 64: at most one 16-wide k slab per wave.  Its B operand is requested before
            // the prologue, so the tile pays one memory round trip, not two.
            float bp[4];
            const int k0 = it0 * 16 + grp * 4;
            load_b<BKC, false, false>(rb, g, n, nok, it0 < it1 ? k0 : (1 << 30), bp);
            head_prologue(ga.head, g, m0, tn, As, red, so);
            if (it0 < it1) {
                float a[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) a[j] = (k0 + j < g.K) ? As[r][k0 + j] : 0.f;
                if constexpr (BF) {
                    const float z[4] = {0.f, 0.f, 0.f, 0.f};      // one slab: the pair's second is zero
                    acc0 = mfma_bf16_2slab(a, z, bp, z, acc0);
                } else {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], bp[0], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], bp[1], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], bp[2], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], bp[3], acc1, 0, 0, 0);
                }
            }
            a_lds = true;
        }
    }
    __shared__ float d3s[ROWK == 4 ? 16 : 1][17];
    if constexpr (MODE == GM_DX && ROWK == 4) {
        // actor.bwd1 with actor.head.bwd folded in (host: one problem, K = H1 <= 256 and a multiple
        // of 16 -- at most one group of 4 whole k slabs per wave -- and Aout <= 8).  The slab operands (Ha2, W1^T and
        // the W3a rows of the generation MFMA) are requested before the prologue, so the tile
        // pays one memory round trip for both.
        auto hbw_loop = [&](auto vt) {
            constexpr bool V = decltype(vt)::value;
            const int Aout = ga.hbw.Aout;
            float a[4][4], b[4][4], w[4][2];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int it = it0 + u;
                const int k0 = it * 16 + grp * 4;
                const int k0e = it < it1 ? k0 : (1 << 30);
                load_a<true, V, false>(ra, g, m, mok, k0e, a[u], rw);
                load_b<true, V>(rb, g, n, nok, k0e, b[u]);
                // generation A operand: lane (r, grp) holds W3a[16 it + r][4 s + grp]
                const int kr = it * 16 + r;
#pragma unroll
                for (int s = 0; s < 2; ++s)
                    w[u][s] = bload(rw, boff(it < it1 && kr < g.K && 4 * s + grp < Aout, kr * Aout + 4 * s + grp));
            }
            head_bwd_prologue(ga.hbw, m0, tn, d3s, so);
            // generation B operand: Da3[m0 + r][4 s + grp] (zeros past Aout)
            float d3[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) d3[s] = d3s[r][4 * s + grp];
            float* Da2 = sr(ga.hbw.Da2, so);
            const bool store = tn == 0 && mok;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                // D'[k][m] = sum_o W3a[k][o] Da3[m][o]: lane (r, grp) gets rows k = 16 it + 4 grp + j
                // of column m = m0 + r -- exactly its A operand elements a[u][j]
                floatx4 pre = {0.f, 0.f, 0.f, 0.f};
                pre = __builtin_amdgcn_mfma_f32_16x16x4f32(w[u][0], d3[0], pre, 0, 0, 0);
                pre = __builtin_amdgcn_mfma_f32_16x16x4f32(w[u][1], d3[1], pre, 0, 0, 0);
                const int k0 = (it0 + u) * 16 + grp * 4;
#pragma unroll
                for (int j = 0; j < 4; ++j) a[u][j] = pre[j] * dact_sel(a[u][j], g.gen_act);
                if (store && it0 + u < it1)
                    *reinterpret_cast<float4*>(&Da2[(size_t)m * g.K + k0]) = float4{a[u][0], a[u][1], a[u][2], a[u][3]};
            }
            if constexpr (BF) {
                acc0 = mfma_bf16_2slab(a[0], a[1], b[0], b[1], acc0);
                acc1 = mfma_bf16_2slab(a[2], a[3], b[2], b[3], acc1);
                return;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0], b[u][0], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1], b[u][1], acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][2], b[u][2], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][3], b[u][3], acc1, 0, 0, 0);
            }
        };
        if constexpr (VEC == 1) {
            if (g.vec) hbw_loop(std::true_type{});
            else hbw_loop(std::false_type{});
        } else {
            hbw_loop(std::false_type{});
        }
        a_lds = true;
    }
    // rowk 6 (model.fwd0 of the fit): this lane's A row is replay record phys(idx[m]) and its
    // tile row's (t >> 4) the one whose target columns the tile stores; every address is valid
    // (clamped row, in-record columns) and out-of-range values are masked after the arithmetic
    const float* grow = nullptr;
    float traw0 = 0.f, traw1 = 0.f, tmu = 0.f, tden = 1.f;
    int tcol = 0;
    bool tstore = false;
    if constexpr (MODE == GM_FWD && ROWK == 6) {
        const MGatherArgs& mg = ga.mg;
        const int64_t seq = mg.ctl->mfit_seq, start = mg.ctl->start;
        const int32_t* ir = mg.idx_ring + (seq % mg.idx_cap) * (int64_t)(mg.nm * mg.mb) + (int64_t)p * mg.mb;
        auto rec_of = [&](int row) {
            int64_t phys = start + ir[min(row, g.M - 1)];
            phys = phys >= mg.cap ? phys - mg.cap : phys;
            return mg.replay + phys * (int64_t)mg.stride;
        };
        grow = rec_of(m);
        // targets T[row][c] (get_loss :286-296): c < S the normalised delta sp - s, c == S the reward
        const int S = mg.S, A = mg.A;
        const float* trec = rec_of(mm);
        tcol = tn * 16 + col;
        tstore = mm < g.M && tcol <= S;
        const int c = min(tcol, S);
        traw0 = c < S ? trec[S + A + c] : trec[2 * S + A];
        traw1 = c < S ? trec[c] : 0.f;
        tmu = c < S ? mg.d_mean[c] : mg.r_norm[0];
        tden = c < S ? mg.d_den[c] : mg.r_norm[1];
    }
    auto gather_a = [&](int k0, float (&a)[4], auto vt) {
        constexpr bool V = decltype(vt)::value;
        const MGatherArgs& mg = ga.mg;
        const bool live = mok && k0 < g.K;
        const int kb = k0 < g.K ? k0 : 0;
        float raw[4];
        if constexpr (V) {      // 16-B aligned: record stride and k0 are multiples of 4, r4(K) <= stride
            const float4 q = *reinterpret_cast<const float4*>(grow + kb);
            raw[0] = q.x; raw[1] = q.y; raw[2] = q.z; raw[3] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) raw[j] = grow[min(kb + j, g.K - 1)];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int kc = min(kb + j, g.K - 1);
            const float* mu = kc < mg.S ? mg.s_mean + kc : mg.a_mean + (kc - mg.S);
            const float* den = kc < mg.S ? mg.s_den + kc : mg.a_den + (kc - mg.S);
            float x = (raw[j] - *mu) / *den;          // k_mgather's normalisation
            asm("" : "+v"(x));
            a[j] = (live && kb + j < g.K) ? x : 0.f;
        }
        if (tn == 0 && mok && k0 < g.lda)        // X for model.adam's layer-0 dW (zero pad columns)
            *reinterpret_cast<float4*>(const_cast<float*>(g.A) + (size_t)m * g.lda + k0) = float4{a[0], a[1], a[2], a[3]};
    };
    if constexpr (MODE == GM_DX && ROWK == 7) {
        // model.bwd1 with model.bwd2 folded in (host: g_o <= 32, every problem a generated one).
        // D3 operand of the generation, per output slab t and pair member j: lane (r, grp) holds
        // D3[m0 + r][16 t + 4 grp + j] (zero past g_o / M), as model.bwd2's A operand
        float d3[2][4];
        const __amdgpu_buffer_rsrc_t rd = rs(g.gd);
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int o = 16 * t2 + 4 * grp + j;
                d3[t2][j] = bload(rd, boff(mok && o < g.g_o, m * g.gd_ld + o));
            }
        const bool store = tn == 0 && mok;
        auto gen_loop = [&](auto vt) {
            constexpr bool V = decltype(vt)::value;
            for (int it = it0; it < it1; it += 4) {
                float a[4][4], b[4][4], w[4][2][4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k0 = (it + u) * 16 + grp * 4;
                    const int k0e = (it + u < it1) ? k0 : (1 << 30);
                    load_a<true, V, false>(ra, g, m, mok, k0e, a[u], rw);      // H2
                    load_b<true, V>(rb, g, n, nok, k0e, b[u]);
                    // generation A operand: lane (r, grp) holds W2[16 (it + u) + r][16 t + 4 grp + j],
                    // one 16-B load per slab t at a 4-B aligned offset (the host requires unaligned
                    // dX loads); elements past g_o (the next row's) are zeroed
                    const int kr = (it + u) * 16 + r;
                    const bool kok = it + u < it1 && kr < g.K;
#pragma unroll
                    for (int t2 = 0; t2 < 2; ++t2) {
                        const int o0 = 16 * t2 + 4 * grp;
                        const float4 q = bload4(rw, boff(kok && o0 < g.g_o, kr * g.g_o + o0));
                        w[u][t2][0] = q.x;
                        w[u][t2][1] = o0 + 1 < g.g_o ? q.y : 0.f;
                        w[u][t2][2] = o0 + 2 < g.g_o ? q.z : 0.f;
                        w[u][t2][3] = o0 + 3 < g.g_o ? q.w : 0.f;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    // D2^T slab = W2 rows x D3^T: lane (r, grp) gets rows k = 16 (it+u) + 4 grp + q of
                    // column m0 + r, exactly its A elements a[u][q]; per output slab the pairs
                    // (j 0, 2) and (1, 3) accumulate apart, then the slabs add in wave order
                    floatx4 pt[2];
                    // an MFMA whose operands are zero in every lane (output columns 16 t + j past
                    // g_o for all grp) is left out: it would add +0, which the +0 of the wave sum
                    // below makes indistinguishable
#pragma unroll
                    for (int t2 = 0; t2 < 2; ++t2) {
                        floatx4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = {0.f, 0.f, 0.f, 0.f};
                        const int live = g.g_o - 16 * t2;      // uniform
                        if (live > 0) x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[u][t2][0], d3[t2][0], x0, 0, 0, 0);
                        if (live > 1) x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[u][t2][1], d3[t2][1], x1, 0, 0, 0);
                        if (live > 2) x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[u][t2][2], d3[t2][2], x0, 0, 0, 0);
                        if (live > 3) x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w[u][t2][3], d3[t2][3], x1, 0, 0, 0);
                        pt[t2] = x0 + x1;
                    }
                    const int k0 = (it + u) * 16 + grp * 4;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float v = pt[0][q] + pt[1][q];
                        v = v + 0.f;          // model.bwd2's idle waves 2 and 3
                        v = v + 0.f;
                        a[u][q] = v * dact_f(a[u][q], g.gen_act);
                    }
                    if (store && it + u < it1)
                        *reinterpret_cast<float4*>(&g.gst[(size_t)m * g.gst_ld + k0]) = float4{a[u][0], a[u][1], a[u][2], a[u][3]};
                }
                if constexpr (BF) {
                    acc0 = mfma_bf16_2slab(a[0], a[1], b[0], b[1], acc0);
                    acc1 = mfma_bf16_2slab(a[2], a[3], b[2], b[3], acc1);
                    continue;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0], b[u][0], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1], b[u][1], acc1, 0, 0, 0);
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][2], b[u][2], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][3], b[u][3], acc1, 0, 0, 0);
                }
            }
        };
        if constexpr (VEC == 1) {
            if (g.vec) gen_loop(std::true_type{});
            else gen_loop(std::false_type{});
        } else {
            gen_loop(std::false_type{});
        }
        a_lds = true;
    }
    // float4 operand loads per problem (g.vec): a launch can mix problems with and without
    // them, and the loop is unswitched on the flag
    auto main_loop = [&](auto vt) {
    constexpr bool V = decltype(vt)::value;
    for (int it = it0; !a_lds && it < it1; it += 4) {
        float a[4][4], b[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            // iterations past it1 read a clamped (valid) slab and are zeroed
            const int k0 = (it + u) * 16 + grp * 4;
            const int k0e = (it + u < it1) ? k0 : (1 << 30);
            if constexpr (MODE == GM_FWD && ROWK == 6) gather_a(k0e, a[u], vt);
            else load_a<AKC, V && AKC, MODE == GM_DX>(ra, g, m, mok, k0e, a[u], rw);
            load_b<BKC, V && BKC, MODE == GM_DW>(rb, g, n, nok, k0e, b[u]);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (BF) {
            // slabs (0, 1) and (2, 3) of the group, one v_mfma_f32_16x16x32_bf16 each
            acc0 = mfma_bf16_2slab(a[0], a[1], b[0], b[1], acc0);
            acc1 = mfma_bf16_2slab(a[2], a[3], b[2], b[3], acc1);
            continue;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0], b[u][0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1], b[u][1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][2], b[u][2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][3], b[u][3], acc1, 0, 0, 0);
        }
    }
    };
    if constexpr (VEC == 1) {
        if (g.vec) main_loop(std::true_type{});
        else main_loop(std::false_type{});
    } else {
        main_loop(std::false_type{});
    }
    GEMM_PH(2);
    if constexpr (MODE == GM_FWD && ROWK == 6) {
        const MGatherArgs& mg = ga.mg;
        if (tstore) {
            float y = tcol < mg.S ? ((traw0 - traw1) - tmu) / tden : (traw0 - tmu) / tden;
            const float cl = tcol < mg.S ? mg.clip_d : mg.clip_r;
            if (cl > 0.f) y = fminf(fmaxf(y, -cl), cl);
            mg.T[(size_t)(p * mg.mb + mm) * (mg.S + 1) + tcol] = y;
        }
    }
    const floatx4 acc = acc0 + acc1;
#pragma unroll
    for (int q = 0; q < 4; ++q) red[wave][q][lane] = acc[q];
    __syncthreads();
    GEMM_PH(3);

    // (row, col) lives in lane (row>>2)*16+col, register row&3 of each wave's tile
    const int L = ((row >> 2) << 4) | col, R = row & 3;
    float v = red[0][R][L] + red[1][R][L];
    v = v + red[2][R][L];
    v = v + red[3][R][L];
    if constexpr (MODE == GM_FWD && ROWK == 8) {
        if (g.mse) {          // uniform: the expert MSE / fit-loss epilogue (all 256 threads take part)
            const bool fit = (g.mse & MSE_FIT) != 0;
            float pred = v + e0;
            // --delta_clip_pred (base_world_model.py:80-82): clip, no gradient outside [-c, c]
            const bool pass = g.dclip <= 0.f || (pred >= -g.dclip && pred <= g.dclip);
            if (g.dclip > 0.f) pred = fminf(fmaxf(pred, -g.dclip), g.dclip);
            const float sp_hat = e1 + (pred * e4 + e3);
            const float diff = fit ? e1 - pred : e2 - sp_hat;
            const float gscale = -es.eps * g.grad_scale;
            const bool rcl = fit && !(g.mse & MSE_NOREW) && nn == g.N - 1;
            const float cf = rcl ? g.fcoef : 1.f;     // the reward column
            float sq = out_ok ? diff * diff * cf : 0.f;
            float dout = fit ? -diff * (cf * g.grad_scale) : (pass ? (gscale * diff) * e4 : 0.f);
            if (g.mse & MSE_GAUSS) {
                // GaussianModel.get_loss (continuous_models.py:101-131) on the delta columns:
                // q = (T - out) / e^l; loss ds (q^2 + 2 l + log 2 pi) (x 0.5 / mb in mfit_final);
                // d / d out = -(q / e^l) ds / mb; d / d l = ds / mb (1 - q^2), summed over rows
                __shared__ float lg_sh[4][16];
                __shared__ float ds_sh[4];
                const int Sd = (g.mse & MSE_NOREW) ? g.N : g.N - 1;     // the logstd columns
                float ds = 1.f;
                if (g.mse & MSE_SCALE) {     // --scale_model_loss: stop_gradient(mean(exp(logstd)^2)) (:122-127)
                    const __amdgpu_buffer_rsrc_t rl = rs(g.spe_raw);
                    float q2 = 0.f;
                    for (int j = t; j < Sd; j += 256) {
                        const float e = expf(bload(rl, (uint32_t)j * 4u));
                        q2 += e * e;
                    }
                    q2 = wave_sum(q2);
                    if ((t & 63) == 0) ds_sh[t >> 6] = q2;
                    __syncthreads();
                    ds = ((ds_sh[0] + ds_sh[1]) + (ds_sh[2] + ds_sh[3])) / (float)Sd;
                }
                float lg = 0.f;
                if (!rcl) {
                    const float el = expf(e2);
                    const float q = diff / el;
                    sq = out_ok ? ds * ((q * q + 2.f * e2) + LOG2PI_F) : 0.f;
                    dout = -(q / el) * (ds * g.grad_scale);
                    lg = out_ok ? 1.f - q * q : 0.f;
                }
                lg += __shfl_xor(lg, 16);      // the wave's 4 rows of this column
                lg += __shfl_xor(lg, 32);
                if ((t & 63) < 16) lg_sh[t >> 6][col] = lg;
                __syncthreads();
                if (t < 16 && n0 + t < Sd)
                    st_out(&g.ppart[(size_t)tm * Sd + n0 + t], (lg_sh[0][t] + lg_sh[1][t]) + (lg_sh[2][t] + lg_sh[3][t]));
            }
            sq += __shfl_xor(sq, 8, 16);   // the 16 columns of this thread's tile row
            sq += __shfl_xor(sq, 4, 16);
            sq += __shfl_xor(sq, 2, 16);
            sq += __shfl_xor(sq, 1, 16);
            if (!out_ok) return;
            st_out(&g.C[(size_t)mm * g.ldc + nn], dout);
            if (col == 0) st_out(&g.part[(size_t)mm * g.tiles_n + tn], sq);
            return;
        }
    }
    if constexpr (PART) {
        if (g.ppart != nullptr) {        // uniform over the problem
            if (mm >= g.M) return;       // whole 16-lane rows
            float x;
            if constexpr (MODE == GM_DX) x = nn < g.N ? v * dact_f(e0, g.act) : 0.f;
            else x = nn < g.N ? act_f(v + e0, g.act) : 0.f;
            float mine = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                // sum over the 16 columns of this thread's tile row (16-lane DPP row); lane j's
                // association order is fixed, so its stored value is deterministic
                float s = x * pwv[j];
                s = s + dpp<0xB1>(s);
                s = s + dpp<0x4E>(s);
                s = s + dpp<0x124>(s);
                s = s + dpp<0x128>(s);
                mine = col == j ? s : mine;
            }
            if (col < g.pw_n) st_out(&g.ppart[((size_t)mm * g.pw_n + col) * g.tiles_n + tn], mine);
            if (g.C == nullptr || !out_ok) return;
            st_out(&g.C[(size_t)mm * g.ldc + nn], x);
            return;
        }
    }
    if constexpr (MODE == GM_FWD) {
        if (!out_ok) return;
        st_out(&g.C[(size_t)mm * g.ldc + nn], act_f(v + e0, g.act));
    } else if constexpr (MODE == GM_DX) {
        if (!out_ok) return;
        st_out(&g.C[(size_t)mm * g.ldc + nn], v * dact_f(e0, g.act));
    } else {
        if (g.epi == EPI_STORE) {    // data-parallel: the local gradient, Adam after the all-reduce
            if (out_ok) st_out(&g.P[pidx + 3 * ga.p_stride], v * g.grad_scale);
            return;
        }
        // every lane computes (clamped operands) so the shadow stores can gather across lanes
        const float lr_t = adam_lr(ga.adam, g.group, es.t + 1 - ga.t_adv);
        const float gr = v * g.grad_scale;
        const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
        const float mm1 = e1 + (gr - e1) * (1.f - b1);
        const float vv1 = e2 + (gr * gr - e2) * (1.f - b2);
        const float pn = e0 - (mm1 * lr_t) / (sqrtf(vv1) + eps);
        if (out_ok) {
            st_out(&g.P[pidx], pn);
            st_mom(&g.P[pidx + ga.p_stride], mm1);
            st_mom(&g.P[pidx + 2 * ga.p_stride], vv1);
            wbf_store(g.wbf, g, mm, nn, pn);
        }
        if (g.T != nullptr) {
            const int64_t nts = (int64_t)__builtin_amdgcn_readfirstlane((int)(es.nts >> 32)) << 32 |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)es.nts);
            const int64_t tui = ga.adam.target_update_int > 0 ? ga.adam.target_update_int : 1;
            if (nts % tui == 0) {
                const float tv = e3 * ga.adam.tau_keep + pn * ga.adam.tau_take;
                if (out_ok) {
                    st_out(&g.T[pidx], tv);
                    wbf_store(g.obf, g, mm, nn, tv);
                }
            }
        }
    }
}

// ktime (measurement graphs only): workgroup b stores its first / last s_memrealtime tick
// (100 MHz) at ktime[2b], ktime[2b+1]; the host takes the launch's span from min / max.
#ifndef SACX_T32_WGS
#define SACX_T32_WGS 6
#endif
#ifndef SACX_T32_DW_WGS
#define SACX_T32_DW_WGS 1
#endif
// bf16 operands (config C5) need ~110 VGPRs in the 32x32 forward / dX tiles: at 6 workgroups per
// CU (80 VGPRs) they spilled 12-80 registers to scratch (36-136 B per lane); 4 fit without
// (Humanoid bf16 6.08k -> 7.1k updates/s, tools/ab_ns.sh)
#ifndef SACX_T32_BF_WGS
#define SACX_T32_BF_WGS 4
#endif
// fp32 32x32 dX tiles with the Q-head rows (rowk 1) spill 17-18 VGPRs at 6 per CU; 5 per CU
// (no spill) measured neutral (Humanoid +0.2 %, HC 8 seeds -0.7 %, tools/ab_qh.sh), so 6 stays
#ifndef SACX_T32_QH_WGS
#define SACX_T32_QH_WGS SACX_T32_WGS
#endif
// bf16 forward tiles without world-model head rows (rowk != 8: no mse epilogue operands held over the
// main loop) fit 5 per CU: a 1,024-tile Humanoid q.fwd launch then runs in one round even with the
// side stream's sampler holding a CU
#ifndef SACX_T32_BF_FWD_WGS
#define SACX_T32_BF_FWD_WGS 5
#endif
#define SACX_T32_OCC                                                                                         \
    (T32 ? (MODE != GM_DW ? (BF ? (MODE == GM_FWD && ROWK != 8 ? SACX_T32_BF_FWD_WGS : SACX_T32_BF_WGS)          \
                                : (MODE == GM_DX && ROWK == 1 ? SACX_T32_QH_WGS : SACX_T32_WGS))              \
                          : SACX_T32_DW_WGS)                                                                 \
         : 1)
template <int MODE, int VEC, int ROWK = 0, int NQ = 4, bool BF = false, bool PK = false, bool T32 = false>
__global__ __launch_bounds__(256, SACX_T32_OCC) void k_gemm(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3,
                                                           GemmArgs ga) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#ifdef SACX_GEMM_PHASES
    if (threadIdx.x == 0) g_gemm_ph[blockIdx.x][0] = t0;
#endif
    gemm_core<MODE, VEC, ROWK, NQ, BF, PK, T32>(KHdr{{h0, h1, h2, h3}}, ga);
    GEMM_PH(4);
    if (SACX_T32_STAMP && T32) {   // (diagnostic: the phase stamp is the end stamp)
        if (ga.ktime != nullptr && threadIdx.x == 0) ga.ktime[2 * ktime_wg()] = t0;
    } else if (ga.ktime != nullptr) {
        __syncthreads();
        if (threadIdx.x == 0) {
            ga.ktime[2 * ktime_wg()] = t0;
            ga.ktime[2 * ktime_wg() + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// q.fwd0 with the actor head folded in: 1,024 tiles + 128 head-row workgroups must be
// resident at once (5 workgroups per CU), so registers are capped at 96 per lane
template <int VEC, int NQ, bool BF, bool PK = false>
__global__ __launch_bounds__(256, 5) void k_gemm_head(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3, GemmArgs ga) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    gemm_core<GM_FWD, VEC, 3, NQ, BF, PK>(KHdr{{h0, h1, h2, h3}}, ga);
    if (ga.ktime != nullptr) {
        __syncthreads();
        if (threadIdx.x == 0) {
            ga.ktime[2 * ktime_wg()] = t0;
            ga.ktime[2 * ktime_wg() + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// ==================================================================== k_dwl
// dW + Keras Adam for long reductions (K = batch rows >= 512: Humanoid's B = 1,024): 32x32
// output tiles whose operand rows stream into LDS by LDS-DMA (global_load_lds), several 16-row
// slabs ahead of the MFMAs.  The 16x16 dW tile reads each of its K rows as 64-B column pieces
// straight into the MFMA operand layout (fragment-shaped loads: half cache lines, 12 dependent
// dword loads per lane and slab) and runs L2-bound; here each row piece is a whole 128-B line,
// and the loads of slab i + NST - 1 are in flight while slab i is multiplied.
// Summation order is gemm_core's 16x16 path, sub-tile by sub-tile: wave w owns the same quarter
// of K, each MFMA the same four k (16 it + 4 grp + j), the same acc0 / acc1 split and the same
// 4-wave reduction order, so all three dW tilings give bit-identical results.
#ifndef SACX_DWL_NST
#define SACX_DWL_NST 4    // slabs in flight per wave (LDS 4 waves x NST x 4.25 KB: 2 workgroups per CU)
#endif
// floats per slab stage: X [16][32], D [16][16 NH], bscale [64] (16 used)
template <int NH>
constexpr int dwl_stg() { return 512 + 256 * NH + 64; }

typedef __attribute__((address_space(3))) void* lds_vp;
__device__ __forceinline__ uint32_t lds_addr(const float* p) { return (uint32_t)(uintptr_t)(lds_vp)(p); }
// One LDS-DMA wave-instruction: lane l's 16 (V4) or 4 bytes from g land at LDS byte address
// l0 + l * size.  Inline asm rather than __builtin_amdgcn_global_load_lds: knowing of the DMA,
// hipcc waits vmcnt(0) before every LDS read of the slab loop, which drains the pipeline; the
// loop orders its reads by explicit counted waits instead.  m0 is saved and restored.
template <bool V4>
__device__ __forceinline__ void glds(const float* g, uint32_t l0) {
    uint32_t keep;
    if constexpr (V4)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(l0) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(l0) : "memory");
}

// LDS column c of slab row `row` holds operand column c ^ dwl_sw(row): rows 4-7 and 12-15 swap
// their 16-column halves, so the two row groups of one ds_read_b32 lane group (grp 0 / 1, 2 / 3)
// fall into different banks
__device__ __forceinline__ int dwl_sw(int row) { return ((row >> 2) & 1) << 4; }

// one slab (rows k0 .. k0 + 15, columns c0 .. c0 + NC - 1) of a row-major [K][ld] operand into
// the LDS image at byte address l0: V4 by 16-B pieces (ld % 4 == 0, 16-B aligned base), else by
// dwords.  NC = 32: image [16][32], columns swizzled by dwl_sw.  NC = 16: image [16][16] whose
// row slot q holds row q ^ ((q >> 2) & 1) (rows 4-7, 12-15 swapped in pairs), the same bank split
// for 64-B rows.  Rows past K and columns past the row repeat valid elements; the reader masks
// them exactly where load_a / load_b read zeros.
__device__ __forceinline__ int dwl_slot(int row) { return row ^ ((row >> 2) & 1); }
template <bool V4, int NC>
__device__ __forceinline__ void dwl_issue(const float* base, int ld, int k0, int K, int c0, uint32_t l0, int lane) {
    if constexpr (NC == 32) {
        if constexpr (V4) {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int row = 8 * q + (lane >> 3);
                const int col = min(c0 + (((lane & 7) << 2) ^ dwl_sw(row)), ld - 4);
                const int k = min(k0 + row, K - 1);
                glds<true>(base + (size_t)k * ld + col, l0 + q * 1024);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int row = 2 * q + (lane >> 5);
                const int col = min(c0 + ((lane & 31) ^ dwl_sw(row)), ld - 1);
                const int k = min(k0 + row, K - 1);
                glds<false>(base + (size_t)k * ld + col, l0 + q * 256);
            }
        }
    } else {
        if constexpr (V4) {
            const int row = dwl_slot(lane >> 2);
            const int col = min(c0 + ((lane & 3) << 2), ld - 4);
            const int k = min(k0 + row, K - 1);
            glds<true>(base + (size_t)k * ld + col, l0);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = dwl_slot(4 * q + (lane >> 4));
                const int col = min(c0 + (lane & 15), ld - 1);
                const int k = min(k0 + row, K - 1);
                glds<false>(base + (size_t)k * ld + col, l0 + q * 256);
            }
        }
    }
}

// NH: 16-column halves per tile -- 2: 32x32 tiles, 1: 32x16 (twice the workgroups, two or three
// per CU: more waves per SIMD to hide each slab's non-MFMA instructions)
template <bool BF, bool PK, int NH>
__global__ __launch_bounds__(256, 2) void k_dwl(uint32_t h0, uint32_t h1, uint32_t h2, uint32_t h3, GemmArgs ga) {
    constexpr int STG = dwl_stg<NH>(), NS = 2 * NH;     // stage floats; sub-tiles per thread
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#ifdef SACX_GEMM_PHASES
    if (threadIdx.x == 0) g_gemm_ph[blockIdx.x][0] = t0;
#endif
    __shared__ float lds[4 * SACX_DWL_NST * STG];    // the one LDS object (staging, then reduction)
    const int64_t so = PK ? seed_off(ga.sstride) : 0;
    const KHdr kh{{h0, h1, h2, h3}};
    int total_tiles, xcd_map, nprob;
    int tb[GEMM_MAXP];
    const uint32_t kf = khdr_flags(kh);
    if (kf & 0x80u) {            // the launch header (gemm_core)
        total_tiles = (int)khdr_field(kh, 0);
        tb[0] = 0;
#pragma unroll
        for (int i = 1; i < GEMM_MAXP; ++i) tb[i] = (int)khdr_field(kh, i + 1);
        nprob = (int)(kf & 15u);
        xcd_map = (int)((kf >> 6) & 1u);
    } else {
        total_tiles = ga.total_tiles; xcd_map = ga.xcd_map; nprob = ga.nprob;
#pragma unroll
        for (int i = 0; i < GEMM_MAXP; ++i) tb[i] = ga.probs[i].tile_begin;
        asm volatile("" ::"s"(total_tiles), "s"(xcd_map), "s"(nprob), "s"(tb[1]), "s"(tb[2]), "s"(tb[3]), "s"(tb[4]),
                     "s"(tb[5]), "s"(tb[6]), "s"(tb[7]));
    }
    int tile = (int)blockIdx.x;
    if (xcd_map) tile = xcd_tile(tile, total_tiles);
    int p = 0;
#pragma unroll
    for (int i = 1; i < GEMM_MAXP; ++i)
        if (i < nprob && tile >= tb[i]) p = i;
    GemmProb g = ga.probs[p];
    asm volatile("" ::"s"(g.A), "s"(g.B), "s"(g.lda), "s"(g.ldb), "s"(g.M), "s"(g.N), "s"(g.K), "s"(g.tiles_n),
                 "s"(g.tile_begin), "s"(g.bscale), "s"(g.P), "s"(g.T), "s"(g.ldp), "s"(g.ones_row), "s"(g.group),
                 "s"(g.epi), "s"(g.grad_scale), "s"(g.vec), "s"(ga.adam.lr[0]), "s"(ga.adam.lr[1]), "s"(ga.adam.lr[2]),
                 "s"(ga.adam.lr[3]), "s"(ga.adam.tau_keep), "s"(ga.adam.tau_take), "s"(ga.adam.target_update_int));
    reloc(g, so);
    const int lt = tile - g.tile_begin;
    const int tm = lt / g.tiles_n, tn = lt - tm * g.tiles_n;
    const int m0 = tm * 32, n0 = tn * 16 * NH;
    const int wave = wave_id(), lane = threadIdx.x & 63;     // wave uniform: the slab loop is scalar
    const int r = lane & 15, grp = lane >> 4;
    const int t = threadIdx.x, row = t >> 4, col = t & 15;

    // ---- epilogue operands of this thread's outputs first (sub-tile s = NH i + j: rows +16 i,
    // cols +16 j), as gemm_tile32
    float e0[NS], e1[NS], e2[NS], e3[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int mm = m0 + 16 * (s / NH) + row, nn = n0 + 16 * (s % NH) + col;
        const size_t pidx = (size_t)min(mm, g.M - 1) * g.ldp + min(nn, g.N - 1);
#ifdef SACX_DWL_NOEPI       // diagnostic builds: no epilogue operand loads
        e0[s] = e1[s] = e2[s] = e3[s] = (float)pidx;
        continue;
#endif
        e0[s] = g.P[pidx];
        e1[s] = g.P[pidx + ga.p_stride];
        e2[s] = g.P[pidx + 2 * ga.p_stride];
        e3[s] = bload(make_rsrc(g.T, g.T != nullptr ? 0x7fffffffu : 0u), (uint32_t)pidx * 4u);
    }
    const EpiScalars es = epi_scalars(sr(ga.ctl, so), g.group);

    const int nIt = (g.K + 15) >> 4;
    const int per = (nIt + 3) >> 2;
    const int it0 = wave * per;
    const int n = max(0, min(nIt, it0 + per) - it0);      // this wave's slabs (uniform per wave)
    float* wl = lds + wave * (SACX_DWL_NST * STG);
    const uint32_t wl_addr = __builtin_amdgcn_readfirstlane(lds_addr(wl));
    // Operand values.  Rows past M and columns past N of a tile only feed outputs that are never
    // stored, so they need no masking; the bias-gradient row (m == ones_row) takes 1.0 for X, and
    // reduction rows past K (their DMA repeats row K - 1) take a zero scale, as load_a / load_b
    // read zeros there (a zero of either sign contributes nothing to a sum that starts at +0).
    bool isone[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) isone[h] = m0 + 16 * h + r == g.ones_row;
    // lane (r, grp) reads rows 4 grp + j: its swizzle is dwl_sw(4 grp + j) = 16 (grp & 1)
    const int sx = 16 * (grp & 1);
    floatx4 acc0[NS], acc1[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        acc0[s] = floatx4{0.f, 0.f, 0.f, 0.f};
        acc1[s] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    // the raw LDS values of one slab in this lane's MFMA layout (X, D, bscale)
    struct Slab { float x[2][4], d[NH][4], bs[4]; };
    auto read_slab = [&](int i, Slab& v) {
        const float* st = wl + (i % SACX_DWL_NST) * STG;
        const float4 b4 = *reinterpret_cast<const float4*>(st + 512 + 256 * NH + 4 * grp);
        v.bs[0] = b4.x; v.bs[1] = b4.y; v.bs[2] = b4.z; v.bs[3] = b4.w;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int o = (4 * grp + j) * 32 + ((16 * h) ^ sx) + r;
                v.x[h][j] = st[o];
                if constexpr (NH == 2) v.d[h][j] = st[512 + o];
                else if (h == 0) v.d[0][j] = st[512 + dwl_slot(4 * grp + j) * 16 + r];
            }
    };
    auto body = [&](auto xv, auto dv) {
        constexpr bool XV = decltype(xv)::value, DV = decltype(dv)::value;
        constexpr int G = (XV ? 2 : 8) + (DV ? NH : 4 * NH) + 1;      // LDS-DMA instructions per slab
        constexpr int NST = SACX_DWL_NST;
        auto issue = [&](int i) {
#ifdef SACX_DWL_NOLOAD      // diagnostic builds (tools/dw_bench.hip): the loop without its loads
            return;
#endif
            const uint32_t st = wl_addr + (uint32_t)((i % NST) * STG * 4);
            const int k0 = (it0 + i) * 16;
            dwl_issue<XV, 32>(g.A, g.lda, k0, g.K, m0, st, lane);
            dwl_issue<DV, 16 * NH>(g.B, g.ldb, k0, g.K, n0, st + 2048, lane);
            glds<false>(g.bscale + min(k0 + (lane & 15), g.K - 1), st + 2048 + 1024 * NH);
        };
        if (n == 0) return;
#pragma unroll
        for (int i = 0; i < NST - 1; ++i)
            if (i < n) issue(i);
        if (n >= NST - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * G) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        GEMM_PH(1);
        Slab cur, nxt;
        read_slab(0, cur);
        // retire slab 0's reads here, in hipcc's own wait bookkeeping: left pending into the loop
        // they make it wait (on every iteration) for the reads of the next slab as well
        asm volatile("" ::"v"(cur.x[0][0]), "v"(cur.x[0][1]), "v"(cur.x[0][2]), "v"(cur.x[0][3]), "v"(cur.x[1][0]),
                     "v"(cur.x[1][1]), "v"(cur.x[1][2]), "v"(cur.x[1][3]), "v"(cur.bs[0]), "v"(cur.bs[1]),
                     "v"(cur.bs[2]), "v"(cur.bs[3]));
#pragma unroll
        for (int h = 0; h < NH; ++h)
            asm volatile("" ::"v"(cur.d[h][0]), "v"(cur.d[h][1]), "v"(cur.d[h][2]), "v"(cur.d[h][3]));
        float pa[2][4], pb[NH][4];     // bf16: the even slab of the pair
        for (int i = 0; i < n; ++i) {
            // Slab i's values are in registers.  Refill the stage slab i - 1 left (its reads
            // retired), wait for slab i + 1 and request its values, then multiply slab i: the
            // LDS round trip of slab i + 1 runs under the MFMAs of slab i.
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (i + NST - 1 < n) {
                issue(i + NST - 1);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * G) : "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (i + 1 < n) read_slab(i + 1, nxt);
            const int kb = (it0 + i) * 16 + 4 * grp;
            float a[2][4], b[NH][4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float sc = kb + j < g.K ? cur.bs[j] : 0.f;
#pragma unroll
                for (int h = 0; h < 2; ++h) a[h][j] = isone[h] ? 1.f : cur.x[h][j];
#pragma unroll
                for (int h = 0; h < NH; ++h) b[h][j] = cur.d[h][j] * sc;
            }
            if constexpr (BF) {
                // slab pairs (it0 + 2q, it0 + 2q + 1), alternately into acc0 / acc1 (gemm_core's
                // groups of four from it0); an odd last slab pairs with zeros
                const bool last = i == n - 1;
                if ((i & 1) == 0 && !last) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) pa[h][j] = a[h][j];
#pragma unroll
                        for (int h = 0; h < NH; ++h) pb[h][j] = b[h][j];
                    }
                } else {
                    const bool odd = (i & 1) != 0;
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        float a0[4], a1[4], b0[4], b1[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            a0[j] = odd ? pa[s / NH][j] : a[s / NH][j];
                            a1[j] = odd ? a[s / NH][j] : 0.f;
                            b0[j] = odd ? pb[s % NH][j] : b[s % NH][j];
                            b1[j] = odd ? b[s % NH][j] : 0.f;
                        }
                        if ((i >> 1) & 1) acc1[s] = mfma_bf16_2slab(a0, a1, b0, b1, acc1[s]);
                        else acc0[s] = mfma_bf16_2slab(a0, a1, b0, b1, acc0[s]);
                    }
                }
            } else {
#ifdef SACX_DWL_NOMFMA      // diagnostic builds: the loop without its MFMAs
                acc0[0][0] += a[0][0] + b[0][0] + a[1][3] + b[1][3];
#else
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        if (j & 1) acc1[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s / NH][j], b[s % NH][j], acc1[s], 0, 0, 0);
                        else acc0[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s / NH][j], b[s % NH][j], acc0[s], 0, 0, 0);
                    }
#endif
            }
            cur = nxt;
        }
    };
    if (g.vec & 1) {
        if (g.vec & 2) body(std::true_type{}, std::true_type{});
        else body(std::true_type{}, std::false_type{});
    } else {
        if (g.vec & 2) body(std::false_type{}, std::true_type{});
        else body(std::false_type{}, std::false_type{});
    }
    GEMM_PH(2);
    // reduction through the wave's own (retired) staging: sub-tile s of wave w at wl + s * 256
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const floatx4 acc = acc0[s] + acc1[s];
#pragma unroll
        for (int q = 0; q < 4; ++q) wl[s * 256 + q * 64 + lane] = acc[q];
    }
    __syncthreads();
    GEMM_PH(3);
    const int L = ((row >> 2) << 4) | col, R = row & 3;
    const int64_t nts = (int64_t)__builtin_amdgcn_readfirstlane((int)(es.nts >> 32)) << 32 |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)es.nts);
    const int64_t tui = ga.adam.target_update_int > 0 ? ga.adam.target_update_int : 1;
    const bool polyak = nts % tui == 0;
    constexpr int WS = SACX_DWL_NST * STG;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int o = s * 256 + R * 64 + L;
        float v = lds[o] + lds[WS + o];
        v = v + lds[2 * WS + o];
        v = v + lds[3 * WS + o];
        const int mm = m0 + 16 * (s / NH) + row, nn = n0 + 16 * (s % NH) + col;
        const bool ok = mm < g.M && nn < g.N;
        const size_t pidx = (size_t)mm * g.ldp + nn;
        if (g.epi == EPI_STORE) {    // data-parallel: the local gradient, Adam after the all-reduce
            if (ok) st_out(&g.P[pidx + 3 * ga.p_stride], v * g.grad_scale);
            continue;
        }
        // every lane computes (clamped operands) so the shadow stores can gather across lanes
        const float lr_t = adam_lr(ga.adam, g.group, es.t + 1 - ga.t_adv);
        const float gr = v * g.grad_scale;
        const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
        const float mm1 = e1[s] + (gr - e1[s]) * (1.f - b1);
        const float vv1 = e2[s] + (gr * gr - e2[s]) * (1.f - b2);
        const float pn = e0[s] - (mm1 * lr_t) / (sqrtf(vv1) + eps);
        const float tv = e3[s] * ga.adam.tau_keep + pn * ga.adam.tau_take;
        if (ok) {
            st_out(&g.P[pidx], pn);
            st_mom(&g.P[pidx + ga.p_stride], mm1);
            st_mom(&g.P[pidx + 2 * ga.p_stride], vv1);
            wbf_store(g.wbf, g, mm, nn, pn);
            if (g.T != nullptr && polyak) {
                st_out(&g.T[pidx], tv);
                wbf_store(g.obf, g, mm, nn, tv);
            }
        }
    }
    GEMM_PH(4);
    if (ga.ktime != nullptr) {
        __syncthreads();
        if (threadIdx.x == 0) {
            ga.ktime[2 * ktime_wg()] = t0;
            ga.ktime[2 * ktime_wg() + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

#define KH_ARGS kh.h[0], kh.h[1], kh.h[2], kh.h[3], a
// SACX_KHDR=0: launch headers marked invalid (the kernels' GemmArgs path; tests compare both)
static bool khdr_enabled() {            // (read at every launch enqueue: graph captures are rare)
    const char* e = std::getenv("SACX_KHDR");
    return !(e && std::atoi(e) == 0);
}

template <bool PK, bool T32>
static void launch_gemm_t(const GemmArgs& a, hipStream_t s) {
    const KHdr kh = khdr_of(a, khdr_enabled());
    const unsigned z = seeds_z(a.nseeds);
    const dim3 grid(a.total_tiles + (a.has_final ? 1 : 0) + (a.has_mfinal ? 1 : 0), 1, z), block(256);
    switch (a.mode) {
    case GM_FWD:
        if (a.rowk == 3) {                 // q.fwd0 with the actor head folded in
            const dim3 gh(a.total_tiles + (a.has_final ? 1 : 0) + a.row_blocks, 1, z);
            const bool h8 = a.head.H1 > 256;
#define SACX_FH(V, Q)                                                                               \
    do {                                                                                           \
        if (a.bf16) hipLaunchKernelGGL((k_gemm_head<V, Q, true, PK>), gh, block, 0, s, KH_ARGS);              \
        else hipLaunchKernelGGL((k_gemm_head<V, Q, false, PK>), gh, block, 0, s, KH_ARGS);                   \
    } while (0)
            if (a.vec) { if (h8) SACX_FH(1, 8); else SACX_FH(1, 4); }
            else { if (h8) SACX_FH(0, 8); else SACX_FH(0, 4); }
#undef SACX_FH
        } else if (a.rowk == 5) {          // actor.fwd1 (+alpha) writing the head partials
            if (a.bf16) {
                if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 5, 4, true, PK, T32>), grid, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 5, 4, true, PK, T32>), grid, block, 0, s, KH_ARGS);
            } else {
                if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 5, 4, false, PK, T32>), grid, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 5, 4, false, PK, T32>), grid, block, 0, s, KH_ARGS);
            }
        } else if (a.rowk == 6) {          // model.fwd0 of the fit, gathering its rows (one seed, 16x16)
            if constexpr (!PK && !T32) {
                if (a.bf16) {
                    if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 6, 4, true, false, false>), grid, block, 0, s, KH_ARGS);
                    else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 6, 4, true, false, false>), grid, block, 0, s, KH_ARGS);
                } else {
                    if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 6, 4, false, false, false>), grid, block, 0, s, KH_ARGS);
                    else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 6, 4, false, false, false>), grid, block, 0, s, KH_ARGS);
                }
            }
        } else if (a.rowk == 8) {          // with world-model head rows (mse problems)
            if (a.bf16) {
                if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 8, 4, true, PK, T32>), grid, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 8, 4, true, PK, T32>), grid, block, 0, s, KH_ARGS);
            } else {
                if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 8, 4, false, PK, T32>), grid, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 8, 4, false, PK, T32>), grid, block, 0, s, KH_ARGS);
            }
        } else if (a.bf16) {
            if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 0, 4, true, PK, T32>), grid, block, 0, s, KH_ARGS);
            else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 0, 4, true, PK, T32>), grid, block, 0, s, KH_ARGS);
        } else {
            if (a.vec) hipLaunchKernelGGL((k_gemm<GM_FWD, 1, 0, 4, false, PK, T32>), grid, block, 0, s, KH_ARGS);
            else hipLaunchKernelGGL((k_gemm<GM_FWD, 0, 0, 4, false, PK, T32>), grid, block, 0, s, KH_ARGS);
        }
        break;
    case GM_DX: {
        const dim3 gx(a.total_tiles + (a.rowk && a.rowk < 3 ? a.row_blocks : 0) + (a.has_mfinal ? 1 : 0), 1, z);
        const bool q8 = a.rowk && a.qh.H1 > 256;
#define SACX_DX(V, R, Q)                                                                            \
    do {                                                                                           \
        if (a.bf16) hipLaunchKernelGGL((k_gemm<GM_DX, V, R, Q, true, PK, T32>), gx, block, 0, s, KH_ARGS);          \
        else hipLaunchKernelGGL((k_gemm<GM_DX, V, R, Q, false, PK, T32>), gx, block, 0, s, KH_ARGS);                      \
    } while (0)
        if (a.rowk == 7) {                 // model.bwd1 with model.bwd2 folded in (one seed, 16x16)
            if constexpr (!PK && !T32) {
                if (a.bf16) {
                    if (a.vec) hipLaunchKernelGGL((k_gemm<GM_DX, 1, 7, 4, true, false, false>), gx, block, 0, s, KH_ARGS);
                    else hipLaunchKernelGGL((k_gemm<GM_DX, 0, 7, 4, true, false, false>), gx, block, 0, s, KH_ARGS);
                } else {
                    if (a.vec) hipLaunchKernelGGL((k_gemm<GM_DX, 1, 7, 4, false, false, false>), gx, block, 0, s, KH_ARGS);
                    else hipLaunchKernelGGL((k_gemm<GM_DX, 0, 7, 4, false, false, false>), gx, block, 0, s, KH_ARGS);
                }
            }
        } else if (a.rowk == 4) {                 // actor.bwd1 with actor.head.bwd folded in (16x16 only)
            if (a.bf16) {
                if (a.vec) hipLaunchKernelGGL((k_gemm<GM_DX, 1, 4, 4, true, PK, false>), gx, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_DX, 0, 4, 4, true, PK, false>), gx, block, 0, s, KH_ARGS);
            } else {
                if (a.vec) hipLaunchKernelGGL((k_gemm<GM_DX, 1, 4, 4, false, PK, false>), gx, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_DX, 0, 4, 4, false, PK, false>), gx, block, 0, s, KH_ARGS);
            }
        } else if (a.rowk == 1) {
            if (a.vec) { if (q8) SACX_DX(1, 1, 8); else SACX_DX(1, 1, 4); }
            else { if (q8) SACX_DX(0, 1, 8); else SACX_DX(0, 1, 4); }
        } else if (a.rowk == 2) {
            if (a.vec) { if (q8) SACX_DX(1, 2, 8); else SACX_DX(1, 2, 4); }
            else { if (q8) SACX_DX(0, 2, 8); else SACX_DX(0, 2, 4); }
        } else {
            if (a.vec) SACX_DX(1, 0, 4);
            else SACX_DX(0, 0, 4);
        }
#undef SACX_DX
        break;
    }
    default:
        if (a.rowk == 3) {                 // dW + Adam with the policy rows of actor.head beside it
            const dim3 gh(a.total_tiles + a.row_blocks, 1, z);
            const bool h8 = a.head.H1 > 256;
            if (a.bf16) {
                if (h8) hipLaunchKernelGGL((k_gemm<GM_DW, 0, 3, 8, true, PK, T32>), gh, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_DW, 0, 3, 4, true, PK, T32>), gh, block, 0, s, KH_ARGS);
            } else {
                if (h8) hipLaunchKernelGGL((k_gemm<GM_DW, 0, 3, 8, false, PK, T32>), gh, block, 0, s, KH_ARGS);
                else hipLaunchKernelGGL((k_gemm<GM_DW, 0, 3, 4, false, PK, T32>), gh, block, 0, s, KH_ARGS);
            }
        } else if (a.bf16) {
            hipLaunchKernelGGL((k_gemm<GM_DW, 0, 0, 4, true, PK, T32>), grid, block, 0, s, KH_ARGS);
        } else {
            hipLaunchKernelGGL((k_gemm<GM_DW, 0, 0, 4, false, PK, T32>), grid, block, 0, s, KH_ARGS);
        }
    }
}

// ==================================================================== k_fwd2
#ifndef SACX_FWD2_NW
#define SACX_FWD2_NW 16   // waves per k_fwd2 workgroup (8 or 16)
#endif

// Two forward layers of a small-input net in ONE launch (GM_FWD2; one seed, fp32, 16x16 MFMA
// tiles): a workgroup owns 16 rows x 64 columns of layer 1.  Its four waves first compute the 16
// rows' whole layer 0 (wave w: the column tiles w, w + 4, ... of H0 <= 256; K0 <= 32) into LDS --
// each 16-wide k slab's partial in k_gemm's acc0 / acc1 pattern, the slab partials added in the
// order k_gemm's LDS reduction adds its waves', then bias and activation -- and column group 0's
// workgroups store layer 0 for the backward.  Then layer 1: K = H0 split over the four waves as in
// k_gemm (one group of <= 4 slabs each), A read from LDS, the partials reduced through LDS in wave
// order, bias, activation, and (actor.fwd1, rowk 5) the head's per-tile partial dots.  Every output
// is bit-identical to the two k_gemm launches; the launch boundary between them and layer 1's cold
// operand round trip are gone.
// HEAD (the target / critic pair of plain SAC, rowk 3): the first row_blocks workgroups are actor-head
// rows (4 waves each: the previous update's alpha rows, whose last block then finalises that update's
// alpha, k_alpha_final's work, when has_final), and the target nets' tiles (headp) compute their 16
// rows' evaluate() actions in a prologue (head_prologue, actor.fwd1's partial dots) into the LDS A tile
// H0X: the largest layer-0 width of the variant (256, or 512: the world-model fit's model.fwd0/1 pair).
// GATHER (rowk 6, the fit): layer 0's A rows are replay records gathered by the step's minibatch indices
// and normalised on load (k_gemm rowk 6's arithmetic); wave 0 of column group 0 stores them to X and the
// group's threads store the rows' targets T (get_loss :286-296) -- model.gather+fwd0+fwd1 in one launch
#ifndef SACX_DW_DIAG_XBF
#define SACX_DW_DIAG_XBF 0
#endif
// SACX_FWD2_STAMP (diagnostic builds): the end stamp of each workgroup is taken after phase P
// instead -- 1: layer 0 done (its operands and, for target tiles, the head prologue), 2: layer 1's
// MFMAs reduced, 3: the problem's kernel arguments loaded, 5 / 6 (target tiles of the HEAD variant):
// the head prologue done / its operands arrived
#ifndef SACX_FWD2_STAMP
#define SACX_FWD2_STAMP 0
#endif

#define F2_STAMP(P)                                                                          \
    do {                                                                                     \
        if (SACX_FWD2_STAMP == (P) && ga.ktime != nullptr) {                                 \
            __syncthreads();                                                                 \
            if (threadIdx.x == 0) {                                                          \
                ga.ktime[2 * f2_slot(ga, g1, lt, HEAD)] = t0;                                \
                ga.ktime[2 * f2_slot(ga, g1, lt, HEAD) + 1] = __builtin_amdgcn_s_memrealtime(); \
            }                                                                                \
        }                                                                                    \
    } while (0)
// k_fwd2's timestamp slot of tile lt of a pair (the host's linear order: head rows, then each pair's tiles)
__device__ __forceinline__ int f2_slot(const GemmArgs& ga, const GemmProb& g1, int lt, bool head) {
    return (head ? ga.row_blocks : 0) + g1.tile_begin + lt;
}
template <int VEC, int NW, bool HEAD, int FIN = 0, int H0X = 256, bool GATHER = false>
__global__ __launch_bounds__(NW * 64, HEAD ? 2 * NW / 4 : 1) void k_fwd2(GemmArgs ga) {   // (min waves per SIMD)
    // (FIN: ga.has_final as a template parameter -- each variant holds one finalisation form)
    // NW waves: layer 0 by column tiles (wave w: tiles w, w + NW, ... of H0 <= H0X), layer 1 as
    // k_gemm's four-way K split (wave w: quarter w & 3) for CTW of the group's four column tiles
    constexpr int L0T = (H0X / 16) / NW, CTW = 16 / NW, PU = H0X / 64;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    __shared__ float hs[16][H0X + 4];
    __shared__ float red2[4][4][4][64];    // [K quarter][column tile][q][lane]
    // grid (tiles of the largest pair, pairs (+ 1)): the problem pair is blockIdx.y and launch_gemm
    // interleaves the pairs' problems (layer 0 of pair p at 2p, layer 1 at 2p + 1), so a workgroup's
    // arguments arrive in ONE scalar round trip (no tile-range table to read first)
    int p = (int)blockIdx.y;
    if constexpr (HEAD) {
        if (p == 0) {                         // actor-head rows, dispatched first: NW / 4 blocks of 4
            const int tile = (int)blockIdx.x;
            if (tile >= ga.row_blocks) return;
            const int blk = ga.head_block0 + (NW / 4) * tile;
            actor_head_body<4, 0, FIN>(ga.head, ga.hfin, blk, 0, ga.fin);
            if (ga.ktime != nullptr) {
                __syncthreads();
                if (threadIdx.x == 0) {
                    ga.ktime[2 * tile] = t0;
                    ga.ktime[2 * tile + 1] = __builtin_amdgcn_s_memrealtime();
                }
            }
            return;
        }
        --p;
    }
    const GemmProb g0 = ga.probs[2 * p], g1 = ga.probs[2 * p + 1];
    const int lt = (int)blockIdx.x;
    if (lt >= ((g1.M + 15) >> 4) * g1.tiles_n) return;   // (a pair with fewer tiles than the grid's x)
    if (SACX_FWD2_STAMP == 3) {               // diagnostic: the problem's arguments have arrived
        asm volatile("" ::"s"(g0.N), "s"(g1.N), "s"(g0.A), "s"(g1.B));
        F2_STAMP(3);
    }
    const int tm = lt / g1.tiles_n, cg = lt - tm * g1.tiles_n;
    const int m0 = tm * 16;
    const int wave = wave_id(), lane = threadIdx.x & 63, r = lane & 15, grp = lane >> 4;
    const int kq = wave & 3, ch = wave >> 2;     // K quarter, column-tile group
    const bool headp = HEAD && g0.headp;
    const int m = m0 + r;
    const bool mok = m < g0.M;
    const int H0 = g0.N, N1 = g1.N;
    const int nIt0 = (g0.K + 15) >> 4;       // <= 2 (host)
    const int per1 = (H0 + 63) >> 6;         // layer-1 slabs per K quarter (H0 = 64 per1)

    // ---- every operand requested up front: the target tiles' head prologue first (its arithmetic
    // then overlaps the weights' round trip)
    HeadPre hpre;
    if constexpr (HEAD)
        if (headp && threadIdx.x < 256) head_pre_load(ga.head, g0, m0, 0, true, hpre);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(g0.A, 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rw0 = make_rsrc(g0.B, 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rw1 = make_rsrc(g1.B, 0x7fffffffu);
    const __amdgpu_buffer_rsrc_t rnull = rs(nullptr);
    float xa[2][4];
    const float* trec = nullptr;             // GATHER: the record of this thread's target row
    if constexpr (GATHER) {
        // k_gemm rowk 6: row m of problem p is record start + idx_ring[seq][p][m] of the replay ring
        const MGatherArgs& mg = ga.mg;
        const int64_t seq = mg.ctl->mfit_seq, start = mg.ctl->start;
        const int32_t* ir = mg.idx_ring + (seq % mg.idx_cap) * (int64_t)(mg.nm * mg.mb) + (int64_t)p * mg.mb;
        auto rec_of = [&](int rr) {
            int64_t phys = start + ir[min(rr, g0.M - 1)];
            phys = phys >= mg.cap ? phys - mg.cap : phys;
            return mg.replay + phys * (int64_t)mg.stride;
        };
        const float* grow = rec_of(m);
        trec = rec_of(m0 + ((threadIdx.x & 255) >> 4));
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int k0 = s2 < nIt0 ? s2 * 16 + grp * 4 : (1 << 30);
            const bool live = mok && k0 < g0.K;
            const int kb = k0 < g0.K ? k0 : 0;
            float raw[4];
            if constexpr (VEC == 1) {        // 16-B aligned records (host: stride and ldQ multiples of 4)
                const float4 q = *reinterpret_cast<const float4*>(grow + kb);
                raw[0] = q.x; raw[1] = q.y; raw[2] = q.z; raw[3] = q.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) raw[j] = grow[min(kb + j, g0.K - 1)];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int kc = min(kb + j, g0.K - 1);
                const float* mu = kc < mg.S ? mg.s_mean + kc : mg.a_mean + (kc - mg.S);
                const float* den = kc < mg.S ? mg.s_den + kc : mg.a_den + (kc - mg.S);
                float x = (raw[j] - *mu) / *den;          // k_mgather's normalisation
                asm("" : "+v"(x));
                xa[s2][j] = (live && kb + j < g0.K) ? x : 0.f;
            }
            // X for model.adam's layer-0 dW (zero pad columns): one wave of column group 0
            if (cg == 0 && wave == 0 && mok && k0 < g0.lda)
                *reinterpret_cast<float4*>(const_cast<float*>(g0.A) + (size_t)m * g0.lda + k0) =
                    float4{xa[s2][0], xa[s2][1], xa[s2][2], xa[s2][3]};
        }
    } else {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
            load_a<true, VEC == 1, false>(rx, g0, m, mok && !headp, s2 < nIt0 ? s2 * 16 + grp * 4 : (1 << 30), xa[s2], rnull);
    }
    float w0[L0T][2][4], b0[L0T];
#pragma unroll
    for (int i = 0; i < L0T; ++i) {
        const int c = wave + NW * i;          // layer-0 column tile
        const int nc = 16 * c + r;
        const bool cok = nc < H0;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) load_b<false, false>(rw0, g0, nc, cok, s2 < nIt0 && cok ? s2 * 16 + grp * 4 : (1 << 30), w0[i][s2]);
        b0[i] = bload(rs(g0.bias), boff(cok, nc));
    }
    float w1[CTW][PU][4];
#pragma unroll
    for (int j2 = 0; j2 < CTW; ++j2) {
        const int ct = CTW * ch + j2;
        const int n1 = 64 * cg + 16 * ct + r;
        const bool nok = n1 < N1;
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            const int it = kq * per1 + u;
            load_b<false, false>(rw1, g1, n1, nok, u < per1 ? it * 16 + grp * 4 : (1 << 30), w1[j2][u]);
        }
    }
    // epilogue: thread t owns (row, col) of the column tiles CTW (t >> 8) + j2
    const int te = threadIdx.x & 255, eh = threadIdx.x >> 8;
    const int row = te >> 4, col = te & 15;
    float b1[CTW];
    constexpr int NPW = HEAD ? 1 : 8;         // (the head pair never writes the head's partial dots)
    float pwv[CTW][NPW];                      // head partial-dot weights of this thread's columns (rowk 5)
#pragma unroll
    for (int j2 = 0; j2 < CTW; ++j2) {
        const int nn = 64 * cg + 16 * (CTW * eh + j2) + col;
        b1[j2] = bload(rs(g1.bias), boff(nn < N1, nn));
        if constexpr (!HEAD) {
            const __amdgpu_buffer_rsrc_t rpw = rs(ga.rowk == 5 ? g1.pw : nullptr);
#pragma unroll
            for (int j = 0; j < NPW; ++j)
                pwv[j2][j] = bload(rpw, boff(j < g1.pw_n && nn < N1, j * g1.pw_ld + min(nn, N1 - 1) * g1.pw_cs));
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (GATHER) {
        // the targets T[row][c] (get_loss :286-296): c < S the normalised delta sp - s, c == S the
        // reward, clipped by --delta_clip_loss / --reward_clip_loss; column group 0, 16 columns per
        // 256 threads (k_gemm rowk 6's arithmetic)
        const MGatherArgs& mg = ga.mg;
        const int S = mg.S, A = mg.A, tcol = 16 * eh + col, mmr = m0 + row;
        if (cg == 0 && mmr < g0.M && tcol <= S) {
            const int c = tcol;
            const float traw0 = c < S ? trec[S + A + c] : trec[2 * S + A];
            const float traw1 = c < S ? trec[c] : 0.f;
            const float tmu = c < S ? mg.d_mean[c] : mg.r_norm[0];
            const float tden = c < S ? mg.d_den[c] : mg.r_norm[1];
            float y = c < S ? ((traw0 - traw1) - tmu) / tden : (traw0 - tmu) / tden;
            const float cl = c < S ? mg.clip_d : mg.clip_r;
            if (cl > 0.f) y = fminf(fmaxf(y, -cl), cl);
            mg.T[(size_t)(p * mg.mb + mmr) * (S + 1) + c] = y;
        }
    }
    if constexpr (HEAD) {
        // the target rows' A tile [sp_n | evaluate() actions], as k_gemm_head's tile prologue; column
        // group 0 stores the rows' neglogp for q.head (host: the head's partial dots exist, so the
        // prologue has no barrier of its own)
        __shared__ float As[16][68];
        if (headp) {                          // uniform
            if (SACX_FWD2_STAMP == 6) {       // diagnostic: the prologue's operands have arrived
                const float mu6 = head_pre_mu(hpre);
                asm volatile("" ::"v"(mu6), "v"(hpre.xs[3]), "v"(hpre.u));
                F2_STAMP(6);
            }
            if (threadIdx.x < 256) head_pre_finish(ga.head, g0, m0, cg, As, hpre, head_pre_mu(hpre), 0);
            __syncthreads();
            F2_STAMP(5);                      // diagnostic: the prologue is done
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int k = s2 * 16 + grp * 4 + j;
                    xa[s2][j] = (s2 < nIt0 && k < g0.K) ? As[r][k] : 0.f;
                }
        }
    }

    // ---- layer 0: per column tile, slab s2 is k_gemm's wave s2 (K0 <= 32: one slab per wave)
#pragma unroll
    for (int i = 0; i < L0T; ++i) {
        const int c = wave + NW * i;
        if (16 * c >= H0) break;              // uniform
        floatx4 ps[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            floatx4 x0 = {0.f, 0.f, 0.f, 0.f}, x1 = {0.f, 0.f, 0.f, 0.f};
            x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s2][0], w0[i][s2][0], x0, 0, 0, 0);
            x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s2][1], w0[i][s2][1], x1, 0, 0, 0);
            x0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s2][2], w0[i][s2][2], x0, 0, 0, 0);
            x1 = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[s2][3], w0[i][s2][3], x1, 0, 0, 0);
            ps[s2] = x0 + x1;
        }
        const floatx4 v4 = ((ps[0] + ps[1]) + floatx4{0.f, 0.f, 0.f, 0.f}) + floatx4{0.f, 0.f, 0.f, 0.f};
        // lane (r, grp) holds rows 4 grp + q of column 16 c + r
        const int nc = 16 * c + r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float h = act_f(v4[q] + b0[i], g0.act);
            hs[4 * grp + q][nc] = h;
            const int mm = m0 + 4 * grp + q;
            if (cg == 0 && mm < g0.M && nc < H0) st_out(&g0.C[(size_t)mm * g0.ldc + nc], h);
        }
    }
    F2_STAMP(1);
    __syncthreads();

    // ---- layer 1: K quarter kq (slabs kq * per1 + u), A from LDS, CTW column tiles
    float a1[PU][4];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
        const int k0 = (kq * per1 + u) * 16 + grp * 4;
        const float4 q4 = u < per1 ? *reinterpret_cast<const float4*>(&hs[r][k0]) : float4{0.f, 0.f, 0.f, 0.f};
        a1[u][0] = q4.x; a1[u][1] = q4.y; a1[u][2] = q4.z; a1[u][3] = q4.w;
    }
#pragma unroll
    for (int j2 = 0; j2 < CTW; ++j2) {
        floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < PU; ++u) {
            if (u >= per1) break;             // uniform (k_gemm's zero slabs add +0)
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u][0], w1[j2][u][0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u][1], w1[j2][u][1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u][2], w1[j2][u][2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u][3], w1[j2][u][3], acc1, 0, 0, 0);
        }
        const floatx4 acc = acc0 + acc1;
#pragma unroll
        for (int q = 0; q < 4; ++q) red2[kq][CTW * ch + j2][q][lane] = acc[q];
    }
    __syncthreads();
    F2_STAMP(2);
    // (row, col) lives in lane (row >> 2) * 16 + col, register row & 3 of each quarter's tile
    const int L = ((row >> 2) << 4) | col, R = row & 3;
    const int mm = m0 + row;
    const int tiles16 = (N1 + 15) >> 4;
#pragma unroll
    for (int j2 = 0; j2 < CTW; ++j2) {
        const int ct = CTW * eh + j2;
        const int nn = 64 * cg + 16 * ct + col;
        if (64 * cg + 16 * ct >= N1) break;   // uniform per wave
        float v = red2[0][ct][R][L] + red2[1][ct][R][L];
        v = v + red2[2][ct][R][L];
        v = v + red2[3][ct][R][L];
        const float x = nn < N1 ? act_f(v + b1[j2], g1.act) : 0.f;
        if (!HEAD && ga.rowk == 5 && g1.ppart != nullptr) {
            // the actor head's partial dots (k_gemm rowk 5), per 16-column tile
            if (mm < g1.M) {
                float mine = 0.f;
#pragma unroll
                for (int j = 0; j < NPW; ++j) {
                    float sdot = x * pwv[j2][j];
                    sdot = sdot + dpp<0xB1>(sdot);
                    sdot = sdot + dpp<0x4E>(sdot);
                    sdot = sdot + dpp<0x124>(sdot);
                    sdot = sdot + dpp<0x128>(sdot);
                    mine = col == j ? sdot : mine;
                }
                if (col < g1.pw_n)
                    st_out(&g1.ppart[((size_t)mm * g1.pw_n + col) * tiles16 + 4 * cg + ct], mine);
            }
        }
        if (mm < g1.M && nn < N1 && g1.C != nullptr) st_out(&g1.C[(size_t)mm * g1.ldc + nn], x);
    }
    if (SACX_FWD2_STAMP == 0 && ga.ktime != nullptr) {
        __syncthreads();
        if (threadIdx.x == 0) {
            ga.ktime[2 * f2_slot(ga, g1, lt, HEAD)] = t0;
            ga.ktime[2 * f2_slot(ga, g1, lt, HEAD) + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

void launch_gemm(const GemmArgs& a, hipStream_t s) {
    if (a.mode == GM_FWD2) {       // two forward layers in one launch (host: one seed, fp32, 16x16)
        // the kernel's layout: pair p's problems at 2p / 2p + 1, grid (tiles of the largest pair,
        // pairs, + a plane of head rows first for HEAD)
        GemmArgs b = a;
        const int np = a.nprob / 2;
        int most = 1;
        for (int i = 0; i < np; ++i) {
            b.probs[2 * i] = a.probs[i];
            b.probs[2 * i + 1] = a.probs[np + i];
            most = std::max(most, ((a.probs[np + i].M + 15) / 16) * a.probs[np + i].tiles_n);
        }
        const dim3 block(SACX_FWD2_NW * 64), grid2(most, np);
        if (a.rowk == 3) {          // the target / critic pair with the actor-head rows
            const dim3 grid(std::max(most, a.row_blocks), np + 1), hblock(SACX_FWD2_HEAD_NW * 64);
#define SACX_F2H(V, F) hipLaunchKernelGGL((k_fwd2<V, SACX_FWD2_HEAD_NW, true, F>), grid, hblock, 0, s, b)
            if (a.has_final == 2) { if (a.vec) SACX_F2H(1, 2); else SACX_F2H(0, 2); }
            else if (a.has_final) { if (a.vec) SACX_F2H(1, 1); else SACX_F2H(0, 1); }
            else { if (a.vec) SACX_F2H(1, 0); else SACX_F2H(0, 0); }
#undef SACX_F2H
        } else if (a.rowk == 6) {   // the world-model fit's gather + two layers (16 waves, H0 <= 512)
            if (a.vec) hipLaunchKernelGGL((k_fwd2<1, 16, false, 0, 512, true>), grid2, dim3(1024), 0, s, b);
            else hipLaunchKernelGGL((k_fwd2<0, 16, false, 0, 512, true>), grid2, dim3(1024), 0, s, b);
        } else if (a.rowk == 9) {   // the fit's two layers on pre-gathered rows (16 waves, H0 <= 512)
            if (a.vec) hipLaunchKernelGGL((k_fwd2<1, 16, false, 0, 512, false>), grid2, dim3(1024), 0, s, b);
            else hipLaunchKernelGGL((k_fwd2<0, 16, false, 0, 512, false>), grid2, dim3(1024), 0, s, b);
        } else {
            if (a.vec) hipLaunchKernelGGL((k_fwd2<1, SACX_FWD2_NW, false>), grid2, block, 0, s, b);
            else hipLaunchKernelGGL((k_fwd2<0, SACX_FWD2_NW, false>), grid2, block, 0, s, b);
        }
        return;
    }
    if (a.dwl) {   // dW + Adam with LDS-staged rows: plain problems only (no fused rows, no alpha.final)
        const dim3 grid(a.total_tiles, 1, seeds_z(a.nseeds)), block(256);
        const KHdr kh = khdr_of(a, khdr_enabled());
#define SACX_DWLL(NH)                                                                                  \
    do {                                                                                              \
        if (a.nseeds > 1) {                                                                           \
            if (a.bf16) hipLaunchKernelGGL((k_dwl<true, true, NH>), grid, block, 0, s, KH_ARGS);            \
            else hipLaunchKernelGGL((k_dwl<false, true, NH>), grid, block, 0, s, KH_ARGS);                  \
        } else {                                                                                      \
            if (a.bf16) hipLaunchKernelGGL((k_dwl<true, false, NH>), grid, block, 0, s, KH_ARGS);           \
            else hipLaunchKernelGGL((k_dwl<false, false, NH>), grid, block, 0, s, KH_ARGS);                 \
        }                                                                                             \
    } while (0)
        if (a.dwl == 2) SACX_DWLL(1);      // 32x16 tiles
        else SACX_DWLL(2);                 // 32x32 tiles
#undef SACX_DWLL
        return;
    }
    // 32x32 tiles: plain FWD / DX / DW launches only (the host never sets t32 elsewhere)
    const bool t32 = a.t32 && !(a.mode == GM_FWD && a.rowk == 3);
    if (a.nseeds > 1) {
        if (t32) launch_gemm_t<true, true>(a, s);
        else launch_gemm_t<true, false>(a, s);
    } else {
        if (t32) launch_gemm_t<false, true>(a, s);
        else launch_gemm_t<false, false>(a, s);
    }
}

// ==================================================================== k_rng
// NumPy legacy RandomState stream, one workgroup, per update of the batch:
//   randint(cur_size, n_int)  masked rejection on 32-bit words
//   n_norm x legacy_gauss     polar method, cached second value
// (mtrand legacy_gauss / random_bounded_uint64_fill restated; bit-exact, tests/test_gpu_engine.py)
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

// two flags per thread, candidate sets A (thread order) then B (thread order): the exclusive
// ranks of this thread's A and B candidates among all flagged ones, and the total
__device__ __forceinline__ void block_rank2(bool fa, bool fb, int* wtot, int& ra, int& rb, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long ba = __ballot(fa), bb = __ballot(fb);
    const unsigned long long lo = (1ULL << lane) - 1ULL;
    if (lane == 0) {
        wtot[w] = __popcll(ba);
        wtot[RNG_THREADS / 64 + w] = __popcll(bb);
    }
    __syncthreads();
    int offa = 0, tota = 0, offb = 0, totb = 0;
#pragma unroll
    for (int i = 0; i < RNG_THREADS / 64; ++i) {
        const int ca = wtot[i], cb = wtot[RNG_THREADS / 64 + i];
        offa += (i < w) ? ca : 0;
        tota += ca;
        offb += (i < w) ? cb : 0;
        totb += cb;
    }
    __syncthreads();
    ra = offa + __popcll(ba & lo);
    rb = tota + offb + __popcll(bb & lo);
    total = tota + totb;
}

// The stream lives in an LDS ring of raw (untempered) MT words: stream word q (words 0..623 =
// the state's key) sits at ring[q % RNG_RW].  MT19937 as a word recurrence is
//   x[n] = x[n-227] ^ g(n-624),   g(m) = twist(x[m], x[m+1])      (n >= 624)
// and unrolled three times
//   x[n] = x[n-681] ^ g(n-624) ^ g(n-851) ^ g(n-1078)
//        = x[n-681] ^ twist(x[n-624] ^ x[n-851] ^ x[n-1078], x[n-623] ^ x[n-850] ^ x[n-1077])
// (twist is linear over GF(2) in its two words, so the three are one twist of the xors),
// whose operands all lie below n-622: 623 consecutive words are independent, so the whole
// workgroup produces 623 words per step with one barrier (the first 454 words after the key
// use the 227-wide form, which needs no history before it).  Consumption is one candidate
// per thread (a word for randint, 4 words for a polar pair), accepted ones ranked by a
// block-wide ballot prefix.  The state written back is (block holding the last consumed word,
// position); the ring keeps that block resident and it is generated to its end first.
// The ring's first RNG_MIR words are mirrored past its end, so the 1079-word operand window of
// any word is contiguous from one base address and every read is that base plus an immediate
// offset.
#define RNG_RW 32768          // ring words (a power of two: the index wraps with a mask)
#define RNG_MIR 1080          // mirrored head (>= the 1078-word reach of the recurrence, even)

struct RngShared {
    uint32_t ring[RNG_RW + RNG_MIR];
    int wtot[2 * RNG_THREADS / 64];
    int last;
    int has;
    double gauss;
};

__device__ __forceinline__ uint32_t& rng_at(RngShared& S, int q) { return S.ring[(unsigned)q & (RNG_RW - 1u)]; }
__device__ __forceinline__ uint32_t rng_g(RngShared& S, int m) {
    const uint32_t y = (rng_at(S, m) & 0x80000000U) | (rng_at(S, m + 1) & 0x7fffffffU);
    return (y >> 1) ^ ((0U - (y & 1U)) & 0x9908b0dfU);
}

// stores stream word q (and its mirror copy)
__device__ __forceinline__ void rng_put(RngShared& S, int q, uint32_t v) {
    const unsigned p = (unsigned)q & (RNG_RW - 1u);
    S.ring[p] = v;
    if (p < RNG_MIR) S.ring[RNG_RW + p] = v;
}
__device__ __forceinline__ uint32_t mt_g(uint32_t a, uint32_t b) {
    const uint32_t y = (a & 0x80000000U) | (b & 0x7fffffffU);
    return (y >> 1) ^ ((0U - (y & 1U)) & 0x9908b0dfU);
}

// all threads: stream words [w0, w1), w0 >= 624.  Steps of RNG_RUN * 207 <= 623 words, RNG_RUN
// consecutive words per thread (operands shared between them; reads at odd lane strides are
// free of bank conflicts)
#ifndef RNG_RUN
#define RNG_RUN 1
#endif
__device__ void rng_twist(RngShared& S, int w0, int w1) {
#ifdef SACX_DIAG_NOTWIST
    return;   // diagnostic builds only (tools/build_variant.sh): wrong words, the twist's cost removed
#endif
    const int t = threadIdx.x;
    int n0 = w0;
    while (n0 < w1 && n0 < 1078) {               // 227-wide steps (history from the key only)
        const int n1 = min(min(w1, 1078), n0 + 227);
        const int n = n0 + t;
        if (n < n1) rng_put(S, n, rng_at(S, n - 227) ^ rng_g(S, n - 624));
        __syncthreads();
        n0 = n1;
    }
    constexpr int STEP = RNG_RUN == 1 ? 623 : RNG_RUN * (623 / RNG_RUN);
    while (n0 < w1) {
        const int n1 = min(w1, n0 + STEP);
        const int n = n0 + RNG_RUN * t;
        if (n < n1) {
            const unsigned p = (unsigned)n & (RNG_RW - 1u);
            const uint32_t* b = S.ring + (p >= 1078u ? p : p + RNG_RW) - 1078u;   // b[i] = word n - 1078 + i
            uint32_t a[RNG_RUN + 1], c[RNG_RUN + 1], e[RNG_RUN], f[RNG_RUN + 1];
#pragma unroll
            for (int i = 0; i <= RNG_RUN; ++i) {
                a[i] = b[i];            // n-1078 ..
                c[i] = b[227 + i];      // n-851 ..
                f[i] = b[454 + i];      // n-624 ..
                if (i < RNG_RUN) e[i] = b[397 + i];   // n-681 ..
            }
#pragma unroll
            for (int i = 0; i < RNG_RUN; ++i)
                if (RNG_RUN == 1 || n + i < n1)
                    // g is GF(2)-linear in its two words: the three twists as one of the xors
                    rng_put(S, n + i, e[i] ^ mt_g(f[i] ^ c[i] ^ a[i], f[i + 1] ^ c[i + 1] ^ a[i + 1]));
        }
        __syncthreads();
        n0 = n1;
    }
}

// tools/rng_bench.hip builds with SACX_RNG_PROF: thread 0 accumulates 100 MHz ticks of the
// twist bursts [0], randint chunks [1], gauss chunks [2], whole kernel [3], bursts [4], chunks [5]
#ifdef SACX_RNG_PROF
__device__ unsigned long long g_rng_prof[16];
#define RNG_PROF_T(v) const uint64_t v = __builtin_amdgcn_s_memrealtime()
#define RNG_PROF_ADD(i, v) do { if (threadIdx.x == 0) g_rng_prof[i] += (v); } while (0)
#else
#define RNG_PROF_T(v)
#define RNG_PROF_ADD(i, v) do { } while (0)
#endif

__device__ __forceinline__ uint32_t rng_word(const RngShared& S, int q) {
    return S.ring[(unsigned)q & (RNG_RW - 1u)];
}

__device__ __forceinline__ void rng_body(const RngArgs& a_in, RngShared& S) {
    RngArgs a = a_in;
    {
        const int64_t so = seed_off(a_in.sstride);
        a.st = sr(a_in.st, so); a.ctl = sr(a_in.ctl, so);
        a.out_idx = sr(a_in.out_idx, so); a.out_norm = sr(a_in.out_norm, so);
        a.pairs = sr(a_in.pairs, so); a.pairs_oi = sr(a_in.pairs_oi, so);
        a.backup = sr(a_in.backup, so);
    }
    const int t = threadIdx.x;
    for (int i = t; i < 624; i += RNG_THREADS) rng_put(S, i, a.st->key[i]);
    const int pos0 = a.st->pos;
    if (t == 0) {
        S.has = a.st->has_gauss;
        S.gauss = a.st->gauss;
    }
    if (a.backup != nullptr) {          // the state before this draw (undo of a speculative draw)
        for (int i = t; i < 624; i += RNG_THREADS) a.backup->key[i] = a.st->key[i];
        if (t == 0) {
            a.backup->pos = pos0;
            a.backup->has_gauss = a.st->has_gauss;
            a.backup->gauss = a.st->gauss;
        }
    }
    // randint(high): masked rejection on 32-bit words (legacy bounded uint64 path, rng < 2^32)
    const uint64_t high = a.size_fixed > 0 ? (uint64_t)a.size_fixed : (uint64_t)a.ctl->cur_size;
    const uint64_t rng = high > 0 ? high - 1 : 0;
    uint64_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
    // expected words of the whole launch: bursts twist no further than the batch needs
    const double ints = (a.n_int > 0 && rng > 0) ? (double)a.n_int * ((double)(mask + 1) / (double)(rng + 1)) : 0.0;
    const double pairs = (double)((a.n_norm + 1) >> 1) * (4.0 / 0.78539816339744831);
    int est_rem = (int)(((ints + pairs) * 1.01 + 32.0) * a.nupd);
    int q = pos0;        // next stream word (block 0 word 0 = 0)
    int gen = 624;       // stream words [0, gen) exist; [gen - RNG_RW, gen) resident
    __syncthreads();

    // makes words [q, q_end) resident (uniform; q_end - q <= RNG_RW - 1248)
    auto ensure = [&](int q_end) {
        if (q_end <= gen) return;
        RNG_PROF_T(p0);
        const int keep = q > 0 ? ((q - 1) / 624) * 624 : 0;   // the last consumed word's block stays
        int tgt = max(q_end, q + est_rem);
        tgt = min(tgt, keep + RNG_RW);
        rng_twist(S, gen, tgt);
        gen = tgt;
        RNG_PROF_T(p1);
        RNG_PROF_ADD(0, p1 - p0);
        RNG_PROF_ADD(4, 1);
    };
    RNG_PROF_T(k0);

    for (int u = 0; u < a.nupd; ++u) {
        // update u of the batch: its randint + normals, in stream order, into slot (slot + u)
        int32_t* const out_idx = a.out_idx ? (int32_t*)((char*)a.out_idx + u * a.slot_bytes) : nullptr;
        float* const out_norm = (float*)((char*)a.out_norm + u * a.slot_bytes);
        const int q_upd = q;

        // ---------------- randint(high, n_int): one word per candidate
        if (a.n_int > 0) {
            if (rng == 0) {
                for (int i = t; i < a.n_int; i += RNG_THREADS) out_idx[i] = 0;
            } else {
                int done = 0;
                while (done < a.n_int) {
                    ensure(q + RNG_THREADS);
                    RNG_PROF_T(c0);
                    const uint32_t w = mt_temper(rng_word(S, q + t));
                    uint32_t v;
                    bool acc;
                    if (rng == 0xFFFFFFFFULL) { v = w; acc = true; }
                    else { v = w & (uint32_t)mask; acc = (uint64_t)v <= rng; }
                    int total;
                    const int rank = block_rank(acc, S.wtot, total);
                    const int nd = a.n_int - done;
                    if (acc && rank < nd) out_idx[done + rank] = (int32_t)v;
                    if (acc && rank == nd - 1) S.last = t;
                    __syncthreads();
                    if (total >= nd) {
                        q += S.last + 1;
                        done = a.n_int;
                    } else {
                        q += RNG_THREADS;
                        done += total;
                    }
                    RNG_PROF_T(c1);
                    RNG_PROF_ADD(1, c1 - c0);
                    RNG_PROF_ADD(5, 1);
                }
            }
        }

        // ---------------- n_norm x legacy_gauss (polar method, 4 words per candidate pair)
        int oi = 0;
        const bool cached = a.n_norm > 0 && S.has;   // every thread reads before thread 0 clears it
        __syncthreads();
        if (cached) {
            if (t == 0) {
                out_norm[0] = (float)S.gauss;
                S.has = 0;
                S.gauss = 0.0;     // NumPy clears the cached value with the flag
            }
            oi = 1;
        }
        const int need_pairs = (a.n_norm - oi + 1) >> 1;
        uint32_t* const pairs_u = a.pairs ? a.pairs + (size_t)u * a.pcap * 4 : nullptr;
        if (a.pairs && t == 0) a.pairs_oi[u] = oi;
        int got = 0;
        // two candidates per thread and round: words [q, q + 4096) (set A) and [q + 4096, q + 8192)
        // (set B), ranked in stream order -- half the barrier rounds of one candidate per thread
        while (got < need_pairs) {
            ensure(q + 8 * RNG_THREADS);
            RNG_PROF_T(c0);
            uint32_t w[2][4];
            double x1[2], x2[2], r2[2];
            bool acc[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int c = q + 4 * (t + k * RNG_THREADS);
#pragma unroll
                for (int i = 0; i < 4; ++i) w[k][i] = mt_temper(rng_word(S, c + i));
                const double u1 = ((double)(int32_t)(w[k][0] >> 5) * 67108864.0 + (double)(int32_t)(w[k][1] >> 6)) / 9007199254740992.0;
                const double u2 = ((double)(int32_t)(w[k][2] >> 5) * 67108864.0 + (double)(int32_t)(w[k][3] >> 6)) / 9007199254740992.0;
                x1[k] = 2.0 * u1 - 1.0;
                x2[k] = 2.0 * u2 - 1.0;
                r2[k] = x1[k] * x1[k] + x2[k] * x2[k];
                acc[k] = (r2[k] < 1.0) && (r2[k] != 0.0);
            }
            int rk[2], total;
            block_rank2(acc[0], acc[1], S.wtot, rk[0], rk[1], total);
            const int np = need_pairs - got;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (!(acc[k] && rk[k] < np)) continue;
                const int o = oi + 2 * (got + rk[k]);
                if (pairs_u) {
                    // k_polar computes this pair's normals; the cached second value of an odd
                    // count is state, so that one pair's transform also runs here (same code)
                    *reinterpret_cast<uint4*>(pairs_u + 4 * (got + rk[k])) = make_uint4(w[k][0], w[k][1], w[k][2], w[k][3]);
                    if (o + 1 >= a.n_norm) {
                        S.gauss = sqrt(-2.0 * log(r2[k]) / r2[k]) * x1[k];
                        S.has = 1;
                    }
                } else {
#ifdef SACX_DIAG_NOPOLAR
                    const double f = r2[k];   // diagnostic builds only: the transform's cost removed
#else
                    const double f = sqrt(-2.0 * log(r2[k]) / r2[k]);
#endif
                    out_norm[o] = (float)(f * x2[k]);
                    if (o + 1 < a.n_norm) {
                        out_norm[o + 1] = (float)(f * x1[k]);
                    } else {
                        S.gauss = f * x1[k];
                        S.has = 1;
                    }
                }
                if (rk[k] == np - 1) S.last = t + k * RNG_THREADS;   // the candidate that completes the draw
            }
            __syncthreads();
            if (total >= np) {
                q += 4 * (S.last + 1);
                got = need_pairs;
            } else {
                q += 8 * RNG_THREADS;
                got += total;
            }
            RNG_PROF_T(c1);
            RNG_PROF_ADD(2, c1 - c0);
            RNG_PROF_ADD(5, 1);
        }
        est_rem -= q - q_upd;
    }

    RNG_PROF_T(k1);
    RNG_PROF_ADD(3, k1 - k0);
    // state: the block holding the last consumed word (generated to its end) and the position
    if (q > pos0) {
        const int b = (q - 1) / 624;
        ensure(624 * (b + 1));
        for (int i = t; i < 624; i += RNG_THREADS) a.st->key[i] = rng_at(S, 624 * b + i);
        if (t == 0) a.st->pos = q - b * 624;
    }
    if (t == 0) {
        a.st->has_gauss = S.has;
        a.st->gauss = S.gauss;
        if (a.slot >= 0) {
            // reset_seq = 1 + k: the update after the next k (a deferred alpha.final, sacx.cpp)
            const int64_t seq = a.reset_seq ? a.ctl->step_seq + (a.reset_seq - 1) : a.ctl->rng_seq;
            for (int u = 0; u < a.nupd; ++u) a.ctl->pseq[a.slot + u] = seq + u;
            a.ctl->rng_seq = seq + a.nupd;
        }
    }
}

__global__ __launch_bounds__(RNG_THREADS) void k_rng(RngArgs a) {
    __shared__ RngShared S;
    rng_body(a, S);
}

// The polar transform of the pairs k_rng accepted (legacy_gauss, mtrand): one thread per pair of
// every update of the batch, the same fp64 arithmetic as k_rng's own path (bit-identical output)
// A few workgroups per update, striding over its pairs: off the update chain, so it need not be
// fast, but a wide grid would take CUs from the chain's launches running beside it.
#ifndef SACX_POLAR_WGS
#define SACX_POLAR_WGS 8
#endif
// pairs j = j0, j0 + stride, ... of one update: its normals from the leading cached one (oi) on
__device__ __forceinline__ void polar_pairs(const uint32_t* pairs, int oi, int n_norm, float* out, int j0, int stride) {
    const int np = (n_norm - oi + 1) >> 1;
    for (int j = j0; j < np; j += stride) {
        const uint4 w = *reinterpret_cast<const uint4*>(pairs + (size_t)j * 4);
        const double u1 = ((double)(int32_t)(w.x >> 5) * 67108864.0 + (double)(int32_t)(w.y >> 6)) / 9007199254740992.0;
        const double u2 = ((double)(int32_t)(w.z >> 5) * 67108864.0 + (double)(int32_t)(w.w >> 6)) / 9007199254740992.0;
        const double x1 = 2.0 * u1 - 1.0;
        const double x2 = 2.0 * u2 - 1.0;
        const double r2 = x1 * x1 + x2 * x2;
        const double f = sqrt(-2.0 * log(r2) / r2);
        const int o = oi + 2 * j;
        out[o] = (float)(f * x2);
        if (o + 1 < n_norm) out[o + 1] = (float)(f * x1);
    }
}

__global__ __launch_bounds__(256) void k_polar(RngArgs a) {
    const int64_t so = seed_off(a.sstride);
    const int u = blockIdx.y;
    polar_pairs(sr(a.pairs, so) + (size_t)u * a.pcap * 4, sr(a.pairs_oi, so)[u], a.n_norm,
                (float*)((char*)sr(a.out_norm, so) + (int64_t)u * a.slot_bytes), blockIdx.x * 256 + threadIdx.x,
                gridDim.x * 256);
}

// ==================================================================== segmented sampler (k_mtj_*)
// The same draws as k_rng (bit-exact), for batches of many words (Humanoid: ~134k words per
// update), without k_rng's two serial limits -- one workgroup twisting 623-word rounds and
// ranking the candidates with block-wide ballots:
//   k_mtj_head     key block -> words [0, MTJ_HEAD) of the batch's raw stream (one WG)
//   k_mtj_jump     the 624-word windows at k*L + 1, k = 1 .. S-1, as XORs of head words
//                  selected by x^(kL) mod phi (mt_jump.h), 63 partial XORs each
//   k_mtj_seg      S workgroups twist S segments of L words at once
//   k_mtj_flags    per word: randint acceptance and polar acceptance of the 4-word group starting
//                  there, as bitmaps, with per-chunk counts (per residue mod 4 for the groups)
//   k_mtj_resolve  chunk prefixes, then per update the position of its n-th accepted word /
//                  group from the current position (binary search + one wave), the state
//                  (a batch that outran the generated words -- never at the sizes used, forced in
//                  tests -- is redrawn there by rng_body from the unchanged state)
//   k_mtj_emit     every accepted candidate -> its output slot (rank = prefix difference),
//                  the polar transform in place
// Stream words are numbered from the key block (words 0 .. 623 = st->key), as in rng_body.
#define MTJ_RW 4096
// global-address-space pointers: global_load / global_store (a pointer loaded from the kernel
// arguments is otherwise generic, and its accesses flat ones that also wait on the LDS counter)
#define MTJ_G __attribute__((address_space(1)))

__device__ __forceinline__ bool polar_acc(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, double& x1,
                                          double& x2, double& r2) {
    const double u1 = ((double)(int32_t)(w0 >> 5) * 67108864.0 + (double)(int32_t)(w1 >> 6)) / 9007199254740992.0;
    const double u2 = ((double)(int32_t)(w2 >> 5) * 67108864.0 + (double)(int32_t)(w3 >> 6)) / 9007199254740992.0;
    x1 = 2.0 * u1 - 1.0;
    x2 = 2.0 * u2 - 1.0;
    r2 = x1 * x1 + x2 * x2;
    return (r2 < 1.0) && (r2 != 0.0);
}

__device__ __forceinline__ void mtj_put(uint32_t* ring, int q, uint32_t v) {
    const unsigned p = (unsigned)q & (MTJ_RW - 1u);
    ring[p] = v;
    if (p < RNG_MIR) ring[MTJ_RW + p] = v;
}

// words [n0, n1) into the LDS ring and sw.  The words from `base` on are resident (a 624-word
// window at base, or the 1,078 before n0); words below base + 1078 take the 227-wide form
__device__ void mtj_twist(uint32_t* ring, MTJ_G uint32_t* __restrict__ sw, int base, int n0, int n1) {
    const int t = threadIdx.x;
    while (n0 < n1 && n0 < base + 1078) {
        const int e = min(min(n1, base + 1078), n0 + 227);
        const int n = n0 + t;
        if (n < e) {
            const uint32_t v = ring[(unsigned)(n - 227) & (MTJ_RW - 1u)] ^
                               mt_g(ring[(unsigned)(n - 624) & (MTJ_RW - 1u)], ring[(unsigned)(n - 623) & (MTJ_RW - 1u)]);
            mtj_put(ring, n, v);
            sw[n] = v;
        }
        __syncthreads();
        n0 = e;
    }
    while (n0 < n1) {
        const int e = min(n1, n0 + 623);
        const int n = n0 + t;
        if (n < e) {
            const unsigned p = (unsigned)n & (MTJ_RW - 1u);
            const uint32_t* b = ring + (p >= 1078u ? p : p + MTJ_RW) - 1078u;   // b[i] = word n - 1078 + i
            const uint32_t v = b[397] ^ mt_g(b[454] ^ b[227] ^ b[0], b[455] ^ b[228] ^ b[1]);
            mtj_put(ring, n, v);
            sw[n] = v;
        }
        __syncthreads();
        n0 = e;
    }
}

// the work area's pointers are in the global address space (MTJ_G)
struct MtjPtrs {
    MTJ_G uint32_t* sw;
    MTJ_G uint32_t* fi;
    MTJ_G uint32_t* fp;
    MTJ_G int32_t* cnt;
    MTJ_G int32_t* pre;
    MTJ_G int32_t* res;
    MTJ_G uint32_t* part;
    MTJ_G int32_t* ptag;
    MTJ_G uint32_t* pfbm;
};
__device__ __forceinline__ MtjPtrs mtj_ptrs(const RngArgs& a, int64_t so) {
    uint32_t* jw = sr(a.jw, so);
    const MtjLayout y = mtj_layout(a.jL, a.jsmax);
    MtjPtrs p;
    p.sw = (MTJ_G uint32_t*)(jw + y.sw); p.fi = (MTJ_G uint32_t*)(jw + y.fi); p.fp = (MTJ_G uint32_t*)(jw + y.fp);
    p.cnt = (MTJ_G int32_t*)(jw + y.cnt); p.pre = (MTJ_G int32_t*)(jw + y.pre); p.res = (MTJ_G int32_t*)(jw + y.res);
    p.part = (MTJ_G uint32_t*)(jw + y.part);
    p.ptag = (MTJ_G int32_t*)(jw + y.ptag);
    p.pfbm = (MTJ_G uint32_t*)(jw + y.pfbm);
    return p;
}
__device__ __forceinline__ uint64_t mtj_u64(const MTJ_G int32_t* r) { return ((uint64_t)(uint32_t)r[1] << 32) | (uint32_t)r[0]; }

// The key block of a batch that followed a segmented batch is (normally) a block of that batch's
// stream, and the words [0, MTJ_HEAD) it needs were generated there too (the estimate keeps
// MTJ_HEAD words of margin): copied instead of twisted when the key still equals them (res[8]:
// the block's offset, res[9]: the words of that batch, res[10]: MTJ_CHAIN while valid).
#define MTJ_CHAIN 0x6d746a31
__global__ __launch_bounds__(1024) void k_mtj_head(RngArgs a) {
    __shared__ uint32_t ring[MTJ_RW + RNG_MIR];
    __shared__ int reuse;
    const int64_t so = seed_off(a.sstride);
    const RngState* st = sr(a.st, so);
    const Ctl* ctl = sr(a.ctl, so);
    RngState* bk = sr(a.backup, so);
    const MtjPtrs p = mtj_ptrs(a, so);
    const int t = threadIdx.x;
    const int off = p.res[8];
    if (t == 0) {
        const int64_t wcap = mtj_layout(a.jL, a.jsmax).wcap;
        reuse = p.res[10] == MTJ_CHAIN && off >= MTJ_HEAD && off % 624 == 0 && (int64_t)off + MTJ_HEAD <= p.res[9] &&
                p.res[9] <= wcap;
    }
    __syncthreads();
    const bool chained = reuse;
    if (chained)
        for (int i = t; i < 624; i += 1024)
            if (st->key[i] != p.sw[off + i]) reuse = 0;   // the state was set from outside
    __syncthreads();
    const bool copy = reuse;
    for (int i = t; i < 624; i += 1024) {
        const uint32_t v = st->key[i];
        if (!copy) {
            mtj_put(ring, i, v);
            p.sw[i] = v;
        }
        if (bk) bk->key[i] = v;      // the state before this draw (undo of a speculative draw)
    }
    if (t == 0) {
        // randint's bound, read once for the whole batch (ctl->cur_size may move meanwhile)
        const uint64_t high = a.size_fixed > 0 ? (uint64_t)a.size_fixed : (uint64_t)ctl->cur_size;
        const uint64_t rng = high > 0 ? high - 1 : 0;
        uint64_t mask = rng;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
        mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
        p.res[0] = 0;
        p.res[1] = a.jS * a.jL + 1;
        p.res[2] = st->pos;
        p.res[3] = st->pos;
        p.res[4] = (int32_t)(uint32_t)rng; p.res[5] = (int32_t)(uint32_t)(rng >> 32);
        p.res[6] = (int32_t)(uint32_t)mask; p.res[7] = (int32_t)(uint32_t)(mask >> 32);
        p.res[10] = 0;               // k_mtj_resolve re-validates
        // the chunks within 3 of each update's expected randint / polar end (the resolve walk's
        // searches land within a few hundred words of them), in increasing order
        const int nchk = (a.jS * a.jL + 1 + MTJ_CHK - 1) / MTJ_CHK;
        int n = 0, last = -1;
        auto window = [&](double pos) {
            const int c = (int)(pos / MTJ_CHK);
            for (int k = max(last + 1, c - 3); k <= min(c + 3, nchk - 1) && n < MTJ_PF; ++k) p.ptag[n++] = last = k;
        };
        double q = st->pos;
        window(q);
        for (int u = 0; u < a.nupd; ++u) {
            if (a.n_int > 0 && rng > 0) {
                q += (double)a.n_int * ((double)(mask + 1) / (double)(rng + 1));
                window(q);
            }
            q += (double)((a.n_norm + 1) >> 1) * (4.0 / 0.78539816339744831);
            window(q);
        }
        while (n < MTJ_PF) p.ptag[n++] = -1;
        if (bk) {
            bk->pos = st->pos;
            bk->has_gauss = st->has_gauss;
            bk->gauss = st->gauss;
        }
    }
    if (copy) {
        for (int i = t; i < MTJ_HEAD; i += 1024) p.sw[i] = p.sw[off + i];   // off >= MTJ_HEAD: disjoint
        return;
    }
    __syncthreads();
    mtj_twist(ring, p.sw, 0, 624, MTJ_HEAD);
}

// window k (words k L + 1 .. k L + 624) = XOR_{c_i = 1} words i + 1 .. i + 624, i < 19937:
// workgroup (c, k) takes coefficients [c MTJ_CH, (c + 1) MTJ_CH), as the host-built list of their
// set bits (mt_jump_lists), eight at a time (24 independent LDS reads per step), and writes its
// partial XOR
__global__ __launch_bounds__(256) void k_mtj_jump(RngArgs a) {
    __shared__ uint32_t win[MTJ_CH + 624];
    const int64_t so = seed_off(a.sstride);
    const MtjPtrs p = mtj_ptrs(a, so);
    const int c = blockIdx.x, k = blockIdx.y + 1;
    const int i0 = c * MTJ_CH;
    const int nb = min(MTJ_CH, 19937 - i0);
    for (int l = threadIdx.x; l < nb + 623; l += 256) win[l] = p.sw[i0 + 1 + l];
    __shared__ int ents[MTJ_CH];
    const int32_t* jl = reinterpret_cast<const int32_t*>(sr(a.jc, so));
    const int g = (k - 1) * MTJ_NC + c;
    const int e0 = jl[g], ne = jl[g + 1] - e0;
    const int32_t* ent = jl + (a.jsmax - 1) * MTJ_NC + 1 + e0;
    for (int l = threadIdx.x; l < ne; l += 256) ents[l] = ent[l];   // the list, in the window's round
    __syncthreads();
    const int j0 = threadIdx.x, j1 = j0 + 256, j2 = min(j0 + 512, 623);   // j2 > 623: computed, not stored
    uint32_t s0 = 0, s1 = 0, s2 = 0;
    int e = 0;
    for (; e + 8 <= ne; e += 8) {
        int ii[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) ii[r] = ents[e + r];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            s0 ^= win[ii[r] + j0];
            s1 ^= win[ii[r] + j1];
            s2 ^= win[ii[r] + j2];
        }
    }
    for (; e < ne; ++e) {
        const int i = ents[e];
        s0 ^= win[i + j0];
        s1 ^= win[i + j1];
        s2 ^= win[i + j2];
    }
    MTJ_G uint32_t* out = p.part + ((size_t)(k - 1) * MTJ_NC + c) * 624;
    out[j0] = s0;
    out[j1] = s1;
    if (j0 + 512 < 624) out[j2] = s2;
}

// segment k: words [k L + 1, (k + 1) L + 1) (segment 0: [0, L + 1), its head from k_mtj_head)
__global__ __launch_bounds__(1024) void k_mtj_seg(RngArgs a) {
    __shared__ uint32_t ring[MTJ_RW + RNG_MIR];
    const int64_t so = seed_off(a.sstride);
    const MtjPtrs p = mtj_ptrs(a, so);
    const int k = blockIdx.x, t = threadIdx.x;
    const int n1 = (k + 1) * a.jL + 1;
    int base, n0;
    if (k == 0) {
        if (n1 <= MTJ_HEAD) return;
        base = 0;
        n0 = MTJ_HEAD;
        for (int q = n0 - 1078 + t; q < n0; q += 1024) mtj_put(ring, q, p.sw[q]);
    } else {
        base = k * a.jL + 1;
        n0 = base + 624;
        const MTJ_G uint32_t* pt = p.part + (size_t)(k - 1) * MTJ_NC * 624;
        for (int j = t; j < 624; j += 1024) {
            uint32_t v = 0;
#pragma unroll
            for (int c = 0; c < MTJ_NC; ++c) v ^= pt[c * 624 + j];   // all 63 loads in one round
            mtj_put(ring, base + j, v);
            p.sw[base + j] = v;
        }
    }
    __syncthreads();
    mtj_twist(ring, p.sw, base, n0, n1);
}

// chunk c: acceptance bitmaps of its MTJ_CHK words and the counts [randint, group at residue 0..3]
__global__ __launch_bounds__(256) void k_mtj_flags(RngArgs a) {
    __shared__ int wc[4][5];
    __shared__ uint32_t bmw[2][MTJ_CHK / 32];
    const int64_t so = seed_off(a.sstride);
    const MtjPtrs p = mtj_ptrs(a, so);
    const int W = a.jS * a.jL + 1;
    const uint64_t rng = mtj_u64(p.res + 4), mask = mtj_u64(p.res + 6);
    const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    int cnt[5] = {0, 0, 0, 0, 0};
    uint32_t wd[MTJ_CHK / 256][4];   // the eight positions' 4-word groups, loaded before any use
#pragma unroll
    for (int i = 0; i < MTJ_CHK / 256; ++i) {
        const int m = c * MTJ_CHK + i * 256 + t;
#pragma unroll
        for (int r = 0; r < 4; ++r) wd[i][r] = m + r < W ? p.sw[m + r] : 0u;
    }
#pragma unroll
    for (int i = 0; i < MTJ_CHK / 256; ++i) {
        const int m = c * MTJ_CHK + i * 256 + t;
        bool fi = false, fp = false;
        if (m < W) {
            const uint32_t w0 = mt_temper(wd[i][0]);
            fi = rng == 0xFFFFFFFFULL || (uint64_t)(w0 & (uint32_t)mask) <= rng;
            if (m + 3 < W) {
                double x1, x2, r2;
                fp = polar_acc(w0, mt_temper(wd[i][1]), mt_temper(wd[i][2]), mt_temper(wd[i][3]), x1, x2, r2);
            }
        }
        const uint64_t bi = __ballot(fi), bp = __ballot(fp);
        if (lane == 0) {
            const int w32 = (m - lane) >> 5;
            p.fi[w32] = (uint32_t)bi; p.fi[w32 + 1] = (uint32_t)(bi >> 32);
            p.fp[w32] = (uint32_t)bp; p.fp[w32 + 1] = (uint32_t)(bp >> 32);
            const int l32 = w32 - c * (MTJ_CHK / 32);
            bmw[0][l32] = (uint32_t)bi; bmw[0][l32 + 1] = (uint32_t)(bi >> 32);
            bmw[1][l32] = (uint32_t)bp; bmw[1][l32 + 1] = (uint32_t)(bp >> 32);
        }
        cnt[0] += __popcll(bi);
#pragma unroll
        for (int r = 0; r < 4; ++r) cnt[1 + r] += __popcll(bp & (0x1111111111111111ULL << r));
    }
    if (lane == 0)
        for (int k = 0; k < 5; ++k) wc[wv][k] = cnt[k];
    __syncthreads();
    if (t < 5) p.cnt[c * 8 + t] = wc[0][t] + wc[1][t] + wc[2][t] + wc[3][t];
    if (wv == 0) {   // a predicted chunk: its bitmaps also to its k_mtj_resolve prefetch slot
        const unsigned long long b0 = __ballot(p.ptag[lane] == c), b1 = __ballot(p.ptag[64 + lane] == c);
        if (b0 | b1) {
            const int sl = b0 ? (int)__builtin_ctzll(b0) : 64 + (int)__builtin_ctzll(b1);
            p.pfbm[sl * 128 + lane] = bmw[0][lane];
            p.pfbm[sl * 128 + 64 + lane] = bmw[1][lane];
        }
    }
}

// Wave-wide integer scans on DPP lane moves (row_shr within 16-lane rows, then the row
// broadcasts), a few cycles each instead of ds_bpermute's LDS round trip; all 64 lanes active
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ int wave_isum(int v) { return __builtin_amdgcn_readlane(wave_incl_scan(v), 63); }
__device__ __forceinline__ uint32_t mtj_rmask(int kind) { return kind == 0 ? 0xFFFFFFFFu : (0x11111111u << (kind - 1)); }

// the chunk prefixes (phase 1) share LDS with rng_body's ring (the fallback, after phase 2)
union MtjResolveShared {
    struct {
        int pre[(MTJ_MAXCHK + 1) * 5];
        int wsum[16][5];
        int ctag[MTJ_PF];
        uint32_t cbm[MTJ_PF][2][64];
    } r;
    RngShared fb;
};

__global__ __launch_bounds__(1024) void k_mtj_resolve(RngArgs a) {
    __shared__ MtjResolveShared U;
    __shared__ int sh_q, sh_ovf, sh_has;
    __shared__ double sh_gauss;
    __shared__ int sh_ru[NBATCH_MAX][8];     // the walk's per-update results (stored after it)
    __shared__ float sh_g0[NBATCH_MAX];      // update u's leading cached normal (sh_ru[u][6] = 1)
    int* const pre = U.r.pre;
    const int64_t so = seed_off(a.sstride);
    const MtjPtrs p = mtj_ptrs(a, so);
    RngState* st = sr(a.st, so);
    Ctl* ctl = sr(a.ctl, so);
    const int W = a.jS * a.jL + 1;
    const int nchk = (W + MTJ_CHK - 1) / MTJ_CHK;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    RNG_PROF_T(r0);
    const uint64_t rng = mtj_u64(p.res + 4);
    const int pos0 = p.res[3];

    // ---- exclusive prefixes of the chunk counts (nchk <= MTJ_MAXCHK = blockDim); the predicted
    // chunks' bitmaps (k_mtj_head's list, copied by k_mtj_flags) into LDS in the same round
    int v[5], incl[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) v[k] = t < nchk ? p.cnt[t * 8 + k] : 0;
    if (t < MTJ_PF) U.r.ctag[t] = p.ptag[t];
    for (int i = t; i < MTJ_PF * 128; i += 1024) U.r.cbm[i >> 7][(i >> 6) & 1][i & 63] = p.pfbm[i];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        incl[k] = wave_incl_scan(v[k]);
        if (lane == 63) U.r.wsum[wv][k] = incl[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        int off = 0;
        for (int i = 0; i < wv; ++i) off += U.r.wsum[i][k];
        if (t < nchk) pre[t * 5 + k] = off + incl[k] - v[k];
        if (t == nchk - 1) pre[nchk * 5 + k] = off + incl[k];
    }
    __syncthreads();
    for (int i = t; i < (nchk + 1) * 5; i += 1024) p.pre[(i / 5) * 8 + i % 5] = pre[i];
    RNG_PROF_T(r1);
    RNG_PROF_ADD(8, r1 - r0);

    // ---- the updates in stream order (wave 0).  The wave holds one chunk's two bitmaps in
    // registers (lane l: word l of the chunk), so the prefix where a search ended needs no load;
    // LDS is addressed through U directly (ds_read), the work area through MTJ_G pointers
    if (wv == 0) {
        int cc = -1;
        uint32_t fiw = 0, fpw = 0;
        auto hold = [&](int c) {
            if (c == cc) return;
            const unsigned long long b0 = __ballot(U.r.ctag[lane] == c), b1 = __ballot(U.r.ctag[64 + lane] == c);
            if (b0 | b1) {
                const int sl = b0 ? (int)__builtin_ctzll(b0) : 64 + (int)__builtin_ctzll(b1);
                fiw = U.r.cbm[sl][0][lane];
                fpw = U.r.cbm[sl][1][lane];
            } else {     // outside the predicted windows: one global round trip
                fiw = p.fi[c * (MTJ_CHK / 32) + lane];
                fpw = p.fp[c * (MTJ_CHK / 32) + lane];
            }
            cc = c;
        };
        // candidates of `kind` accepted at positions < m (kind 0: randint words; 1 + r: groups at r mod 4)
        auto prefix = [&](int kind, int m) -> int {
            const int c = m / MTJ_CHK;
            if (c >= nchk) return U.r.pre[nchk * 5 + kind];
            hold(c);
            const int o = m - c * MTJ_CHK;
            uint32_t w = (kind == 0 ? fiw : fpw) & mtj_rmask(kind);
            const int lw = o >> 5;
            if (lane > lw) w = 0;
            else if (lane == lw) w &= (1u << (o & 31)) - 1u;
            return U.r.pre[c * 5 + kind] + wave_isum(__popc(w));
        };
        // the position of the T-th (1-based) accepted candidate of `kind`; -1 past the generated words
        auto find = [&](int kind, int T) -> int {
            if (T > U.r.pre[nchk * 5 + kind]) return -1;
            // the last chunk whose exclusive prefix is < T: among 16-chunk groups, then within one
            const int g = lane * 16;
            const int l1 = 63 - __clzll(__ballot(g < nchk && U.r.pre[g * 5 + kind] < T));
            const int c2 = l1 * 16 + lane;
            const int c = l1 * 16 + 63 - __clzll(__ballot(lane < 16 && c2 < nchk && U.r.pre[c2 * 5 + kind] < T));
            hold(c);
            const int rem = T - 1 - U.r.pre[c * 5 + kind];
            uint32_t w = (kind == 0 ? fiw : fpw) & mtj_rmask(kind);
            const int n = __popc(w);
            const int incl = wave_incl_scan(n);
            const bool mine = incl - n <= rem && rem < incl;
            int pos = 0;
            if (mine) {
                for (int i = incl - n; i < rem; ++i) w &= w - 1u;
                pos = c * MTJ_CHK + lane * 32 + __builtin_ctz(w);
            }
            return __builtin_amdgcn_readlane(pos, (int)__builtin_ctzll(__ballot(mine)));
        };
        int q = pos0, ovf = 0;
        int has = st->has_gauss;
        double gauss = st->gauss;
        for (int u = 0; u < a.nupd && !ovf; ++u) {
            int32_t* const out_idx = a.out_idx ? (int32_t*)((char*)sr(a.out_idx, so) + u * a.slot_bytes) : nullptr;
            int ib = q, ie = q, ibase = 0;
            if (a.n_int > 0) {
                if (rng == 0) {
                    for (int i = lane; i < a.n_int; i += 64) out_idx[i] = 0;
                } else {
                    ibase = prefix(0, q);
                    const int m = find(0, ibase + a.n_int);
                    if (m < 0) { ovf = 1; break; }
                    ie = q = m + 1;
                }
            }
            int oi = 0;
            if (a.n_norm > 0 && has) {
                if (lane == 0) sh_g0[u] = (float)gauss;
                has = 0;
                gauss = 0.0;     // NumPy clears the cached value with the flag
                oi = 1;
            }
            const int need = (a.n_norm - oi + 1) >> 1;
            int pb = q, pe = q, pbase = 0;
            if (need > 0) {
                const int kind = 1 + (q & 3);
                pbase = prefix(kind, q);
                const int m = find(kind, pbase + need);
                if (m < 0) { ovf = 1; break; }
                pe = q = m + 4;
                if ((a.n_norm - oi) & 1) {   // the last pair's second normal is cached
                    double x1, x2, r2;
                    polar_acc(mt_temper(p.sw[m]), mt_temper(p.sw[m + 1]), mt_temper(p.sw[m + 2]), mt_temper(p.sw[m + 3]),
                              x1, x2, r2);
                    gauss = sqrt(-2.0 * log(r2) / r2) * x1;
                    has = 1;
                }
            }
            if (lane == 0) {   // LDS: a global store here would be waited for by the next search's loads
                sh_ru[u][0] = ib; sh_ru[u][1] = ie; sh_ru[u][2] = ibase;
                sh_ru[u][3] = pb; sh_ru[u][4] = pe; sh_ru[u][5] = pbase; sh_ru[u][6] = oi;
            }
        }
        if (!ovf && q > pos0 && 624 * ((q - 1) / 624 + 1) > W) ovf = 1;   // the state block must exist
        if (lane == 0) {
            sh_q = q; sh_ovf = ovf; sh_has = has; sh_gauss = gauss;
            p.res[0] = ovf;
            p.res[2] = q;
        }
    }
    __syncthreads();
    RNG_PROF_T(r2);
    RNG_PROF_ADD(9, r2 - r1);
    if (sh_ovf) {   // the batch outran the generated words: rng_body redraws it from the unchanged state
        RngArgs b = a;
        b.pairs = nullptr;
        b.backup = nullptr;     // k_mtj_head saved it
        rng_body(b, U.fb);
        return;
    }
    if (t < a.nupd * 7) p.res[16 + 16 * (t / 7) + t % 7] = sh_ru[t / 7][t % 7];
    if (t < a.nupd && sh_ru[t][6]) *(float*)((char*)sr(a.out_norm, so) + t * a.slot_bytes) = sh_g0[t];
    const int q = sh_q;
    if (q > pos0) {
        const int b = (q - 1) / 624;
        for (int i = t; i < 624; i += 1024) st->key[i] = p.sw[624 * b + i];
        if (t == 0) {
            st->pos = q - b * 624;
            p.res[8] = 624 * b;      // the next batch's head may copy its words from here
            p.res[9] = W;
            p.res[10] = MTJ_CHAIN;
        }
    }
    if (t == 0) {
        st->has_gauss = sh_has;
        st->gauss = sh_gauss;
        if (a.slot >= 0) {
            const int64_t seq = a.reset_seq ? ctl->step_seq + (a.reset_seq - 1) : ctl->rng_seq;
            for (int u = 0; u < a.nupd; ++u) ctl->pseq[a.slot + u] = seq + u;
            ctl->rng_seq = seq + a.nupd;
        }
    }
    RNG_PROF_T(r3);
    RNG_PROF_ADD(10, r3 - r2);
    RNG_PROF_ADD(11, 1);
}

// Chunk c's randint values are stored directly; its accepted polar groups are first compacted
// into an LDS list, so that the fp64 transform runs on every lane (one in four positions of a
// range is a candidate)
#define MTJ_EMIT_CAP (MTJ_CHK / 4 + NBATCH_MAX + 8)
__global__ __launch_bounds__(256) void k_mtj_emit(RngArgs a) {
    __shared__ uint32_t bm[2][64];
    __shared__ int wpre[64][5];
    __shared__ uint32_t lw[MTJ_EMIT_CAP][4];
    __shared__ int lo[MTJ_EMIT_CAP], lu[MTJ_EMIT_CAP];
    __shared__ int ln;
    const int64_t so = seed_off(a.sstride);
    RNG_PROF_T(e0);
    const MtjPtrs p = mtj_ptrs(a, so);
    if (p.res[0]) return;
    const int c = blockIdx.x, t = threadIdx.x;
    const int qf = p.res[2];
    if (c * MTJ_CHK >= qf) return;
    const uint64_t rng = mtj_u64(p.res + 4), mask = mtj_u64(p.res + 6);
    if (t < 64) {      // wave 0: the bitmaps and their exclusive prefix over the chunk's words, per kind
        const uint32_t fi = p.fi[c * (MTJ_CHK / 32) + t], fp = p.fp[c * (MTJ_CHK / 32) + t];
        bm[0][t] = fi;
        bm[1][t] = fp;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const int n = __popc((k == 0 ? fi : fp) & mtj_rmask(k));
            wpre[t][k] = p.pre[c * 8 + k] + wave_incl_scan(n) - n;
        }
    }
    if (t == 0) ln = 0;
    __syncthreads();
    RNG_PROF_T(e1);
    const int lane = t & 63;
    // what each of the thread's eight positions is: 1 an accepted randint word of update uu
    // (output o = its rank), 2 an accepted polar group (o = its first output), 0 neither.  The
    // update ranges are uniform (scalar loads), the bitmap words and prefixes of all eight
    // positions are read from LDS in one batch: no dependent LDS round trips per position
    const int kp = 1 + (t & 3);          // a position's residue class (chunk and step are multiples of 4)
    int rr[NBATCH_MAX][7];
#pragma unroll
    for (int u = 0; u < NBATCH_MAX; ++u)
#pragma unroll
        for (int k = 0; k < 7; ++k) rr[u][k] = u < a.nupd ? p.res[16 + 16 * u + k] : 0;
    uint32_t b0[MTJ_CHK / 256], b1[MTJ_CHK / 256];
    int w0[MTJ_CHK / 256], w1[MTJ_CHK / 256];
#pragma unroll
    for (int i = 0; i < MTJ_CHK / 256; ++i) {
        const int wl = (i * 256 + t) >> 5;
        b0[i] = bm[0][wl]; b1[i] = bm[1][wl];
        w0[i] = wpre[wl][0]; w1[i] = wpre[wl][kp];
    }
    int what[MTJ_CHK / 256], uu[MTJ_CHK / 256], o[MTJ_CHK / 256];
#pragma unroll
    for (int i = 0; i < MTJ_CHK / 256; ++i) {
        const int m = c * MTJ_CHK + i * 256 + t;
        const uint32_t bit = 1u << (m & 31), below = bit - 1u;
        what[i] = 0; uu[i] = 0; o[i] = 0;
#pragma unroll
        for (int u = 0; u < NBATCH_MAX; ++u) {
            if (u >= a.nupd || m >= qf) break;
            if (m >= rr[u][0] && m < rr[u][1] && (b0[i] & bit)) {
                what[i] = 1; uu[i] = u;
                o[i] = w0[i] + __popc(b0[i] & below) - rr[u][2];
            }
            if (m >= rr[u][3] && m < rr[u][4] && ((m - rr[u][3]) & 3) == 0 && (b1[i] & bit)) {
                what[i] = 2; uu[i] = u;
                o[i] = rr[u][6] + 2 * (w1[i] + __popc(b1[i] & mtj_rmask(kp) & below) - rr[u][5]);
            }
        }
    }
    // the candidates' words, all requested in one round
    uint32_t wd[MTJ_CHK / 256][4];
#pragma unroll
    for (int i = 0; i < MTJ_CHK / 256; ++i) {
        const int m = c * MTJ_CHK + i * 256 + t;
#pragma unroll
        for (int r = 0; r < 4; ++r) wd[i][r] = (what[i] == 2 || (what[i] == 1 && r == 0)) ? p.sw[m + r] : 0u;
    }
#pragma unroll
    for (int i = 0; i < MTJ_CHK / 256; ++i) {
        if (what[i] == 1) {
            const uint32_t w = mt_temper(wd[i][0]);
            int32_t* out_idx = (int32_t*)((char*)sr(a.out_idx, so) + uu[i] * a.slot_bytes);
            if ((unsigned)o[i] < (unsigned)a.n_int) out_idx[o[i]] = (int32_t)(rng == 0xFFFFFFFFULL ? w : (w & (uint32_t)mask));
        }
        // the wave's accepted groups appended to the list: one LDS atomic per wave
        const bool take = what[i] == 2;
        const unsigned long long bal = __ballot(take);
        if (bal) {
            const int first = (int)__builtin_ctzll(bal);
            int base = 0;
            if (lane == first) base = atomicAdd(&ln, __popcll(bal));
            base = __builtin_amdgcn_readlane(base, first);
            const int e = base + __popcll(bal & ((1ULL << lane) - 1ULL));
            if (take && e < MTJ_EMIT_CAP) {
#pragma unroll
                for (int r = 0; r < 4; ++r) lw[e][r] = wd[i][r];
                lo[e] = o[i];
                lu[e] = uu[i];
            }
        }
    }
    __syncthreads();
    RNG_PROF_T(e2);
    const int n = min(ln, MTJ_EMIT_CAP);
    for (int e = t; e < n; e += 256) {
        double x1, x2, r2;
        polar_acc(mt_temper(lw[e][0]), mt_temper(lw[e][1]), mt_temper(lw[e][2]), mt_temper(lw[e][3]), x1, x2, r2);
        const double f = sqrt(-2.0 * log(r2) / r2);
        float* out = (float*)((char*)sr(a.out_norm, so) + lu[e] * a.slot_bytes);
        const int o = lo[e];
        if ((unsigned)o < (unsigned)a.n_norm) out[o] = (float)(f * x2);
        if ((unsigned)(o + 1) < (unsigned)a.n_norm) out[o + 1] = (float)(f * x1);
    }
    RNG_PROF_T(e3);
#ifdef SACX_RNG_PROF
    if (t == 0) {    // per workgroup: loads, ranks, transforms (sums) and the span's first start / last end
        atomicAdd(&g_rng_prof[12], e1 - e0);
        atomicAdd(&g_rng_prof[13], e2 - e1);
        atomicAdd(&g_rng_prof[14], e3 - e2);
        atomicAdd(&g_rng_prof[15], 1ULL);
    }
#endif
}

// words a launch of `a` expects to draw (randint at acceptance >= 1/2) and whether it takes the
// segmented path, with its segment count
static int mtj_segments(const RngArgs& a) {
    if (a.jw == nullptr || a.jL < MTJ_HEAD || a.nupd > NBATCH_MAX) return 0;
    const double per = 2.0 * a.n_int + (double)((a.n_norm + 1) >> 1) * (4.0 / 0.78539816339744831);
    const double words = a.nupd * per;
    if (words < (double)a.jmin) return 0;
    // + MTJ_HEAD: the next batch's head words (k_mtj_head copies them)
    const double est = 624.0 + 1.02 * words + 8.0 * sqrt(words) + 64.0 * a.nupd + 1024.0 + MTJ_HEAD;
    int S = (int)ceil((est - 1.0) / a.jL);
    if (a.junder > 0) S = std::max(1, std::min(S, a.junder));   // tests: too few segments (the fallback)
    const int64_t W = (int64_t)S * a.jL + 1;
    if (S > a.jsmax || (W + MTJ_CHK - 1) / MTJ_CHK > MTJ_MAXCHK) return 0;
    return S;
}

void launch_rng(const RngArgs& a0, hipStream_t s) {
    if (const int S = mtj_segments(a0)) {
        RngArgs a = a0;
        a.jS = S;
        const int z = seeds_z(a.nseeds);
        const int nchk = (int)(((int64_t)S * a.jL + 1 + MTJ_CHK - 1) / MTJ_CHK);
        hipLaunchKernelGGL(k_mtj_head, dim3(1, 1, z), dim3(1024), 0, s, a);
        if (S > 1) hipLaunchKernelGGL(k_mtj_jump, dim3(MTJ_NC, S - 1, z), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_mtj_seg, dim3(S, 1, z), dim3(1024), 0, s, a);
        hipLaunchKernelGGL(k_mtj_flags, dim3(nchk, 1, z), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_mtj_resolve, dim3(1, 1, z), dim3(1024), 0, s, a);
        hipLaunchKernelGGL(k_mtj_emit, dim3(nchk, 1, z), dim3(256), 0, s, a);
        return;
    }
    const RngArgs& a = a0;
    hipLaunchKernelGGL(k_rng, dim3(1, 1, seeds_z(a.nseeds)), dim3(RNG_THREADS), 0, s, a);
    if (a.pairs != nullptr && a.n_norm > 0)
        hipLaunchKernelGGL(k_polar, dim3(std::min((a.pcap + 255) / 256, SACX_POLAR_WGS), a.nupd, seeds_z(a.nseeds)),
                           dim3(256), 0, s, a);
}

// ==================================================================== k_gather
// one wave per sampled row (then per expert row); rows are [s | a | sp | r | d]
__global__ __launch_bounds__(256) void k_gather(GatherArgs ga) {
    const int rwgs = (ga.B + ga.ne + 3) >> 2;
    if ((int)blockIdx.x >= rwgs) {      // the speculative draw's polar transform (one update, one seed)
        polar_pairs(ga.pairs, ga.pairs_oi[0], ga.n_norm, ga.norm, ((int)blockIdx.x - rwgs) * 256 + threadIdx.x,
                    ga.polar_wgs * 256);
        return;
    }
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    // slot (ga.slot + blockIdx.y): every slot buffer sits at a fixed distance from slot 0's
    GatherArgs g = ga;
    {
        const int64_t so = seed_off(ga.sstride);
        const int64_t off = (int64_t)blockIdx.y * ga.slot_bytes + so;
        auto sh = [off](auto* p) { return p ? (decltype(p))((char*)p + off) : p; };
        g.idx = sh(ga.idx); g.Xa = sh(ga.Xa); g.Xq = sh(ga.Xq); g.Xt = sh(ga.Xt); g.Xp = sh(ga.Xp);
        g.Xm = sh(ga.Xm); g.r = sh(ga.r); g.d = sh(ga.d); g.se_raw = sh(ga.se_raw); g.spe_raw = sh(ga.spe_raw);
        g.xbfq = sh(ga.xbfq);
        g.slot = ga.slot + (int)blockIdx.y;
        g.replay = sr(ga.replay, so); g.ctl = sr(ga.ctl, so);
        g.s_mean = sr(ga.s_mean, so); g.s_den = sr(ga.s_den, so); g.a_mean = sr(ga.a_mean, so); g.a_den = sr(ga.a_den, so);
        g.ms_mean = sr(ga.ms_mean, so); g.ms_den = sr(ga.ms_den, so);
        g.exp_s = sr(ga.exp_s, so); g.exp_sp = sr(ga.exp_sp, so); g.perm_ring = sr(ga.perm_ring, so);
    }
    const int S = g.S, A = g.A;
    const __amdgpu_buffer_rsrc_t rsm = rs(g.s_mean), rsd = rs(g.s_den), ram = rs(g.a_mean), rad = rs(g.a_den);
    if (row < g.B) {
        const int64_t li = g.idx[row];
        const int64_t phys = (g.ctl->start + li) % g.cap;
        // resource based at the record: the ring itself may exceed 32-bit offsets
        const __amdgpu_buffer_rsrc_t rR = make_rsrc(g.replay + phys * (int64_t)g.stride, (uint32_t)g.stride * 4u);
        const float r_v = bload(rR, (uint32_t)(2 * S + A) * 4u);
        const float d_v = bload(rR, (uint32_t)(2 * S + A + 1) * 4u);
        for (int c = lane; c < g.ldQ; c += 64) {
            const bool cs = c < S, ca = c >= S && c < S + A;
            const float xs = bload(rR, boff(cs, c)), xsp = bload(rR, boff(cs, S + A + c));
            const float xa = bload(rR, boff(ca, c));
            const float ms = bload(rsm, boff(cs, c)), ds = bload(rsd, boff(cs, c));
            const float ma = bload(ram, boff(ca, c - S)), da = bload(rad, boff(ca, c - S));
            const float sn = cs ? (xs - ms) / ds : 0.f;
            const float spn = cs ? (xsp - ms) / ds : 0.f;
            const float an = ca ? (xa - ma) / da : 0.f;
            if (c < g.ldS) {
                g.Xa[(size_t)row * g.ldS + c] = spn;
                g.Xa[(size_t)(g.B + row) * g.ldS + c] = sn;
            }
            g.Xq[(size_t)row * g.ldQ + c] = cs ? sn : an;
            if (g.xbfq != nullptr && c < S + A)     // (critic.adam's layer-0 A operand, transposed)
                g.xbfq[(size_t)c * wbf_ld_of(g.B) + wbf_pos(row, wbf_per_of(g.B))] = (uint16_t)bf16_bits(cs ? sn : an);
            if (!ca) {
                g.Xt[(size_t)row * g.ldQ + c] = spn;
                g.Xp[(size_t)row * g.ldQ + c] = sn;
            }
        }
        if (lane == 0) {
            g.r[row] = r_v;
            g.d[row] = d_v;
        }
    } else if (row < g.B + g.ne) {
        const int e = row - g.B;
        // 2+ models: the update's self.rng.shuffle permutation (SAC_expert.py:301-303), whose first ne
        // entries are array_split's first two sections; one model takes the expert rows in order
        // (:290-295, no perm ring)
        const int64_t slot = g.ctl->pseq[g.slot] % g.perm_cap;
        const int src = g.perm_ring != nullptr ? g.perm_ring[slot * g.perm_ld + e] : e;
        const __amdgpu_buffer_rsrc_t rse = rs(g.exp_s + (size_t)src * S), rspe = rs(g.exp_sp + (size_t)src * S);
        // the actor row takes the actor's normaliser, the world-model row the models' (the same
        // values unless --only_model_normalizer, SAC_expert.py:139-144)
        const __amdgpu_buffer_rsrc_t rmm = rs(g.ms_mean), rmd = rs(g.ms_den);
        for (int c = lane; c < g.ldQ; c += 64) {
            const bool cs = c < S;
            const float xs = bload(rse, boff(cs, c)), xsp = bload(rspe, boff(cs, c));
            const float ms = bload(rsm, boff(cs, c)), ds = bload(rsd, boff(cs, c));
            const float mms = bload(rmm, boff(cs, c)), mds = bload(rmd, boff(cs, c));
            const float sn = cs ? (xs - ms) / ds : 0.f;
            const float smn = cs ? (xs - mms) / mds : 0.f;
            if (cs) {
                g.se_raw[(size_t)e * S + c] = xs;
                g.spe_raw[(size_t)e * S + c] = xsp;
            }
            if (c < g.ldS) g.Xa[(size_t)(2 * g.B + e) * g.ldS + c] = sn;
            if (c < S || c >= S + A) g.Xm[(size_t)e * g.ldQ + c] = smn;
        }
    }
}

void launch_gather(const GatherArgs& a, hipStream_t s) {
    const int rows = a.B + a.ne;
    hipLaunchKernelGGL(k_gather, dim3((rows + 3) / 4 + a.polar_wgs, a.nupd > 0 ? a.nupd : 1, seeds_z(a.nseeds)),
                       dim3(256), 0, s, a);
}

// one wave: alpha Adam + clamp and the statistics row of the update
__global__ __launch_bounds__(64) void k_alpha_final(FinalArgs f_in) {
    FinalArgs f = f_in;
    reloc(f, seed_off(f_in.sstride));
    finalize_update(f, f.nred);
}

void launch_alpha_final(const FinalArgs& f, hipStream_t s) {
    hipLaunchKernelGGL(k_alpha_final, dim3(1, 1, seeds_z(f.nseeds)), dim3(64), 0, s, f);
}

// ==================================================================== k_actor_head
// one wave per actor row: mu = h2 . W3 + b, then evaluate()/sample() per column.
// The wave sums are broadcast, so lane j keeps output j in a register.
// FIN (k_fwd2's fused q launch, the previous update's alpha finalisation ffin): 1 (TICKET) the alpha
// blocks take a ticket after storing their partial, and the last of them finalises in the same
// launch; 2 (split, SACX_AFIN) the alpha blocks store their partials only and the first one snapshots
// the finalisation's other operands (ffin.pre) and writes the update's loss statistics: the next
// launch's target rows finish the alpha step (qhead_block)
template <int NQ, int OW, int FIN>
__device__ __forceinline__ void actor_head_body(const HeadArgs& h, const FinalArgs& f, int block, int64_t so,
                                                const FinalArgs& ffin) {
    // a workgroup of 4 G waves runs G blocks of 4 rows (block + wave >> 2): per block the same partial
    __shared__ float red_s[16];
    __shared__ int last_s[4];
    __shared__ float w3s[OW > 0 ? 256 * OW : 1];
    if constexpr (OW > 0) {
        // W3 (H1 x Aout, row-major) copied whole into LDS by the workgroup: contiguous loads,
        // all in flight together, before any row exits
        static_assert(NQ == 4, "LDS-staged W3: H1 <= 256");
        const __amdgpu_buffer_rsrc_t rW0 = rs(sr(h.W3, so));
        const int n = h.H1 * h.Aout;
        float wv[OW];
#pragma unroll
        for (int c = 0; c < OW; ++c) wv[c] = bload(rW0, boff((int)threadIdx.x + 256 * c < n, threadIdx.x + 256 * c));
#pragma unroll
        for (int c = 0; c < OW; ++c)
            if ((int)threadIdx.x + 256 * c < n) w3s[threadIdx.x + 256 * c] = wv[c];
        __syncthreads();
    }
    const int wave = wave_id() & 3, lane = threadIdx.x & 63, g4 = wave_id() >> 2;
    constexpr bool TICKET = FIN == 1;
    FinPre fpre;
    if constexpr (FIN == 2) {
        // the first alpha block's wave 0 requests the snapshot's operands under the rows' own loads
        if (threadIdx.x < 64 && h.alpha_mode && block * 4 == h.alpha_row0) fin_prefetch(ffin, fpre);
    }
    if constexpr (TICKET && SACX_FIN_PRE) {
        // wave 0 of a workgroup holding alpha blocks (the one that may finalise) requests the
        // finalisation's other operands now, under the rows' own loads
        const int last_blk = block + (int)(blockDim.x >> 8) - 1;
        if (threadIdx.x < 64 && h.alpha_mode && last_blk * 4 >= h.alpha_row0 && block * 4 < h.total_rows)
            fin_prefetch(ffin, fpre);
    }
    block += g4;
    const int row = block * 4 + wave;
    float row_ent = 0.f;
    int sidx = 0;
    for (int i = 1; i < h.nseg; ++i)
        if (row >= h.seg[i].r0) sidx = i;
    if (row < h.total_rows && row < h.seg[sidx].r1) {     // rows in the pad before alpha_row0 idle
        HeadSeg sg = h.seg[sidx];
        reloc(sg, so);
        const int A = h.A, Aout = h.Aout;
        const bool jok = lane < A;
        // everything this row reads is issued up front: its H2 row, or (h.part) the per-column-tile
        // partials of H2 . W3 written by actor.fwd1 -- lane o < Aout sums output o's
        const bool hp = h.part != nullptr;
        float hv[NQ];
        float4 pv[4];
        if (hp) {
            const __amdgpu_buffer_rsrc_t rp = rs(sr(h.part, so));
#pragma unroll
            for (int i = 0; i < 4; ++i) pv[i] = bload4(rp, boff(lane < Aout && 4 * i < h.tq, (row * Aout + lane) * h.tq + 4 * i));
        } else {
            load_row(rs(sr(h.H2, so)), row * h.ldh, h.H1, hv);
        }
        const __amdgpu_buffer_rsrc_t rW = rs(sr(h.W3, so));
        const float u_pf = bload(rs(sg.noise), boff(jok, (row - sg.r0) * A + lane));
        const float ls_pf = bload(rs(sr(h.logstd, so)), boff(jok && !h.per_state_std, lane));
        // sample segments (mode 1) feed the world models: their normaliser for the action columns
        const bool msg = sg.mode == 1 && h.ma_mean != nullptr;
        const float am_pf = bload(rs(sr(msg ? h.ma_mean : h.a_mean, so)), boff(jok, lane));
        const float ad_pf = bload(rs(sr(msg ? h.ma_den : h.a_den, so)), boff(jok, lane));
        const float bmu = bload(rW, boff(jok, h.H1 * Aout + lane));
        const float bls = bload(rW, boff(jok && h.per_state_std, h.H1 * Aout + A + lane));
        float mu = 0.f, lraw = 0.f;
        if (hp) {
            float v = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v = v + pv[i].x; v = v + pv[i].y; v = v + pv[i].z; v = v + pv[i].w;
            }
            mu = v;
            lraw = __shfl(v, min(lane + A, 63), 64);
        } else if constexpr (OW > 0) {        // Aout <= OW, H1 <= 256 (host-checked): W3 from LDS
            float so_[OW];
            rowdot_lds<NQ, OW>(hv, w3s, h.H1, Aout, so_);
#pragma unroll
            for (int u = 0; u < OW; ++u) {
                mu = (lane == u) ? so_[u] : mu;
                lraw = (lane + A == u) ? so_[u] : lraw;
            }
        } else {
            for (int o0 = 0; o0 < Aout; o0 += 8) {
                float s8[8];
                rowdot8(hv, rW, h.H1, Aout, o0, Aout, s8);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int o = o0 + u;
                    mu = (lane == o) ? s8[u] : mu;
                    lraw = (lane + A == o) ? s8[u] : lraw;
                }
            }
        }
        mu = mu + bmu;
        lraw = h.per_state_std ? lraw + bls : ls_pf;
        if (sg.mode == 2) {
            // GaussianActor.sample (continuous_actors.py:74-123), no squash: optional output
            // normalisation of the mean, logstd = log(softplus(out)) (per_state_std) or the
            // variable, + logstd_init, floored at log(1e-3); a = mean + exp(logstd) * u
            float m = mu;
            if (h.output_norm) {
                const float s = wave_sum(jok ? fabsf(mu) : 0.f) / (float)A;
                m = mu / fmaxf(s, 1.f);
            }
            if (jok) {
                float l = h.per_state_std ? logf(softplus_f(lraw)) : lraw;
                l = fmaxf(l + h.logstd_init, logf(1e-3f));
                const float a = m + expf(l) * u_pf;
                if (sg.pi_out != nullptr) sg.pi_out[(size_t)(row - sg.r0) * A + lane] = a;
            }
            return;
        }
        float nlp_vec = 0.f, nlp_corr = 0.f;
        if (jok) {
            const int j = lane;
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
            if (sg.pi_out != nullptr) sg.pi_out[(size_t)(row - sg.r0) * A + j] = pi;
            if (row >= h.cache_row0 && row < h.cache_row1 && h.c_t != nullptr) {
                const size_t ci = (size_t)(row - h.cache_row0) * A + j;
                sr(h.c_t, so)[ci] = t;
                sr(h.c_std, so)[ci] = sd;
                sr(h.c_u, so)[ci] = u;
                sr(h.c_mask, so)[ci] = (lraw >= -5.f && lraw <= 2.f) ? 1.f : 0.f;
            }
        }
        if (sg.mode == 0) {
            const float nlp = 0.5f * wave_sum(nlp_vec) + wave_sum(nlp_corr);
            if (lane == 0 && sg.nlp_out != nullptr) sg.nlp_out[row - sg.r0] = nlp;
            row_ent = -nlp + f.target_entropy;
        }
    }
    // (a group whose block is past the rows -- the last workgroup of k_fwd2's rows -- ends here too)
    if (!h.alpha_mode || block * 4 < h.alpha_row0 || block * 4 >= h.total_rows) return;
    if constexpr (FIN == 2) {
        if (threadIdx.x < 64 && block * 4 == h.alpha_row0) {
            // (the first alpha block is group 0 of its workgroup: the host aligns alpha_row0 to one)
            // the update's loss statistics (finalize_update's sums, same order) and the snapshot
            const float q1 = wave_sum(fpre.ps[0]) / (float)ffin.B;
            const float q2 = wave_sum(fpre.ps[1]) / (float)ffin.B;
            const float pl = wave_sum(fpre.ps[2]) / (float)ffin.B;
            if (lane == 0) {
                float* st = ffin.stats + (size_t)(fpre.seq0 % ffin.stats_cap) * 8;
                st[0] = q1;
                st[1] = q2;
                st[2] = pl;
                st[5] = 0.f;
                AfinPre* P = ffin.pre;
                P->a_old = fpre.a_old; P->a_m = fpre.a_m; P->a_v = fpre.a_v;
                P->t_sac = fpre.t_sac; P->seq0 = fpre.seq0; P->nts = fpre.nts; P->tsi = fpre.tsi;
            }
        }
    }
    // ---- alpha: block partial of sum(-nlp + H); k_alpha_final reduces them
    if (lane == 0) red_s[4 * g4 + wave] = row_ent;
    if constexpr (TICKET) {
        if (threadIdx.x < 4) last_s[threadIdx.x] = 0;
    }
    __syncthreads();
    if ((threadIdx.x & 255) == 0) {
        float part = red_s[4 * g4] + red_s[4 * g4 + 1];
        part = part + red_s[4 * g4 + 2];
        part = part + red_s[4 * g4 + 3];
        sr(f.red, so)[block - h.alpha_row0 / 4] = part;
        if constexpr (TICKET) {
            // release this partial, count it; the block that brings the count to nred acquires the
            // others' (vector atomics on the control block; self-resetting)
            // (release only: the cache invalidation of an acquire is the last block's alone, below)
            const int old = __hip_atomic_fetch_add(&ffin.ctl->red_counter[0], 1, __ATOMIC_RELEASE,
                                                   __HIP_MEMORY_SCOPE_AGENT);
            last_s[g4] = old == ffin.nred - 1;
        }
    }
    if constexpr (TICKET) {
        __syncthreads();
        if (last_s[0] | last_s[1] | last_s[2] | last_s[3]) {
            // the winning group's RMW saw the count reach nred (every partial was released before its
            // block's increment); after the barrier every wave of this workgroup acquires at agent
            // scope itself, whichever wave's atomic observed the count
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            finalize_update<SACX_FIN_PRE != 0>(ffin, ffin.nred, &fpre);
            if (threadIdx.x == 0) __hip_atomic_store(&ffin.ctl->red_counter[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// per-workgroup first / last tick (measurement graphs only), as k_gemm
__device__ __forceinline__ void ktime_stamp(uint64_t* kt, uint64_t t0) {
    if (kt != nullptr) {
        __syncthreads();
        if (threadIdx.x == 0) {
            kt[2 * ktime_wg()] = t0;
            kt[2 * ktime_wg() + 1] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

template <int NQ, bool PK, int OW = 0>
__global__ __launch_bounds__(256) void k_actor_head(HeadArgs h, FinalArgs f) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    actor_head_body<NQ, OW>(h, f, (int)blockIdx.x, PK ? seed_off(h.sstride) : 0);
    ktime_stamp(h.ktime, t0);
}

void launch_actor_head(const HeadArgs& a, const FinalArgs& f, hipStream_t s) {
    const dim3 grid((a.total_rows + 3) / 4, 1, seeds_z(a.nseeds));
    const bool pk = a.nseeds > 1;
    if (a.H1 <= 256) {
        // more than one 8-column chunk: the whole row's W3 loads in one round trip (NQ = 4
        // keeps w[4][OW] at <= 96 registers)
        if (a.Aout > 8 && a.Aout <= 16) {
            if (pk) hipLaunchKernelGGL((k_actor_head<4, true, 16>), grid, dim3(256), 0, s, a, f);
            else hipLaunchKernelGGL((k_actor_head<4, false, 16>), grid, dim3(256), 0, s, a, f);
        } else if (a.Aout > 16 && a.Aout <= 24) {
            if (pk) hipLaunchKernelGGL((k_actor_head<4, true, 24>), grid, dim3(256), 0, s, a, f);
            else hipLaunchKernelGGL((k_actor_head<4, false, 24>), grid, dim3(256), 0, s, a, f);
        } else if (pk) {
            hipLaunchKernelGGL((k_actor_head<4, true>), grid, dim3(256), 0, s, a, f);
        } else {
            hipLaunchKernelGGL((k_actor_head<4, false>), grid, dim3(256), 0, s, a, f);
        }
    } else {
        if (pk) hipLaunchKernelGGL((k_actor_head<8, true>), grid, dim3(256), 0, s, a, f);
        else hipLaunchKernelGGL((k_actor_head<8, false>), grid, dim3(256), 0, s, a, f);
    }
}

// ==================================================================== k_act_rows
// Behaviour-policy inference on a few rows (SquashedGaussianActor.sample /
// GaussianActor.sample, continuous_actors.py:270-306 / :74-123, on the env loop's one
// observation): one 1,024-thread workgroup per row normalises the observation, runs both
// hidden layers and the head with the vectors in LDS, and samples -- one launch where the
// batched path takes four (obs_norm, two GEMM launches, the head), each of them a few
// microseconds of launch and round trip for a single row.
// Dense layer: the 16 waves split K four ways for 256 output columns at a time (thread
// (q, j) sums k in quarter q of column j: each k reads 1 KB of W contiguously across the
// threads), and the quarters add in order; fp32 FMAs, within the parity tolerance of the
// batched MFMA path (a different summation order, not bit-identical to it).
__device__ __forceinline__ void act_dense(const float* in, int K, const float* W, int N, int act, float* out,
                                          float (&part)[4][ACT_ROWS_DIM]) {
    const int t = threadIdx.x, q = t >> 8, j0 = t & 255;
    const int kq = (K + 3) >> 2, k0 = q * kq, k1 = min(K, k0 + kq);
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, 0x7fffffffu);
    for (int j = j0; j < N; j += 256) {
        float s = 0.f;
        // 32 weights requested per round trip (one unconditional buffer load each, zero past
        // k1), then the FMAs in k order
        for (int kb = k0; kb < k1; kb += 32) {
            float w[32];
#pragma unroll
            for (int i = 0; i < 32; ++i) w[i] = bload(rW, boff(kb + i < k1, (kb + i) * N + j));
#pragma unroll
            for (int i = 0; i < 32; ++i) s = (kb + i < k1) ? fmaf(in[min(kb + i, K - 1)], w[i], s) : s;
        }
        part[q][j] = s;
    }
    __syncthreads();
    for (int j = t; j < N; j += 1024) {
        float v = part[0][j] + part[1][j];
        v = v + part[2][j];
        v = v + part[3][j];
        out[j] = act_f(v + W[(size_t)K * N + j], act);
    }
    __syncthreads();
}

// sampling tail on wave 0 (outs = mu [, raw logstd]); ls / u: this lane's logstd variable and
// noise (already loaded)
__device__ __forceinline__ void act_tail(const ActRowArgs& g, const float* outs, int row, int lane, float ls, float u) {
    const int A = g.A;
    const bool jok = lane < A;
    const float mu = jok ? outs[lane] : 0.f;
    const float lraw = jok ? (g.per_state_std ? outs[A + lane] : ls) : 0.f;
    if (g.mode == 2) {              // as actor_head_body's GaussianActor.sample
        float m = mu;
        if (g.output_norm) {
            const float s = wave_sum(jok ? fabsf(mu) : 0.f) / (float)A;
            m = mu / fmaxf(s, 1.f);
        }
        if (jok) {
            float l = g.per_state_std ? logf(softplus_f(lraw)) : lraw;
            l = fmaxf(l + g.logstd_init, logf(1e-3f));
            g.out[(size_t)row * A + lane] = m + expf(l) * u;
        }
        return;
    }
    if (jok) {                      // SquashedGaussianActor.sample: lim * tanh(mu + exp(clip(l)) u)
        const float l = fminf(fmaxf(lraw, -5.f), 2.f);
        const float x = mu + expf(l) * u;
        g.out[(size_t)row * A + lane] = g.lim * tanhf(x);
    }
}

// PF (S <= 128, H0, H1 <= 256, Aout <= 16): every operand of the row -- the observation and
// its normaliser, all the weights this thread multiplies (<= 32 of W0, <= 64 of W1, <= 4 of W3),
// the biases, logstd and the noise -- is requested before the first barrier, so the row costs
// one memory round trip instead of one per layer.  Same FMA order as the generic path.
struct ActShared {
    float xs[ACT_ROWS_DIM], h1s[ACT_ROWS_DIM], h2s[ACT_ROWS_DIM];
    float part[4][ACT_ROWS_DIM];
    float outs[64];
};
template <bool PF>
__device__ __forceinline__ void act_rows_body(const ActRowArgs& g_in, const int row, ActShared& L) {
    float(&xs)[ACT_ROWS_DIM] = L.xs;
    float(&h1s)[ACT_ROWS_DIM] = L.h1s;
    float(&h2s)[ACT_ROWS_DIM] = L.h2s;
    float(&part)[4][ACT_ROWS_DIM] = L.part;
    float(&outs)[64] = L.outs;
    ActRowArgs g = g_in;
    if (g_in.nseeds > 1) {          // packed seeds: seed z's weights, normaliser and noise; its rows
        const int64_t so = seed_off(g_in.sstride);
        g.s_mean = sr(g.s_mean, so); g.s_den = sr(g.s_den, so); g.W0 = sr(g.W0, so); g.W1 = sr(g.W1, so);
        g.W3 = sr(g.W3, so); g.logstd = sr(g.logstd, so); g.noise = sr(g.noise, so);
        g.obs = g.obs + (size_t)blockIdx.z * g.m * g.S;
        g.out = g.out + (size_t)blockIdx.z * g.m * g.A;
    }
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int S = g.S, A = g.A, Aout = g.Aout;
    const bool jok = wave == 0 && lane < A;
    if constexpr (PF) {
        const int H0 = g.H0, H1 = g.H1;
        const int q = t >> 8, j = t & 255;
        const int kq0 = (S + 3) >> 2, a0 = q * kq0, n0 = min(S, a0 + kq0) - a0;
        const int kq1 = (H0 + 3) >> 2, a1 = q * kq1, n1 = min(H0, a1 + kq1) - a1;
        const __amdgpu_buffer_rsrc_t rW0 = make_rsrc(g.W0, 0x7fffffffu), rW1 = make_rsrc(g.W1, 0x7fffffffu),
                                     rW3 = make_rsrc(g.W3, 0x7fffffffu);
        const float ob = bload(rs(g.obs), boff(t < S, row * S + t));
        const float om = bload(rs(g.s_mean), boff(t < S, t)), od = bload(rs(g.s_den), boff(t < S, t));
        float w0[32], w1[64], w3[4];
#pragma unroll
        for (int i = 0; i < 32; ++i) w0[i] = bload(rW0, boff(i < n0 && j < H0, (a0 + i) * H0 + j));
#pragma unroll
        for (int i = 0; i < 64; ++i) w1[i] = bload(rW1, boff(i < n1 && j < H1, (a1 + i) * H1 + j));
#pragma unroll
        for (int i = 0; i < 4; ++i) w3[i] = bload(rW3, boff(wave < Aout && lane + 64 * i < H1, (lane + 64 * i) * Aout + wave));
        const float b0 = bload(rW0, boff(t < H0, S * H0 + t)), b1 = bload(rW1, boff(t < H1, H0 * H1 + t));
        const float b3 = bload(rW3, boff(wave < Aout, H1 * Aout + wave));
        const float ls = bload(rs(g.logstd), boff(jok && !g.per_state_std, lane));
        const float u = bload(rs(g.noise), boff(jok, row * A + lane));
        if (t < S) xs[t] = (ob - om) / od;
        __syncthreads();
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 32; ++i) s = i < n0 ? fmaf(xs[min(a0 + i, S - 1)], w0[i], s) : s;
        part[q][j] = s;
        __syncthreads();
        if (t < H0) {
            float v = part[0][t] + part[1][t];
            v = v + part[2][t];
            v = v + part[3][t];
            h1s[t] = act_f(v + b0, g.act0);
        }
        __syncthreads();
        s = 0.f;
#pragma unroll
        for (int i = 0; i < 64; ++i) s = i < n1 ? fmaf(h1s[min(a1 + i, H0 - 1)], w1[i], s) : s;
        part[q][j] = s;
        __syncthreads();
        if (t < H1) {
            float v = part[0][t] + part[1][t];
            v = v + part[2][t];
            v = v + part[3][t];
            h2s[t] = act_f(v + b1, g.act1);
        }
        __syncthreads();
        if (wave < Aout) {
            s = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i) s = lane + 64 * i < H1 ? fmaf(h2s[min(lane + 64 * i, H1 - 1)], w3[i], s) : s;
            s = wave_sum(s);
            if (lane == 0) outs[wave] = s + b3;
        }
        __syncthreads();
        if (wave == 0) act_tail(g, outs, row, lane, ls, u);
        return;
    }
    for (int c = t; c < S; c += 1024) xs[c] = (g.obs[(size_t)row * S + c] - g.s_mean[c]) / g.s_den[c];
    __syncthreads();
    act_dense(xs, S, g.W0, g.H0, g.act0, h1s, part);
    act_dense(h1s, g.H0, g.W1, g.H1, g.act1, h2s, part);
    // head: output o on wave o mod 16, lanes over k, one wave sum
    const __amdgpu_buffer_rsrc_t rW3 = make_rsrc(g.W3, 0x7fffffffu);
    for (int o = wave; o < Aout; o += 16) {
        float w[ACT_ROWS_DIM / 64];
#pragma unroll
        for (int i = 0; i < ACT_ROWS_DIM / 64; ++i) w[i] = bload(rW3, boff(lane + 64 * i < g.H1, (lane + 64 * i) * Aout + o));
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < ACT_ROWS_DIM / 64; ++i)
            s = (lane + 64 * i < g.H1) ? fmaf(h2s[min(lane + 64 * i, g.H1 - 1)], w[i], s) : s;
        s = wave_sum(s);
        if (lane == 0) outs[o] = s + g.W3[(size_t)g.H1 * Aout + o];
    }
    __syncthreads();
    if (wave != 0) return;
    const float ls = jok && !g.per_state_std ? g.logstd[lane] : 0.f;
    const float u = (jok && g.noise != nullptr) ? g.noise[(size_t)row * A + lane] : 0.f;
    act_tail(g, outs, row, lane, ls, u);
}

// after a row's outputs: publish them to a polling host (ActRowArgs::done)
__device__ __forceinline__ void act_rows_done(uint32_t* done) {
    if (done == nullptr) return;
    __threadfence_system();            // every thread's output stores, before the count
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool PF>
__global__ __launch_bounds__(1024) void k_act_rows(ActRowArgs g) {
    __shared__ ActShared L;
    act_rows_body<PF>(g, blockIdx.x, L);
    act_rows_done(g.done);
}

// TrajectoryBuffer.add (buffers.py:41-71) as a device ring, by one workgroup so the control-block
// update is ordered after every row write (k_append; k_act_rng's append workgroup)
__device__ void append_body(const AppendArgs& a_in) {
    __shared__ int64_t cur_s, start_s;
    AppendArgs a = a_in;
    if (a_in.nseeds > 1) {          // packed seeds: seed z's ring and counters, its n source rows
        const int64_t so = seed_off(a_in.sstride), z = blockIdx.z;
        a.replay = sr(a.replay, so); a.ctl = sr(a.ctl, so);
        a.s = a.s + z * a.n * a.S; a.a = a.a + z * a.n * a.A; a.sp = a.sp + z * a.n * a.S;
        a.r = a.r + z * a.n; a.d = a.d + z * a.n;
    }
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
    act_rows_done(a.done);   // (uniform: every thread reaches it)
}

// The drop-in loop's deterministic act with the next update's sampler draw beside it: the
// action rows are workgroups 0 .. m - 1 and k_rng's draw is workgroup m, so the draw (one CU,
// ~13 us at HC shapes) runs while the rows run instead of after them.  One LDS image, either
// role's.  (A deterministic act reads no randoms: the two are independent.)  APP: the previous
// call's deferred 1-row append is workgroup m + 1 (the draw then takes the ring size from the
// host, r.size_fixed, instead of reading it beside the append)
union ActRngShared {
    RngShared r;
    ActShared a;
};
template <bool PF, bool APP>
__global__ __launch_bounds__(1024) void k_act_rng(ActRowArgs g, RngArgs r, AppendArgs app) {
    __shared__ ActRngShared U;
    const int m = (int)gridDim.x - 1 - (APP ? 1 : 0);
    if ((int)blockIdx.x < m) {
        act_rows_body<PF>(g, blockIdx.x, U.a);
        act_rows_done(g.done);
    } else if ((int)blockIdx.x == m) {
#ifndef SACX_DIAG_NODRAW
        rng_body(r, U.r);
#endif
    } else if constexpr (APP) {
        append_body(app);
    }
}


void launch_act_rows(const ActRowArgs& a, int m, hipStream_t s) {
    const bool pf = a.S <= 128 && a.H0 <= 256 && a.H1 <= 256 && a.Aout <= 16;
    const dim3 grid(m, 1, seeds_z(a.nseeds));
    if (pf) hipLaunchKernelGGL(k_act_rows<true>, grid, dim3(1024), 0, s, a);
    else hipLaunchKernelGGL(k_act_rows<false>, grid, dim3(1024), 0, s, a);
}

void launch_act_rng(const ActRowArgs& a, int m, const RngArgs& r, hipStream_t s, const AppendArgs* app, bool polar) {
    const bool pf = a.S <= 128 && a.H0 <= 256 && a.H1 <= 256 && a.Aout <= 16;
    const dim3 grid(m + 1 + (app ? 1 : 0), 1, seeds_z(a.nseeds));
    const AppendArgs none{};
    if (app) {
        if (pf) hipLaunchKernelGGL((k_act_rng<true, true>), grid, dim3(1024), 0, s, a, r, *app);
        else hipLaunchKernelGGL((k_act_rng<false, true>), grid, dim3(1024), 0, s, a, r, *app);
    } else {
        if (pf) hipLaunchKernelGGL((k_act_rng<true, false>), grid, dim3(1024), 0, s, a, r, none);
        else hipLaunchKernelGGL((k_act_rng<false, false>), grid, dim3(1024), 0, s, a, r, none);
    }
    if (polar && r.pairs != nullptr && r.n_norm > 0)   // the split sampler's polar transform, as launch_rng
        hipLaunchKernelGGL(k_polar, dim3(std::min((r.pcap + 255) / 256, SACX_POLAR_WGS), r.nupd, seeds_z(r.nseeds)),
                           dim3(256), 0, s, r);
}

// ==================================================================== k_qhead
template <int MODE, int NQ>
__device__ __forceinline__ void qhead_block(const QHeadArgs& q_in, int block, int64_t so, const FinalArgs* fin) {
    __shared__ float buf[4][512];
    QHeadArgs q = q_in;
    reloc(q, so);
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int row = block * 4 + wave;
    const int B = q.B, H1 = q.H1;
    if (row < B) {
        constexpr int nnet = (MODE == 0) ? 4 : 2;
        float alpha;
        if (MODE == 0 && fin != nullptr && fin->pre != nullptr) {
            // the split alpha finalisation (one seed: no relocation): the previous update's alpha step
            // from its partials and the snapshot its first alpha block took -- finalize_update's
            // arithmetic, so every row block computes the same alpha; block 0 stores the results
            const FinalArgs& f = *fin;
            const AfinPre* P = f.pre;
            const float* const xs[1] = {f.red};
            const int ns[1] = {f.nred};
            float p0[1];
            strided_sums<1>(xs, ns, p0);
            const float a_old = P->a_old, a_m = P->a_m, a_v = P->a_v;
            const int64_t t_sac = P->t_sac, seq = P->seq0, nts = P->nts, tsi = P->tsi;
            const float m_ent = wave_sum(p0[0]) / (float)f.B;   // reduce_mean(-nlp + H)
            const int64_t tnew = t_sac + 1;
            const float g = -m_ent;
            const float lr_t = adam_lr(f.adam, GRP_ALPHA, tnew);
            const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
            const float mm = a_m + (g - a_m) * (1.f - b1);
            const float vv = a_v + (g * g - a_v) * (1.f - b2);
            float an = a_old - (mm * lr_t) / (sqrtf(vv) + eps);
            an = fmaxf(an, 1e-5f);                  // SAC_expert.py:348
            alpha = an;
            if (block == 0 && wave == 0 && lane == 0) {
                *f.alpha_m = mm;
                *f.alpha_v = vv;
                *f.alpha = an;
                float* st = f.stats + (size_t)(seq % f.stats_cap) * 8;
                st[3] = -a_old * m_ent;
                st[4] = an;
                st[6] = -(m_ent - f.target_entropy);
                st[7] = (float)seq;
                Ctl* ctl = f.ctl;
                ctl->t_sac = tnew;
                ctl->num_timesteps = nts + tsi;
                ctl->step_seq = seq + 1;
            }
        } else {
            alpha = *q.alpha;
        }
        const float nlp_r = q.nlp[row];
        float r_r = 0.f, d_r = 0.f, rd = 1.f;
        if (MODE == 0) {
            r_r = q.r[row];
            d_r = q.d[row];
            rd = *q.ret_den;
        }
        float hv[4][NQ];
        float wv[4][NQ];
        float bias[4];
        const __amdgpu_buffer_rsrc_t rH = rs(q.H2);
#pragma unroll
        for (int k = 0; k < nnet; ++k) {
            load_row(rH, (k * B + row) * H1, H1, hv[k]);
            const __amdgpu_buffer_rsrc_t rW = rs(q.W3[k]);
            load_row(rW, 0, H1, wv[k]);
            bias[k] = bload(rW, (uint32_t)H1 * 4u);
        }
        float out[4];
#pragma unroll
        for (int k = 0; k < nnet; ++k) {
            float p = 0.f;
#pragma unroll
            for (int i = 0; i < NQ; ++i) p = fmaf(hv[k][i], wv[k][i], p);
            out[k] = wave_sum(p) + bias[k];
        }
        float g0, g1;
        if constexpr (MODE == 0) {
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
            if (lane == 0 && q.g != nullptr) {
                q.g[row] = g0;
                q.g[B + row] = g1;
            }
            if (q.D2 == nullptr) return;   // the dX launch applies g downstream (linearity)
        }
        // differentiated nets: slabs 2,3 (mode 0) or 0,1 (mode 1)
        constexpr int dn = MODE == 0 ? 2 : 0;
        float* d0 = q.D2 + (size_t)row * H1;
        float* d1 = q.D2 + ((size_t)B + row) * H1;
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            const int k = lane + 64 * i;
            if (k < H1) {
                d0[k] = (g0 * wv[dn][i]) * dact_f(hv[dn][i], q.act);
                d1[k] = (g1 * wv[dn + 1][i]) * dact_f(hv[dn + 1][i], q.act);
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
    const __amdgpu_buffer_rsrc_t rW = rs(k ? q.Wm3[1] : q.Wm3[0]);
    float hv[8];
    load_row(rs(q.Hm2), e * Hm, Hm, hv);
    float* ob = buf[wave];
    for (int j0 = 0; j0 < S; j0 += 8) {
        float s8[8];
        rowdot8(hv, rW, Hm, O, j0, S, s8);
        const float bj = bload(rW, boff(j0 + lane < S, Hm * O + j0 + lane));
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (lane == u && j0 + u < S) ob[j0 + u] = s8[u] + bj;
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
    // Dm2[e][i] = (sum_j ob[j] W[i][j]) * act'(h[i]); j in ascending order, 8 loads in flight
    float pacc[8];
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) pacc[qq] = 0.f;
    for (int j0 = 0; j0 < S; j0 += 8) {
        float w[8][8];
#pragma unroll
        for (int qq = 0; qq < 8; ++qq) {
            const int i = lane + 64 * qq;
#pragma unroll
            for (int u = 0; u < 8; ++u) w[qq][u] = bload(rW, boff(i < Hm && j0 + u < S, i * O + j0 + u));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float ou = ob[min(j0 + u, S - 1)];
#pragma unroll
            for (int qq = 0; qq < 8; ++qq) pacc[qq] = (j0 + u < S) ? fmaf(ou, w[qq][u], pacc[qq]) : pacc[qq];
        }
    }
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) {
        const int i = lane + 64 * qq;
        if (i < Hm) q.Dm2[(size_t)e * Hm + i] = pacc[qq] * dact_f(hv[qq], q.mact);
    }
}

template <int MODE, int NQ>
__global__ __launch_bounds__(256) void k_qhead(QHeadArgs q) { qhead_block<MODE, NQ>(q, blockIdx.x, seed_off(q.sstride)); }

void launch_qhead(const QHeadArgs& a, hipStream_t s) {
    const int rows = a.B + (a.mode == 0 ? a.ne : 0);
    const dim3 grid((rows + 3) / 4, 1, seeds_z(a.nseeds));
    if (a.H1 <= 256) {
        if (a.mode == 0) hipLaunchKernelGGL((k_qhead<0, 4>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((k_qhead<1, 4>), grid, dim3(256), 0, s, a);
    } else {
        if (a.mode == 0) hipLaunchKernelGGL((k_qhead<0, 8>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((k_qhead<1, 8>), grid, dim3(256), 0, s, a);
    }
}

// ==================================================================== k_actor_bwd
// one wave per actor row of the loss: action gradient through the Q (policy
// rows) or world-model (expert rows) input columns, tanh-Gaussian backward
// (SURVEY.md §8a A5), then the Dense(H1 -> Aout) backward with the activation
// derivative.  Per-column values live in lane j and are broadcast by shuffles.
template <int NQ, int NQD, bool PK, int OW>
__device__ __forceinline__ void actor_bwd_body(const ActorBwdArgs& b_in) {
    ActorBwdArgs b = b_in;
    // every argument in one batch of kernarg loads (else one dependent batch per branch)
    asm volatile("" ::"s"(b.B), "s"(b.ne), "s"(b.S), "s"(b.A), "s"(b.Aout), "s"(b.H0), "s"(b.H1), "s"(b.Hm0),
                 "s"(b.per_state_std), "s"(b.lim), "s"(b.Dp1), "s"(b.Wq1[0]), "s"(b.Wq1[1]), "s"(b.Dm1),
                 "s"(b.Wm1[0]), "s"(b.Wm1[1]), "s"(b.a_den), "s"(b.ma_den), "s"(b.alpha), "s"(b.ctl), "s"(b.use_expert),
                 "s"(b.c_t), "s"(b.c_std), "s"(b.c_u), "s"(b.c_mask), "s"(b.W3a), "s"(b.Ha2), "s"(b.act),
                 "s"(b.gpol));
    if constexpr (PK) reloc(b, seed_off(b_in.sstride));
    __shared__ float w3s[OW > 0 ? 256 * OW : 1];
    if constexpr (OW > 0) {
        // W3a (H1 x Aout) staged in LDS as in actor_head_body: its lane-strided reads below
        // would be 64 cache lines per load instruction
        static_assert(NQ == 4, "LDS-staged W3: H1 <= 256");
        const __amdgpu_buffer_rsrc_t rW0 = rs(b.W3a);
        const int n = b.H1 * b.Aout;
        float wv[OW];
#pragma unroll
        for (int c = 0; c < OW; ++c) wv[c] = bload(rW0, boff((int)threadIdx.x + 256 * c < n, threadIdx.x + 256 * c));
#pragma unroll
        for (int c = 0; c < OW; ++c)
            if ((int)threadIdx.x + 256 * c < n) w3s[threadIdx.x + 256 * c] = wv[c];
        __syncthreads();
    }
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    const int B = b.B, S = b.S, A = b.A;
    if (row >= B + b.ne) return;
    const bool pol = row < B;
    const bool jok = lane < A;
    const float eps = b.use_expert ? b.ctl->epsilon : 0.f;
    const float alpha = *b.alpha;
    const int ci = row * A + lane;
    const float t_pf = bload(rs(b.c_t), boff(jok, ci));
    const float sd_pf = bload(rs(b.c_std), boff(jok, ci));
    const float u_pf = bload(rs(b.c_u), boff(jok, ci));
    const float mk_pf = bload(rs(b.c_mask), boff(jok, ci));
    const float ad_pf = bload(rs(pol ? b.a_den : b.ma_den), boff(jok, lane));   // expert rows: the models' normaliser
    float h2v[NQ];
    load_row(rs(b.Ha2), row * b.H1, b.H1, h2v);
    // W3's first 8 output columns (all of them when Aout <= 8) load with the phase-1 operands,
    // not after the action-gradient reductions: one memory round trip less per row
    const __amdgpu_buffer_rsrc_t rW3 = rs(b.W3a);
    float w3n[NQ][8];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) {
        const int i = qq * 64 + lane;
#pragma unroll
        for (int u = 0; u < 8; ++u) w3n[qq][u] = OW > 0 ? 0.f : bload(rW3, boff(i < b.H1 && u < b.Aout, i * b.Aout + u));
    }
    const float w_sac = 1.f - eps;
    const float c = -w_sac * alpha * (1.f / (float)B);
    // action gradient: ga_j = sum over the input rows S+j of W1 of the row's layer-1 delta
    // (policy rows: both critics' deltas; expert rows: its world model's delta, no second term)
    const int e = row - B;
    const int km = e < b.ne / 2 ? 0 : 1;
    const int Hd = pol ? b.H0 : b.Hm0;
    float dv0[NQD], dv1[NQD];
    load_row(rs(pol ? b.Dp1 : b.Dm1), pol ? row * b.H0 : e * b.Hm0, Hd, dv0);
    load_row(rs(b.Dp1), (B + row) * b.H0, pol ? Hd : 0, dv1);
    // Dp1 is unscaled (linearity): policy rows scale by their q0 / q1 output gradients,
    // expert rows by 1 (the OOB read gives 0, plus 1)
    const __amdgpu_buffer_rsrc_t rg = rs(b.gpol);
    const float gs0 = bload(rg, boff(pol && b.gpol != nullptr, row)) + ((pol && b.gpol != nullptr) ? 0.f : 1.f);
    const float gs1 = bload(rg, boff(pol && b.gpol != nullptr, B + row)) + ((pol && b.gpol != nullptr) ? 0.f : 1.f);
    const __amdgpu_buffer_rsrc_t rWa = rs(pol ? b.Wq1[0] : (km ? b.Wm1[1] : b.Wm1[0]));
    const __amdgpu_buffer_rsrc_t rWb = rs(b.Wq1[1]);
    const int Hb = pol ? Hd : 0;
    float ga = 0.f;
    for (int j0 = 0; j0 < A; j0 += 8) {
        float w0[8][NQD], w1[8][NQD];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool uok = j0 + u < A;
            const int jr = S + j0 + u;
#pragma unroll
            for (int i = 0; i < NQD; ++i) {
                const int k = lane + 64 * i;
                w0[u][i] = bload(rWa, boff(uok && k < Hd, jr * Hd + k));
                w1[u][i] = bload(rWb, boff(uok && k < Hb, jr * Hd + k));
            }
        }
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            p[u] = 0.f;
#pragma unroll
            for (int i = 0; i < NQD; ++i) {
                p[u] = fmaf(gs0 * dv0[i], w0[u][i], p[u]);
                p[u] = fmaf(gs1 * dv1[i], w1[u][i], p[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float sj = wave_sum(p[u]);
            ga = (lane == j0 + u) ? sj : ga;
        }
    }
    ga = ga / ad_pf;
    float gx = 0.f, dl = 0.f;
    if (jok) {
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
    // Da2[row][i] = (sum_o Da3[row][o] W3a[i][o]) * act'(Ha2[row][i]); columns o live in lanes
    float pacc[NQ];
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) pacc[qq] = 0.f;
    if constexpr (OW > 0) {     // all OW columns (zeros past Aout, as the 8-chunks give)
#pragma unroll
        for (int u = 0; u < OW; ++u) {
            const float src = (u < A) ? __shfl(gx, min(u, 63), 64) : __shfl(dl, min(max(u - A, 0), 63), 64);
            const float d3 = (u < b.Aout) ? src : 0.f;
#pragma unroll
            for (int qq = 0; qq < NQ; ++qq) {
                const int i = qq * 64 + lane;
                const float w = (i < b.H1 && u < b.Aout) ? w3s[i * b.Aout + u] : 0.f;
                pacc[qq] = fmaf(d3, w, pacc[qq]);
            }
        }
    }
    for (int o0 = 0; OW == 0 && o0 < b.Aout; o0 += 8) {
        float w[NQ][8];
        if (o0 == 0) {
#pragma unroll
            for (int qq = 0; qq < NQ; ++qq)
#pragma unroll
                for (int u = 0; u < 8; ++u) w[qq][u] = w3n[qq][u];
        } else {
#pragma unroll
            for (int qq = 0; qq < NQ; ++qq) {
                const int i = qq * 64 + lane;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    w[qq][u] = bload(rW3, boff(i < b.H1 && o0 + u < b.Aout, i * b.Aout + o0 + u));
            }
        }
        float d3[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int o = o0 + u;
            const float src = (o < A) ? __shfl(gx, min(o, 63), 64) : __shfl(dl, min(max(o - A, 0), 63), 64);
            d3[u] = (o < b.Aout) ? src : 0.f;
        }
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq)
#pragma unroll
            for (int u = 0; u < 8; ++u) pacc[qq] = fmaf(d3[u], w[qq][u], pacc[qq]);
    }
#pragma unroll
    for (int qq = 0; qq < NQ; ++qq) {
        const int i = qq * 64 + lane;
        if (i < b.H1) b.Da2[(size_t)row * b.H1 + i] = pacc[qq] * dact_f(h2v[qq], b.act);
    }
}

template <int NQ, int NQD, bool PK, int OW = 0>
__global__ __launch_bounds__(256) void k_actor_bwd(ActorBwdArgs b) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    actor_bwd_body<NQ, NQD, PK, OW>(b);
    ktime_stamp(b.ktime, t0);
}

void launch_actor_bwd(const ActorBwdArgs& a, hipStream_t s) {
    const int rows = a.B + a.ne;
    const dim3 grid((rows + 3) / 4, 1, seeds_z(a.nseeds));
    const int hd = std::max(a.H0, a.use_expert ? a.Hm0 : 0);
    const bool q8 = a.H1 > 256, d8 = hd > 256;
#define SACX_AB(Q, D, ...)                                                                                  \
    do {                                                                                                    \
        if (a.nseeds > 1) hipLaunchKernelGGL((k_actor_bwd<Q, D, true, ##__VA_ARGS__>), grid, dim3(256), 0, s, a); \
        else hipLaunchKernelGGL((k_actor_bwd<Q, D, false, ##__VA_ARGS__>), grid, dim3(256), 0, s, a);            \
    } while (0)
    if (q8) {
        if (d8) SACX_AB(8, 8);
        else SACX_AB(8, 4);
    } else if (a.Aout > 8 && a.Aout <= 24) {   // W3a staged in LDS (see actor_bwd_body)
        if (d8) SACX_AB(4, 8, 24);
        else SACX_AB(4, 4, 24);
    } else {
        if (d8) SACX_AB(4, 8);
        else SACX_AB(4, 4);
    }
#undef SACX_AB
}

// ==================================================================== k_append
// TrajectoryBuffer.add (buffers.py:41-71) as a device ring (append_body, above)
__global__ __launch_bounds__(256) void k_append(AppendArgs a_in) { append_body(a_in); }

void launch_append(const AppendArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_append, dim3(1, 1, seeds_z(a.nseeds)), dim3(256), 0, s, a);
}

}  // namespace sacx

namespace sacx {
// per-call control values as kernel arguments (graph/stream ordered, no host buffer lifetime issues)
// busy-waits ~us microseconds (100 MHz realtime counter): lets the host queue a whole
// step of launches + events behind it, so the event deltas are device back-to-back time
__global__ void k_spin(int64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
}

void launch_spin(double us, hipStream_t s) {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(1), 0, s, (int64_t)(us * 100.0));
}

// BaseActor._transform_state (base_actor.py:35-39): X[i][c] = (obs[i][c] - mean[c]) / den[c], 0 in the pad
__global__ __launch_bounds__(256) void k_obs_norm(const float* obs, int64_t n, int S, const float* mean,
                                                  const float* den, float* X, int ldX) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * ldX) return;
    const int64_t i = t / ldX;
    const int c = (int)(t - i * ldX);
    X[t] = c < S ? (obs[i * S + c] - mean[c]) / den[c] : 0.f;
}

void launch_obs_norm(const float* obs, int64_t n, int S, const float* mean, const float* den, float* X, int ldX,
                     hipStream_t s) {
    const int64_t tot = n * ldX;
    hipLaunchKernelGGL(k_obs_norm, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, obs, n, S, mean, den, X, ldX);
}

// ==================================================================== k_diag
// Expert diagnostics.  mode 0: one wave per row normalises s_e into the actor
// input and the state columns of the model input, and (a_e != null) a_e into its action
// columns.  modes 1-3: one workgroup of 1024 threads, n <= 2048 rows.
#define DIAG_THREADS 1024
#define DIAG_MAXN 2048

__device__ __forceinline__ float diag_pred(const DiagArgs& g, int k, int i, int j) {
    float dn = g.O[((int64_t)k * g.n + i) * (g.S + 1) + j];
    if (g.clip_d > 0.f) dn = fminf(fmaxf(dn, -g.clip_d), g.clip_d);
    if (g.mnoise != nullptr)        // GaussianModel.sample(deterministic=False) (continuous_models.py:60-62)
        dn = dn + expf(g.mlogstd[k][j]) * g.mnoise[((int64_t)k * g.n + i) * g.S + j];
    return g.s_e[(int64_t)i * g.S + j] + (dn * g.d_den[j] + g.d_mean[j]);   // MSEModel.sample
}

__device__ float block_sum_1024(float v, float* sh) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    float t = 0.f;
    if (threadIdx.x < 64) t = wave_sum(threadIdx.x < DIAG_THREADS / 64 ? sh[threadIdx.x] : 0.f);
    if (threadIdx.x == 0) sh[0] = t;
    __syncthreads();
    return sh[0];
}

__global__ __launch_bounds__(256) void k_diag_prep(DiagArgs g) {
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= g.n) return;
    for (int j = lane; j < g.S; j += 64) {
        const float x = g.s_e[(int64_t)i * g.S + j];
        g.X[(int64_t)i * g.ldS + j] = (x - g.s_mean[j]) / g.s_den[j];
        g.Xm[(int64_t)i * g.ldQ + j] = (x - g.ms_mean[j]) / g.ms_den[j];
    }
    if (g.a_e)
        for (int j = lane; j < g.A; j += 64)
            g.Xm[(int64_t)i * g.ldQ + g.S + j] = (g.a_e[(int64_t)i * g.A + j] - g.a_mean[j]) / g.a_den[j];
}

__global__ __launch_bounds__(DIAG_THREADS) void k_diag(DiagArgs g) {
    __shared__ float sh[DIAG_MAXN];
    __shared__ float red[DIAG_THREADS / 64];
    const int n = g.n, S = g.S;
    if (g.mode == 1 || g.mode == 2) {
        // per model: mean_i 0.5 sum_j (sp_pred - sp_e)^2; then np.mean over the models' f32 values
        // (sequential below 8 values, numpy's 8-way pairwise block at 8)
        const int nmod = g.nmod;
        float m[MAX_MODELS];
        for (int k = 0; k < nmod; ++k) {
            float acc = 0.f;
            for (int i = threadIdx.x; i < n; i += DIAG_THREADS) {
                float se = 0.f;
                for (int j = 0; j < S; ++j) {
                    const float d = diag_pred(g, k, i, j) - g.sp_e[(int64_t)i * S + j];
                    se += d * d;
                }
                acc += 0.5f * se;
            }
            const float mk = block_sum_1024(acc, red) / (float)n;
            if (threadIdx.x == 0) m[k] = mk;
        }
        if (threadIdx.x == 0) {
            float sum;
            if (nmod >= 8) {
                sum = ((m[0] + m[1]) + (m[2] + m[3])) + ((m[4] + m[5]) + (m[6] + m[7]));
            } else {
                sum = m[0];
                for (int k = 1; k < nmod; ++k) sum += m[k];
            }
            const int o = g.mode == 1 ? 0 : 1;
            g.out[o] = sum / (float)nmod;
            for (int k = 0; k < nmod; ++k) g.out[2 + nmod * (g.mode - 1) + k] = m[k];
        }
        return;
    }
    // mode 3: s_disc_i = || sp_pred0 - sp_pred1 ||_2; total, max, median, ratio
    float acc = 0.f;
    for (int i = threadIdx.x; i < DIAG_MAXN; i += DIAG_THREADS) {
        float v = __builtin_inff();
        if (i < n) {
            float q = 0.f;
            for (int j = 0; j < S; ++j) {
                const float d = diag_pred(g, 0, i, j) - diag_pred(g, 1, i, j);
                q += d * d;
            }
            v = sqrtf(q);
            acc += v;
        }
        sh[i] = v;
    }
    const float total = block_sum_1024(acc, red);
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int kk = 2; kk <= n2; kk <<= 1)           // bitonic sort of sh[0, n2) ascending
        for (int jj = kk >> 1; jj > 0; jj >>= 1) {
            __syncthreads();
            for (int i = threadIdx.x; i < n2; i += DIAG_THREADS) {
                const int l = i ^ jj;
                if (l > i) {
                    const float a = sh[i], b = sh[l];
                    const bool up = (i & kk) == 0;
                    if ((a > b) == up) { sh[i] = b; sh[l] = a; }
                }
            }
        }
    __syncthreads();
    if (threadIdx.x == 0) {
        g.out[0] = total;
        g.out[1] = sh[n - 1];
        g.out[2] = (n & 1) ? sh[n / 2] : (sh[n / 2 - 1] + sh[n / 2]) * 0.5f;
    }
    for (int i = threadIdx.x; i < n; i += DIAG_THREADS) {
        float q = 0.f;
        for (int j = 0; j < S; ++j) {
            const float d = diag_pred(g, 0, i, j) - diag_pred(g, 1, i, j);
            q += d * d;
        }
        g.out[3 + i] = sqrtf(q) / total;
    }
}

void launch_diag(const DiagArgs& a, hipStream_t s) {
    if (a.mode == 0) hipLaunchKernelGGL(k_diag_prep, dim3((a.n + 3) / 4), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_diag, dim3(1), dim3(DIAG_THREADS), 0, s, a);
}

// ==================================================================== data-parallel Adam
// k_adam_apply: element i of a parameter range, gradient = all-reduced sum * (1 / ranks);
// the arithmetic of the fused GM_DW epilogue, so one rank reproduces it bit for bit.
__global__ __launch_bounds__(256) void k_adam_apply(AdamApplyArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const Ctl* ctl = a.ctl;
    const int64_t tstep = (a.group == GRP_MODEL ? ctl->t_model : ctl->t_sac) + 1 - a.t_adv;
    const float lr_t = adam_lr(a.adam, a.group, tstep);
    float* P = a.P + i;
    float gr = P[3 * a.p_stride] * a.grad_scale;
    if (a.scale_dev != nullptr) gr = gr * a.scale_dev[0];
    const float e0 = P[0], e1 = P[a.p_stride], e2 = P[2 * a.p_stride];
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-7f;
    const float mm1 = e1 + (gr - e1) * (1.f - b1);
    const float vv1 = e2 + (gr * gr - e2) * (1.f - b2);
    const float pn = e0 - (mm1 * lr_t) / (sqrtf(vv1) + eps);
    P[0] = pn;
    P[a.p_stride] = mm1;
    P[2 * a.p_stride] = vv1;
    if (a.t_off != 0) {
        const int64_t tui = a.adam.target_update_int > 0 ? a.adam.target_update_int : 1;
        if (ctl->num_timesteps % tui == 0) P[a.t_off] = P[a.t_off] * a.adam.tau_keep + pn * a.adam.tau_take;
    }
}

void launch_adam_apply(const AdamApplyArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_adam_apply, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
}

// sacx_dp_local_step's reduce: the ranks' gradient ranges summed in rank order, the sum written
// back to every rank (ncclAllReduce(sum)'s result; with two ranks a + b, exactly RCCL's)
__global__ __launch_bounds__(256) void k_dp_sum(DpSumArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    float v = a.buf[0][i];
    for (int r = 1; r < a.nranks; ++r) v = v + a.buf[r][i];
    for (int r = 0; r < a.nranks; ++r) a.buf[r][i] = v;
}

void launch_dp_sum(const DpSumArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_dp_sum, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
}

// the alpha half of finalize_update that follows the all-reduce of the alpha gradient
__global__ void k_alpha_apply(FinalArgs f) {
    if (threadIdx.x != 0) return;
    Ctl* ctl = f.ctl;
    const int64_t tnew = ctl->t_sac + 1;
    const float lr_t = adam_lr(f.adam, GRP_ALPHA, tnew);
    float an = adam_update(f.alpha, f.alpha_m, f.alpha_v, *f.alpha_g * f.grad_scale, lr_t);
    an = fmaxf(an, 1e-5f);                      // SAC_expert.py:348
    *f.alpha = an;
    const int64_t seq = ctl->step_seq;
    f.stats[(size_t)(seq % f.stats_cap) * 8 + 4] = an;
    ctl->t_sac = tnew;
    ctl->num_timesteps += ctl->ts_increment;
    ctl->step_seq = seq + 1;
}

void launch_alpha_apply(const FinalArgs& f, hipStream_t s) {
    hipLaunchKernelGGL(k_alpha_apply, dim3(1), dim3(64), 0, s, f);
}

// ==================================================================== k_roll
// one wave per trajectory row.  mode 0 (prep): s_t (s_init at t = 0, copied to s_out) is
// normalised into the actor input and the state columns of the model input
// (BaseActor._transform_state, BaseWorldModel._forward: same s_rms).  mode 1 (finish):
// MSEModel.step -- s_{t+1} = s_t + denorm_delta(clip(delta_n)), r = denorm_r(clip(r_n)),
// d = False (tf.ones_like(r) == 0) -- and the stores of samplers.py:98-116.
__global__ __launch_bounds__(256) void k_roll(RollArgs g) {
    const int wave = wave_id(), lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wave;
    if (i >= g.n) return;
    const int S = g.S, A = g.A;
    const int64_t o = (int64_t)i * g.H + g.t;
    if (g.mode == 0) {
        const float* src = (g.t == 0 && g.s_init) ? g.s_init + (int64_t)i * S : g.s_out + o * S;
        for (int j = lane; j < S; j += 64) {
            const float v = src[j];
            if (g.t == 0 && g.s_init) g.s_out[o * S + j] = v;
            g.X[(int64_t)i * g.ldS + j] = (v - g.s_mean[j]) / g.s_den[j];
            g.Xm[(int64_t)i * g.ldQ + j] = (v - g.ms_mean[j]) / g.ms_den[j];
        }
        return;
    }
    const float* Oi = g.O + (int64_t)i * (S + 1);
    for (int j = lane; j < S; j += 64) {
        float dn = Oi[j];
        if (g.clip_d > 0.f) dn = fminf(fmaxf(dn, -g.clip_d), g.clip_d);
        if (g.mnoise != nullptr)    // GaussianModel.step (continuous_models.py:38-41)
            dn = dn + expf(g.mlogstd[j]) * g.mnoise[(int64_t)i * S + j];
        const float sp = g.s_out[o * S + j] + (dn * g.d_den[j] + g.d_mean[j]);
        g.sp_out[o * S + j] = sp;
        if (g.t + 1 < g.H) g.s_out[(o + 1) * S + j] = sp;
    }
    for (int j = lane; j < A; j += 64) g.a_out[o * A + j] = g.a_raw[(int64_t)i * A + j];
    if (lane == 0) {
        float rn = Oi[S];
        if (g.clip_r > 0.f) rn = fminf(fmaxf(rn, -g.clip_r), g.clip_r);
        g.r_out[o] = rn * g.r_norm[1] + g.r_norm[0];
        g.d_out[o] = 0;
    }
}

void launch_roll(const RollArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_roll, dim3((a.n + 3) / 4), dim3(256), 0, s, a);
}

// ==================================================================== k_net_io
// The reference objects' standalone network calls around the GEMM launches:
//   mode 0: [s_rms.normalize(s) | a_rms.normalize(a) | 0] -> X (QCritic._forward,
//           critics.py:89-94; BaseWorldModel._forward, base_world_model.py:67-70; the actor's
//           _transform_state with a == null), one thread per element;
//   mode 1: QCritic._forward -> [n, 1], value -> squeeze * max(ret_std, 1e-8)
//           (critics.py:96-103), one thread per row;
//   mode 2: BaseWorldModel._forward's clips + MSEModel.sample / step
//           (continuous_models.py:225-254): sp = s + delta_rms.denormalize(delta_n),
//           r = r_rms.denormalize(r_n); one wave per row;
//   mode 3: MSEModel.get_loss (continuous_models.py:280-302) over a chunk of rows, one
//           workgroup; the chunk sums chain through out0 in stream order, the last chunk
//           writes reduce_mean to out1.
__global__ __launch_bounds__(256) void k_net_io_elem(NetIOArgs g) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g.mode == 0) {
        if (t >= (int64_t)g.n * g.ldX) return;
        const int64_t i = t / g.ldX;
        const int c = (int)(t - i * g.ldX);
        float x = 0.f;
        if (c < g.S) x = (g.s[i * g.S + c] - g.s_mean[c]) / g.s_den[c];
        else if (g.a != nullptr && c < g.S + g.A) x = (g.a[i * g.A + (c - g.S)] - g.a_mean[c - g.S]) / g.a_den[c - g.S];
        g.X[t] = x;
        return;
    }
    if (t >= g.n) return;                   // mode 1
    const float q = g.O[t * g.ldO];
    g.out0[t] = g.value ? q * g.ret_den[0] : q;
}

__global__ __launch_bounds__(256) void k_net_io_rows(NetIOArgs g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int S = g.S, O = S + 1;
    if (g.mode == 2) {
        const int64_t i = (int64_t)blockIdx.x * 4 + wave;
        if (i >= g.n) return;
        const float* Oi = g.O + i * g.ldO;
        for (int j = lane; j <= S; j += 64) {
            float v = Oi[j];
            const float cl = j < S ? g.clip_d : g.clip_r;
            if (cl > 0.f) v = fminf(fmaxf(v, -cl), cl);
            if (g.out0 != nullptr) g.out0[i * O + j] = v;
            if (j < S) {
                if (g.mnoise != nullptr)    // GaussianModel.sample(deterministic=False) / step (:36-70)
                    v = v + expf(g.mlogstd[j]) * g.mnoise[i * S + j];
                if (g.out1 != nullptr) g.out1[i * S + j] = g.s[i * S + j] + (v * g.d_den[j] + g.d_mean[j]);
            } else if (g.out2 != nullptr) {
                g.out2[i] = v * g.r_norm[1] + g.r_norm[0];
            }
        }
        return;
    }
    // mode 3: 0.5 ||clip(norm(sp - s)) - delta_pred||^2 + coef * 0.5 (clip(norm(r)) - r_pred)^2
    // (GaussianModel: ds * 0.5 sum_j (((dn - pred) / e^l)^2 + 2 l + log 2 pi), continuous_models.py:111-129)
    __shared__ float part[4];
    float ds = 1.f;
    if (g.mlogstd != nullptr && g.lscale) {      // stop_gradient(reduce_mean(square(exp(logstd))))
        float q2 = 0.f;
        for (int j = lane; j < S; j += 64) {
            const float e = expf(g.mlogstd[j]);
            q2 += e * e;
        }
        ds = wave_sum(q2) / (float)S;
    }
    float acc = 0.f;
    for (int64_t i = wave; i < g.n; i += 4) {
        const float* Oi = g.O + i * g.ldO;
        float sq = 0.f;
        for (int j = lane; j < S; j += 64) {
            float dn = ((g.sp[i * S + j] - g.s[i * S + j]) - g.d_mean[j]) / g.d_den[j];
            if (g.clip_d > 0.f) dn = fminf(fmaxf(dn, -g.clip_d), g.clip_d);
            const float e = dn - Oi[j];
            if (g.mlogstd != nullptr) {
                const float l = g.mlogstd[j], q = e / expf(l);
                sq = sq + ((q * q + 2.f * l) + LOG2PI_F);
            } else {
                sq = sq + e * e;
            }
        }
        const float tot = g.mlogstd != nullptr ? ds * wave_sum(sq) : wave_sum(sq);
        float rn = (g.r[i] - g.r_norm[0]) / g.r_norm[1];
        if (g.clip_r > 0.f) rn = fminf(fmaxf(rn, -g.clip_r), g.clip_r);
        const float er = rn - Oi[S];
        acc = acc + (0.5f * tot + g.reward_coef * (0.5f * (er * er)));
    }
    if (lane == 0) part[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float sum = (part[0] + part[1]) + (part[2] + part[3]);
        const float run = g.first ? sum : g.out0[0] + sum;
        g.out0[0] = run;
        if (g.last) g.out1[0] = run / (float)g.n_total;
    }
}

void launch_net_io(const NetIOArgs& a, hipStream_t s) {
    if (a.mode == 0) {
        const int64_t tot = (int64_t)a.n * a.ldX;
        hipLaunchKernelGGL(k_net_io_elem, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, a);
    } else if (a.mode == 1) {
        hipLaunchKernelGGL(k_net_io_elem, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
    } else if (a.mode == 2) {
        hipLaunchKernelGGL(k_net_io_rows, dim3((unsigned)((a.n + 3) / 4)), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_net_io_rows, dim3(1), dim3(256), 0, s, a);
    }
}

// k_wbf_refresh: thread (n, 8 shadow positions) of matrix blockIdx.y; the 8 positions are one lane
// group's operand values of a slab pair (k = s0 + 4 grp + j, then s1 + 4 grp + j), read down
// column n of W (coalesced across the threads' n) and stored as one 16-B row piece; positions
// past K or of an unpaired slab get zeros
__global__ __launch_bounds__(256) void k_wbf_refresh(WbfArgs a) {
    const int mi = blockIdx.y;
    if (mi >= a.nmat) return;
    const int64_t so = a.nseeds > 1 ? (int64_t)blockIdx.z * a.sstride : 0;
    const float* W = sr(a.W[mi], so);
    uint16_t* S = sr(a.S[mi], so);
    const int K = a.K[mi], N = a.N[mi], per = wbf_per_of(K), ld = wbf_ld_of(K), ppw = (per + 1) >> 1;
    const int nIt = (K + 15) >> 4;
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int n = (int)(idx % N);
    const int64_t q = idx / N;                 // 8-position group of row n
    if (q >= ld / 8) return;
    const int pair = (int)(q >> 2), grp = (int)(q & 3);
    const int w = pair / ppw, i0 = (pair - w * ppw) * 2;
    uint16_t v[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int i = i0 + h, sl = w * per + i;
        const bool sok = i < per && sl < nIt;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = sl * 16 + grp * 4 + j;
            const float x = (sok && k < K) ? W[(size_t)k * N + n] : 0.f;
            v[h * 4 + j] = __builtin_bit_cast(uint16_t, (__bf16)x);
        }
    }
    uint4 o;
    o.x = v[0] | ((uint32_t)v[1] << 16); o.y = v[2] | ((uint32_t)v[3] << 16);
    o.z = v[4] | ((uint32_t)v[5] << 16); o.w = v[6] | ((uint32_t)v[7] << 16);
    *reinterpret_cast<uint4*>(S + (size_t)n * ld + q * 8) = o;
}

void launch_wbf_refresh(const WbfArgs& a, hipStream_t s) {
    int64_t most = 0;
    for (int i = 0; i < a.nmat; ++i) most = std::max<int64_t>(most, (int64_t)a.N[i] * (wbf_ld_of(a.K[i]) / 8));
    const dim3 grid((unsigned)((most + 255) / 256), (unsigned)a.nmat, (unsigned)seeds_z(a.nseeds));
    hipLaunchKernelGGL(k_wbf_refresh, grid, dim3(256), 0, s, a);
}

__global__ void k_set_pseq(Ctl* ctl, int slot, int64_t sstride) {
    ctl = sr(ctl, seed_off(sstride));
    ctl->pseq[slot] = ctl->step_seq;
}

void launch_set_pseq(Ctl* ctl, int slot, int64_t sstride, int nseeds, hipStream_t s) {
    hipLaunchKernelGGL(k_set_pseq, dim3(1, 1, seeds_z(nseeds)), dim3(1), 0, s, ctl, slot, sstride);
}

__global__ void k_set_ctl(Ctl* ctl, int64_t num_timesteps, int64_t ts_increment, int64_t sstride) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        ctl = sr(ctl, seed_off(sstride));
        ctl->num_timesteps = num_timesteps;
        ctl->ts_increment = ts_increment;
    }
}
void launch_set_ctl(Ctl* ctl, int64_t num_timesteps, int64_t ts_increment, int64_t sstride, int nseeds,
                    hipStream_t s) {
    hipLaunchKernelGGL(k_set_ctl, dim3(1, 1, seeds_z(nseeds)), dim3(64), 0, s, ctl, num_timesteps, ts_increment,
                       sstride);
}
}  // namespace sacx

namespace sacx {
// ==================================================================== world-model fitting
// MSEModel.get_loss (continuous_models.py:280-302) summed over the two models
// and one Keras Adam over all their variables (mbrl_onpolicy_alg.py:301-319).
__global__ __launch_bounds__(256) void k_mgather(MGatherArgs g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    const int R2 = g.nm * g.mb;
    if (row >= R2) return;
    const int S = g.S, A = g.A;
    // one step (grid y = 1), or step j = blockIdx.y of a pre-gathered block into staging slot j
    const int j = (int)blockIdx.y;
    float* X = g.X + (size_t)j * R2 * g.ldQ;
    float* T = g.T + (size_t)j * R2 * (S + 1);
    const int64_t slot = (g.ctl->mfit_seq + j) % g.idx_cap;
    const int64_t li = g.idx_ring[slot * R2 + row];
    const int64_t phys = (g.ctl->start + li) % g.cap;
    const float* rec = g.replay + phys * (int64_t)g.stride;
    for (int c = lane; c < g.ldQ; c += 64) {
        float x = 0.f;
        if (c < S) x = (rec[c] - g.s_mean[c]) / g.s_den[c];
        else if (c < S + A) x = (rec[c] - g.a_mean[c - S]) / g.a_den[c - S];
        X[(size_t)row * g.ldQ + c] = x;
    }
    for (int c = lane; c <= S; c += 64) {
        float y;
        if (c < S) y = ((rec[S + A + c] - rec[c]) - g.d_mean[c]) / g.d_den[c];
        else y = (rec[2 * S + A] - g.r_norm[0]) / g.r_norm[1];
        const float cl = c < S ? g.clip_d : g.clip_r;
        if (cl > 0.f) y = fminf(fmaxf(y, -cl), cl);
        T[(size_t)row * (S + 1) + c] = y;
    }
}

__global__ __launch_bounds__(256) void k_mloss(MLossArgs g) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= g.nm * g.mb) return;
    const int S = g.S, O = S + 1;
    const float inv = 1.f / (float)g.mb;
    float sq = 0.f, er = 0.f;
    for (int c = lane; c <= S; c += 64) {
        const float e = g.T[(size_t)row * O + c] - g.O[(size_t)row * O + c];
        if (c < S) {
            sq = sq + e * e;
            g.D3[(size_t)row * g.ldD + c] = -e * inv;
        } else {
            er = e;
            g.D3[(size_t)row * g.ldD + c] = -e * (g.reward_coef * inv);
        }
    }
    const float tot = wave_sum(sq);
    const float e_r = wave_sum(er);
    if (lane == 0) g.loss_rows[row] = 0.5f * tot + g.reward_coef * (0.5f * (e_r * e_r));
}

__global__ __launch_bounds__(64) void k_mfinal(MFinalArgs f) { mfit_final(f); }

void launch_mgather(const MGatherArgs& a, hipStream_t s, int nsteps) {
    hipLaunchKernelGGL(k_mgather, dim3((a.nm * a.mb + 3) / 4, std::max(1, nsteps)), dim3(256), 0, s, a);
}
void launch_mloss(const MLossArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_mloss, dim3((a.nm * a.mb + 3) / 4), dim3(256), 0, s, a);
}

// clip_by_global_norm of the model gradients (see GNormArgs): per-chunk sums of squares in a
// fixed order, then the norm and scale in one wave
__global__ __launch_bounds__(256) void k_gnorm_part(GNormArgs a) {
    __shared__ float red[4];
    const int64_t chunk = (a.n + GNORM_PARTS - 1) / GNORM_PARTS;
    const int64_t b0 = (int64_t)blockIdx.x * chunk, b1 = min(a.n, b0 + chunk);
    float acc = 0.f;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += 256) acc = acc + a.g[i] * a.g[i];
    const float w = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) a.part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(64) void k_gnorm_final(GNormArgs a) {
    float acc = 0.f;
    for (int i = threadIdx.x; i < GNORM_PARTS; i += 64) acc = acc + a.part[i];
    const float tot = wave_sum(acc);
    if (threadIdx.x == 0) {
        const float norm = sqrtf(tot);
        a.scale_out[0] = a.clip * fminf(1.f / norm, 1.f / a.clip) + (norm - norm);
    }
}

// ==================================================================== k_ln (actor layer norm)
template <int NQ>
__global__ __launch_bounds__(256) void k_ln(LNArgs a) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t so = seed_off(a.sstride);
    const int H = a.H;
    const float inv_h = 1.f / (float)H;
    int row = blockIdx.x * 4 + wave;
    const float* gamma = sr(a.gamma, so);
    if (a.mode == 0) {
        // rows [r0, r1) then [r2, r3), as one index space
        const int n0 = a.r[1] - a.r[0];
        if (row >= n0 + (a.nrange > 1 ? a.r[3] - a.r[2] : 0)) return;
        row = row < n0 ? a.r[0] + row : a.r[2] + (row - n0);
        float* z = sr(a.Z, so) + (size_t)row * H;
        float v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) v[q] = (lane + 64 * q < H) ? z[lane + 64 * q] : 0.f;
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q) s += v[q];
        const float mu = wave_sum(s) * inv_h;
        float ss = 0.f;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const float d = (lane + 64 * q < H) ? v[q] - mu : 0.f;
            ss += d * d;
        }
        const float var = wave_sum(ss) * inv_h;
        const float rstd = 1.f / sqrtf(var + 1e-3f);     // Keras LayerNormalization epsilon
        const bool cache = row < a.cache_rows && a.xhat != nullptr;
        float* xh = cache ? sr(a.xhat, so) + (size_t)row * H : nullptr;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int j = lane + 64 * q;
            if (j < H) {
                const float x = (v[q] - mu) * rstd;
                if (cache) xh[j] = x;
                z[j] = tanhf(gamma[j] * x + gamma[H + j]);
            }
        }
        if (cache && lane == 0) sr(a.rstd, so)[row] = rstd;
        return;
    }
    // mode 1: dY -> dZ = rstd (g - mean(g) - xhat mean(g xhat)), g = dY gamma
    if (row >= a.r[1]) return;
    float* d = sr(a.Z, so) + (size_t)row * H;
    const float* xh = sr(a.xhat, so) + (size_t)(row + a.xrow0) * H;
    const float rstd = sr(a.rstd, so)[row + a.xrow0];
    float dy[NQ], x[NQ];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int j = lane + 64 * q;
        dy[q] = j < H ? d[j] : 0.f;
        x[q] = j < H ? xh[j] : 0.f;
        const float g = j < H ? dy[q] * gamma[j] : 0.f;
        s1 += g;
        s2 += g * x[q];
    }
    const float m1 = wave_sum(s1) * inv_h, m2 = wave_sum(s2) * inv_h;
    float* gy = sr(a.gy, so) + (size_t)row * H;
    float* gb = sr(a.gb, so) + (size_t)row * H;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int j = lane + 64 * q;
        if (j < H) {
            d[j] = rstd * ((dy[q] * gamma[j] - m1) - x[q] * m2);
            gy[j] = dy[q] * x[q];
            gb[j] = dy[q];
        }
    }
}

void launch_ln(const LNArgs& a, hipStream_t s) {
    const int rows = a.mode == 0 ? (a.r[1] - a.r[0]) + (a.nrange > 1 ? a.r[3] - a.r[2] : 0) : a.r[1];
    const dim3 grid((rows + 3) / 4, 1, seeds_z(a.nseeds));
    if (a.H <= 256) hipLaunchKernelGGL(k_ln<4>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_ln<8>, grid, dim3(256), 0, s, a);
}

void launch_gnorm(const GNormArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_gnorm_part, dim3(GNORM_PARTS), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_gnorm_final, dim3(1), dim3(64), 0, s, a);
}
void launch_mfinal(const MFinalArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_mfinal, dim3(1), dim3(64), 0, s, a);
}
}  // namespace sacx
