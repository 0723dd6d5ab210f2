// Internal structures shared by the host plan builder (sacx.cpp) and the
// gfx950 kernels (k_*.hip).  Not part of the public ABI.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace sacx {

enum Act { ACT_RELU = 0, ACT_TANH = 1, ACT_ELU = 2, ACT_NONE = 3 };

// Device control block (lives in the arena, segment "ctl", int64 x CTL_WORDS).
// update-input slots: the sampler + gather fill them a batch of NBATCH updates at a time,
// ahead of the updates that consume them (and an update's alpha rows are read one update
// later by the folded launches); the ring holds at least two batches (sacx_handle::nslot)
#define NBATCH_MAX 8
#define MAX_MODELS 8        // world models (--num_models, sacx.h SACX_MAX_MODELS)
#define NSLOT 32
#define CTL_WORDS 48

struct Ctl {
    int64_t t_sac;          // completed updates (Adam iterations of q / pi / alpha optimisers)
    int64_t t_model;        // model optimiser iterations
    int64_t num_timesteps;  // SAC_expert.py:475 gating of the Polyak sync
    int64_t ts_increment;
    int64_t cur_size;       // TrajectoryBuffer.current_size
    int64_t start;          // physical ring index of logical row 0
    int64_t step_seq;       // update sequence number (stats / perm ring index)
    int64_t n_expert;       // expert rows currently set
    int32_t red_counter[8]; // last-arriver tickets (self-resetting)
    float epsilon;          // expert weight
    float pad_f[3];
    int64_t mfit_seq;       // model-fit step sequence (index ring / stats)
    int64_t rng_seq;        // update number the next sampler launch draws for
    int64_t pseq[NSLOT];    // update number whose randoms slot k holds (expert perm ring index)
};
static_assert(sizeof(Ctl) <= CTL_WORDS * 8, "ctl segment is CTL_WORDS int64");

struct RngState {          // NumPy legacy RandomState (MT19937) state
    uint32_t key[624];
    int32_t pos;
    int32_t has_gauss;
    double gauss;
};

// Adam constants for the optimiser groups.
enum { GRP_Q = 0, GRP_PI = 1, GRP_ALPHA = 2, GRP_MODEL = 3 };
struct AdamConsts {
    float lr[4];
    float tau_keep;   // f32(1 - tau)
    float tau_take;   // f32(tau)
    int32_t target_update_int;
    int32_t pad;
};

// ---------------------------------------------------------------- grouped GEMM
// C[M,N] = A[M,K] * B[K,N] on 16x16 output tiles, fp32 MFMA (v_mfma_f32_16x16x4_f32),
// K split over the 4 waves of a 256-thread workgroup and reduced through LDS.
enum Epi { EPI_FWD = 0, EPI_DACT = 1, EPI_ADAM = 2, EPI_STORE = 3 };
// launch-uniform operand/epilogue mode of k_gemm (template parameter)
// GM_FWD2: two forward layers of small-input nets in one launch (k_fwd2): probs[0, n) are layer 0,
// probs[n, 2n) layer 1 of the same nets (layer 1 reads layer 0's output); the layer-1 problems'
// tile_begin / tiles_n count (16-row block, 64-column group) workgroups
enum GemmMode { GM_FWD = 0, GM_DX = 1, GM_DW = 2, GM_FWD2 = 3 };
// waves per k_fwd2 workgroup of the pair that carries actor-head rows (rowk 3): two workgroups per CU,
// so the 256 tiles and the head rows run in one round; its head rows take NW / 4 blocks of 4 rows each
#define SACX_FWD2_HEAD_NW 8

enum { MSE_EXPERT = 1, MSE_FIT = 2, MSE_GAUSS = 4, MSE_SCALE = 8, MSE_NOREW = 16 };
struct GemmProb {
    const float* A;        // a_kc: A[m*lda + k]   else A[k*lda + m] (row ones_row = 1.0)
    const float* B;        // b_kc: B[n*ldb + k]   else B[k*ldb + n]
    float* C;
    const float* bias;     // EPI_FWD
    const float* H;        // EPI_DACT: activation output whose derivative multiplies
    float* P;              // EPI_ADAM: parameter tile base (m/v at +P_stride, +2*P_stride floats)
    float* T;              // EPI_ADAM: Polyak target (nullable)
    int32_t lda, ldb, ldc, ldh, ldp;
    int32_t M, N, K;
    int32_t a_kc, b_kc, ones_row;
    int32_t epi, act, group;
    int32_t tiles_n, tile_begin;
    float grad_scale;
    // GM_DX: when set, A is generated on load as wgen[k] * act'(A[m][k]) -- the delta at the
    // layer-2 output of a scalar-output net for a unit output gradient (the per-row gradient
    // is applied downstream: the result is linear in it)
    const float* wgen;
    int32_t gen_act;       // the activation whose derivative the generated A takes (layer 2's)
    // GM_DW: B[k][n] is scaled by bscale[k] on load (per-row output gradient; a ones vector
    // when unscaled, so every problem takes the same path)
    const float* bscale;
    // GM_FWD with mse: the world-model head on expert rows (SAC_expert.py:319-332): the output
    // is the normalised delta; C receives d loss / d out = (-eps * grad_scale * diff) * d_den,
    // diff = sp_e - (s_e + out * d_den + d_mean); part[row * tiles_n + tn] = sum of diff^2 over
    // the tile's columns (row stride of se_raw / spe_raw is N)
    // mse = 2: the world-model FIT loss (MSEModel.get_loss, continuous_models.py:280-302, in the
    // model.fwd2 epilogue): se_raw = the normalised targets T [M, N]; C = d loss / d out =
    // -(T - out) * (cf / mb) with cf = fcoef (reward_loss_coef) on column N - 1, else 1
    // (grad_scale = 1 / mb); part[row * tiles + tn] = sum over the tile's columns of cf (T - out)^2
    // Fit heads are mse = MSE_FIT | flags (ABI 7): the targets' row stride is ldp (T is [rows, S+1]
    // whatever the head's N); the reward column N - 1 takes fcoef, none with MSE_NOREW (the model
    // net beside a separate reward net); MSE_GAUSS: GaussianModel.get_loss (continuous_models.py:
    // 101-131) on the delta columns, spe_raw = the model's logstd [Sd] (Sd = N - 1, or N with
    // MSE_NOREW), with MSE_SCALE times the stop-gradient ds = mean(exp(2 logstd)) of
    // --scale_model_loss: q = (T - out) / e^l, C = -(q / e^l) (ds / mb), part sums ds (q^2 + 2 l +
    // log 2 pi), and ppart[tm * Sd + n] = sum over the tile's rows of 1 - q^2 (the logstd gradient's
    // partials, x ds / mb in mfit_final; a fit head has no partial dots, so ppart is free)
    int32_t mse;
    float fcoef;
    float dclip;            // --delta_clip_pred on `out` (clipped, zero gradient outside); 0: off
    const float *se_raw, *spe_raw, *dmean, *dden;
    float* part;
    // GM_FWD: the A operand's last columns [K - A, K) are the actor's evaluate() actions of the
    // tile's rows, computed in the tile's prologue from GemmArgs::head (seg[0]); columns
    // [0, K - A) are read from A as usual (the target rows: actor.head folded into q.fwd0)
    int32_t headp;
    // GM_FWD / GM_DX: this problem's operands take float4 loads along k (host-checked strides and
    // alignment); the launch's VEC template only says whether any problem does
    int32_t vec;
    // GM_DX in a q-head launch (rowk 2) / GM_FWD in an actor launch (rowk 5): per-row partial
    // dots of the tile's output row with the rows of pw -- ppart[(m * pw_n + j) * tiles_n + tn] =
    // sum over the tile's 16 columns n of C[m][n] * pw[j * pw_ld + n * pw_cs], j < pw_n <= 8.
    // rowk 2: the policy rows' action gradient through the critic's layer-0 action rows (summed
    // by the folded actor head backward; C may then be null).  rowk 5: the actor head
    // mu / logstd rows = Ha2 . W3 (summed, + bias, by the head rows and prologues).
    const float* pw;
    float* ppart;
    int32_t pw_ld, pw_cs, pw_n;
    // GM_DX with rowk 4: the folded actor head backward problem (GemmArgs::hbw)
    int32_t hbw;
    // GM_DX with rowk 7 (model.bwd1 of the fit with model.bwd2 folded in): the A operand, the
    // layer-2 delta D2 = (D3 . W2^T) (.) act'(H2), is generated on load from A = H2 [M, K] and
    // gd = D3 [M, g_o] (row stride gd_ld) through wgen = W2_ext [K (+1), g_o] (row stride g_o),
    // with model.bwd2's exact MFMA sequence (16-wide output slabs t, j = 0 2 / 1 3 pairs, the
    // slabs as waves summed in order; g_o <= 32); column tile 0 stores D2 to gst (ld gst_ld)
    const float* gd;
    union {
        float* gst;
        // config C5, GM_FWD on 32x32 tiles: the output's transposed bf16 image, rows n of C^T in the
        // wbf_pos layout of K = M (one 8-B piece per 4 consecutive rows) -- a later dW problem's A
        // operand (abf of GM_DW below; M % 4 == 0)
        uint16_t* tbf;
    };
    int32_t gd_ld, g_o, gst_ld;
    // config C5 (bf16 GEMMs) with 32x32 forward tiles: bf16 shadows of operands in the MFMA pair
    // layout of wbf_pos, read as one bf16x8 per lane and k-slab pair (null: the fp32 operand,
    // converted on load).  Weights: each row n of W^T; GM_FWD reads B from wbf, GM_DW + Adam stores
    // the updated rows k < wbf_k of P into wbf and the Polyak target into obf.  Activations (the
    // hidden layer-0 outputs, K = H0 a multiple of 128: rows of K positions): GM_FWD reads A from
    // abf (row stride K) and stores its own output into obf (row stride N) beside C.  GM_DW on
    // 32x32 tiles reads its A (= X^T) from abf when set: rows m < ones_row of wbf_ld_of(K)
    // positions (the ones row generated), written by the producer of X (tbf above, or k_gather's
    // xbfq for the critic input rows).
    uint16_t* wbf;
    uint16_t* obf;
    const uint16_t* abf;
    int32_t wbf_ld, wbf_per, wbf_k;
};

// Shadow row layout: the consumer's K is split over 4 waves of `per` 16-wide slabs (gemm_core's
// split: per = ceil(ceil(K / 16) / 4)); a wave's slabs pair up from its first, (it0, it0 + 1),
// (it0 + 2, it0 + 3), ..., and each pair takes 32 consecutive bf16: lane group grp's 8 operand
// values, k = s0 + 4 grp + j then s1 + 4 grp + j (j < 4) -- the order in which the bf16 MFMA
// path packs a converted pair, so a 16-B load yields the same operand bit for bit.  Positions
// of k >= K and of a wave's unpaired last slab stay zero.
__host__ __device__ inline int wbf_per_of(int K) { return (((K + 15) >> 4) + 3) >> 2; }
__host__ __device__ inline int wbf_ld_of(int K) { return 4 * ((wbf_per_of(K) + 1) >> 1) * 32; }
__host__ __device__ inline int wbf_pos(int k, int per) {
    const int s = k >> 4;
    if ((per & 1) == 0)        // every wave starts on an even slab: pair s / 2, half s % 2
        return (s >> 1) * 32 + ((k >> 2) & 3) * 8 + (s & 1) * 4 + (k & 3);
    const int w = s / per, i = s - w * per;
    return (w * ((per + 1) >> 1) + (i >> 1)) * 32 + ((k >> 2) & 3) * 8 + (i & 1) * 4 + (k & 3);
}

#define WBF_MAXM 12
// k_wbf_refresh: every shadow rebuilt from its fp32 weights (at each sacx_sac_step entry, so host
// writes of the parameters reach it; the Adam epilogues keep it current inside a step)
struct WbfArgs {
    const float* W[WBF_MAXM];    // [K x N] row-major (the first K rows of W_ext)
    uint16_t* S[WBF_MAXM];       // [N x ld]
    int32_t K[WBF_MAXM], N[WBF_MAXM];
    int32_t nmat;
    int64_t sstride;             // packed seeds: grid z = seed
    int32_t nseeds;
};

// rowk 4 (GM_DX, actor.bwd1): the actor head backward (k_actor_bwd's policy-row work) runs as
// the tile prologue.  Per row: ga = (g0 * sum ppart_q0 + g1 * sum ppart_q1) / a_den, the
// tanh-Gaussian backward (A5) -> Da3[row][0, Aout) (and E), then the A operand
// Da2[row][k] = (sum_o Da3[row][o] W3a[k][o]) * act'(Ha2[row][k]) is generated on load by a
// small MFMA (W3a = the problem's wgen, Ha2 = its A); column tile 0 stores Da2 for actor.adam.
struct HeadBwdArgs {
    int32_t B, A, Aout, per_state_std, tq;   // tq: partials per row and critic (H0 / 16 tiles)
    float lim;
    const float* part;      // [2, B, A, tq]
    const float* gpol;      // [2, B] output gradients of q0, q1 (the partials are unscaled)
    const float* a_den;
    const float* alpha;
    const float *c_t, *c_std, *c_u, *c_mask;   // backward cache rows [0, B + ne)
    float* Da3; float* E; float* Da2;
    // SAC-EO: rows [B, B + ne) are the expert rows, whose action gradient comes through their
    // world model's layer-0 action rows: partials [ne, A, tqm] written by model.bwd1 (unscaled
    // by any output gradient: the model head's MSE gradient already carries epsilon); the
    // policy rows' alpha term takes (1 - epsilon) (SAC_expert.py:305-338)
    int32_t ne, tqm;
    const float* mpart;
    const Ctl* ctl;         // epsilon (use_expert)
    const float* ma_den;    // the world models' action normaliser (expert rows; --only_model_normalizer)
};

// The split alpha finalisation of k_fwd2's fused q launch (SACX_AFIN, default): the first alpha block
// of that launch snapshots what finalize_update reads besides the alpha partials, so that the NEXT
// launch (q.head+critic.bwd1) can finish the alpha step in every one of its target row blocks (the
// same arithmetic, the same value) while its block 0 alone stores the results
struct AfinPre {
    float a_old, a_m, a_v, pad;
    int64_t t_sac, seq0, nts, tsi;
};

struct FinalArgs {
    float* alpha; float* alpha_m; float* alpha_v;
    Ctl* ctl;
    AdamConsts adam;
    float target_entropy;
    int32_t B, ne, use_expert;
    const float* lq;        // [2, B]
    const float* lp;        // [B]
    const float* mse_rows;  // [ne, mse_tiles] per-column-tile partial sums of diff^2
    float* red;             // partial slots
    int32_t nred;           // number of partials (alpha.head workgroups)
    int32_t nm;             // SAC-EO world models (1: every expert row through model 0)
    int32_t mse_tiles;      // partials per expert row in mse_rows
    float* stats; int32_t stats_cap;
    // data-parallel mode: the local alpha gradient goes here (then an all-reduce and
    // k_alpha_apply do the Adam, clamp, stats[4] and counters); null: all in place.
    // The split finalisation (never in the data-parallel modes, which do not fold): the snapshot
    union {
        float* alpha_g;
        AfinPre* pre;
    };
    float grad_scale;       // k_alpha_apply: 1 / ranks
    // packed seeds (sacx_config.seeds): grid z = nseeds independent learners whose arena blocks
    // sit sstride bytes apart; every arena pointer is relocated by blockIdx.z * sstride
    int64_t sstride;
    int32_t nseeds;
};

struct QHeadArgs {
    // target/critic mode (mode 0): nets t0,t1 on H2 slabs [0],[1]; q0,q1 on slabs [2],[3]
    // actor-loss mode (mode 1): q0,q1 on slabs [0],[1]
    int32_t mode;
    int32_t B, H1;
    const float* H2;        // [nslab, B, H1]
    const float* W3[4];     // W3_ext of the nets, [(H1+1) x 1]
    int32_t act;
    float* D2;              // [2, B, H1] delta at the layer-2 output of the trained / differentiated nets
    float* g;               // [2, B]     delta at the outputs of the two differentiated nets (nullable)
    float* loss_rows;       // mode 0: [2, B] 0.5 e^2 ; mode 1: [B] -alpha*nlp - minQ
    const float* alpha;
    const float* nlp;       // mode 0: nlp of the target actions; mode 1: nlp of the policy actions
    const float* r; const float* d;
    float gamma, ret_den_unused;
    const float* ret_den;
    float w_sac;            // (1 - epsilon) for SAC-EO, 1 for SAC
    // SAC-EO model rows (mode 0 only): rows [B, B+ne) handle the expert MSE
    int32_t ne, Hm1, S;
    const float* Hm2;       // [ne, Hm1]
    const float* Wm3[2];    // [(Hm1+1), S+1]
    int32_t mact;
    const float* se_raw; const float* spe_raw;
    const float *d_mean, *d_den;
    const Ctl* ctl;         // epsilon
    float* Dm2;             // [ne, Hm1]
    float* mse_rows;        // [ne]
    // packed seeds (sacx_config.seeds): grid z = nseeds independent learners whose arena blocks
    // sit sstride bytes apart; every arena pointer is relocated by blockIdx.z * sstride
    int64_t sstride;
    int32_t nseeds;
};

struct HeadSeg {
    int32_t r0, r1;        // actor rows [r0, r1)
    int32_t mode;          // 0 = evaluate (neglogp), 1 = sample (no neglogp), 2 = GaussianActor.sample
                           // (no squash; pi_out only)
    int32_t xq_row0;       // first row in xq_out
    const float* noise;    // [r1-r0, A]
    float* xq_out;         // normalised action -> xq_out[(xq_row0 + i) * ldQ + S + j]
    float* nlp_out;        // [r1-r0] (evaluate)
    float* pi_out;         // raw action lim*tanh(x) -> pi_out[(i) * A + j] (nullable)
};

struct HeadArgs {
    const float* H2; int32_t ldh;
    const float* W3;       // W3_ext [(H1+1), Aout]
    const float* logstd;   // [A] global logstd (per_state_std == 0)
    int32_t H1, A, Aout, S, ldQ, per_state_std;
    float lim;
    const float *a_mean, *a_den;
    // mode-1 (sample) segments write world-model inputs: their actions take the models'
    // normaliser (SAC_expert.py:139-144 --only_model_normalizer; the same values otherwise)
    const float *ma_mean, *ma_den;
    float logstd_init;     // mode 2: GaussianActor.logstd_init (continuous_actors.py:39-44)
    int32_t output_norm;   // mode 2: --actor_output_norm (continuous_actors.py:68-72)
    // nullable: the head's Ha2 . W3 as per-column-tile partials written by actor.fwd1 (rowk 5),
    // part[(row * Aout + o) * tq + i], i < tq (<= 16, a multiple of 4); row = the H2 row
    const float* part;
    int32_t tq;
    int32_t nseg;
    HeadSeg seg[4];
    int32_t total_rows;
    // backward cache (rows >= cache_row0 are cached at [row - cache_row0])
    int32_t cache_row0, cache_row1;
    float* c_t; float* c_std; float* c_u; float* c_mask;
    // alpha mode: rows >= alpha_row0 (a multiple of 4: whole workgroups) are the alpha
    // evaluate() of an update; their workgroups write partials of sum(-nlp + H) to fin.red
    int32_t alpha_mode;
    int32_t alpha_row0;
    uint64_t* ktime;        // measurement only (as GemmArgs::ktime)
    // packed seeds (sacx_config.seeds): grid z = nseeds independent learners whose arena blocks
    // sit sstride bytes apart; every arena pointer is relocated by blockIdx.z * sstride
    int64_t sstride;
    int32_t nseeds;
};

// world-model fit inputs: the step's minibatch rows gathered from the replay ring (k_mgather, or
// on load by model.fwd0's tiles: GemmArgs rowk 6)
struct MGatherArgs {        // rows [0, 2*mb): model k = row / mb
    const float* replay; int64_t cap; int32_t stride;
    int32_t S, A, mb;
    const int32_t* idx_ring; int32_t idx_cap;   // [idx_cap, 2*mb] replay-logical rows
    const Ctl* ctl;
    const float *s_mean, *s_den, *a_mean, *a_den, *d_mean, *d_den, *r_norm;   // r_norm = (mean, den)
    float* X; int32_t ldQ;      // [2mb, ldQ] = [s_n | a_n | 0]
    float* T;                   // [2mb, S+1] = [norm(sp - s) | norm(r)]
    int32_t nm;                 // world models fitted (rows [0, nm*mb))
    float clip_d, clip_r;       // > 0: --delta_clip_loss / --reward_clip_loss on T (get_loss :286-296)
};
#define MFIT_PRE 64                 // fit steps one pre-gather block holds (= the steps of a fit graph)

// end of a world-model fitting step (k_mfinal, or folded into a launch of the step)
struct MFinalArgs {
    Ctl* ctl;
    const float* loss_rows; int32_t mb, nm;
    float* mstats; int32_t mstats_cap;
    // nt > 0: loss_rows holds nt partials per row (the fit-loss epilogue's, sums of cf e^2 over a
    // column tile: the loss is 0.5 x their sum); 0: one loss per row (k_mloss)
    int32_t nt;
    // --separate_reward_nn: the reward heads' loss partials, nt2 per row (same 0.5 x sum), right after
    // the nm * mb * nt of loss_rows; 0: none
    int32_t nt2;
    // GaussianModel: the logstd gradient, (ds / mb) x the sum over the ntm row tiles of lgpart (model k
    // at lgpart + k ntm S), then Keras Adam on logstd[k] (m / v at +p_stride / +2 p_stride) at the
    // advanced step, or (gstore, --model_max_grad_norm) the gradient stored at +3 p_stride for the
    // global-norm clip; ds = mean(exp(2 logstd)) with lscale, else 1
    const float* lgpart; int32_t ntm, S, lscale, gstore;
    float* logstd;          // model 0's; model k's at + k * lstride floats (equal per-model parameter blocks)
    int64_t lstride;
};

#define GEMM_MAXP 8
struct GemmArgs {
    GemmProb probs[GEMM_MAXP];   // by value: no dependent global load to find a tile's problem
    int32_t nprob;
    int32_t mode;          // GemmMode, uniform over the launch's problems
    int32_t vec;           // GM_FWD/GM_DX: float4 loads along k (ld % 4 == 0, K % 4 == 0, aligned);
    int32_t total_tiles;
    int32_t xcd_map;       // 1: each XCD takes a contiguous tile range (see xcd_tile)
    int32_t bf16;          // 1: bf16 MFMA operands (rounded on load), fp32 accumulate (config C5)
    int32_t t32;           // 1: 32x32 output tiles per workgroup (tile_begin / tiles_n count those)
    int32_t dwl;           // GM_DW: k_dwl (32x32 tiles, LDS-DMA staged rows; probs[].vec bit 0 / 1:
                           // A / B rows by 16-B pieces)
    int64_t p_stride;      // floats between params / adam_m / adam_v blocks
    const Ctl* ctl;
    AdamConsts adam;
    // one extra workgroup (blockIdx == total_tiles) finalises the PREVIOUS update's alpha
    // (alpha.final folded into a launch of the next update, see get_graph)
    int32_t has_final;
    FinalArgs fin;
    // GM_DX: rowk = 1 / 2 appends row_blocks workgroups running k_qhead<0> / <1> on qh
    // (horizontal fusion: the heads and the unscaled dX GEMM are independent)
    int32_t rowk, row_blocks;
    QHeadArgs qh;
    // GM_FWD with rowk = 3: the actor head (GemmArgs::head) -- seg[0] in the prologue of the
    // headp problems, the other rows as row_blocks extra workgroups (from row head_block0 * 4);
    // hfin: the alpha-row partials (alpha_mode)
    HeadArgs head;
    FinalArgs hfin;
    int32_t head_block0;
    HeadBwdArgs hbw;       // rowk 4 (GM_DX)
    uint64_t* ktime;       // measurement only: per-workgroup start / end ticks (nullable)
    // packed seeds (sacx_config.seeds): grid z = nseeds independent learners whose arena blocks
    // sit sstride bytes apart; every arena pointer is relocated by blockIdx.z * sstride
    int64_t sstride;
    int32_t nseeds;
    // world-model fit (ROWK 0 launches): one extra workgroup after the tiles finalises the fit step
    // (k_mfinal's work: loss statistics, t_model and mfit_seq advance)
    int32_t has_mfinal;
    // GM_DW: the optimiser step counter was already advanced in this step (the folded model
    // finalisation runs before model.adam): the Adam step is t + 1 - t_adv
    int32_t t_adv;
    MFinalArgs mfin;
    // GM_FWD rowk 6 (model.fwd0 of the fit): problem p's A rows are replay records gathered by the
    // step's indices (model p's minibatch) and normalised on load; column tile 0 stores them to
    // the problem's A (X, read by model.adam) and each tile stores its 16 columns of the targets
    MGatherArgs mg;
};
static_assert(sizeof(GemmArgs) <= 4096 - 16, "GemmArgs travels as kernel arguments, behind a KHdr");

// The scalars that pick a k_gemm / k_dwl workgroup's role and problem (total_tiles, row_blocks,
// the problems' first tiles, nprob, has_final, xcd_map), packed as 9 x 12-bit fields + 8 flag bits
// into 4 dwords that travel AHEAD of GemmArgs as plain kernel arguments and are preloaded into
// SGPRs at dispatch (gfx950 kernarg preload, hipcc -mllvm -amdgpu-kernarg-preload-count=4): the
// workgroup then reads its problem's fields in ONE scalar round trip instead of two.  valid = 0
// (a value past 12 bits) falls back to reading them from GemmArgs.
struct KHdr {
    uint32_t h[4];
};
__host__ __device__ inline uint32_t khdr_field(const KHdr& k, int i) {   // 12-bit field i (i <= 9)
    const int b = 12 * i, w = b >> 5, o = b & 31;
    const uint64_t v = ((uint64_t)(w + 1 < 4 ? k.h[w + 1] : 0u) << 32) | k.h[w];
    return (uint32_t)(v >> o) & 0xfffu;
}
// flags: bits 108.. : nprob (4), has_final (2), xcd_map (1), valid (1)
__host__ __device__ inline uint32_t khdr_flags(const KHdr& k) { return (k.h[3] >> 12) & 0xffu; }
// The launch header of a k_gemm / k_dwl launch (sacx_internal.h: KHdr); invalid (all zero) when a
// value does not fit 12 bits, and the kernel then reads the same values from GemmArgs
inline KHdr khdr_of(const GemmArgs& a, bool enabled = true) {
    KHdr k{};
    if (!enabled) return k;              // (SACX_KHDR=0: every launch reads GemmArgs)
    uint32_t v[9];
    v[0] = (uint32_t)a.total_tiles;
    v[1] = (uint32_t)a.row_blocks;
    for (int i = 1; i < GEMM_MAXP; ++i) v[i + 1] = i < a.nprob ? (uint32_t)a.probs[i].tile_begin : 0xfffu;
    bool ok = a.nprob <= 15 && a.has_final >= 0 && a.has_final <= 3 && (a.xcd_map & ~1) == 0;
    for (int i = 0; i < 9; ++i) ok = ok && v[i] <= 0xfffu;
    // (problems past nprob never match: the selection loop checks i < nprob first)
    if (!ok) return k;
    uint64_t bits[2] = {0, 0};
    for (int i = 0; i < 9; ++i) {
        const int b = 12 * i;
        bits[b >> 6] |= (uint64_t)v[i] << (b & 63);
        if ((b & 63) + 12 > 64) bits[(b >> 6) + 1] |= (uint64_t)v[i] >> (64 - (b & 63));
    }
    const uint32_t flags = (uint32_t)a.nprob | ((uint32_t)a.has_final << 4) | ((uint32_t)a.xcd_map << 6) | 0x80u;
    bits[1] |= (uint64_t)flags << (108 - 64);
    k.h[0] = (uint32_t)bits[0]; k.h[1] = (uint32_t)(bits[0] >> 32);
    k.h[2] = (uint32_t)bits[1]; k.h[3] = (uint32_t)(bits[1] >> 32);
    return k;
}


// ---------------------------------------------------------------- sampler + gather
struct RngArgs {
    RngState* st;
    Ctl* ctl;              // reads cur_size at run time; advances rng_seq / pseq
    int32_t n_int;
    int32_t n_norm;
    int32_t* out_idx;
    float* out_norm;
    int32_t slot;          // writes ctl->pseq[slot]; -1: a draw outside the updates (no stamp)
    int32_t reset_seq;     // first sampler launch of a chain: rng_seq = step_seq
    int32_t nupd;          // consecutive updates drawn by this launch (slots slot .. slot+nupd-1)
    int64_t slot_bytes;    // distance between consecutive slots' buffers
    // the speculative draw of the drop-in loop (sacx_sac_step(1)): randint's bound given by the
    // host (the ring size after the append to come) instead of ctl->cur_size, and the state
    // before the draw saved to `backup` so the draw can be undone
    int64_t size_fixed;    // > 0: randint(size_fixed)
    RngState* backup;      // nullable
    // packed seeds (sacx_config.seeds): grid z = nseeds independent learners whose arena blocks
    // sit sstride bytes apart; every arena pointer is relocated by blockIdx.z * sstride
    int64_t sstride;
    int32_t nseeds;
    // split sampler: k_rng stores each accepted polar pair's four tempered words at
    // pairs[(u * pcap + j) * 4] and update u's leading cached normal (0 / 1) at pairs_oi[u];
    // k_polar (launched by launch_rng after it) computes the normals.  nullptr: k_rng does both
    uint32_t* pairs;
    int32_t* pairs_oi;
    int32_t pcap;
    // segmented sampler (launch_rng: a batch of many words): the batch's raw stream is generated
    // as jS segments of jL words, each but the first started from a window jumped to from the
    // key block (mt_jump.h), then consumed by flag / prefix / resolve / emit launches over the
    // GPU (k_mtj_*).  jw: the work area (mtj_layout, per seed); nullptr: the one-workgroup k_rng
    uint32_t* jw;
    const uint32_t* jc;    // jump coefficients x^(k jL) mod phi, k = 1 .. jsmax - 1 (624 words each)
    int32_t jL;
    int32_t jsmax;         // segments the work area holds
    int32_t jS;            // segments of this launch (launch_rng)
    int32_t jmin;          // launches expecting fewer words stay on k_rng
    int32_t junder;        // > 0: at most this many segments (tests: forces the redraw fallback;
                           // SACX_MTJ_UNDER, read once at sacx_bind)
};

// ---------------------------------------------------------------- segmented sampler layout
#define MTJ_CH 320                                   // jump coefficient bits per workgroup
#define MTJ_NC ((19937 + MTJ_CH - 1) / MTJ_CH)       // jump workgroups per window (63)
#define MTJ_HEAD (19937 + 624)                       // words [0, MTJ_HEAD) feed every jump
#define MTJ_CHK 2048                                 // flag chunk (words)
#define MTJ_MAXCHK 1024                              // chunks the resolve workgroup scans
#define MTJ_RES_WORDS (16 + 16 * NBATCH_MAX)
#define MTJ_PF 128                                   // chunks k_mtj_resolve finds in LDS
// res words: [0] overflow, [1] words generated, [2] final position, [3] pos0, [4..5] rng,
// [6..7] mask; update u at 16 + 16 u: [0] ib [1] ie [2] ibase [3] pb [4] pe [5] pbase [6] oi
// ptag: the chunks around each update's predicted boundaries (k_mtj_head), pfbm: their two
// bitmaps, copied there by k_mtj_flags
struct MtjLayout {
    int64_t sw, part, fi, fp, cnt, pre, res, ptag, pfbm, total, wcap;
    int32_t nchk;
};
__host__ __device__ inline MtjLayout mtj_layout(int64_t L, int smax) {
    MtjLayout y{};
    y.wcap = ((smax * L + 1 + 8 + MTJ_CHK - 1) / MTJ_CHK) * MTJ_CHK;
    y.nchk = (int32_t)(y.wcap / MTJ_CHK);
    y.sw = 0;
    y.part = y.wcap;
    y.fi = y.part + (int64_t)(smax - 1) * MTJ_NC * 624;
    y.fp = y.fi + y.wcap / 32;
    y.cnt = y.fp + y.wcap / 32;
    y.pre = y.cnt + (int64_t)y.nchk * 8;
    y.res = y.pre + (int64_t)(y.nchk + 1) * 8;
    y.ptag = y.res + MTJ_RES_WORDS;
    y.pfbm = y.ptag + MTJ_PF;
    y.total = y.pfbm + (int64_t)MTJ_PF * 128;
    return y;
}

struct GatherArgs {
    const float* replay;   // [cap, stride]
    int64_t cap;
    int32_t stride;
    int32_t S, A, B, ne;
    const int32_t* idx;
    const Ctl* ctl;
    int32_t slot;          // expert permutation of update ctl->pseq[slot]
    int32_t nupd;          // consecutive slots gathered by this launch (blockIdx.y)
    int64_t slot_bytes;    // distance between consecutive slots' buffers
    const float *s_mean, *s_den, *a_mean, *a_den;
    const float *ms_mean, *ms_den;   // the world models' state normaliser: Xm's state columns
    float* Xa;  int32_t ldS;   // actor rows [sp(B) ; s(B) ; s_e(ne)]
    float* Xq;  float* Xt; float* Xp; float* Xm; int32_t ldQ;
    float* r; float* d;
    const float* exp_s; const float* exp_sp; const int32_t* perm_ring; int32_t perm_cap;
    int32_t perm_ld;            // permutation length (expert_batch; ne = the rows used, <= perm_ld)
    float* se_raw; float* spe_raw;
    // config C5: the critic rows' transposed bf16 image (columns c < S + A of Xq as rows of
    // wbf_ld_of(B) positions, wbf_pos layout): critic.adam's layer-0 A operand; null: not written
    uint16_t* xbfq;
    // the drop-in loop's speculative draw (k_act_rng, plain SAC, one update): the draw stored its
    // accepted polar pairs' words (pairs, pairs_oi[0]); polar_wgs more workgroups turn them into the
    // slot's n_norm normals at norm with k_polar's arithmetic.  polar_wgs 0: none
    const uint32_t* pairs;
    const int32_t* pairs_oi;
    float* norm;
    int32_t n_norm;
    int32_t polar_wgs;
    // packed seeds (sacx_config.seeds): grid z = nseeds independent learners whose arena blocks
    // sit sstride bytes apart; every arena pointer is relocated by blockIdx.z * sstride
    int64_t sstride;
    int32_t nseeds;
};

// ---------------------------------------------------------------- actor head rows

// ---------------------------------------------------------------- Q heads


// ---------------------------------------------------------------- actor backward head
struct ActorBwdArgs {
    int32_t B, ne, S, A, Aout, H0, H1, Hm0, per_state_std;
    float lim;
    const float* Dp1;       // [2, B, H0]
    const float* Wq1[2];    // W1_ext of q0, q1 [(S+A+1), H0]
    const float* Dm1;       // [ne, Hm0]
    const float* Wm1[2];    // W1_ext of the models [(S+A+1), Hm0]
    const float *a_den;
    const float* ma_den;    // the world models' action normaliser (expert rows)
    const float* alpha;
    const Ctl* ctl;         // epsilon
    int32_t use_expert;
    const float *c_t, *c_std, *c_u, *c_mask;   // cache rows [0, B+ne)
    const float* W3a;       // [(H1+1), Aout]
    const float* Ha2;       // actor layer-2 outputs of rows [B, ...) ; row i at Ha2[i*H1]
    int32_t act;
    float* Da3; float* Da2; float* E;
    const float* gpol;      // [2, B] output gradients of q0, q1 for the policy rows (Dp1 is unscaled)
    uint64_t* ktime;        // measurement only (as GemmArgs::ktime)
    // packed seeds (sacx_config.seeds): grid z = nseeds independent learners whose arena blocks
    // sit sstride bytes apart; every arena pointer is relocated by blockIdx.z * sstride
    int64_t sstride;
    int32_t nseeds;
};

// ---------------------------------------------------------------- finalize (alpha + stats)


struct AppendArgs {
    float* replay; int64_t cap; int32_t stride; int32_t S, A;
    const float *s, *a, *r, *sp, *d;
    int64_t n;
    Ctl* ctl;
    // pinned counter the workgroup bumps once it has read the source rows (k_act_rng's held
    // append: the host reuses the staging buffer without an event marker); null: none
    uint32_t* done;
    // packed seeds (sacx_buffer_append_host_seeds): grid z = seed; replay / ctl move by z * sstride,
    // the source rows by z * n rows (arrays [seeds, n, ...])
    int64_t sstride;
    int32_t nseeds;
};

// ---------------------------------------------------------------- world-model fitting
// ---------------------------------------------------------------- reference object methods
// The standalone network calls of the reference's actor / critic / model objects
// (sacx_critic_forward, sacx_actor_evaluate, sacx_model_forward, sacx_model_loss): the
// rows a caller hands over, normalised into a GEMM input, and the net output turned into
// what the reference method returns.
struct NetIOArgs {
    int32_t mode;               // 0: prep [norm s | norm a | 0] -> X; 1: critic output; 2: model
                                // output (sample / step); 3: model loss (get_loss) of a chunk
    int32_t n, S, A, ldX, ldO;
    const float *s, *a, *sp, *r;   // caller rows of this chunk (a nullable in mode 0)
    float* X;                      // mode 0: [n, ldX]
    const float* O;                // modes 1-3: net output [n, ldO]
    const float *s_mean, *s_den, *a_mean, *a_den, *d_mean, *d_den, *r_norm, *ret_den;
    float clip_d, clip_r;          // > 0: clip_by_value(-clip, clip)
    float reward_coef;
    int32_t value;                 // mode 1: 1 = QCritic.value (x ret sigma), 0 = _forward
    float* out0;                   // mode 1: [n]; mode 2: pred [n, S+1]; mode 3: running sum [1]
    float* out1;                   // mode 2: sp [n, S]; mode 3: loss [1] (written on the last chunk)
    float* out2;                   // mode 2: r [n]
    int32_t first, last;           // mode 3: first / last chunk of the call
    int64_t n_total;               // mode 3: rows of the whole call (reduce_mean)
    // GaussianModel (ABI 7): mode 2 adds exp(mlogstd) * mnoise[i * S + j] to the clipped delta_n when
    // mnoise is set (sample(deterministic=False) / step); mode 3 takes the Gaussian NLL of
    // continuous_models.py:101-131 for the delta columns (x mean(exp(2 l)) with lscale)
    const float* mlogstd; const float* mnoise; int32_t lscale;
};

struct MLossArgs {
    int32_t S, mb, nm;
    const float* T; const float* O;   // [2mb, S+1]
    float* D3;                        // dL/dout [2mb, ldD]
    int32_t ldD;                      // r4(S+1): float4 rows for model.bwd2's operand loads
    float* loss_rows;                 // [2mb]
    float reward_coef;
};

// ---------------------------------------------------------------- data-parallel Adam (C4)
// After the gradient all-reduce: Keras Adam over a contiguous parameter range with the
// summed gradients at +3 p_stride (scaled by 1/ranks), Polyak into P + t_off when t_off != 0.
struct AdamApplyArgs {
    float* P;
    int64_t n, p_stride, t_off;
    int32_t group;
    float grad_scale;
    const float* scale_dev;     // nullable: gradients also times *scale_dev (clip_by_global_norm)
    const Ctl* ctl;
    AdamConsts adam;
    int32_t t_adv;              // as GemmArgs::t_adv
};

// In-process data-parallel reduce (sacx_dp_local_step): buf[r][i] = sum over r' of buf[r'][i], in
// rank order, for every rank r -- what ncclAllReduce(sum) leaves on each rank.
#define DP_LOCAL_MAX 8
struct DpSumArgs {
    float* buf[DP_LOCAL_MAX];
    int32_t nranks;
    int64_t n;
};

// ---------------------------------------------------------------- actor layer norm (A3)
// --actor_layer_norm: layer 0 is Dense -> LayerNormalization (epsilon 1e-3, gamma / beta) -> tanh
// (nn_utils.py:110-119).  The layer-0 GEMM writes the pre-norm Z; k_ln mode 0 turns rows of Z
// into tanh(gamma xhat + beta) in place (caching xhat, rstd for rows < cache_rows); mode 1 turns
// dY (the gradient at the norm's output, after tanh') into dZ in place and writes dY*xhat and
// dY for the gamma / beta column sums.  One wave per row, H <= 512.
struct LNArgs {
    int32_t mode;
    int32_t H;
    float* Z;                   // [rows, H] (mode 0: Z -> H1; mode 1: dY -> dZ)
    int32_t nrange, r[4];       // mode 0: row ranges [r0, r1) (+ [r2, r3)); mode 1: rows [0, r1)
    const float* gamma;         // [H] (beta = gamma + H)
    float* xhat; float* rstd;   // cache (mode 0 writes rows < cache_rows, mode 1 reads row + xrow0)
    int32_t cache_rows, xrow0;
    float* gy; float* gb;       // mode 1: [rows, H] dY * xhat and dY
    int64_t sstride;
    int32_t nseeds;
};

// clip_by_global_norm (mbrl_onpolicy_alg.py:315-317 over TF's clip_ops): k_gnorm_part sums g^2
// over contiguous chunks of the gradient range, k_gnorm_final forms norm = sqrt(sum) and
// scale = clip * min(1 / norm, 1 / clip) (+ (norm - norm): NaN when the norm is not finite)
#define GNORM_PARTS 128
struct GNormArgs {
    const float* g; int64_t n;
    float* part;                // [GNORM_PARTS]
    float* scale_out;           // [1]
    float clip;
};

// ---------------------------------------------------------------- model rollout (F2)
// batch_simtrajectory_sampler (samplers.py:73-122) over MSEModel.step
// (continuous_models.py:225-242): one chunk of rows, output row i at (i * H + t)
struct RollArgs {
    int32_t mode;               // 0: prep step t (s_t -> actor / model inputs), 1: finish step t
    int32_t n, S, A, H, t, ldS, ldQ;
    const float* s_init;        // [n, S] (mode 0, t == 0)
    float* s_out; float* a_out; float* r_out; float* sp_out; uint8_t* d_out;
    const float* O;             // model output [n, S+1] = [delta_n | r_n]
    const float* a_raw;         // actor sample [n, A]
    float* X; float* Xm;        // actor input [n, ldS], model input [n, ldQ] (columns < S)
    const float *s_mean, *s_den, *d_mean, *d_den, *r_norm;   // r_norm = (mean, den); d / r: the model's
    const float *ms_mean, *ms_den;   // the model's state normaliser (Xm); s_*: the actor's (X)
    float clip_d, clip_r;       // > 0: clip_by_value(-clip, clip) (delta_clip_pred / reward_clip_pred)
    // GaussianModel.step (continuous_models.py:36-54): exp(mlogstd) * mnoise [n, S] added to the clipped
    // delta_n (mode 1); null: MSEModel
    const float* mlogstd; const float* mnoise;
};

// ---------------------------------------------------------------- expert diagnostics (F3)
// SAC_expert.py:554-608 (model MSE on expert data / on counterfactual actions) and
// _calc_disc :427-460 (discrepancy of the two models).  O holds model 0's output on rows
// [0, n) and model 1's on rows [n, 2n) for the same inputs.
struct DiagArgs {
    int32_t mode;               // 0: prep inputs; 1: MSE (expert actions); 2: MSE (counterfactual); 3: disc
    int32_t n, S, A, ldS, ldQ;
    const float *s_e, *a_e, *sp_e;
    const float* O;             // [2n, S+1]
    float* X; float* Xm;        // actor input [n, ldS]; model input [n, ldQ]
    const float *s_mean, *s_den, *a_mean, *a_den, *d_mean, *d_den;   // s: the actor's; a, d: the models'
    const float *ms_mean, *ms_den;   // the models' state normaliser (Xm)
    float clip_d;
    float* out;
    // mode 3 (_calc_disc, deterministic=False) with GaussianModels: model k's delta_n gets
    // exp(mlogstd[k]) * mnoise[(k n + i) * S + j] (null: MSEModel)
    const float* mlogstd[2]; const float* mnoise;
    int32_t nmod;               // modes 1 / 2: models whose outputs O holds (rows [k n, (k+1) n)), 2 .. MAX_MODELS
};

// sacx_actor_act on a few rows (the env loop's one observation): one workgroup per row runs
// the normaliser, both hidden layers and the sampling head (k_act_rows)
#define ACT_ROWS_MAX 16       // rows per call that take k_act_rows
#define ACT_ROWS_DIM 1024     // S, H0, H1 bound (LDS vectors)
struct ActRowArgs {
    const float* obs;          // [m, S]
    const float *s_mean, *s_den;
    const float *W0, *W1, *W3; // Keras (in, out) with the bias as the last row
    const float* logstd;       // [A] (per_state_std == 0)
    const float* noise;        // [m, A] or null (deterministic)
    float* out;                // [m, A]
    int32_t S, A, Aout, H0, H1, act0, act1;
    int32_t mode;              // 1: SquashedGaussianActor.sample, 2: GaussianActor.sample
    int32_t per_state_std, output_norm;
    float lim, logstd_init;
    // packed seeds (sacx_actor_act_host_seeds): grid z = seed; the arena pointers (normaliser,
    // weights, noise) move by z * sstride, obs / out by z * m rows (arrays [seeds, m, S / A])
    int64_t sstride;
    int32_t nseeds, m;
    // host-mapped completion counter (nullable): each row's workgroup adds 1 (system-scope
    // release) once its outputs are written, so a synchronous host caller can take the actions
    // without waiting for the rest of the launch (k_act_rng's sampler workgroup)
    uint32_t* done;
};

// launchers (defined in k_sac.hip)
void launch_act_rows(const ActRowArgs& a, int m, hipStream_t s);
// rows + the sampler draw beside them (+ a deferred 1-row append as one more workgroup when app is set)
void launch_act_rng(const ActRowArgs& a, int m, const RngArgs& r, hipStream_t s, const AppendArgs* app = nullptr, bool polar = true);
void launch_gemm(const GemmArgs& a, hipStream_t s);
void launch_rng(const RngArgs& a, hipStream_t s);
void launch_gather(const GatherArgs& a, hipStream_t s);
void launch_actor_head(const HeadArgs& a, const FinalArgs& f, hipStream_t s);
void launch_qhead(const QHeadArgs& a, hipStream_t s);
void launch_actor_bwd(const ActorBwdArgs& a, hipStream_t s);
void launch_append(const AppendArgs& a, hipStream_t s);
// nsteps > 0: the pre-gather of a block of fit steps (SACX_MPRE): step j of the block (ctl->mfit_seq + j)
// into slot j of the staging that a.X / a.T point to ([MFIT_PRE, 2mb, ldQ] / [MFIT_PRE, 2mb, S+1]), which
// that step's launches read; 0: this step's rows into X / T
void launch_mgather(const MGatherArgs& a, hipStream_t s, int nsteps = 0);
void launch_mloss(const MLossArgs& a, hipStream_t s);
void launch_mfinal(const MFinalArgs& a, hipStream_t s);
void launch_set_ctl(Ctl* ctl, int64_t num_timesteps, int64_t ts_increment, int64_t sstride, int nseeds, hipStream_t s);
void launch_set_pseq(Ctl* ctl, int slot, int64_t sstride, int nseeds, hipStream_t s);
void launch_wbf_refresh(const WbfArgs& a, hipStream_t s);
void launch_spin(double us, hipStream_t s);
void launch_obs_norm(const float* obs, int64_t n, int S, const float* mean, const float* den, float* X, int ldX,
                     hipStream_t s);
void launch_alpha_final(const FinalArgs& f, hipStream_t s);
void launch_roll(const RollArgs& a, hipStream_t s);
void launch_net_io(const NetIOArgs& a, hipStream_t s);
void launch_gnorm(const GNormArgs& a, hipStream_t s);
void launch_ln(const LNArgs& a, hipStream_t s);
void launch_diag(const DiagArgs& a, hipStream_t s);
void launch_adam_apply(const AdamApplyArgs& a, hipStream_t s);
void launch_alpha_apply(const FinalArgs& f, hipStream_t s);
void launch_dp_sum(const DpSumArgs& a, hipStream_t s);

}  // namespace sacx
