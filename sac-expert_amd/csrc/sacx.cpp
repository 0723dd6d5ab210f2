// libsacx host side: arena layout, launch plan of one SAC / SAC-EO update,
// hipGraph capture and the C ABI declared in include/sacx.h.
//
// One update (SAC_expert.py:463-477) is planned as this launch sequence
// (reference function each stage restates in brackets):
//   rng            sampler: randint + all normals of the update   [buffers.py:136, continuous_actors.py:351]
//   gather         replay rows -> normalised staging               [buffers.py:137-141, normalizer.py:36-41]
//   actor.fwd0/1   actor MLP on [sp ; s ; s_expert]               [continuous_actors.py:327-331]
//   actor.head     evaluate(sp), evaluate(s), sample(s_expert)     [continuous_actors.py:270-379]
//   q.fwd0/1       target nets on (sp,a'), critics on (s,a), models on (s_e, c_a)
//   q.head         min target, TD target, critic loss grads, expert MSE  [SAC_expert.py:211-250, 321-334]
//   critic.bwd1    dX through critic layer 2 (+ model layer 2)
//   critic.adam    dW of q0/q1 + Keras Adam + Polyak into t0/t1  [SAC_expert.py:243,250,362-373]
//   pi.q.fwd0/1    updated critics on (s, pi(s))                  [SAC_expert.py:314-317]
//   pi.q.head      min + policy loss grads                        [SAC_expert.py:317-319]
//   pi.q.bwd1      dX through critic layer 2
//   actor.head.bwd action grads -> tanh-Gaussian backward -> actor layer 3 dX
//   actor.bwd1     dX through actor layer 2
//   actor.adam     dW of the actor (+ logstd) + Keras Adam        [SAC_expert.py:336-338]
//   alpha.fwd0/1   updated actor on s                              [SAC_expert.py:341-343]
//   alpha.head     evaluate + alpha loss + Adam + clamp + stats   [SAC_expert.py:345-356]
#include "sacx.h"
#include "sacx_internal.h"
#include "mt_jump.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <chrono>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

using namespace sacx;

namespace {

std::string g_create_error;

inline int64_t r4(int64_t x) { return (x + 3) & ~int64_t(3); }

struct RollKey {             // sacx_rollout graph cache key (memcmp'd: no padding holes)
    int32_t model;
    int32_t seed;             // packed seeds: the selected seed (its arena block)
    int64_t n;
    int32_t horizon, deterministic;
    float delta_clip, reward_clip;
    const void* ptrs[6];
};
static_assert(sizeof(RollKey) == 4 + 4 + 8 + 4 + 4 + 4 + 4 + 6 * 8, "RollKey is packed");

struct SegInfo {
    std::string name;
    uint64_t off;
    int64_t rows, cols;
    int dtype, role;
};

struct Launch {
    enum Kind { RNG, GATHER, GEMM, AHEAD, QHEAD, ABWD, FINAL, MGATHER, MLOSS, MFINAL, ALLREDUCE, APPLY, AAPPLY,
                GNORM, LNORM } kind;
    std::string name;
    RngArgs rng;
    GatherArgs gather;
    GemmArgs gemm;
    HeadArgs head;
    FinalArgs fin;
    QHeadArgs qh;
    ActorBwdArgs ab;
    MGatherArgs mg;
    MLossArgs ml;
    MFinalArgs mf;
    AdamApplyArgs ap;          // APPLY
    GNormArgs gn;              // GNORM
    LNArgs ln;                 // LNORM
    float* ar_buf = nullptr;   // ALLREDUCE: in-place sum over the data-parallel ranks
    int64_t ar_count = 0;
    int grid = 0, block = 256;
    int pre_steps = 0;         // MGATHER: > 0 the pre-gather of that many fit steps (launch_mgather)
    double flops = 0, bytes = 0;
    int gemm_first = 0;  // index of the first problem in the host table (GEMM)
    bool after_final = false;  // graph: waits for the previous update's alpha branch
    bool alpha_branch = false; // graph: runs on the side stream beside the next update's first launches
    bool frees_slot = false;   // graph: the launch that carries the folded alpha rows (last reader of a slot)
    // graph: the critics' forward on the buffer rows (s, a) runs on its own stream, between
};

const char* kernel_family(Launch::Kind k) {
    switch (k) {
        case Launch::RNG: return "k_rng";
        case Launch::GATHER: return "k_gather";
        case Launch::GEMM: return "k_gemm";
        case Launch::AHEAD: return "k_actor_head";
        case Launch::QHEAD: return "k_qhead";
        case Launch::ABWD: return "k_actor_bwd";
        case Launch::FINAL: return "k_alpha_final";
        case Launch::MGATHER: return "k_mgather";
        case Launch::MLOSS: return "k_mloss";
        case Launch::MFINAL: return "k_mfinal";
        case Launch::ALLREDUCE: return "rccl_allreduce";
        case Launch::APPLY: return "k_adam_apply";
        case Launch::AAPPLY: return "k_alpha_apply";
        case Launch::GNORM: return "k_gnorm";
        case Launch::LNORM: return "k_ln";
    }
    return "?";
}

}  // namespace

// One net's hidden layers: create_nn's layers list and its activations (nn_utils.py:100-138)
struct NetDims {
    std::vector<int> h, act;
    int D() const { return (int)h.size(); }
};

struct sacx_handle {
    sacx_config cfg{};
    std::string err;
    // dims
    int S = 0, A = 0, H0 = 0, H1 = 0, B = 0, Aout = 0, ne = 0, Hm0 = 0, Hm1 = 0, ecap = 0;
    int Hc0 = 0, Hc1 = 0;     // the critics' hidden sizes (--critic_layers; H0 / H1 are the actor's)
    int ldS = 0, ldQ = 0, stride = 0, Ra = 0, Rb = 0, n_norm = 0;
    // hidden-layer activations per net and layer (nn_utils.py:5-22 create_activations): actor,
    // critics, world models
    int aact[2] = {0, 0}, cact[2] = {0, 0}, macts[2] = {0, 0};
    int64_t cap = 0;
    int graph_steps = 128, stats_cap = 4096, perm_cap = 4096, mb = 0, mfit_cap = 1024;
    int nm = 0;               // SAC-EO world models (--num_models: 1 .. SACX_MAX_MODELS)
    int ne_perm = 0;          // expert rows per update permutation (expert_batch); ne = the rows the update
                              // uses: all of them (1 or 2 models), else the first two array_split sections
    // hidden layers of [actor, critics, world models, reward nets]; H0 / H1 (Hc*, Hm*, Hr*) and the act
    // pairs above are the first and the last hidden layer of each
    NetDims nd[4];
    bool deep = false;        // a net of other than 2 hidden layers: the generic plans (build_plan_generic)
    // world-model variants (ABI 7): GaussianModel (a logstd per model, the NLL fit loss, noise in
    // sample / step) and --separate_reward_nn (a reward net r<k> beside each model net m<k>)
    bool gm = false, srn = false, lscale = false;
    int Om = 0;               // model-net outputs: S + 1 (the reward as the last column), or S (srn)
    int Hr0 = 0, Hr1 = 0;     // the reward nets' hidden sizes (srn)
    int racts[2] = {0, 0};    // their hidden-layer activations
    bool ln = false;          // --actor_layer_norm: Dense -> LayerNorm -> tanh on the actor's layer 0
    // layout
    std::vector<SegInfo> segs;
    std::map<std::string, size_t> seg_index;
    uint64_t arena_bytes = 0;
    uint64_t param_off = 0;
    int64_t p_stride = 0;  // floats
    // packed seeds: K learners in K arena blocks seed_bytes apart; `arena` is the block of the
    // selected seed (the per-seed calls), arena0 seed 0's (the plans: grid z covers the rest)
    int seeds = 1, sel = 0;
    int plan_seeds = 1;       // the seed count the plan's shape decisions see (1 with single_seed_plan)
    uint64_t seed_bytes = 0;
    char* arena0 = nullptr;
    // binding
    char* arena = nullptr;
    hipStream_t stream = nullptr;
    hipStream_t cap_stream = nullptr, rng_stream = nullptr;
    bool bound = false;
    std::vector<Launch> plan[NSLOT];
    int64_t slot_bytes = 0;   // distance between consecutive update-input slots
    int nbatch = 4;           // sampler batch (updates per k_rng launch)
    int nslot = 8;            // update-input slots the ring rotates over (a multiple of nbatch, >= 2 nbatch)
    // bf16 weight shadows (SACX_WBF, default on): the matrices (segment "wbf.<name>") and whether
    // add_gemm wires them into the problems it builds (the update plans only)
    struct WbfMat { std::string name; int K, N; };
    std::vector<WbfMat> wbf_mats;
    int wbf_enabled = 3;      // SACX_WBF: 0 off, 1 weights + layer-0 activations, 2 weights only, 3 activations only
    int xbf = 0;              // transposed bf16 images of critic.adam's X operands (SACX_XBF; C5, B % 128 == 0):
                              // 0 off, 1 the critic rows (k_gather) and layer-0 outputs (q.fwd0), 2 the rows only
    bool wbf_attach = false;
    bool wbf_live = false;    // the update plans read / maintain the shadows (refreshed per step call)
    hipEvent_t seg_start = nullptr;   // run_segments: the call's start on the bound stream (before set_ctl)
    // run_segments' cross-stream edges as stream memory operations on signal memory instead of
    // event markers (SACX_SEG_SIG: 1 the side stream's batch-ready edges, 2 (default) also batch
    // 0's, whose marker on the bound stream held segment 0 back: the driver's command 16.00-16.03k
    // -> 16.20-16.23k, r06_ab_seg_sig_v1.txt); 0 where the device lacks stream wait-value
    int seg_sig = 2;
    uint64_t* sig_mem[2] = {nullptr, nullptr};   // batches drawn (side stream), batch 0 drawn (bound stream)
    uint64_t sig_seq[2] = {0, 0};
    std::vector<std::string> abf_segs;          // activation segments with a bf16 shadow ("abf.<name>")
    std::vector<std::pair<const float*, const float*>> abf_written;   // plan build: ranges a wired producer stores
    bool rng_split = false;   // k_rng + k_polar (rng.pairs): the polar transform spread over the GPU
    int pcap = 0;             // polar pairs per update (rng.pairs rows per update)
    // the drop-in loop's draw beside the act (k_act_rng, plain SAC, no split sampler) stores its
    // accepted pairs' words in rng.spairs and the gather queued behind it computes the normals on
    // spare workgroups: the fp64 log / sqrt leave the draw's one workgroup (SACX_SPEC_POLAR)
    bool spec_polar = false;
    bool spec_polar_live = false;   // the queued speculative draw stored pairs
    int spcap = 0;
    bool rng_jump = false;    // segmented sampler (k_mtj_*): the update sampler's launches
    int jL = 0;               // its segment length (words)
    int jsmax = 0;            // segments its work area holds
    int mtj_ramp = 3;         // a graph's first mtj_ramp sampler batches take it (SACX_MTJ_RAMP), the rest k_rng
    int mtj_under = 0;        // tests: cap its segment count (SACX_MTJ_UNDER: forces the redraw fallback)
    int tile32 = 0;           // plan GEMMs on 32x32 workgroup tiles: 1 all, 2 FWD / DX only (SACX_T32)
    int tile32_plan = 0;      // the tile32 a plan of plan_seeds seeds would take: the folds follow it
    int dwl = 0;              // dW + Adam launches on k_dwl: 0 never, 1 when K >= 512, 2 always (SACX_DWL)
    int dwl_nh = 1;           // k_dwl tile width in 16-column halves (SACX_DWL_NH: 1 -> 32x16, 2 -> 32x32)
    int mfuse = 2;            // model fit folds (SACX_MFUSE): 1 the loss into model.fwd2's epilogue and k_mfinal
                              // into model.bwd2, 2 also k_mgather into model.fwd0's operand loads (default);
                              // 3 also model.bwd2 into model.bwd1 (generated operand, heads of <= 32
                              // outputs; bit-identical, measured slower: HC 49.7 vs 46.9 us per step)
    int unaligned_b = 1;      // dX launches: float4 loads of W_ext rows at any 4-B offset (SACX_UNALIGNED)
    int fwd2 = 1;             // two-layer forward pairs as one k_fwd2 launch where they qualify (SACX_FWD2)
    int mtile = 1;            // model fit tiles: 0 16x16, 1 16x16 + wide dW on 32x32, 2 the handle's (SACX_MTILE)
    int mt32 = 5;             // fit launches on 32x32 tiles under mtile 1 (SACX_MT32): 1 model.bwd1, 2 model.fwd1, 4 model.bwd2, 8 model.fwd2
    int dw_round_tiles = 1280;  // 16x16 dW tiles resident at once (SACX_DW_ROUND)
                              // (32x32 tiles accumulate as 16x16 ones: only the folds change sums)
    int xcd_map = 1;          // GEMM tiles XCD-contiguous (xcd_tile)
    int afin = 1;             // k_fwd2's folded alpha finalisation split over q.head's rows (SACX_AFIN; 0: ticket)
    int mfwd2 = 1;            // the fit's gather + model.fwd0 + model.fwd1 as one k_fwd2 launch (SACX_MFWD2)
    int mpre = 1;             // the fit's minibatch rows pre-gathered for a block of steps (SACX_MPRE): the
                              // steps read the staging slots mfit.Xs / mfit.Ts instead of gathering on load
    // data-parallel mode (sacx_dp_init): each rank's local-batch gradients are summed over
    // dp_ranks by RCCL inside the update graph, then every rank applies the same Adam
    int dp_ranks = 0, dp_rank = 0;
    bool dp_local = false;    // sacx_dp_init_local: the ranks are handles of this process (no RCCL)
    ncclComm_t comm = nullptr;
    bool nccl_failed = false;
    // world-model fitting, per seed (packed seeds fit one seed at a time: its arena block's plan)
    std::vector<std::vector<Launch>> mplans;
    std::vector<Launch> mpres;   // per seed: the pre-gather launch of its fit plan (kind RNG: none)
    std::vector<std::map<int, hipGraphExec_t>> mgraphs;   // per seed: fit steps per graph -> graph
    std::vector<int64_t> mfit_hosts;   // model steps issued per seed (mirror ctl->mfit_seq)
    std::vector<GemmProb> probs;
    int probs_cursor = 0;
    std::map<std::tuple<int, int, int>, hipGraphExec_t> graphs;   // (G, with_rng, skipped kind)
    std::vector<std::pair<RollKey, hipGraphExec_t>> roll_graphs;     // sacx_rollout replays
    std::vector<hipEvent_t> events;
    uint32_t* done_host = nullptr;   // pinned completion counter of act_host's rows (ActRowArgs::done)
    uint32_t* done_dev = nullptr;
    uint32_t done_seq = 0;           // its value once every row launched so far has finished
    bool act_poll = true;            // act_host waits on the counter, not on the stream (SACX_ACT_POLL=0: event)
    float* pin = nullptr;            // pinned host staging (2 x STAGE_CAP floats), the _host entry points:
    float* pin_dev = nullptr;        // [0, STAGE_CAP) appends, [STAGE_CAP, 2 STAGE_CAP) acts; pin_dev is its
                                     // device-side address (kernels read / write it in place)
    hipEvent_t pin_ev = nullptr;     // the last kernel that reads it
    bool pin_pending = false;
    int64_t seq_host = 0;  // updates issued (mirrors ctl->step_seq)
    // Speculative sampler of the drop-in loop (the reference's cadence act -> _update -> env.step ->
    // add, SAC_expert.py:779-797): when the caller steps one update at a time, sacx_actor_act_host
    // queues the next update's randint + normals right behind the action kernel and returns once
    // the action is back, so the draw runs while the host has the action; the next
    // sacx_sac_step(1) then replays a graph without the sampler if the ring still holds the size
    // the draw assumed.  Every other consumer of the RNG stream first undoes the draw (spec_cancel).
    bool spec_enabled = true;  // SACX_SPEC=0: off
    bool spec_live = false;    // a speculative draw is queued
    bool last_step_one = false;  // the last sacx_sac_step was a plain one-update step
    // k_act_rng's held append signals its reads of the staging rows through done_host[1] instead of
    // an event recorded behind it (SACX_APP_CTR); app_seq = the count the host expects
    bool app_ctr = true;         // (and the acts record act_ev only when the host does not poll)
    bool app_ctr_pending = false;
    uint32_t app_seq = 0;
    bool act_ev_live = true;     // act_ev marks the last act (false: nothing recorded, poll only)
    int64_t spec_size = 0;     // the ring size it assumed
    int64_t spec_hits = 0;     // one-update steps that used a speculative draw (sacx_spec_hits)
    int spec_slot = 1;         // the slot the queued draw fills (1 or 2: never the pending alpha's)
    // The alpha branch (alpha.fwd, alpha.head, alpha.final) of the last speculative one-update
    // step is deferred into the next one (merged_body, as inside a captured multi-update graph):
    // the next act needs the updated actor, not alpha.  alpha_pending = that update's slot, or -1;
    // every entry point that could observe or disturb it runs it first (settle).
    int alpha_pending = -1;
    // k_set_ctl skipped when the control block already holds the values: a speculative step(1)
    // right after another with num_timesteps advanced by ts_increment (the folded alpha.final's
    // add) -- the drop-in loop's cadence.  settle() and resync forget it.
    // Deferred append (SACX_APP_DEFER): a 1-row append_host right after a one-update step is held
    // (its row in the pinned staging) and runs as one more workgroup of the next act's k_act_rng
    // launch -- the drop-in cadence's act -> step(1) -> append; every other entry point queues it
    // first (flush_append, from settle and the ring's other users)
    bool app_defer = true;
    bool app_pending = false;
    AppendArgs app_args{};
    bool ctl_skip = true;     // SACX_CTL_SKIP=0: always launch it
    // a fork / join graph's first sampler batch (one update) on the chain's own stream, as the segment
    // graphs do: the chain's first update then does not wait on a cross-queue edge (SACX_G_INLINE0)
    bool g_inline0 = true;
    bool ctl_known = false;
    int64_t ctl_nts = 0;
    int32_t ctl_inc = 0;
    int64_t cur_size_host = 0; // mirrors ctl->cur_size (appends, resync)
    int64_t n_appends = 0;     // sacx_buffer_append calls (a full ring changes content, not size)
    int64_t spec_appends = 0;  // n_appends when the speculative draw was queued
    bool act_rng = true;       // deterministic act + speculative draw in one launch (k_act_rng; SACX_ACT_RNG=0: two)
    hipEvent_t act_ev = nullptr;   // end of the last act_host kernel chain (its actions are on the host)

    uint64_t add(const std::string& name, int64_t rows, int64_t cols, int dtype, int role) {
        const int esz = (dtype == SACX_I64 || dtype == SACX_F64) ? 8 : 4;
        const uint64_t off = (arena_bytes + 255) & ~uint64_t(255);
        segs.push_back({name, off, rows, cols, dtype, role});
        seg_index[name] = segs.size() - 1;
        arena_bytes = off + (uint64_t)(rows * cols * esz);
        return off;
    }
    void alias(const std::string& name, uint64_t off, int64_t rows, int64_t cols, int dtype, int role) {
        segs.push_back({name, off, rows, cols, dtype, role});
        seg_index[name] = segs.size() - 1;
    }
    const SegInfo& seg(const std::string& n) const { return segs.at(seg_index.at(n)); }
    uint64_t off_of(const std::string& n) const { return seg(n).off; }
    template <class T>
    T* ptr(const std::string& n) const { return reinterpret_cast<T*>(arena + seg(n).off); }
    float* f(const std::string& n) const { return ptr<float>(n); }
    // seed 0's segment (the packed launches relocate it by blockIdx.z * seed_bytes)
    float* f0(const std::string& n) const { return reinterpret_cast<float*>(arena0 + seg(n).off); }
    Ctl* ctl() const { return ptr<Ctl>("ctl"); }
    Ctl* ctl0() const { return reinterpret_cast<Ctl*>(arena0 + seg("ctl").off); }
    uint64_t total_bytes() const { return seeds > 1 ? (uint64_t)seeds * seed_bytes : arena_bytes; }
};

namespace {

// a segment of the normaliser set the world models use: mnorm.* (SAC-EO) -- or norm.* on a handle
// without models, where only the update's own normaliser exists
std::string mnorm(const sacx_handle* h, const char* x) {
    return std::string(h->cfg.use_expert ? "mnorm." : "norm.") + x;
}

// the actor's output head (the Dense layer after its last hidden one)
std::string actor_head_name(const sacx_handle* h) { return "actor.l" + std::to_string(h->nd[0].D()); }

int fail(sacx_handle* h, const std::string& msg) {
    if (h) h->err = msg;
    return -1;
}

// Undoes a queued speculative draw (drawn on the bound stream, so stream order alone puts the
// restore after it): restores the RNG state it started from.  keep_state: nothing to restore
// (the caller overwrites the state anyway).
int spec_cancel(sacx_handle* h, bool keep_state = false) {
    if (!h->spec_live) return 0;
    h->spec_live = false;
    // every seed's state (packed seeds: one block per seed, seed_bytes apart)
    const size_t pitch = h->seeds > 1 ? (size_t)h->seed_bytes : sizeof(RngState);
    if (!keep_state &&
        hipMemcpy2DAsync(h->arena0 + h->off_of("rng"), pitch, h->arena0 + h->off_of("rng.spec"), pitch,
                         sizeof(RngState), (size_t)h->seeds, hipMemcpyDeviceToDevice, h->stream) != hipSuccess)
        return fail(h, "spec restore");
    return 0;
}

// the handles the speculative draw applies to: one learner, its own RNG stream
bool spec_mode(const sacx_handle* h) {
    return h->spec_enabled && h->dp_ranks == 0 && !h->dp_local && h->nslot >= 3;
}

#define HIPCHK(h, x)                                                                    \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) return fail((h), std::string(#x " -> ") + hipGetErrorString(e_)); \
    } while (0)

constexpr int ACT_CAP = 1024;   // rows per sacx_actor_act launch chain
constexpr int MFIT_GRAPH = 64;      // model-fit steps per captured graph (then 8, then 1)
static_assert(MFIT_GRAPH <= MFIT_PRE, "a fit graph's steps fit one pre-gather block");
constexpr int STAGE_CAP = SACX_STAGE_FLOATS;   // floats in the pinned host staging buffer of the _host entry points
constexpr int ROLL_CAP = 4096;  // trajectories per sacx_rollout launch chain

void build_layout(sacx_handle* h) {
    const int S = h->S, A = h->A, H0 = h->H0, H1 = h->H1, B = h->B;
    const int F = SACX_F32;
    // ---------------- parameters (Keras W_ext = [W ; b] per Dense layer)
    h->arena_bytes = 0;
    // Keras Dense layers l0 .. l<D> (the last one the output head) of a net with hidden widths w
    auto net = [&](const std::string& n, int in, int out, int role, const std::vector<int>& w) {
        int k = in;
        for (size_t l = 0; l < w.size(); ++l) {
            h->add(n + ".l" + std::to_string(l), k + 1, w[l], F, role);
            k = w[l];
        }
        h->add(n + ".l" + std::to_string(w.size()), k + 1, out, F, role);
    };
    net("actor", S, h->Aout, SACX_ROLE_PARAM, h->nd[0].h);
    if (h->ln) h->add("actor.ln", 2, H0, F, SACX_ROLE_PARAM);     // LayerNormalization gamma ; beta
    h->add("actor.logstd", 1, A, F, SACX_ROLE_PARAM);
    const int Hc0 = h->Hc0, Hc1 = h->Hc1;      // the critics' (--critic_layers)
    net("q0", S + A, 1, SACX_ROLE_PARAM, h->nd[1].h);
    net("q1", S + A, 1, SACX_ROLE_PARAM, h->nd[1].h);
    net("t0", S + A, 1, SACX_ROLE_TARGET, h->nd[1].h);
    net("t1", S + A, 1, SACX_ROLE_TARGET, h->nd[1].h);
    h->add("alpha", 1, 1, F, SACX_ROLE_PARAM);
    if (h->cfg.use_expert) {
        // per model, in model.trainable order (continuous_models.py:27-32, :216-221): the model net,
        // GaussianModel's logstd, the separate reward net -- one contiguous range (the global-norm clip)
        for (int k = 0; k < h->nm; ++k) {
            const std::string m = "m" + std::to_string(k);
            net(m, S + A, h->Om, SACX_ROLE_PARAM, h->nd[2].h);
            if (h->gm) h->add(m + ".logstd", 1, S, F, SACX_ROLE_PARAM);
            if (h->srn) net("r" + std::to_string(k), S + A, 1, SACX_ROLE_PARAM, h->nd[3].h);
        }
    }
    const uint64_t pbytes = (h->arena_bytes + 255) & ~uint64_t(255);
    h->param_off = 0;
    h->p_stride = (int64_t)(pbytes / 4);
    h->alias("params", 0, 1, h->p_stride, F, SACX_ROLE_PARAM);
    h->arena_bytes = pbytes;
    h->add("adam_m", 1, h->p_stride, F, SACX_ROLE_STATE);
    h->add("adam_v", 1, h->p_stride, F, SACX_ROLE_STATE);
    h->add("grad", 1, h->p_stride, F, SACX_ROLE_WORK);   // data-parallel gradients (+3 p_stride)
    // ---------------- normalisers (normalizer.py: (x - mean) / max(std, 1e-8))
    h->add("norm.s_mean", 1, S, F, SACX_ROLE_STATE);
    h->add("norm.s_den", 1, S, F, SACX_ROLE_STATE);
    h->add("norm.a_mean", 1, A, F, SACX_ROLE_STATE);
    h->add("norm.a_den", 1, A, F, SACX_ROLE_STATE);
    h->add("norm.d_mean", 1, S, F, SACX_ROLE_STATE);
    h->add("norm.d_den", 1, S, F, SACX_ROLE_STATE);
    h->add("norm.r", 1, 2, F, SACX_ROLE_STATE);  // r_mean, r_den
    h->add("norm.ret_den", 1, 1, F, SACX_ROLE_STATE);
    // bf16 shadows of the SAC nets' hidden-layer weights (config C5, 32x32 forward tiles): the
    // forward launches read B from them (wbf_pos layout), the Adam epilogues keep them current
    h->wbf_mats.clear();
    if (h->cfg.gemm_bf16 && !h->deep && (h->wbf_enabled == 1 || h->wbf_enabled == 2)) {
        const char* nets[] = {"actor", "q0", "q1", "t0", "t1"};
        for (const char* n : nets) {
            const bool act = std::string(n) == "actor";
            const int in = act ? S : S + A, h0 = act ? H0 : Hc0, h1 = act ? H1 : Hc1;
            for (int l = 0; l < 2; ++l) {
                const int K = l == 0 ? in : h0, N = l == 0 ? h0 : h1;
                const std::string w = std::string(n) + ".l" + std::to_string(l);
                h->add("wbf." + w, N, wbf_ld_of(K) / 2, SACX_U32, SACX_ROLE_WORK);
                h->wbf_mats.push_back({w, K, N});
            }
        }
    }
    // the world models' own normaliser set (SAC_expert.py:53-54, :139-144): a copy of norm.*
    // unless --only_model_normalizer gives the models a RunningNormalizers of their own
    if (h->cfg.use_expert) {
        h->add("mnorm.s_mean", 1, S, F, SACX_ROLE_STATE);
        h->add("mnorm.s_den", 1, S, F, SACX_ROLE_STATE);
        h->add("mnorm.a_mean", 1, A, F, SACX_ROLE_STATE);
        h->add("mnorm.a_den", 1, A, F, SACX_ROLE_STATE);
        h->add("mnorm.d_mean", 1, S, F, SACX_ROLE_STATE);
        h->add("mnorm.d_den", 1, S, F, SACX_ROLE_STATE);
        h->add("mnorm.r", 1, 2, F, SACX_ROLE_STATE);
    }
    // ---------------- control + RNG
    h->add("ctl", 1, CTL_WORDS, SACX_I64, SACX_ROLE_STATE);
    const uint64_t roff = h->add("rng", 1, sizeof(RngState) / 4, SACX_U32, SACX_ROLE_STATE);
    h->alias("rng.key", roff, 1, 624, SACX_U32, SACX_ROLE_STATE);
    h->alias("rng.pos", roff + offsetof(RngState, pos), 1, 2, SACX_I32, SACX_ROLE_STATE);
    h->alias("rng.gauss", roff + offsetof(RngState, gauss), 1, 1, SACX_F64, SACX_ROLE_STATE);
    h->add("rng.spec", 1, sizeof(RngState) / 4, SACX_U32, SACX_ROLE_WORK);   // state before a speculative draw
    // Split sampler (many normals per update, Humanoid): k_rng ranks the accepted polar pairs and
    // stores their four words; k_polar turns them into normals over the whole GPU
    h->rng_split = h->n_norm > 16384;
    if (const char* e = std::getenv("SACX_RNG_SPLIT")) h->rng_split = std::atoi(e) != 0;
    if (h->rng_split) {
        h->pcap = (h->n_norm + 1) / 2;
        h->add("rng.pairs", (int64_t)NBATCH_MAX * h->pcap, 4, SACX_U32, SACX_ROLE_WORK);
        h->add("rng.pairs_oi", 1, NBATCH_MAX, SACX_I32, SACX_ROLE_WORK);
    }
    h->spec_polar = !h->rng_split && !h->cfg.use_expert && h->n_norm > 0;
    if (const char* e = std::getenv("SACX_SPEC_POLAR")) h->spec_polar = h->spec_polar && std::atoi(e) != 0;
    if (h->spec_polar) {
        h->spcap = (h->n_norm + 1) / 2;
        h->add("rng.spairs", h->spcap, 4, SACX_U32, SACX_ROLE_WORK);
        h->add("rng.spairs_oi", 1, 1, SACX_I32, SACX_ROLE_WORK);
    }
    // Segmented sampler (k_mtj_*): a sampler batch of many words (Humanoid: ~135k per update)
    // is twisted as ~16 segments of L words from jumped-ahead windows and ranked over the GPU
    // instead of on one workgroup.  L: a 4-update batch in ~16 segments, >= the 20,561 words
    // every jump reads; the work area holds a batch of NBATCH_MAX updates
    {
        const double per = 2.0 * h->B + (double)((h->n_norm + 1) >> 1) * (4.0 / 0.78539816339744831);
        h->rng_jump = per >= 40000.0;
        if (const char* e = std::getenv("SACX_RNG_JUMP")) h->rng_jump = std::atoi(e) != 0;
        if (h->rng_jump) {
            int64_t L = ((int64_t)std::ceil(per * 1.02 / 4.0) + 63) / 64 * 64;
            if (const char* e = std::getenv("SACX_MTJ_L")) L = std::atoll(e);
            L = std::max<int64_t>(L, MTJ_HEAD);
            const double words = NBATCH_MAX * per;
            const double est = 624.0 + 1.02 * words + 8.0 * std::sqrt(words) + 64.0 * NBATCH_MAX + 1024.0 + MTJ_HEAD;
            int smax = (int)std::ceil((est - 1.0) / (double)L) + 1;
            smax = (int)std::max<int64_t>(2, std::min<int64_t>(smax, ((int64_t)MTJ_MAXCHK * MTJ_CHK - 9) / L));
            h->jL = (int)L;
            h->jsmax = smax;
            h->add("rng.jw", 1, mtj_layout(L, smax).total, SACX_U32, SACX_ROLE_WORK);
            // x^(kL) mod phi as per-chunk set-bit lists (mt_jump_lists), uploaded at bind
            h->add("rng.jc", 1, mt_jump_lists_words(smax - 1, MTJ_CH), SACX_I32, SACX_ROLE_STATE);
        }
    }
    // per-slot update inputs: the sampler + gather run ahead of the updates on a side stream,
    // so everything they write rotates over a ring of slots.  A cheap sampler (HC: 1,536 normals
    // per update) gets 32 slots: a graph of up to 32 updates draws every input at its start,
    // with no sampler launch waiting on the update chain (a 20-update graph otherwise waits
    // ~0.1 ms at update 8 for a sampler batch the runtime releases only when the chain reaches
    // it); an expensive one (Humanoid: 10 MB of slot rows per update) keeps 8, the footprint
    // the caches hold
    h->nslot = h->n_norm <= 16384 ? NSLOT : 8;
    if (const char* e = std::getenv("SACX_NSLOT")) h->nslot = std::max(2, std::min(NSLOT, std::atoi(e)));
    const int ne1 = std::max(1, h->ne);
    // config C5: critic.adam's bf16 32x32 tiles read X^T (the critic rows, the critics' layer-0
    // outputs) from transposed images their producers write (k_gather, q.fwd0's epilogue) instead
    // of converting strided fp32 columns; B % 128 == 0, so the images have no pad positions
    h->xbf = 0;
    if (const char* e = std::getenv("SACX_CTL_SKIP")) h->ctl_skip = std::atoi(e) != 0;
    if (const char* e = std::getenv("SACX_APP_CTR")) h->app_ctr = std::atoi(e) != 0;
    if (const char* e = std::getenv("SACX_SEG_SIG")) h->seg_sig = std::atoi(e);
    if (const char* e = std::getenv("SACX_G_INLINE0")) h->g_inline0 = std::atoi(e) != 0;
    if (const char* e = std::getenv("SACX_APP_DEFER")) h->app_defer = std::atoi(e) != 0;
    if (const char* e = std::getenv("SACX_XBF"))
        if (h->cfg.gemm_bf16 && !h->deep && B % 128 == 0) h->xbf = std::max(0, std::min(2, std::atoi(e)));
    for (int s = 0; s < h->nslot; ++s) {
        const std::string sl = "slot" + std::to_string(s);
        h->add(sl + ".idx", 1, B, SACX_I32, SACX_ROLE_WORK);
        h->add(sl + ".noise", 1, h->n_norm, F, SACX_ROLE_WORK);
        h->add(sl + ".Xa", h->Ra, h->ldS, F, 0);   // actor rows [sp ; s ; s_e] (normalised)
        h->add(sl + ".Xq", B, h->ldQ, F, 0);       // critic rows [s | a]
        h->add(sl + ".Xt", B, h->ldQ, F, 0);       // target rows [sp | pi(sp)]
        h->add(sl + ".Xp", B, h->ldQ, F, 0);       // policy rows [s | pi(s)]
        h->add(sl + ".Xm", ne1, h->ldQ, F, 0);     // expert rows [s_e | pi(s_e)]
        h->add(sl + ".r", 1, B, F, 0);
        h->add(sl + ".d", 1, B, F, 0);
        h->add(sl + ".se_raw", ne1, S, F, 0);
        h->add(sl + ".spe_raw", ne1, S, F, 0);
        if (h->xbf) h->add(sl + ".xbfq", S + A, wbf_ld_of(B) / 2, SACX_U32, SACX_ROLE_WORK);
    }
    h->slot_bytes = (int64_t)(h->off_of("slot1.idx") - h->off_of("slot0.idx"));
    for (int k = 1; k < h->nslot; ++k)   // the batched sampler / gather address slot k as slot 0 + k * slot_bytes
        for (const char* nm : {".idx", ".noise", ".Xa", ".Xq", ".Xt", ".Xp", ".Xm", ".r", ".d", ".se_raw", ".spe_raw", ".xbfq"})
            if ((std::string(nm) != ".xbfq" || h->xbf) &&
                (h->off_of("slot" + std::to_string(k) + nm) != h->off_of(std::string("slot0") + nm) + k * (uint64_t)h->slot_bytes)) {
                fprintf(stderr, "sacx: slot layout is not uniform\n");
                abort();
            }
    // ---------------- data
    h->add("replay", h->cap, h->stride, F, SACX_ROLE_STATE);
    const int ecap = std::max(1, h->ecap);
    h->add("expert.s", ecap, S, F, SACX_ROLE_STATE);
    h->add("expert.sp", ecap, S, F, SACX_ROLE_STATE);
    h->add("perm", h->perm_cap, std::max(1, h->ne_perm), SACX_I32, SACX_ROLE_STATE);
    h->add("stats", h->stats_cap, 8, F, SACX_ROLE_STATE);
    h->add("red", 1, std::max(1024, (B + 3) / 4), F, SACX_ROLE_WORK);
    h->add("ws.afin", 1, sizeof(AfinPre) / 4, F, SACX_ROLE_WORK);   // the split alpha finalisation's snapshot
    // ---------------- workspace
    const int Ra = h->Ra, Rb = h->Rb, Hm0 = std::max(1, h->Hm0), Hm1 = std::max(1, h->Hm1);
    // actor activations; rows [Ra4, Ra4 + B) hold the alpha evaluate() of an update
    // (aliased ws.Hl1 / ws.Hl2) so one grouped head launch can serve both
    const int Ra4 = (Ra + 3) & ~3;
    // a chain's per-layer buffers: <p>1 = hidden layer 0, <p>2 = the last hidden layer -- one segment
    // each at two layers (the fused plans' layout), with one layer <p>2 aliases <p>1; the middle layers
    // <p>m<i> of deeper nets (the generic plans) are added at the end of the workspace (mids)
    auto last = [&](const std::string& n2, const std::string& n1, int64_t rows, int w2, int D) -> uint64_t {
        if (D >= 2) return h->add(n2, rows, w2, F, 0);
        const SegInfo& s1 = h->seg(n1);
        h->alias(n2, s1.off, s1.rows, s1.cols, F, 0);
        return s1.off;
    };
    struct Mid { std::string p; int64_t rows; int net; };
    std::vector<Mid> mids;
    const int Da = h->nd[0].D(), Dc = h->nd[1].D(), Dm = h->nd[2].D(), Dr = h->nd[3].D();
    const uint64_t oHa1 = h->add("ws.Ha1", Ra4 + B, H0, F, 0);
    const uint64_t oHa2 = last("ws.Ha2", "ws.Ha1", Ra4 + B, H1, Da);
    mids.push_back({"ws.Ham", Ra4 + B, 0});
    // Ha2 . W3 per 16-column tile of actor.fwd1 (rows as ws.Ha2), summed by the head rows
    h->add("ws.hpart", Ra4 + B, (int64_t)h->Aout * ((H1 + 15) / 16), F, 0);
    h->add("ws.c_t", Rb, A, F, 0);
    h->add("ws.c_std", Rb, A, F, 0);
    h->add("ws.c_u", Rb, A, F, 0);
    h->add("ws.c_mask", Rb, A, F, 0);
    h->add("ws.nlp_t", 1, B, F, 0);
    h->add("ws.nlp_p", 1, B, F, 0);
    h->add("ws.nlp3", 1, B, F, 0);
    h->add("ws.Hq1", 4 * B, Hc0, F, 0);
    last("ws.Hq2", "ws.Hq1", 4 * B, Hc1, Dc);
    if (Dc >= 2) h->add("ws.Dq2", 2 * B, Hc1, F, 0);
    h->add("ws.Dq1", 2 * B, Hc0, F, 0);
    if (Dc < 2) last("ws.Dq2", "ws.Dq1", 2 * B, Hc1, Dc);
    mids.push_back({"ws.Hqm", 4 * B, 1});
    mids.push_back({"ws.Dqm", 2 * B, 1});
    h->add("ws.gq", 2, B, F, 0);
    h->add("ws.lq", 2, B, F, 0);
    h->add("ws.Hp1", 2 * B, Hc0, F, 0);
    last("ws.Hp2", "ws.Hp1", 2 * B, Hc1, Dc);
    h->add("ws.Dp1", 2 * B, Hc0, F, 0);
    if (h->deep) {                    // the generic plan's policy-row deltas (the fused one keeps partials)
        last("ws.Dp2", "ws.Dp1", 2 * B, Hc1, Dc);
        mids.push_back({"ws.Hpm", 2 * B, 1});
        mids.push_back({"ws.Dpm", 2 * B, 1});
    }
    h->add("ws.lp", 1, B, F, 0);
    h->add("ws.gp", 2, B, F, 0);                 // policy-row output gradients of q0, q1
    h->add("ws.apart", 2 * B, ((Hc0 + 15) / 16) * A, F, 0);  // their action-gradient partials (folded head bwd)
    h->add("ws.mpart", ne1, ((Hm0 + 15) / 16) * A, F, 0);       // the expert rows' ones (SAC-EO, model.bwd1)
    h->add("ws.ones", 1, std::max(std::max(Rb, B), std::max(1, h->mb)) + 4, F, SACX_ROLE_STATE);
    h->add("ws.Hm1", ne1, Hm0, F, 0);
    last("ws.Hm2", "ws.Hm1", ne1, Hm1, Dm);
    if (Dm >= 2) h->add("ws.Dm2", ne1, Hm1, F, 0);
    h->add("ws.Dm1", ne1, Hm0, F, 0);
    if (Dm < 2) last("ws.Dm2", "ws.Dm1", ne1, Hm1, Dm);
    if (h->cfg.use_expert) {
        mids.push_back({"ws.Hmm", ne1, 2});
        mids.push_back({"ws.Dmm", ne1, 2});
    }
    h->add("ws.mse", ne1, (S + 15) / 16, F, 0);       // per-column-tile partials of the expert MSE
    h->add("ws.dout", ne1, S, F, 0);                  // d loss / d model output (expert rows)
    h->add("ws.Da3", Rb, h->Aout, F, 0);
    if (Da >= 2) h->add("ws.Da2", Rb, H1, F, 0);
    h->add("ws.Da1", Rb, H0, F, 0);
    if (Da < 2) last("ws.Da2", "ws.Da1", Rb, H1, Da);
    mids.push_back({"ws.Dam", Rb, 0});
    h->add("ws.E", Rb, A, F, 0);
    h->alias("ws.Hl1", oHa1 + (uint64_t)Ra4 * H0 * 4, B, H0, F, 0);
    h->alias("ws.Hl2", oHa2 + (uint64_t)Ra4 * H1 * 4, B, H1, F, 0);
    // bf16 shadows of the layer-0 outputs the 32x32 bf16 forward tiles of layer 1 read as A
    // (H0 a multiple of 128: every shadow position holds a k < H0; not under the layer norm,
    // which rewrites the actor's layer-0 output after the GEMM)
    h->abf_segs.clear();
    if (h->cfg.gemm_bf16 && !h->deep && (h->wbf_enabled == 1 || h->wbf_enabled == 3))
        for (const char* n : {"ws.Ha1", "ws.Hq1", "ws.Hp1"}) {
            const bool act = std::string(n) == "ws.Ha1";
            const int w = act ? H0 : Hc0;
            if (w % 128 != 0 || (act && h->ln)) continue;
            const auto& sg = h->seg(n);
            h->add(std::string("abf.") + n, sg.rows, w / 2, SACX_U32, SACX_ROLE_WORK);
            h->abf_segs.push_back(n);
        }
    // (config C5) the critics' layer-0 outputs transposed: one image per q.fwd0 problem (t0 t1 q0 q1)
    if (h->xbf == 1) h->add("xbf.ws.Hq1", 4 * (int64_t)Hc0, wbf_ld_of(B) / 2, SACX_U32, SACX_ROLE_WORK);
    // behaviour-policy inference (sacx_actor_act), up to ACT_CAP rows per launch chain
    h->add("act.X", ACT_CAP, h->ldS, F, 0);
    // (sacx_critic_forward's too; the generic plans' nets alternate between the two: any layer's width)
    auto wmax = [&](int n) { return *std::max_element(h->nd[n].h.begin(), h->nd[n].h.end()); };
    h->add("act.H1", ACT_CAP, h->deep ? std::max(wmax(0), wmax(1)) : std::max(H0, Hc0), F, 0);
    h->add("act.H2", ACT_CAP, h->deep ? std::max(wmax(0), wmax(1)) : std::max(H1, Hc1), F, 0);
    h->add("act.noise", 1, (int64_t)ACT_CAP * A, F, 0);
    if (h->ln) {                      // layer-norm caches of the update's actor rows
        h->add("ws.ln_xhat", h->Ra, H0, F, 0);
        h->add("ws.ln_rstd", 1, h->Ra, F, 0);
        h->add("ws.ln_gy", h->Rb, H0, F, 0);
        h->add("ws.ln_gb", h->Rb, H0, F, 0);
    }
    h->add("act.Xq", ACT_CAP, h->ldQ, F, 0);          // sacx_critic_forward input [norm s | norm a]
    h->add("act.Q", ACT_CAP, 1, F, 0);                // sacx_critic_forward output
    if (h->cfg.use_expert) {          // world-model fitting (A16)
        const int R2 = h->nm * h->mb, O = S + 1;
        // the models' output rows: a rollout chunk, or every model on the diagnostics' <= 2048 rows
        const int64_t RR = std::max<int64_t>(ROLL_CAP, (int64_t)h->nm * 2048);
        h->add("mfit.idx", h->mfit_cap, R2, SACX_I32, SACX_ROLE_WORK);
        h->add("ws.gnorm", 1, GNORM_PARTS + 1, F, 0);   // clip_by_global_norm partials + scale
        h->add("mstats", h->stats_cap, 2, F, SACX_ROLE_STATE);
        h->add("ws.Xf", R2, h->ldQ, F, 0);
        h->add("ws.Tf", R2, O, F, 0);
        h->add("mfit.Xs", MFIT_PRE, (int64_t)R2 * h->ldQ, F, 0);   // pre-gathered rows / targets of a block of steps
        h->add("mfit.Ts", MFIT_PRE, (int64_t)R2 * O, F, 0);
        h->add("ws.Hf1", R2, Hm0, F, 0);
        last("ws.Hf2", "ws.Hf1", R2, Hm1, Dm);
        h->add("ws.Of", R2, O, F, 0);
        h->add("ws.Df3", R2, r4(O), F, 0);    // float4 rows: model.bwd2's A operand
        if (Dm >= 2) h->add("ws.Df2", R2, Hm1, F, 0);
        h->add("ws.Df1", R2, Hm0, F, 0);
        if (Dm < 2) last("ws.Df2", "ws.Df1", R2, Hm1, Dm);
        mids.push_back({"ws.Hfm", R2, 2});
        mids.push_back({"ws.Dfm", R2, 2});
        // fit-loss partials (per row: k_mloss); --separate_reward_nn: then one per row of the reward heads
        h->add("ws.lf", 1, (int64_t)R2 * ((O + 15) / 16) + (h->srn ? R2 : 0), F, 0);
        if (h->srn) {                 // the reward nets' fit activations / deltas
            const int Hr0 = h->Hr0, Hr1 = h->Hr1;
            h->add("ws.Hrf1", R2, Hr0, F, 0);
            last("ws.Hrf2", "ws.Hrf1", R2, Hr1, Dr);
            h->add("ws.Drf3", R2, 4, F, 0);         // d loss / d reward (float4 rows)
            if (Dr >= 2) h->add("ws.Drf2", R2, Hr1, F, 0);
            h->add("ws.Drf1", R2, Hr0, F, 0);
            if (Dr < 2) last("ws.Drf2", "ws.Drf1", R2, Hr1, Dr);
            mids.push_back({"ws.Hrfm", R2, 3});
            mids.push_back({"ws.Drfm", R2, 3});
            h->add("roll.R1", RR, h->deep ? wmax(3) : Hr0, F, 0);
            h->add("roll.R2", RR, h->deep ? wmax(3) : Hr1, F, 0);
        }
        if (h->gm) {                  // logstd-gradient partials per model, 16-row tile and column
            h->add("ws.lgp", h->nm * ((h->mb + 15) / 16), S, F, 0);
            h->add("roll.mnoise", 1, RR * S, F, 0);   // exp(logstd) * u noise (sample / step, every model's)
        }
        // model rollout (sacx_rollout), up to ROLL_CAP trajectories per launch chain
        h->add("roll.X", ROLL_CAP, h->ldS, F, 0);
        h->add("roll.H1", ROLL_CAP, h->deep ? wmax(0) : H0, F, 0);
        h->add("roll.H2", ROLL_CAP, h->deep ? wmax(0) : H1, F, 0);
        h->add("roll.noise", 1, (int64_t)ROLL_CAP * A, F, 0);
        h->add("roll.A", ROLL_CAP, A, F, 0);
        h->add("roll.Xm", ROLL_CAP, h->ldQ, F, 0);
        h->add("roll.M1", RR, h->deep ? wmax(2) : Hm0, F, 0);
        h->add("roll.M2", RR, h->deep ? wmax(2) : Hm1, F, 0);
        h->add("roll.O", RR, O, F, 0);
    }
    // the middle hidden layers (1 .. D-2) of nets deeper than two layers: <p>m<i>
    for (const Mid& m : mids)
        for (int i = 1; i + 1 < h->nd[m.net].D(); ++i)
            h->add(m.p + std::to_string(i), m.rows, h->nd[m.net].h[i], F, 0);
    h->arena_bytes = (h->arena_bytes + 255) & ~uint64_t(255);
}

// ---------------------------------------------------------------- GEMM problem helpers
GemmProb prob_fwd(const float* X, int ldx, int M, int K, const float* Wext, int N, float* C, int act) {
    GemmProb p{};
    p.A = X; p.lda = ldx; p.a_kc = 1; p.ones_row = -1;
    p.B = Wext; p.ldb = N; p.b_kc = 0;
    p.M = M; p.N = N; p.K = K;
    p.bias = Wext + (size_t)K * N;
    p.C = C; p.ldc = N;
    p.epi = EPI_FWD; p.act = act;
    return p;
}

// C = (D * W^T) (.) act'(Hprev), W_ext is [(K_in+1) x N_out]; C is [M x K_in]
GemmProb prob_dx(const float* D, int M, int Nout, const float* Wext, int Kin, const float* Hprev, float* C, int act) {
    GemmProb p{};
    p.A = D; p.lda = Nout; p.a_kc = 1; p.ones_row = -1;
    p.B = Wext; p.ldb = Nout; p.b_kc = 1;   // B[k][n] = W[n][k]
    p.M = M; p.N = Kin; p.K = Nout;
    p.H = Hprev; p.ldh = Kin;
    p.C = C; p.ldc = Kin;
    p.epi = EPI_DACT; p.act = act;
    return p;
}

// dW_ext = [X | 1]^T * D over R rows, then Adam (+ Polyak into T)
GemmProb prob_dw(const float* X, int ldx, int Kin, int R, const float* D, int Nout, float* P, float* T, int group) {
    GemmProb p{};
    p.A = X; p.lda = ldx; p.a_kc = 0; p.ones_row = Kin;
    p.B = D; p.ldb = Nout; p.b_kc = 0;
    p.M = Kin + 1; p.N = Nout; p.K = R;
    p.P = P; p.T = T; p.ldp = Nout;
    p.epi = EPI_ADAM; p.group = group; p.grad_scale = 1.f;
    return p;
}

// algorithmic counts (the fused layer 0 counted once, not per column tile)
double gemm_flops(const GemmProb& p) { return 2.0 * p.M * p.N * p.K; }
double gemm_bytes(const GemmProb& p) {
    double b = 4.0 * ((double)p.M * p.K + (double)p.K * p.N + (double)p.M * p.N);
    if (p.epi == EPI_ADAM) b += 4.0 * p.M * p.N * (p.T ? 8 : 6) - 4.0 * p.M * p.N;
    if (p.epi == EPI_DACT) b += 4.0 * p.M * p.N;
    return b;
}

// The bf16 weight shadows of a problem (SACX_WBF): a forward problem on 32x32 tiles reads the
// shadow of its B; a dW + Adam problem stores the shadows of the P and T it updates
void wbf_wire(sacx_handle* h, GemmProb& p, int mode, bool t32) {
    auto find = [&](const float* w) -> const sacx_handle::WbfMat* {
        for (const auto& m : h->wbf_mats)
            if (w != nullptr && w == h->f(m.name)) return &m;
        return nullptr;
    };
    if (mode == GM_FWD && t32) {
        const auto* m = find(p.B);
        if (m && m->K == p.K && m->N == p.N && p.ldb == p.N) {
            p.wbf = h->ptr<uint16_t>("wbf." + m->name);
            p.wbf_ld = wbf_ld_of(m->K);
            p.wbf_per = wbf_per_of(m->K);
        }
        // activations: a plain forward problem whose output lies in a shadowed segment stores its
        // shadow; a layer-1 problem reads A from the shadow when a wired producer of this plan
        // stores every row it reads (ranges recorded in build order: producers come first)
        for (const auto& n : h->abf_segs) {
            const auto& sg = h->seg(n);
            const float* base = h->f(n);
            const float* end = base + (size_t)sg.rows * sg.cols;
            if (p.C && p.C >= base && p.C < end && p.ldc == sg.cols && p.N == sg.cols && p.mse == 0 &&
                p.C + (size_t)p.M * p.ldc <= end) {
                p.obf = h->ptr<uint16_t>("abf." + n) + (p.C - base);
                h->abf_written.push_back({p.C, p.C + (size_t)p.M * p.ldc});
            }
            if (p.A >= base && p.A < end && p.lda == sg.cols && p.K == sg.cols && p.headp == 0) {
                const float* a1 = p.A + (size_t)p.M * p.lda;
                bool covered = false;
                for (const auto& w : h->abf_written) covered = covered || (p.A >= w.first && a1 <= w.second);
                if (covered) p.abf = h->ptr<uint16_t>("abf." + n) + (p.A - base);
            }
        }
    } else if (mode == GM_DW && p.epi == EPI_ADAM) {
        const auto* m = find(p.P);
        if (!m || m->K != p.M - 1 || m->N != p.N || p.ldp != p.N) return;
        p.wbf = h->ptr<uint16_t>("wbf." + m->name);
        p.wbf_ld = wbf_ld_of(m->K);
        p.wbf_per = wbf_per_of(m->K);
        p.wbf_k = m->K;
        if (const auto* t = find(p.T)) p.obf = h->ptr<uint16_t>("wbf." + t->name);
    }
}

AdamConsts adam_consts(const sacx_handle* h) {
    AdamConsts c{};
    c.lr[GRP_Q] = h->cfg.lr_q;
    c.lr[GRP_PI] = h->cfg.lr_pi;
    c.lr[GRP_ALPHA] = h->cfg.lr_alpha;
    c.lr[GRP_MODEL] = h->cfg.lr_model;
    c.tau_keep = (float)(1.0 - (double)h->cfg.tau);
    c.tau_take = h->cfg.tau;
    c.target_update_int = h->cfg.target_update_int;
    return c;
}

void add_gemm(sacx_handle* h, std::vector<Launch>& plan, const std::string& name, std::vector<GemmProb> ps,
              bool record_probs, bool allow_dwl = true) {
    Launch L{};
    L.kind = Launch::GEMM;
    L.name = name;
    // 32x32 workgroup tiles for plain FWD / DX / DW launches when the handle asks for them
    // (packed seeds: many tiles per launch); head-prologue and fused two-layer launches stay 16x16
    // (tile32 = 2: forward / dX launches only -- the dW + Adam epilogue's registers cost occupancy)
    bool t32 = h->tile32 > 0;
    // tile32 = 2 keeps dW + Adam on 16x16 tiles (their registers cost occupancy), except a launch
    // whose 16x16 tiles exceed what is resident at once (5 workgroups on each of 256 CUs): there
    // the last tiles start a whole workgroup time late (Humanoid critic.adam: 1,378 tiles, 11 us
    // of skew in a 23 us launch), and 32x32 tiles -- bit-identical sums -- run in one round
    // (tools/dw_bench.hip: Humanoid critic.adam 23.7 -> 21.0 us fp32, 21.1 -> 14.3 us bf16)
    int tiles16 = 0;
    for (auto& p : ps) tiles16 += ((p.M + 15) / 16) * ((p.N + 15) / 16);
    const bool dw_wide = tiles16 > h->dw_round_tiles;
    for (auto& p : ps)
        t32 = t32 && p.headp == 0 && !(h->tile32 == 2 && p.epi == EPI_ADAM && !dw_wide) && p.hbw == 0;
    // dW + Adam launches with long reductions take k_dwl (32x32 tiles, LDS-DMA staged rows)
    bool dwl = h->dwl > 0 && allow_dwl;   // not where rows ride along (the policy head rows)
    int kmax = 0;
    for (auto& p : ps) {
        dwl = dwl && p.epi == EPI_ADAM;
        kmax = std::max(kmax, (int)p.K);
    }
    dwl = dwl && (h->dwl == 2 || kmax >= 512);
    if (dwl) t32 = false;
    const int ts = (t32 || dwl) ? 32 : 16;
    const int tsn = dwl ? 16 * h->dwl_nh : ts;    // k_dwl: 32 x 16 NH tiles
    int tiles = 0;
    for (auto& p : ps) {
        p.tiles_n = (p.N + tsn - 1) / tsn;
        p.tile_begin = tiles;
        tiles += ((p.M + ts - 1) / ts) * p.tiles_n;
        L.flops += gemm_flops(p);
        L.bytes += gemm_bytes(p);
    }
    L.gemm.t32 = t32 ? 1 : 0;
    // both slot plans address the same (slot-independent) problem table
    L.gemm_first = h->probs_cursor;
    h->probs_cursor += (int)ps.size();
    if (ps.size() > GEMM_MAXP) { fprintf(stderr, "sacx: too many GEMM problems in %s\n", name.c_str()); abort(); }
    // every problem of a launch must share the operand/epilogue mode (k_gemm template)
    auto mode_of = [](const GemmProb& p) {
        return p.epi == EPI_ADAM ? GM_DW : (p.epi == EPI_DACT ? GM_DX : GM_FWD);
    };
    const int mode = mode_of(ps[0]);
    bool vec = false;   // any problem with float4 loads (each problem carries its own flag)
    for (auto& p : ps) {
        // 32-bit buffer offsets: every operand the GEMM reads must stay below 2 GiB
        const double ext = 4.0 * ((double)p.M * p.lda + (double)p.K * p.ldb + p.N);
        if (ext >= 2147483648.0) { fprintf(stderr, "sacx: operand too large in %s\n", name.c_str()); abort(); }
    }
    for (auto& p : ps) {
        if (mode_of(p) != mode) { fprintf(stderr, "sacx: mixed GEMM modes in %s\n", name.c_str()); abort(); }
        const bool akc = p.a_kc != 0, bkc = p.b_kc != 0;
        if (akc != (mode != GM_DW) || bkc != (mode == GM_DX)) { fprintf(stderr, "sacx: bad operand layout in %s\n", name.c_str()); abort(); }
        if (mode == GM_DW && p.bscale == nullptr) p.bscale = h->f("ws.ones");
        // float4 loads along k: a K that is not a multiple of 4 (S+A = 23, 393; S = 17) still
        // qualifies when the row stride holds round4(K) (the zero pad columns of the staging
        // slabs): the over-read elements meet B values that load_b zeroes past K
        const int64_t k4 = r4(p.K);
        const bool v_a = (p.lda % 4 == 0) && (k4 <= p.lda) && ((((uintptr_t)p.A) & 15) == 0) &&
                         ((((uintptr_t)p.wgen) & 15) == 0);
        // dX: B = W_ext rows (n < N = K_in, so a row's float4 over-read past K stays inside W_ext: the
        // bias row follows the last); rows at any 4-B offset with h->unaligned_b (dword-aligned 16-B
        // buffer loads), whose elements past K meet A's zero pad (A rows are 16-B aligned)
        const bool b_al = (p.ldb % 4 == 0) && (k4 <= p.ldb) && ((((uintptr_t)p.B) & 15) == 0);
        const bool v_b = mode == GM_DX ? (b_al || (h->unaligned_b && (((uintptr_t)p.B) & 3) == 0)) : true;
        p.vec = (mode != GM_DW && v_a && v_b && p.K >= 4) ? 1 : 0;
        vec = vec || p.vec;
    }
    if (h->wbf_attach && h->cfg.gemm_bf16)
        for (auto& p : ps) wbf_wire(h, p, mode, t32);
    if (dwl) {
        // 16-B row pieces need 16-B aligned rows in every seed's arena block
        const bool sa = h->seeds <= 1 || h->seed_bytes % 16 == 0;
        for (auto& p : ps) {
            const bool a4 = sa && p.lda >= 4 && p.lda % 4 == 0 && (((uintptr_t)p.A) & 15) == 0;
            const bool b4 = sa && p.ldb >= 4 && p.ldb % 4 == 0 && (((uintptr_t)p.B) & 15) == 0;
            p.vec = (a4 ? 1 : 0) | (b4 ? 2 : 0);
        }
    }
    // forward launches with world-model head rows (mse epilogues) take their own variant (rowk 8),
    // so the others do not hold the mse operands in registers
    for (auto& p : ps)
        if (mode == GM_FWD && p.mse) L.gemm.rowk = 8;
    if (record_probs) h->probs.insert(h->probs.end(), ps.begin(), ps.end());
    L.gemm.dwl = dwl ? (h->dwl_nh == 1 ? 2 : 1) : 0;    // 2: 32x16 tiles, 1: 32x32
    L.gemm.mode = mode;
    L.gemm.vec = vec ? 1 : 0;
    for (size_t i = 0; i < ps.size(); ++i) L.gemm.probs[i] = ps[i];
    L.gemm.nprob = (int)ps.size();
    L.gemm.total_tiles = tiles;
    L.gemm.xcd_map = h->xcd_map;
    L.gemm.bf16 = h->cfg.gemm_bf16 != 0;
    L.gemm.p_stride = h->p_stride;
    L.gemm.ctl = h->ctl();
    L.gemm.adam = adam_consts(h);
    L.grid = tiles;
    plan.push_back(L);
}

// Appends the problems of GEMM launch `b` to launch `a` (same mode; tile ranges follow a's).
// Replaces the plan's last two launches -- the layers 0 and 1 of the same nets, as add_gemm built
// them -- by one k_fwd2 launch (GM_FWD2) when the pair qualifies: fp32, one seed, 16x16 tiles, plain
// forward problems (layer 1 optionally with the actor head's partial dots, rowk 5), at most 4 nets,
// K0 <= 32, H0 a multiple of 64 up to 256, layer 1 reading exactly layer 0's output.  Returns
// whether it fused.
bool fuse_fwd2(sacx_handle* h, std::vector<Launch>& plan, const std::string& name) {
    if (plan.size() < 2) return false;
    Launch& L0 = plan[plan.size() - 2];
    Launch& L1 = plan[plan.size() - 1];
    const GemmArgs &a0 = L0.gemm, &a1 = L1.gemm;
    if (L0.kind != Launch::GEMM || L1.kind != Launch::GEMM || a0.mode != GM_FWD || a1.mode != GM_FWD) return false;
    if (a0.t32 || a1.t32 || a0.dwl || a1.dwl || a0.bf16 || a0.nseeds > 1 || h->seeds > 1) return false;
    // layer 0 may carry the actor head (rowk 3: target tile prologues from the head's partial dots,
    // which keep the prologue free of barriers, and head rows as extra workgroups)
    const bool head = a0.rowk == 3;
    // or layer 0 gathers its rows from the replay ring (rowk 6: the world-model fit's model.fwd0), or
    // reads them pre-gathered (rowk 9): the fit's layer 0, up to 512 wide
    const bool gather = a0.rowk == 6 || a0.rowk == 9;
    if ((a0.rowk != 0 && !head && !gather) || (a1.rowk != 0 && a1.rowk != 5) || ((head || gather) && a1.rowk != 0) ||
        a0.has_final || a1.has_final || a0.nprob != a1.nprob || a0.nprob > 4)
        return false;
    if (head && (a0.head.part == nullptr || a0.head.H1 > 256 || a0.head.A > 16)) return false;
    bool vec = true;
    for (int i = 0; i < a0.nprob; ++i) {
        const GemmProb &p0 = a0.probs[i], &p1 = a1.probs[i];
        if (p0.mse || p1.mse || (p0.headp && !head) || p1.headp || p0.K > 32 || p0.N % 64 != 0 ||
            p0.N > (gather ? 512 : 256) ||
            p1.K != p0.N || p1.A != p0.C || p1.lda != p0.ldc || p1.M != p0.M || p1.N % 16 != 0)
            return false;
        vec = vec && p0.vec;
    }
    Launch F = L1;
    F.name = name;
    GemmArgs& g = F.gemm;
    const int n = a0.nprob;
    int tiles = 0;
    for (int i = 0; i < n; ++i) {
        g.probs[i] = a0.probs[i];
        GemmProb q = a1.probs[i];
        q.tiles_n = (q.N + 63) / 64;
        q.tile_begin = tiles;
        tiles += ((q.M + 15) / 16) * q.tiles_n;
        g.probs[n + i] = q;
    }
    g.nprob = 2 * n;
    g.mode = GM_FWD2;
    g.vec = vec ? 1 : 0;
    g.total_tiles = tiles;
    g.rowk = head ? 3 : gather ? a0.rowk : a1.rowk;
    if (a0.rowk == 6) g.mg = a0.mg;
    if (head) {
        g.head = a0.head;
        g.hfin = a0.hfin;
        g.head_block0 = a0.head_block0;
    }
    if (head && a0.row_blocks != 0) return false;   // plain SAC: the head rows come with merged_body only
    g.row_blocks = 0;
    F.grid = tiles;
    F.frees_slot = L0.frees_slot || L1.frees_slot;
    F.block = head ? SACX_FWD2_HEAD_NW * 64 : 1024;     // k_fwd2 waves (16; the fit's gather variant too)
    F.flops = L0.flops + L1.flops;
    F.bytes = L0.bytes + L1.bytes;
    F.gemm_first = L0.gemm_first;
    plan.pop_back();
    plan.pop_back();
    plan.push_back(F);
    return true;
}

bool merge_gemm(GemmArgs& a, const GemmArgs& b) {
    if (a.mode == GM_FWD2 || b.mode == GM_FWD2) {
        // two k_fwd2 launches: layer-0 problems, then layer-1 problems, each launch's in order
        const int na = a.nprob / 2, nb = b.nprob / 2;
        if (a.mode != b.mode || na + nb > 4 || a.vec != b.vec) return false;
        GemmProb l0[4], l1[4];
        for (int i = 0; i < na; ++i) { l0[i] = a.probs[i]; l1[i] = a.probs[na + i]; }
        for (int i = 0; i < nb; ++i) {
            l0[na + i] = b.probs[i];
            l1[na + i] = b.probs[nb + i];
            l1[na + i].tile_begin += a.total_tiles;
        }
        for (int i = 0; i < na + nb; ++i) { a.probs[i] = l0[i]; a.probs[na + nb + i] = l1[i]; }
        a.nprob = 2 * (na + nb);
        a.total_tiles += b.total_tiles;
        if (b.rowk == 5) a.rowk = 5;           // head partials: per problem (ppart null or not)
        return true;
    }
    if (a.mode != b.mode || a.t32 != b.t32 || a.dwl != b.dwl || a.nprob + b.nprob > GEMM_MAXP) return false;
    for (int i = 0; i < b.nprob; ++i) {
        GemmProb p = b.probs[i];
        p.tile_begin += a.total_tiles;
        a.probs[a.nprob + i] = p;
    }
    a.nprob += b.nprob;
    a.total_tiles += b.total_tiles;
    a.vec = a.vec || b.vec;
    if (b.rowk == 8) {             // world-model head rows: the forward variant with mse operands
        if (a.rowk != 0 && a.rowk != 8) return false;
        a.rowk = 8;
    }
    return true;
}

// Packed seeds: every launch of an update plan runs all seeds (grid z), relocating its
// seed-0 arena pointers by blockIdx.z * seed_bytes.
void pack_seeds(Launch& L, int64_t stride, int n) {
    L.rng.sstride = L.gather.sstride = L.gemm.sstride = L.head.sstride = L.fin.sstride = L.qh.sstride =
        L.ab.sstride = stride;
    L.rng.nseeds = L.gather.nseeds = L.gemm.nseeds = L.head.nseeds = L.fin.nseeds = L.qh.nseeds = L.ab.nseeds = n;
    L.ln.sstride = stride;
    L.ln.nseeds = n;
}

// Data-parallel mode: the dW launch `L` stores its local gradients (+3 p_stride) instead of
// running Adam; RCCL sums the contiguous gradient range [first, last] over the ranks and
// k_adam_apply runs the Adam (and Polyak into the same range at `targ`) with scale 1/ranks.
void dp_split_adam(sacx_handle* h, std::vector<Launch>& plan, const std::string& first, const std::string& last,
                   const std::string& targ, int group, int nlaunch = 1) {
    std::string base;
    for (int j = 0; j < nlaunch; ++j) {        // the last nlaunch dW launches (add_gemm_split's)
        Launch& G = plan[plan.size() - 1 - j];
        for (int i = 0; i < G.gemm.nprob; ++i) G.gemm.probs[i].epi = EPI_STORE;
        base = G.name.substr(0, G.name.find(".adam"));
        G.name = base + ".grad" + G.name.substr(G.name.find(".adam") + 5);
    }
    const AdamConsts gadam = adam_consts(h);
    const uint64_t o0 = h->off_of(first);
    const SegInfo& sl = h->seg(last);
    const int64_t n = (int64_t)((sl.off + (uint64_t)(sl.rows * sl.cols) * 4 - o0) / 4);
    float* P = h->f(first);
    Launch R{};
    R.kind = Launch::ALLREDUCE;
    R.name = base + ".allreduce";
    R.ar_buf = P + 3 * h->p_stride;
    R.ar_count = n;
    R.grid = 0;
    R.bytes = 8.0 * n;
    plan.push_back(R);
    Launch U{};
    U.kind = Launch::APPLY;
    U.name = base + ".adam";
    AdamApplyArgs& a = U.ap;
    a.P = P; a.n = n; a.p_stride = h->p_stride; a.group = group;
    a.t_off = targ.empty() ? 0 : (int64_t)(h->off_of(targ) - o0) / 4;
    a.grad_scale = (float)(1.0 / (double)h->dp_ranks);
    a.ctl = h->ctl();
    a.adam = gadam;
    U.grid = (int)((n + 255) / 256);
    U.bytes = 4.0 * n * (targ.empty() ? 7 : 9);
    plan.push_back(U);
}

// The update's inputs in slot `slot`: the sampler (randint + every normal of the update,
// buffers.py:136, continuous_actors.py:351) and the gather of the replay / expert rows into the
// normalised staging slabs (buffers.py:137-141, normalizer.py:36-41).  Every plan starts with them.
void plan_inputs(sacx_handle* h, std::vector<Launch>& plan, int slot) {
    const int S = h->S, A = h->A, B = h->B, ne = h->ne;
    const int ldS = h->ldS, ldQ = h->ldQ;
    const std::string sl = "slot" + std::to_string(slot);
    auto W = [&](const std::string& n) { return h->f(n); };
    int32_t* idx = h->ptr<int32_t>(sl + ".idx");
    float* noise = h->f(sl + ".noise");
    float *Xa = W(sl + ".Xa"), *Xq = W(sl + ".Xq"), *Xt = W(sl + ".Xt"), *Xp = W(sl + ".Xp"), *Xm = W(sl + ".Xm");
    float *r_in = W(sl + ".r"), *d_in = W(sl + ".d"), *se_raw = W(sl + ".se_raw"), *spe_raw = W(sl + ".spe_raw");
    // ---- sampler
    {
        Launch L{};
        L.kind = Launch::RNG;
        L.name = "rng";
        L.rng.st = h->ptr<RngState>("rng");
        L.rng.ctl = h->ctl();
        L.rng.n_int = B;
        L.rng.n_norm = h->n_norm;
        L.rng.out_idx = idx;
        L.rng.out_norm = noise;
        L.rng.slot = slot;
        L.rng.reset_seq = 1;   // cleared for the chained launches of a captured graph
        L.rng.nupd = 1;
        L.rng.slot_bytes = h->slot_bytes;
        if (h->rng_split) {
            L.rng.pairs = h->ptr<uint32_t>("rng.pairs");
            L.rng.pairs_oi = h->ptr<int32_t>("rng.pairs_oi");
            L.rng.pcap = h->pcap;
        }
        if (h->rng_jump) {
            L.rng.jw = h->ptr<uint32_t>("rng.jw");
            L.rng.jc = h->ptr<uint32_t>("rng.jc");
            L.rng.jL = h->jL;
            L.rng.jsmax = h->jsmax;
            L.rng.junder = h->mtj_under;
        }
        L.grid = 1;
        L.block = 1024;
        L.bytes = 4.0 * (B + h->n_norm) + 2.0 * sizeof(RngState);
        plan.push_back(L);
    }
    // ---- gather
    {
        Launch L{};
        L.kind = Launch::GATHER;
        L.name = "gather";
        GatherArgs& g = L.gather;
        g.replay = W("replay"); g.cap = h->cap; g.stride = h->stride;
        g.S = S; g.A = A; g.B = B; g.ne = ne; g.idx = idx; g.ctl = h->ctl();
        g.s_mean = W("norm.s_mean"); g.s_den = W("norm.s_den");
        g.a_mean = W("norm.a_mean"); g.a_den = W("norm.a_den");
        g.ms_mean = W(mnorm(h, "s_mean")); g.ms_den = W(mnorm(h, "s_den"));
        g.Xa = Xa; g.ldS = ldS; g.Xq = Xq; g.Xt = Xt; g.Xp = Xp; g.Xm = Xm; g.ldQ = ldQ;
        g.r = r_in; g.d = d_in; g.slot = slot; g.nupd = 1; g.slot_bytes = h->slot_bytes;
        g.exp_s = W("expert.s"); g.exp_sp = W("expert.sp");
        g.perm_ring = h->nm == 1 ? nullptr : h->ptr<int32_t>("perm"); g.perm_cap = h->perm_cap;
        g.perm_ld = h->ne_perm;
        g.se_raw = se_raw; g.spe_raw = spe_raw;
        L.grid = (B + ne + 3) / 4;
        L.bytes = 4.0 * (B * (2.0 * S + A + 2) + ne * 2.0 * S) + 4.0 * (B * (2.0 * ldS + 3.0 * ldQ + 2));
        plan.push_back(L);
    }
}

// alpha.final (k_alpha_final: the alpha loss / Adam / clamp, SAC_expert.py:340-356, and the update's
// statistics row) behind the alpha.head launch that ends `plan`; in the data-parallel mode the local
// alpha gradient, its all-reduce and k_alpha_apply
void plan_alpha_final(sacx_handle* h, std::vector<Launch>& plan, int nm) {
    const int B = h->B, ne = h->ne, S = h->S;
    const bool eo = h->cfg.use_expert != 0;
    auto W = [&](const std::string& n) { return h->f(n); };
    {
        const Launch& AH = plan.back();
        Launch L{};
        L.kind = Launch::FINAL;
        L.name = "alpha.final";
        FinalArgs& f = L.fin;
        f.nred = AH.grid;
        f.alpha = W("alpha"); f.alpha_m = f.alpha + h->p_stride; f.alpha_v = f.alpha + 2 * h->p_stride;
        f.ctl = h->ctl();
        f.adam = adam_consts(h);
        f.target_entropy = h->cfg.target_entropy;
        f.B = B; f.ne = ne; f.use_expert = eo; f.nm = nm;
        f.lq = W("ws.lq"); f.lp = W("ws.lp"); f.mse_rows = W("ws.mse"); f.red = W("red");
        f.mse_tiles = (S + 15) / 16;
        f.stats = W("stats"); f.stats_cap = h->stats_cap;
        L.grid = 1;
        L.block = 64;
        L.bytes = 4.0 * (f.nred + 3.0 * B + ne);
        if (h->dp_ranks > 0) {              // alpha gradient: local -> all-reduce -> Adam + counters
            f.alpha_g = W("alpha") + 3 * h->p_stride;
            f.grad_scale = (float)(1.0 / (double)h->dp_ranks);
            L.name = "alpha.grad";
            plan.push_back(L);
            Launch R{};
            R.kind = Launch::ALLREDUCE;
            R.name = "alpha.allreduce";
            R.ar_buf = f.alpha_g;
            R.ar_count = 1;
            plan.push_back(R);
            Launch U{};
            U.kind = Launch::AAPPLY;
            U.name = "alpha.adam";
            U.fin = f;
            U.grid = 1;
            U.block = 64;
            plan.push_back(U);
        } else {
            plan.push_back(L);
        }
    }
}

// Config C5: the bf16 32x32 dW + Adam problems whose X is the slot's critic rows (Xq) or a critic's
// layer-0 output (ws.Hq1, written by a bf16 32x32 forward problem earlier in the plan) read X^T
// from a transposed image instead (GemmProb::abf); its producer -- k_gather (xbfq) or that
// forward problem's epilogue (tbf) -- is told to write it.  Bit-identical: the image holds the
// bf16 values the converting loads make, in the order they pack them.
void xbf_wire(sacx_handle* h, std::vector<Launch>& plan, int slot) {
    if (!h->xbf || !h->wbf_attach) return;
    const int S = h->S, A = h->A, B = h->B, Hc0 = h->Hc0, ld = wbf_ld_of(B);
    const std::string sl = "slot" + std::to_string(slot);
    const float* Xq = h->f(sl + ".Xq");
    const float* Hq1 = h->f("ws.Hq1");
    Launch* gather = nullptr;
    for (Launch& L : plan)
        if (L.kind == Launch::GATHER) gather = &L;
    for (size_t i = 0; i < plan.size(); ++i) {
        Launch& L = plan[i];
        if (L.kind != Launch::GEMM || L.gemm.mode != GM_DW || !L.gemm.t32 || L.gemm.dwl || !L.gemm.bf16) continue;
        for (int j = 0; j < L.gemm.nprob; ++j) {
            GemmProb& p = L.gemm.probs[j];
            if (p.K != B || p.a_kc != 0) continue;
            if (p.A == Xq && p.ones_row == S + A && gather != nullptr) {
                p.abf = h->ptr<uint16_t>(sl + ".xbfq");
                gather->gather.xbfq = h->ptr<uint16_t>(sl + ".xbfq");
                continue;
            }
            const int64_t d = p.A - Hq1;
            if (h->xbf != 1 || d < 0 || d % ((int64_t)B * Hc0) != 0 || d / ((int64_t)B * Hc0) >= 4 || p.lda != Hc0 || p.ones_row != Hc0)
                continue;
            uint16_t* img = h->ptr<uint16_t>("xbf.ws.Hq1") + (size_t)(d / ((int64_t)B * Hc0)) * Hc0 * ld;
            for (size_t q = 0; q < i && p.abf == nullptr; ++q) {
                Launch& F = plan[q];
                if (F.kind != Launch::GEMM || F.gemm.mode != GM_FWD || !F.gemm.t32 || !F.gemm.bf16 || F.gemm.rowk != 0) continue;
                for (int c = 0; c < F.gemm.nprob; ++c) {
                    GemmProb& f = F.gemm.probs[c];
                    if (f.C == p.A && f.M == B && f.N == Hc0 && f.ldc == Hc0 && f.mse == 0 && f.ppart == nullptr) {
                        f.tbf = img;
                        p.abf = img;
                    }
                }
            }
        }
    }
}

void build_plan(sacx_handle* h, int slot, bool record_probs) {
    std::vector<Launch>& plan = h->plan[slot];
    plan.clear();
    h->probs_cursor = 0;
    const int S = h->S, A = h->A, H0 = h->H0, H1 = h->H1, B = h->B, ne = h->ne, Aout = h->Aout;
    const int Hm0 = h->Hm0, Hm1 = h->Hm1, half = ne / 2;
    const int Hc0 = h->Hc0, Hc1 = h->Hc1;   // the critics' hidden sizes (--critic_layers; H0 / H1: the actor's)
    // expert rows of world model k: [k * half, (k + 1) * half) with 2 or more models (the expert term
    // takes models 0 and 1, SAC_expert.py:325-326), all with one
    const int nm = std::min(h->nm, 2), mrows = nm == 1 ? ne : half;
    const int ldS = h->ldS, ldQ = h->ldQ;
    const int a0 = h->aact[0], a1 = h->aact[1], c0 = h->cact[0], c1 = h->cact[1], m0 = h->macts[0], m1 = h->macts[1];
    const bool eo = h->cfg.use_expert != 0;
    const std::string sl = "slot" + std::to_string(slot);
    float* noise = h->f(sl + ".noise");
    float* noise_t = noise;
    float* noise_pi = noise + (size_t)B * A;
    float* noise_e = noise + (size_t)2 * B * A;
    float* noise_al = noise + (size_t)(2 * B + ne) * A;
    auto W = [&](const std::string& n) { return h->f(n); };
    float *Xa = W(sl + ".Xa"), *Xq = W(sl + ".Xq"), *Xt = W(sl + ".Xt"), *Xp = W(sl + ".Xp"), *Xm = W(sl + ".Xm");
    float *r_in = W(sl + ".r"), *d_in = W(sl + ".d"), *se_raw = W(sl + ".se_raw"), *spe_raw = W(sl + ".spe_raw");
    float *Ha1 = W("ws.Ha1"), *Ha2 = W("ws.Ha2");
    float *Hq1 = W("ws.Hq1"), *Hq2 = W("ws.Hq2"), *Dq1 = W("ws.Dq1"), *Dq2 = W("ws.Dq2");
    float *Hp1 = W("ws.Hp1"), *Hp2 = W("ws.Hp2"), *Dp1 = W("ws.Dp1");
    float *Hm1b = W("ws.Hm1"), *Hm2b = W("ws.Hm2"), *Dm1 = W("ws.Dm1"), *Dm2 = W("ws.Dm2");
    float *Da1 = W("ws.Da1"), *Da2 = W("ws.Da2"), *Da3 = W("ws.Da3"), *E = W("ws.E");
    float *Hl1 = W("ws.Hl1"), *Hl2 = W("ws.Hl2");
    const char* qn[4] = {"t0", "t1", "q0", "q1"};

    plan_inputs(h, plan, slot);
    // ---- actor forward on [sp ; s ; s_e]
    // the two forward layers of a net as two launches (a fused two-layer tile recomputing
    // layer 0 per column tile measured slower once the alpha branch and the heads share
    // launches: 12.06k vs 12.33k updates/s)
    auto fwd_pair = [&](const std::string& name, const std::vector<GemmProb>& p0, const std::vector<GemmProb>& p1) {
        add_gemm(h, plan, name + "0", p0, record_probs);
        add_gemm(h, plan, name + "1", p1, record_probs);
    };
    // the same pair as ONE k_fwd2 launch where it qualifies (fuse_fwd2), else the two launches
    auto fwd_pair2 = [&](const std::string& name, const std::vector<GemmProb>& p0, const std::vector<GemmProb>& p1) {
        fwd_pair(name, p0, p1);
        if (h->fwd2) fuse_fwd2(h, plan, name + "01");
    };
    const int Ra4 = (h->Ra + 3) & ~3;       // first row of the alpha rows (ws.Hl1 / ws.Hl2 alias Ha1 / Ha2)
    // --actor_layer_norm: layer 0 writes the pre-norm Z, k_ln turns it into tanh(LN(Z)) in place
    auto ln_fwd = [&](const std::string& name, int r0, int r1) {
        Launch L{};
        L.kind = Launch::LNORM;
        L.name = name;
        LNArgs& a = L.ln;
        a.mode = 0; a.H = H0; a.Z = Ha1; a.nrange = 1; a.r[0] = r0; a.r[1] = r1;
        a.gamma = W("actor.ln"); a.xhat = W("ws.ln_xhat"); a.rstd = W("ws.ln_rstd"); a.cache_rows = h->Ra;
        L.grid = (r1 - r0 + 3) / 4;
        L.flops = 8.0 * (r1 - r0) * H0;
        L.bytes = 4.0 * (r1 - r0) * H0 * 3;
        plan.push_back(L);
    };
    // actor.fwd1 writes the head's Ha2 . W3 as per-column-tile partials (rowk 5), so the head
    // rows and the target-tile prologues sum 16 values per output instead of re-reading Ha2
    // rows.  SACX_HEAD_PART=0 keeps the row dots (A/B measurement).
    const char* hpe = std::getenv("SACX_HEAD_PART");
    const int tqh = (H1 + 15) / 16;
    const bool head_part = Aout <= 8 && H1 <= 256 && H1 % 64 == 0 &&
                           (hpe ? std::atoi(hpe) != 0 : h->tile32_plan == 0);
    float* hpart = W("ws.hpart");
    // layer 1 of the actor on `rows` rows from row r0 of Ha1 / Ha2 (+ the head partials)
    auto actor_fwd1 = [&](int r0, int rows) {
        GemmProb p = prob_fwd(Ha1 + (size_t)r0 * H0, H0, rows, H0, W("actor.l1"), H1, Ha2 + (size_t)r0 * H1, a1);
        if (head_part) {
            p.pw = W("actor.l2"); p.pw_ld = 1; p.pw_cs = Aout; p.pw_n = Aout;   // W3[n][o] at n * Aout + o
            p.ppart = hpart + (size_t)r0 * Aout * tqh;
        }
        return p;
    };
    auto mark_part = [&]() { if (head_part) plan.back().gemm.rowk = 5; };
    if (h->ln) {
        add_gemm(h, plan, "actor.fwd0", {prob_fwd(Xa, ldS, h->Ra, S, W("actor.l0"), H0, Ha1, ACT_NONE)}, record_probs);
        ln_fwd("actor.ln", 0, h->Ra);
        add_gemm(h, plan, "actor.fwd1", {actor_fwd1(0, h->Ra)}, record_probs);
        mark_part();
    } else {
        fwd_pair("actor.fwd", {prob_fwd(Xa, ldS, h->Ra, S, W("actor.l0"), H0, Ha1, a0)}, {actor_fwd1(0, h->Ra)});
        mark_part();
        if (h->fwd2) fuse_fwd2(h, plan, "actor.fwd01");
    }
    // actor.head folded into q.fwd0 (plain SAC): the target tiles compute their rows' actions
    // in a prologue, the policy rows (and the previous update's alpha rows) run as extra
    // workgroups of the same launch.  SACX_FUSE_HEAD=0 keeps the separate launch.
    const char* fh = std::getenv("SACX_FUSE_HEAD");
    // Packed seeds (>= 4) keep the separate launch: the prologue recomputes each tile's 16 rows
    // once per column tile, which a full GPU of seeds pays for (measured 34.3k vs 31.6k updates/s
    // at 8 seeds); one seed gains the launch it saves.
    // SAC-EO as well: the expert rows (sample -> the world models' inputs Xm) ride as row
    // workgroups of q.fwd0, and the models' forward shifts one launch later (layer 0 in q.fwd1,
    // layer 1 in pi.q.fwd0, the MSE head in pi.q.fwd1)
    const bool fuse_head = Aout <= 16 && S + A <= 64 && H1 % 16 == 0 && H1 <= 512 &&
                           (fh ? std::atoi(fh) != 0 : h->plan_seeds < 4);
    HeadArgs head_fused{};
    // actor.head.bwd folded into actor.bwd1 (plain SAC; the expert rows' model gradients keep
    // the row kernel): pi.q.bwd1 writes per-tile partial action gradients, actor.bwd1's tiles
    // finish them.  SACX_FOLD_HBW=0 keeps the separate launch (A/B measurement).
    const char* fhb = std::getenv("SACX_FOLD_HBW");
    const int tq = (Hc0 + 15) / 16;        // action-gradient partials per row (the critics' layer-0 tiles)
    // The folded launch itself keeps 16x16 tiles (its prologue and generated A operand); the
    // partial-writing launches may take 32x32 tiles.  On 32x32 (packed) plans both folds are off
    // by default: there the launches are bound by workgroup residency, not by their number, and
    // the folds' extra work loses (HC 8 seeds, A/B x2: both on 42.3k, hbw fold only 43.4k, head
    // partials only 43.1k, both off 43.9k updates/s; tools/pk_ab.sh).
    const bool fold_hbw = Aout <= 8 && H1 <= 256 && H1 % 16 == 0 && Hc0 <= 256 && Hc0 % 64 == 0 &&
                          (!eo || (Hm0 <= 512 && Hm0 % 64 == 0)) &&
                          (fhb ? std::atoi(fhb) != 0 : h->tile32_plan == 0);
    // ---- actor head
    if (fuse_head) {
        HeadArgs& a = head_fused;
        a.H2 = Ha2; a.ldh = H1; a.W3 = W("actor.l2"); a.logstd = W("actor.logstd");
        a.part = head_part ? hpart : nullptr; a.tq = tqh;
        a.H1 = H1; a.A = A; a.Aout = Aout; a.S = S; a.ldQ = ldQ; a.per_state_std = h->cfg.per_state_std;
        a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
        a.ma_mean = W(mnorm(h, "a_mean")); a.ma_den = W(mnorm(h, "a_den"));
        // q.fwd0 carries the target rows (tile prologues) and, folded, the previous update's
        // alpha rows; the policy rows ride as extra workgroups of critic.adam (policy_head)
        a.nseg = 1;
        a.seg[0] = {0, B, 0, 0, noise_t, nullptr, W("ws.nlp_t")};
        // total_rows = Ra: merged_body appends the previous update's alpha rows at round4(Ra),
        // where their layer-2 outputs live (ws.Hl2 aliases Ha2 from row round4(Ra))
        a.total_rows = h->Ra;
        a.cache_row0 = 1 << 30;             // no backward cache from these rows (target, alpha)
        a.cache_row1 = 1 << 30;
        if (eo) {                           // SAC-EO expert rows: sample() into Xm, cached
            a.nseg = 2;
            a.seg[1] = {2 * B, 2 * B + ne, 1, 0, noise_e, Xm, nullptr};
            a.cache_row0 = B;
            a.cache_row1 = h->Ra;
        }
        a.c_t = W("ws.c_t"); a.c_std = W("ws.c_std"); a.c_u = W("ws.c_u"); a.c_mask = W("ws.c_mask");
        a.alpha_mode = 0;
    } else {
        Launch L{};
        L.kind = Launch::AHEAD;
        L.name = "actor.head";
        L.frees_slot = true;
        HeadArgs& a = L.head;
        a.H2 = Ha2; a.ldh = H1; a.W3 = W("actor.l2"); a.logstd = W("actor.logstd");
        a.part = head_part ? hpart : nullptr; a.tq = tqh;
        a.H1 = H1; a.A = A; a.Aout = Aout; a.S = S; a.ldQ = ldQ; a.per_state_std = h->cfg.per_state_std;
        a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
        a.ma_mean = W(mnorm(h, "a_mean")); a.ma_den = W(mnorm(h, "a_den"));
        a.nseg = eo ? 3 : 2;
        a.seg[0] = {0, B, 0, 0, noise_t, Xt, W("ws.nlp_t")};
        a.seg[1] = {B, 2 * B, 0, 0, noise_pi, Xp, W("ws.nlp_p")};
        a.seg[2] = {2 * B, 2 * B + ne, 1, 0, noise_e, Xm, nullptr};
        a.total_rows = h->Ra;
        a.cache_row0 = B;
        a.cache_row1 = h->Ra;
        a.c_t = W("ws.c_t"); a.c_std = W("ws.c_std"); a.c_u = W("ws.c_u"); a.c_mask = W("ws.c_mask");
        a.alpha_mode = 0;
        L.grid = (h->Ra + 3) / 4;
        L.flops = 2.0 * h->Ra * H1 * Aout;
        L.bytes = 4.0 * h->Ra * (H1 + 6.0 * A);
        plan.push_back(L);
    }
    // ---- target / critic / model forward
    if (fuse_head) {
        std::vector<GemmProb> p0, p1;
        for (int k = 0; k < 4; ++k) {
            const std::string n = qn[k];
            GemmProb q0 = prob_fwd(k < 2 ? Xt : Xq, ldQ, B, S + A, W(n + ".l0"), Hc0, Hq1 + (size_t)k * B * Hc0, c0);
            q0.headp = k < 2;
            GemmProb q1 = prob_fwd(Hq1 + (size_t)k * B * Hc0, Hc0, B, Hc0, W(n + ".l1"), Hc1, Hq2 + (size_t)k * B * Hc1, c1);
            p0.push_back(q0);
            p1.push_back(q1);
        }
        add_gemm(h, plan, "q.fwd0+actor.head", p0, record_probs);
        Launch& L = plan.back();
        L.gemm.rowk = 3;
        L.gemm.head = head_fused;
        L.gemm.head_block0 = eo ? (2 * B) / 4 : ((h->Ra + 3) & ~3) / 4;
        L.gemm.row_blocks = eo ? (h->Ra + 3) / 4 - (2 * B) / 4 : 0;   // + the alpha rows (merged_body)
        L.grid += L.gemm.row_blocks;
        L.flops += 2.0 * B * H1 * Aout;
        L.bytes += 4.0 * B * (H1 + 6.0 * A);
        L.frees_slot = true;
        if (eo) {                           // the models' layer 0 on Xm (written by the rows above)
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                p1.push_back(prob_fwd(Xm + (size_t)k * half * ldQ, ldQ, mrows, S + A, W(n + ".l0"), Hm0,
                                      Hm1b + (size_t)k * half * Hm0, m0));
            }
        }
        add_gemm(h, plan, "q.fwd1", p1, record_probs);
        if (h->fwd2 && !eo) fuse_fwd2(h, plan, "q.fwd01+actor.head");
    } else {
        std::vector<GemmProb> p0, p1;
        for (int k = 0; k < 4; ++k) {
            const std::string n = qn[k];
            p0.push_back(prob_fwd(k < 2 ? Xt : Xq, ldQ, B, S + A, W(n + ".l0"), Hc0, Hq1 + (size_t)k * B * Hc0, c0));
            p1.push_back(prob_fwd(Hq1 + (size_t)k * B * Hc0, Hc0, B, Hc0, W(n + ".l1"), Hc1, Hq2 + (size_t)k * B * Hc1, c1));
        }
        if (eo) {
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                p0.push_back(prob_fwd(Xm + (size_t)k * half * ldQ, ldQ, mrows, S + A, W(n + ".l0"), Hm0,
                                      Hm1b + (size_t)k * half * Hm0, m0));
                p1.push_back(prob_fwd(Hm1b + (size_t)k * half * Hm0, Hm0, mrows, Hm0, W(n + ".l1"), Hm1,
                                      Hm2b + (size_t)k * half * Hm1, m1));
            }
        }
        fwd_pair("q.fwd", p0, p1);
    }
    // ---- critic backward.  By linearity Dq1 = g (.) M1 with M1 = ((w3 (.) act'(Hq2)) Wq1^T) (.) act'(Hq1)
    // independent of the per-row loss gradient g, so the dX GEMM (A generated from Hq2 and w3)
    // shares one launch with the q.head rows (target, g, loss rows, Dq2, expert MSE + Dm2), and
    // critic.adam applies g to layer 0 (row-scaled B).
    {
        QHeadArgs q{};
        q.mode = 0; q.B = B; q.H1 = Hc1; q.H2 = Hq2;
        for (int k = 0; k < 4; ++k) q.W3[k] = W(std::string(qn[k]) + ".l2");
        q.act = c1; q.D2 = Dq2; q.g = W("ws.gq"); q.loss_rows = W("ws.lq");
        q.alpha = W("alpha"); q.nlp = W("ws.nlp_t"); q.r = r_in; q.d = d_in;
        q.gamma = h->cfg.gamma; q.ret_den = W("norm.ret_den"); q.w_sac = 1.f;
        // the SAC-EO world-model head on the expert rows runs as GEMM problems (mse epilogue)
        // in the pi.q.fwd0 launch, not as rows here
        q.ne = 0; q.ctl = h->ctl();
        std::vector<GemmProb> pb;
        for (int k = 0; k < 2; ++k) {
            const std::string n = "q" + std::to_string(k);
            GemmProb p = prob_dx(Hq2 + (size_t)(2 + k) * B * Hc1, B, Hc1, W(n + ".l1"), Hc0,
                                 Hq1 + (size_t)(2 + k) * B * Hc0, Dq1 + (size_t)k * B * Hc0, c0);
            p.wgen = W(n + ".l2");             // w3 column of W3_ext
            p.gen_act = c1;                    // act'(Hq2); the epilogue takes act'(Hq1)
            pb.push_back(p);
        }
        add_gemm(h, plan, "q.head+critic.bwd1", pb, record_probs);
        Launch& L = plan.back();
        L.gemm.rowk = 1;
        L.gemm.row_blocks = (B + 3) / 4;
        L.gemm.qh = q;
        L.grid += L.gemm.row_blocks;
        L.flops += 2.0 * B * Hc1 * 4 + 2.0 * B * Hc1 * 2;
        L.bytes += 4.0 * (4.0 * B * Hc1 + 2.0 * B * Hc1 * 2);
        std::vector<GemmProb> pw;
        for (int k = 0; k < 2; ++k) {
            const std::string n = "q" + std::to_string(k), t = "t" + std::to_string(k);
            GemmProb p0 = prob_dw(Xq, ldQ, S + A, B, Dq1 + (size_t)k * B * Hc0, Hc0, W(n + ".l0"), W(t + ".l0"), GRP_Q);
            p0.bscale = W("ws.gq") + (size_t)k * B;   // Dq1 = g (.) M1
            pw.push_back(p0);
            pw.push_back(prob_dw(Hq1 + (size_t)(2 + k) * B * Hc0, Hc0, Hc0, B, Dq2 + (size_t)k * B * Hc1, Hc1, W(n + ".l1"),
                                 W(t + ".l1"), GRP_Q));
            pw.push_back(prob_dw(Hq2 + (size_t)(2 + k) * B * Hc1, Hc1, Hc1, B, W("ws.gq") + (size_t)k * B, 1,
                                 W(n + ".l2"), W(t + ".l2"), GRP_Q));
        }
        add_gemm(h, plan, "critic.adam", pw, record_probs, !fuse_head);
        if (fuse_head) {                    // the policy rows of actor.head (read from pi.q.fwd0 on)
            Launch& L = plan.back();
            HeadArgs a = head_fused;
            a.nseg = 1;
            a.seg[0] = {B, 2 * B, 0, 0, noise_pi, Xp, W("ws.nlp_p")};
            a.total_rows = 2 * B;
            a.cache_row0 = B;
            a.cache_row1 = h->Ra;
            L.name += "+actor.head";
            L.gemm.rowk = 3;
            L.gemm.head = a;
            L.gemm.head_block0 = B / 4;
            L.gemm.row_blocks = (2 * B + 3) / 4 - B / 4;
            L.grid += L.gemm.row_blocks;
            L.flops += 2.0 * B * H1 * Aout;
            L.bytes += 4.0 * B * (H1 + 6.0 * A);
        }
        if (h->dp_ranks > 0) dp_split_adam(h, plan, "q0.l0", "q1.l2", "t0.l0", GRP_Q);
    }
    // ---- policy loss through the updated critics: the same linearity; pi.q.head's rows
    // (min, tie split, loss rows, g0 / g1) share the unscaled dX launch, actor.head.bwd applies
    // g0 / g1.  The SAC-EO world-model dX (needs q.head's Dm2) rides in the same launch.
    {
        std::vector<GemmProb> p0, p1;
        for (int k = 0; k < 2; ++k) {
            const std::string n = "q" + std::to_string(k);
            p0.push_back(prob_fwd(Xp, ldQ, B, S + A, W(n + ".l0"), Hc0, Hp1 + (size_t)k * B * Hc0, c0));
            p1.push_back(prob_fwd(Hp1 + (size_t)k * B * Hc0, Hc0, B, Hc0, W(n + ".l1"), Hc1, Hp2 + (size_t)k * B * Hc1, c1));
        }
        // SAC-EO: world-model layer 2 on the expert rows + MSE epilogue (needs Hm2 from q.fwd1),
        // riding in the pi.q.fwd0 launch (a launch of its own when that one is fused)
        std::vector<GemmProb> pm;
        const int mtn = (S + 15) / 16;
        if (eo) {
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                GemmProb p{};
                p.A = Hm2b + (size_t)k * half * Hm1; p.lda = Hm1; p.a_kc = 1; p.ones_row = -1;
                p.B = W(n + ".l2"); p.ldb = h->Om; p.b_kc = 0;       // W_ext [(Hm1+1) x Om], Om = S (+1)
                p.M = mrows; p.N = S; p.K = Hm1;                     // delta-s columns only
                p.bias = W(n + ".l2") + (size_t)Hm1 * h->Om;
                p.C = W("ws.dout") + (size_t)k * half * S; p.ldc = S;
                p.epi = EPI_FWD; p.act = ACT_NONE;
                p.mse = 1; p.grad_scale = 1.f / (float)mrows;       // MSE_loss = mean over the rows
                p.dclip = h->cfg.delta_clip_pred > 0.f ? h->cfg.delta_clip_pred : 0.f;
                p.se_raw = se_raw + (size_t)k * half * S; p.spe_raw = spe_raw + (size_t)k * half * S;
                p.dmean = W("mnorm.d_mean"); p.dden = W("mnorm.d_den");
                p.part = W("ws.mse") + (size_t)k * half * mtn;
                pm.push_back(p);
            }
        }
        if (eo && fuse_head) {               // the models' layer 1 on Hm1 (from q.fwd1)
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                p0.push_back(prob_fwd(Hm1b + (size_t)k * half * Hm0, Hm0, mrows, Hm0, W(n + ".l1"), Hm1,
                                      Hm2b + (size_t)k * half * Hm1, m1));
            }
        }
        if (eo) fwd_pair("pi.q.fwd", p0, p1);
        else fwd_pair2("pi.q.fwd", p0, p1);
        if (eo) {                            // plan.back() is pi.q.fwd1: fold into pi.q.fwd0 (or, with
                                             // the fused head, into pi.q.fwd1: Hm2 comes from pi.q.fwd0)
            Launch& F0 = plan[plan.size() - (fuse_head ? 1 : 2)];
            std::vector<Launch> one;
            add_gemm(h, one, "model.head", pm, false);
            h->probs_cursor -= (int)pm.size();
            if (!merge_gemm(F0.gemm, one[0].gemm)) { fprintf(stderr, "sacx: model.head merge\n"); abort(); }
            F0.name += "+model.head";
            F0.grid = F0.gemm.total_tiles;
            F0.flops += one[0].flops;
            F0.bytes += one[0].bytes;
        }
        QHeadArgs q{};
        q.mode = 1; q.B = B; q.H1 = Hc1; q.H2 = Hp2;
        q.W3[0] = W("q0.l2"); q.W3[1] = W("q1.l2"); q.W3[2] = nullptr; q.W3[3] = nullptr;
        q.act = c1; q.D2 = nullptr; q.g = W("ws.gp"); q.loss_rows = W("ws.lp");
        q.alpha = W("alpha"); q.nlp = W("ws.nlp_p");
        q.w_sac = eo ? (float)(1.0 - (double)h->cfg.epsilon) : 1.f;
        q.ret_den = W("norm.ret_den");
        q.ne = 0; q.ctl = h->ctl();
        std::vector<GemmProb> pb;
        for (int k = 0; k < 2; ++k) {
            const std::string n = "q" + std::to_string(k);
            GemmProb p = prob_dx(Hp2 + (size_t)k * B * Hc1, B, Hc1, W(n + ".l1"), Hc0, Hp1 + (size_t)k * B * Hc0,
                                 Dp1 + (size_t)k * B * Hc0, c0);
            p.wgen = W(n + ".l2");
            p.gen_act = c1;
            pb.push_back(p);
        }
        if (eo) {                            // Dm2 = dout . Wm2[:, :S]^T (.) act'(Hm2)
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                GemmProb p = prob_dx(W("ws.dout") + (size_t)k * half * S, mrows, S, W(n + ".l2"), Hm1,
                                     Hm2b + (size_t)k * half * Hm1, Dm2 + (size_t)k * half * Hm1, m1);
                p.ldb = h->Om;                       // B[n][k] = W_ext[n][k], row stride Om
                pb.push_back(p);
            }
        }
        if (fold_hbw) {                      // partial action gradients instead of Dp1 (read by no one else)
            for (int k = 0; k < 2; ++k) {
                GemmProb& p = pb[k];
                p.pw = W("q" + std::to_string(k) + ".l0") + (size_t)S * Hc0;   // action rows of W_ext
                p.pw_ld = Hc0;
                p.pw_cs = 1;
                p.pw_n = A;
                p.ppart = W("ws.apart") + (size_t)k * B * tq * A;
                p.C = nullptr;
            }
        }
        add_gemm(h, plan, "pi.q.head+pi.q.bwd1", pb, record_probs);
        {
            Launch& L = plan.back();
            L.gemm.rowk = 2;
            L.gemm.row_blocks = (B + 3) / 4;
            L.gemm.qh = q;
            L.grid += L.gemm.row_blocks;
            L.flops += 2.0 * B * Hc1 * 2 * 2;
            L.bytes += 4.0 * (2.0 * B * Hc1 * 2);
        }
        if (eo) {                            // Dm1 = Dm2 . Wm1^T (.) act'(Hm1), for actor.head.bwd
            std::vector<GemmProb> pd;
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                pd.push_back(prob_dx(Dm2 + (size_t)k * half * Hm1, mrows, Hm1, W(n + ".l1"), Hm0,
                                     Hm1b + (size_t)k * half * Hm0, Dm1 + (size_t)k * half * Hm0, m0));
            }
            if (fold_hbw) {                  // partial action gradients of the expert rows instead of Dm1
                const int tqm = (Hm0 + 15) / 16;
                for (int k = 0; k < nm; ++k) {
                    GemmProb& p = pd[k];
                    p.pw = W("m" + std::to_string(k) + ".l0") + (size_t)S * Hm0;   // action rows of W_ext
                    p.pw_ld = Hm0;
                    p.pw_cs = 1;
                    p.pw_n = A;
                    p.ppart = W("ws.mpart") + (size_t)k * half * A * tqm;
                    p.C = nullptr;
                }
            }
            add_gemm(h, plan, "model.bwd1", pd, record_probs);
            if (fold_hbw) plan.back().gemm.rowk = 2;   // DX with the partial epilogue (no q-head rows)
        }
    }
    // ---- actor backward
    if (fold_hbw) {
        // actor.head.bwd as the tile prologue of actor.bwd1: Da3 from the partials of pi.q.bwd1,
        // Da2 generated on load (an MFMA from Da3 and W3a), stored by column tile 0
        const int Rb = h->Rb;
        GemmProb p = prob_dx(Ha2 + (size_t)B * H1, Rb, H1, W("actor.l1"), H0, Ha1 + (size_t)B * H0, Da1,
                             h->ln ? ACT_TANH : a0);
        p.wgen = W("actor.l2");              // W3a [(H1+1) x Aout]
        p.gen_act = a1;                      // act'(Ha2)
        p.hbw = 1;
        add_gemm(h, plan, "actor.head.bwd+actor.bwd1", {p}, record_probs);
        Launch& L = plan.back();
        L.gemm.rowk = 4;
        HeadBwdArgs& b = L.gemm.hbw;
        b.B = B; b.A = A; b.Aout = Aout; b.per_state_std = h->cfg.per_state_std; b.tq = tq;
        b.lim = h->cfg.act_limit; b.part = W("ws.apart"); b.gpol = W("ws.gp"); b.a_den = W("norm.a_den");
        b.ma_den = W(mnorm(h, "a_den")); b.alpha = W("alpha");
        b.c_t = W("ws.c_t"); b.c_std = W("ws.c_std"); b.c_u = W("ws.c_u"); b.c_mask = W("ws.c_mask");
        b.Da3 = Da3; b.E = E; b.Da2 = Da2;
        b.ne = ne; b.tqm = (Hm0 + 15) / 16; b.mpart = eo ? W("ws.mpart") : nullptr; b.ctl = eo ? h->ctl() : nullptr;
        L.flops += 2.0 * B * 2 * Hc0 * A + 2.0 * Rb * H1 * Aout;
        L.bytes += 4.0 * (2.0 * B * tq * A + 2.0 * Rb * H1);
    }
    {
        Launch L{};
        L.kind = Launch::ABWD;
        L.name = "actor.head.bwd";
        ActorBwdArgs& b = L.ab;
        b.B = B; b.ne = ne; b.S = S; b.A = A; b.Aout = Aout; b.H0 = Hc0; b.H1 = H1; b.Hm0 = Hm0;   // Dp1 / Wq1: critic
        b.per_state_std = h->cfg.per_state_std; b.lim = h->cfg.act_limit;
        b.Dp1 = Dp1; b.Wq1[0] = W("q0.l0"); b.Wq1[1] = W("q1.l0");
        b.Dm1 = Dm1; b.Wm1[0] = eo ? W("m0.l0") : nullptr; b.Wm1[1] = eo ? W(nm > 1 ? "m1.l0" : "m0.l0") : nullptr;
        b.a_den = W("norm.a_den"); b.ma_den = W(mnorm(h, "a_den")); b.alpha = W("alpha"); b.ctl = h->ctl();
        b.use_expert = eo;
        b.c_t = W("ws.c_t"); b.c_std = W("ws.c_std"); b.c_u = W("ws.c_u"); b.c_mask = W("ws.c_mask");
        b.W3a = W("actor.l2"); b.Ha2 = Ha2 + (size_t)B * H1; b.act = a1;
        b.Da3 = Da3; b.Da2 = Da2; b.E = E;
        b.gpol = W("ws.gp");
        L.grid = (h->Rb + 3) / 4;
        L.flops = 2.0 * B * 2 * Hc0 * A + 2.0 * ne * Hm0 * A + 2.0 * h->Rb * H1 * Aout;
        L.bytes = 4.0 * (2.0 * B * Hc0 + ne * Hm0 + 2.0 * h->Rb * H1);
        const int Rb = h->Rb;
        if (!fold_hbw) {
            plan.push_back(L);
            add_gemm(h, plan, "actor.bwd1",      // layer-norm layer 0: tanh' at its output
                     {prob_dx(Da2, Rb, H1, W("actor.l1"), H0, Ha1 + (size_t)B * H0, Da1, h->ln ? ACT_TANH : a0)},
                     record_probs);
        }
        if (h->ln) {                          // dY -> dZ through the norm; dY*xhat, dY for gamma / beta
            Launch N{};
            N.kind = Launch::LNORM;
            N.name = "actor.ln.bwd";
            LNArgs& a = N.ln;
            a.mode = 1; a.H = H0; a.Z = Da1; a.r[1] = Rb; a.gamma = W("actor.ln");
            a.xhat = W("ws.ln_xhat"); a.rstd = W("ws.ln_rstd"); a.xrow0 = B;
            a.gy = W("ws.ln_gy"); a.gb = W("ws.ln_gb");
            N.grid = (Rb + 3) / 4;
            N.flops = 8.0 * Rb * H0;
            N.bytes = 4.0 * Rb * H0 * 5;
            plan.push_back(N);
        }
        std::vector<GemmProb> pw;
        pw.push_back(prob_dw(Xa + (size_t)B * ldS, ldS, S, Rb, Da1, H0, W("actor.l0"), nullptr, GRP_PI));
        pw.push_back(prob_dw(Ha1 + (size_t)B * H0, H0, H0, Rb, Da2, H1, W("actor.l1"), nullptr, GRP_PI));
        pw.push_back(prob_dw(Ha2 + (size_t)B * H1, H1, H1, Rb, Da3, Aout, W("actor.l2"), nullptr, GRP_PI));
        if (!h->cfg.per_state_std) {
            GemmProb p = prob_dw(E, 1, 0, Rb, E, A, W("actor.logstd"), nullptr, GRP_PI);
            p.ones_row = 0;   // single all-ones row: column sums of E
            pw.push_back(p);
        }
        if (h->ln) {          // gamma, beta: column sums of dY*xhat and dY
            for (int k = 0; k < 2; ++k) {
                float* gsrc = W(k ? "ws.ln_gb" : "ws.ln_gy");
                GemmProb p = prob_dw(gsrc, 1, 0, Rb, gsrc, H0, W("actor.ln") + (size_t)k * H0, nullptr, GRP_PI);
                p.ones_row = 0;
                pw.push_back(p);
            }
        }
        add_gemm(h, plan, "actor.adam", pw, record_probs);
        if (h->dp_ranks > 0) dp_split_adam(h, plan, "actor.l0", "actor.logstd", "", GRP_PI);
    }
    // ---- alpha: updated actor on s, evaluate, Adam on alpha, statistics
    const size_t alpha_first = plan.size();
    // the alpha forward is folded into the next update's actor forward (merged_body): same fusion
    if (h->ln) {
        add_gemm(h, plan, "alpha.fwd0", {prob_fwd(Xa + (size_t)B * ldS, ldS, B, S, W("actor.l0"), H0, Hl1, ACT_NONE)},
                 record_probs);
        ln_fwd("alpha.ln", Ra4, Ra4 + B);
        add_gemm(h, plan, "alpha.fwd1", {actor_fwd1(Ra4, B)}, record_probs);
        mark_part();
    } else {
        fwd_pair("alpha.fwd", {prob_fwd(Xa + (size_t)B * ldS, ldS, B, S, W("actor.l0"), H0, Hl1, a0)},
                 {actor_fwd1(Ra4, B)});
        mark_part();
        // fused as the actor pair is, so merged_body folds one k_fwd2 launch into the other
        if (h->fwd2) fuse_fwd2(h, plan, "alpha.fwd01");
    }
    {
        Launch L{};
        L.kind = Launch::AHEAD;
        L.name = "alpha.head";
        HeadArgs& a = L.head;
        a.H2 = Hl2; a.ldh = H1; a.W3 = W("actor.l2"); a.logstd = W("actor.logstd");
        a.part = head_part ? hpart + (size_t)Ra4 * Aout * tqh : nullptr; a.tq = tqh;
        a.H1 = H1; a.A = A; a.Aout = Aout; a.S = S; a.ldQ = ldQ; a.per_state_std = h->cfg.per_state_std;
        a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
        a.nseg = 1;
        a.seg[0] = {0, B, 0, 0, noise_al, nullptr, W("ws.nlp3")};
        a.total_rows = B;
        a.cache_row0 = 1 << 30;
        a.c_t = nullptr;
        a.alpha_mode = 1;
        L.fin.red = W("red");                       // per-workgroup partials of sum(-nlp + H)
        L.fin.target_entropy = h->cfg.target_entropy;
        L.grid = (B + 3) / 4;
        L.flops = 2.0 * B * H1 * Aout;
        L.bytes = 4.0 * B * H1;
        plan.push_back(L);
    }
    plan_alpha_final(h, plan, nm);
    // alpha.fwd .. alpha.final only feed the next update's q.head
    for (size_t i = alpha_first; i < plan.size(); ++i) plan[i].alpha_branch = true;
    xbf_wire(h, plan, slot);
    for (Launch& L : plan) pack_seeds(L, (int64_t)h->seed_bytes, h->seeds);
}

// Appends one GEMM launch per GEMM_MAXP problems (a launch's problems travel by value): `name`,
// then name.1, name.2, ...  Returns the launches added.
int add_gemm_split(sacx_handle* h, std::vector<Launch>& plan, const std::string& name, const std::vector<GemmProb>& ps,
                   bool record_probs) {
    int n = 0;
    for (size_t i = 0; i < ps.size(); i += GEMM_MAXP, ++n) {
        std::vector<GemmProb> part(ps.begin() + i, ps.begin() + std::min(ps.size(), i + GEMM_MAXP));
        add_gemm(h, plan, n == 0 ? name : name + "." + std::to_string(n), part, record_probs);
    }
    return n;
}

// ---------------------------------------------------------------- the generic update plan
// Nets of any depth (create_nn's layers list, nn_utils.py:100-138; SACX_GENERIC=1 also at two layers,
// the parity check of this plan against the fused one): the update of build_plan in the reference's
// order, with every Dense layer a problem of its depth level's forward, dX or dW + Adam launch and the
// heads on the row kernels -- k_actor_head (evaluate / sample), k_qhead (twin-Q target, critic loss and
// policy-loss gradients, writing the delta at the critics' last hidden layer), k_actor_bwd (the action
// gradient through the first layer of the critics / world models, the tanh-Gaussian backward, the
// delta at the actor's last hidden layer).  No folds and no linearity fusion: each delta is the
// loss-scaled one, the dW launches take unscaled rows.  merged_body folds the alpha branch exactly
// as in the fused plan (alpha.fwd<i> into actor.fwd<i>, alpha.head into actor.head, alpha.final into
// the first forward launch after it).
void build_plan_generic(sacx_handle* h, int slot, bool record_probs) {
    std::vector<Launch>& plan = h->plan[slot];
    plan.clear();
    h->probs_cursor = 0;
    const int S = h->S, A = h->A, H0 = h->H0, H1 = h->H1, B = h->B, ne = h->ne, Aout = h->Aout;
    const int Hm1 = h->Hm1, half = ne / 2, Hc1 = h->Hc1;
    const int nm = std::min(h->nm, 2), mrows = nm == 1 ? ne : half;   // the expert term's models
    const int ldS = h->ldS, ldQ = h->ldQ, Rb = h->Rb;
    const bool eo = h->cfg.use_expert != 0;
    const NetDims &na = h->nd[0], &nc = h->nd[1], &nmd = h->nd[2];
    const int Da = na.D(), Dc = nc.D(), Dm = eo ? nmd.D() : 0;
    const std::string sl = "slot" + std::to_string(slot);
    auto W = [&](const std::string& n) { return h->f(n); };
    auto L_ = [](const std::string& net, int i) { return net + ".l" + std::to_string(i); };
    // hidden-layer buffer i of a chain of D layers: <p>1 (layer 0), <p>2 (the last), <p>m<i>
    auto ch = [&](const std::string& p, int i, int D) -> float* {
        if (i == 0) return W(p + "1");
        if (i == D - 1) return W(p + "2");
        return W(p + "m" + std::to_string(i));
    };
    float* noise = h->f(sl + ".noise");
    float* noise_t = noise;
    float* noise_pi = noise + (size_t)B * A;
    float* noise_e = noise + (size_t)2 * B * A;
    float* noise_al = noise + (size_t)(2 * B + ne) * A;
    float *Xa = W(sl + ".Xa"), *Xq = W(sl + ".Xq"), *Xt = W(sl + ".Xt"), *Xp = W(sl + ".Xp"), *Xm = W(sl + ".Xm");
    float *r_in = W(sl + ".r"), *d_in = W(sl + ".d"), *se_raw = W(sl + ".se_raw"), *spe_raw = W(sl + ".spe_raw");
    const char* qn[4] = {"t0", "t1", "q0", "q1"};
    const int Ra4 = (h->Ra + 3) & ~3;       // first row of the alpha rows in the actor chain's buffers

    plan_inputs(h, plan, slot);
    // ---- actor forward on rows [r0, r0 + M) of its chain from X: --actor_layer_norm puts Dense ->
    // LayerNorm -> tanh on layer 0 (k_ln on the pre-norm output, nn_utils.py:110-119)
    auto actor_fwd = [&](const std::string& name, const float* X, int r0, int M, bool alpha) {
        for (int i = 0; i < Da; ++i) {
            const float* in = i == 0 ? X : ch("ws.Ha", i - 1, Da) + (size_t)r0 * na.h[i - 1];
            const int ldi = i == 0 ? ldS : na.h[i - 1], K = i == 0 ? S : na.h[i - 1];
            const int act = (i == 0 && h->ln) ? ACT_NONE : na.act[i];
            add_gemm(h, plan, name + std::to_string(i),
                     {prob_fwd(in, ldi, M, K, W(L_("actor", i)), na.h[i], ch("ws.Ha", i, Da) + (size_t)r0 * na.h[i], act)},
                     record_probs);
            if (i == 0 && h->ln) {
                Launch L{};
                L.kind = Launch::LNORM;
                L.name = alpha ? "alpha.ln" : "actor.ln";
                LNArgs& a = L.ln;
                a.mode = 0; a.H = H0; a.Z = W("ws.Ha1"); a.nrange = 1; a.r[0] = r0; a.r[1] = r0 + M;
                a.gamma = W("actor.ln"); a.xhat = W("ws.ln_xhat"); a.rstd = W("ws.ln_rstd"); a.cache_rows = h->Ra;
                L.grid = (M + 3) / 4;
                L.flops = 8.0 * M * H0;
                L.bytes = 4.0 * M * H0 * 3;
                plan.push_back(L);
            }
        }
    };
    actor_fwd("actor.fwd", Xa, 0, h->Ra, false);
    float* Ha_last = W("ws.Ha2");
    auto head_base = [&](HeadArgs& a, const float* H2) {
        a.H2 = H2; a.ldh = H1; a.W3 = W(L_("actor", Da)); a.logstd = W("actor.logstd");
        a.part = nullptr; a.tq = (H1 + 15) / 16;
        a.H1 = H1; a.A = A; a.Aout = Aout; a.S = S; a.ldQ = ldQ; a.per_state_std = h->cfg.per_state_std;
        a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
        a.ma_mean = W(mnorm(h, "a_mean")); a.ma_den = W(mnorm(h, "a_den"));
    };
    {   // ---- actor head: evaluate(sp) -> target rows, evaluate(s) -> policy rows, sample(s_e) -> model rows
        Launch L{};
        L.kind = Launch::AHEAD;
        L.name = "actor.head";
        L.frees_slot = true;
        HeadArgs& a = L.head;
        head_base(a, Ha_last);
        a.nseg = eo ? 3 : 2;
        a.seg[0] = {0, B, 0, 0, noise_t, Xt, W("ws.nlp_t")};
        a.seg[1] = {B, 2 * B, 0, 0, noise_pi, Xp, W("ws.nlp_p")};
        a.seg[2] = {2 * B, 2 * B + ne, 1, 0, noise_e, Xm, nullptr};
        a.total_rows = h->Ra;
        a.cache_row0 = B;
        a.cache_row1 = h->Ra;
        a.c_t = W("ws.c_t"); a.c_std = W("ws.c_std"); a.c_u = W("ws.c_u"); a.c_mask = W("ws.c_mask");
        a.alpha_mode = 0;
        L.grid = (h->Ra + 3) / 4;
        L.flops = 2.0 * h->Ra * H1 * Aout;
        L.bytes = 4.0 * h->Ra * (H1 + 6.0 * A);
        plan.push_back(L);
    }
    // ---- target / critic forward (t0, t1 on [sp | pi(sp)], q0, q1 on [s | a]; the world models' hidden
    // layers on the expert rows [s_e | pi(s_e)]), one launch per depth level
    for (int i = 0; i < std::max(Dc, Dm); ++i) {
        std::vector<GemmProb> ps;
        if (i < Dc)
            for (int k = 0; k < 4; ++k) {
                const float* in = i == 0 ? (k < 2 ? Xt : Xq) : ch("ws.Hq", i - 1, Dc) + (size_t)k * B * nc.h[i - 1];
                ps.push_back(prob_fwd(in, i == 0 ? ldQ : nc.h[i - 1], B, i == 0 ? S + A : nc.h[i - 1], W(L_(qn[k], i)),
                                      nc.h[i], ch("ws.Hq", i, Dc) + (size_t)k * B * nc.h[i], nc.act[i]));
            }
        if (i < Dm)
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                const float* in = i == 0 ? Xm + (size_t)k * half * ldQ : ch("ws.Hm", i - 1, Dm) + (size_t)k * half * nmd.h[i - 1];
                ps.push_back(prob_fwd(in, i == 0 ? ldQ : nmd.h[i - 1], mrows, i == 0 ? S + A : nmd.h[i - 1], W(L_(n, i)),
                                      nmd.h[i], ch("ws.Hm", i, Dm) + (size_t)k * half * nmd.h[i], nmd.act[i]));
            }
        add_gemm(h, plan, "q.fwd" + std::to_string(i), ps, record_probs);
    }
    const int mtn = (S + 15) / 16;
    if (eo) {   // the world models' head on the expert rows + the expert MSE (SAC_expert.py:319-332)
        std::vector<GemmProb> pm;
        for (int k = 0; k < nm; ++k) {
            const std::string n = "m" + std::to_string(k);
            GemmProb p{};
            p.A = W("ws.Hm2") + (size_t)k * half * Hm1; p.lda = Hm1; p.a_kc = 1; p.ones_row = -1;
            p.B = W(L_(n, Dm)); p.ldb = h->Om; p.b_kc = 0;       // W_ext [(Hm1+1) x Om], Om = S (+1)
            p.M = mrows; p.N = S; p.K = Hm1;                     // delta-s columns only
            p.bias = W(L_(n, Dm)) + (size_t)Hm1 * h->Om;
            p.C = W("ws.dout") + (size_t)k * half * S; p.ldc = S;
            p.epi = EPI_FWD; p.act = ACT_NONE;
            p.mse = 1; p.grad_scale = 1.f / (float)mrows;       // MSE_loss = mean over the rows
            p.dclip = h->cfg.delta_clip_pred > 0.f ? h->cfg.delta_clip_pred : 0.f;
            p.se_raw = se_raw + (size_t)k * half * S; p.spe_raw = spe_raw + (size_t)k * half * S;
            p.dmean = W("mnorm.d_mean"); p.dden = W("mnorm.d_den");
            p.part = W("ws.mse") + (size_t)k * half * mtn;
            pm.push_back(p);
        }
        add_gemm(h, plan, "model.head", pm, record_probs);
    }
    {   // ---- q.head: min target, TD target, critic losses and the delta at the critics' last hidden layer
        Launch L{};
        L.kind = Launch::QHEAD;
        L.name = "q.head";
        QHeadArgs& q = L.qh;
        q.mode = 0; q.B = B; q.H1 = Hc1; q.H2 = W("ws.Hq2");
        for (int k = 0; k < 4; ++k) q.W3[k] = W(L_(qn[k], Dc));
        q.act = nc.act[Dc - 1]; q.D2 = W("ws.Dq2"); q.g = W("ws.gq"); q.loss_rows = W("ws.lq");
        q.alpha = W("alpha"); q.nlp = W("ws.nlp_t"); q.r = r_in; q.d = d_in;
        q.gamma = h->cfg.gamma; q.ret_den = W("norm.ret_den"); q.w_sac = 1.f;
        q.ne = 0; q.ctl = h->ctl();
        L.grid = (B + 3) / 4;
        L.flops = 2.0 * B * Hc1 * 4;
        L.bytes = 4.0 * (4.0 * B * Hc1 + 2.0 * B * Hc1);
        plan.push_back(L);
    }
    // ---- critic backward (dX down to layer 0's output), then dW + Keras Adam + Polyak into t0 / t1
    for (int i = Dc - 1; i >= 1; --i) {
        std::vector<GemmProb> pb;
        for (int k = 0; k < 2; ++k)
            pb.push_back(prob_dx(ch("ws.Dq", i, Dc) + (size_t)k * B * nc.h[i], B, nc.h[i], W(L_(qn[2 + k], i)), nc.h[i - 1],
                                 ch("ws.Hq", i - 1, Dc) + (size_t)(2 + k) * B * nc.h[i - 1],
                                 ch("ws.Dq", i - 1, Dc) + (size_t)k * B * nc.h[i - 1], nc.act[i - 1]));
        add_gemm(h, plan, "critic.bwd" + std::to_string(i), pb, record_probs);
    }
    {
        std::vector<GemmProb> pw;
        for (int k = 0; k < 2; ++k) {
            const std::string n = "q" + std::to_string(k), t = "t" + std::to_string(k);
            for (int i = 0; i < Dc; ++i) {
                const float* X = i == 0 ? Xq : ch("ws.Hq", i - 1, Dc) + (size_t)(2 + k) * B * nc.h[i - 1];
                const int K = i == 0 ? S + A : nc.h[i - 1];
                pw.push_back(prob_dw(X, i == 0 ? ldQ : K, K, B, ch("ws.Dq", i, Dc) + (size_t)k * B * nc.h[i], nc.h[i],
                                     W(L_(n, i)), W(L_(t, i)), GRP_Q));
            }
            pw.push_back(prob_dw(W("ws.Hq2") + (size_t)(2 + k) * B * Hc1, Hc1, Hc1, B, W("ws.gq") + (size_t)k * B, 1,
                                 W(L_(n, Dc)), W(L_(t, Dc)), GRP_Q));
        }
        const int n = add_gemm_split(h, plan, "critic.adam", pw, record_probs);
        if (h->dp_ranks > 0) dp_split_adam(h, plan, "q0.l0", L_("q1", Dc), "t0.l0", GRP_Q, n);
    }
    // ---- policy loss through the updated critics
    for (int i = 0; i < Dc; ++i) {
        std::vector<GemmProb> ps;
        for (int k = 0; k < 2; ++k) {
            const float* in = i == 0 ? Xp : ch("ws.Hp", i - 1, Dc) + (size_t)k * B * nc.h[i - 1];
            ps.push_back(prob_fwd(in, i == 0 ? ldQ : nc.h[i - 1], B, i == 0 ? S + A : nc.h[i - 1],
                                  W(L_("q" + std::to_string(k), i)), nc.h[i], ch("ws.Hp", i, Dc) + (size_t)k * B * nc.h[i],
                                  nc.act[i]));
        }
        add_gemm(h, plan, "pi.q.fwd" + std::to_string(i), ps, record_probs);
    }
    {   // min, tie split, policy loss rows, the delta at the critics' last hidden layer (x d p / d Q_k)
        Launch L{};
        L.kind = Launch::QHEAD;
        L.name = "pi.q.head";
        QHeadArgs& q = L.qh;
        q.mode = 1; q.B = B; q.H1 = Hc1; q.H2 = W("ws.Hp2");
        q.W3[0] = W(L_("q0", Dc)); q.W3[1] = W(L_("q1", Dc)); q.W3[2] = nullptr; q.W3[3] = nullptr;
        q.act = nc.act[Dc - 1]; q.D2 = W("ws.Dp2"); q.g = W("ws.gp"); q.loss_rows = W("ws.lp");
        q.alpha = W("alpha"); q.nlp = W("ws.nlp_p");
        q.w_sac = eo ? (float)(1.0 - (double)h->cfg.epsilon) : 1.f;
        q.ret_den = W("norm.ret_den");
        q.ne = 0; q.ctl = h->ctl();
        L.grid = (B + 3) / 4;
        L.flops = 2.0 * B * Hc1 * 2;
        L.bytes = 4.0 * (4.0 * B * Hc1);
        plan.push_back(L);
    }
    for (int i = Dc - 1; i >= 1; --i) {
        std::vector<GemmProb> pb;
        for (int k = 0; k < 2; ++k)
            pb.push_back(prob_dx(ch("ws.Dp", i, Dc) + (size_t)k * B * nc.h[i], B, nc.h[i], W(L_("q" + std::to_string(k), i)),
                                 nc.h[i - 1], ch("ws.Hp", i - 1, Dc) + (size_t)k * B * nc.h[i - 1],
                                 ch("ws.Dp", i - 1, Dc) + (size_t)k * B * nc.h[i - 1], nc.act[i - 1]));
        add_gemm(h, plan, "pi.q.bwd" + std::to_string(i), pb, record_probs);
    }
    if (eo)     // the world models' backward to their layer-0 output (the expert rows' action gradient)
        for (int i = Dm; i >= 1; --i) {
            std::vector<GemmProb> pb;
            for (int k = 0; k < nm; ++k) {
                const std::string n = "m" + std::to_string(k);
                const float* D = i == Dm ? W("ws.dout") + (size_t)k * half * S : ch("ws.Dm", i, Dm) + (size_t)k * half * nmd.h[i];
                GemmProb p = prob_dx(D, mrows, i == Dm ? S : nmd.h[i], W(L_(n, i)), nmd.h[i - 1],
                                     ch("ws.Hm", i - 1, Dm) + (size_t)k * half * nmd.h[i - 1],
                                     ch("ws.Dm", i - 1, Dm) + (size_t)k * half * nmd.h[i - 1], nmd.act[i - 1]);
                if (i == Dm) p.ldb = h->Om;          // the head's delta-s columns: B[n][k] = W_ext[n][k], stride Om
                pb.push_back(p);
            }
            add_gemm(h, plan, "model.bwd" + std::to_string(i), pb, record_probs);
        }
    // ---- actor backward: action gradients -> tanh-Gaussian backward -> the delta at the last hidden
    // layer (k_actor_bwd, from the loss-scaled deltas: gpol = null), dX to layer 0, dW + Adam
    {
        Launch L{};
        L.kind = Launch::ABWD;
        L.name = "actor.head.bwd";
        ActorBwdArgs& b = L.ab;
        b.B = B; b.ne = ne; b.S = S; b.A = A; b.Aout = Aout; b.H0 = h->Hc0; b.H1 = H1; b.Hm0 = h->Hm0;
        b.per_state_std = h->cfg.per_state_std; b.lim = h->cfg.act_limit;
        b.Dp1 = W("ws.Dp1"); b.Wq1[0] = W("q0.l0"); b.Wq1[1] = W("q1.l0");
        b.Dm1 = W("ws.Dm1"); b.Wm1[0] = eo ? W("m0.l0") : nullptr; b.Wm1[1] = eo ? W(nm > 1 ? "m1.l0" : "m0.l0") : nullptr;
        b.a_den = W("norm.a_den"); b.ma_den = W(mnorm(h, "a_den")); b.alpha = W("alpha"); b.ctl = h->ctl();
        b.use_expert = eo;
        b.c_t = W("ws.c_t"); b.c_std = W("ws.c_std"); b.c_u = W("ws.c_u"); b.c_mask = W("ws.c_mask");
        b.W3a = W(L_("actor", Da)); b.Ha2 = Ha_last + (size_t)B * H1;
        b.act = (Da == 1 && h->ln) ? ACT_TANH : na.act[Da - 1];   // layer norm: tanh' at the norm's output
        b.Da3 = W("ws.Da3"); b.Da2 = W("ws.Da2"); b.E = W("ws.E");
        b.gpol = nullptr;
        L.grid = (Rb + 3) / 4;
        L.flops = 2.0 * B * 2 * h->Hc0 * A + 2.0 * ne * h->Hm0 * A + 2.0 * Rb * H1 * Aout;
        L.bytes = 4.0 * (2.0 * B * h->Hc0 + ne * h->Hm0 + 2.0 * Rb * H1);
        plan.push_back(L);
    }
    for (int i = Da - 1; i >= 1; --i)
        add_gemm(h, plan, "actor.bwd" + std::to_string(i),
                 {prob_dx(ch("ws.Da", i, Da), Rb, na.h[i], W(L_("actor", i)), na.h[i - 1],
                          ch("ws.Ha", i - 1, Da) + (size_t)B * na.h[i - 1], ch("ws.Da", i - 1, Da),
                          (i == 1 && h->ln) ? ACT_TANH : na.act[i - 1])},
                 record_probs);
    if (h->ln) {                          // dY -> dZ through the norm; dY*xhat, dY for gamma / beta
        Launch N{};
        N.kind = Launch::LNORM;
        N.name = "actor.ln.bwd";
        LNArgs& a = N.ln;
        a.mode = 1; a.H = H0; a.Z = W("ws.Da1"); a.r[1] = Rb; a.gamma = W("actor.ln");
        a.xhat = W("ws.ln_xhat"); a.rstd = W("ws.ln_rstd"); a.xrow0 = B;
        a.gy = W("ws.ln_gy"); a.gb = W("ws.ln_gb");
        N.grid = (Rb + 3) / 4;
        N.flops = 8.0 * Rb * H0;
        N.bytes = 4.0 * Rb * H0 * 5;
        plan.push_back(N);
    }
    {
        std::vector<GemmProb> pw;
        for (int i = 0; i < Da; ++i) {
            const float* X = i == 0 ? Xa + (size_t)B * ldS : ch("ws.Ha", i - 1, Da) + (size_t)B * na.h[i - 1];
            const int K = i == 0 ? S : na.h[i - 1];
            pw.push_back(prob_dw(X, i == 0 ? ldS : K, K, Rb, ch("ws.Da", i, Da), na.h[i], W(L_("actor", i)), nullptr, GRP_PI));
        }
        pw.push_back(prob_dw(Ha_last + (size_t)B * H1, H1, H1, Rb, W("ws.Da3"), Aout, W(L_("actor", Da)), nullptr, GRP_PI));
        if (!h->cfg.per_state_std) {
            GemmProb p = prob_dw(W("ws.E"), 1, 0, Rb, W("ws.E"), A, W("actor.logstd"), nullptr, GRP_PI);
            p.ones_row = 0;   // single all-ones row: column sums of E
            pw.push_back(p);
        }
        if (h->ln) {          // gamma, beta: column sums of dY*xhat and dY
            for (int k = 0; k < 2; ++k) {
                float* gsrc = W(k ? "ws.ln_gb" : "ws.ln_gy");
                GemmProb p = prob_dw(gsrc, 1, 0, Rb, gsrc, H0, W("actor.ln") + (size_t)k * H0, nullptr, GRP_PI);
                p.ones_row = 0;
                pw.push_back(p);
            }
        }
        const int n = add_gemm_split(h, plan, "actor.adam", pw, record_probs);
        if (h->dp_ranks > 0) dp_split_adam(h, plan, "actor.l0", "actor.logstd", "", GRP_PI, n);
    }
    // ---- alpha: the updated actor on s, evaluate, Adam on alpha, statistics
    const size_t alpha_first = plan.size();
    actor_fwd("alpha.fwd", Xa + (size_t)B * ldS, Ra4, B, true);
    {
        Launch L{};
        L.kind = Launch::AHEAD;
        L.name = "alpha.head";
        HeadArgs& a = L.head;
        head_base(a, W("ws.Hl2"));
        a.nseg = 1;
        a.seg[0] = {0, B, 0, 0, noise_al, nullptr, W("ws.nlp3")};
        a.total_rows = B;
        a.cache_row0 = 1 << 30;
        a.c_t = nullptr;
        a.alpha_mode = 1;
        L.fin.red = W("red");                       // per-workgroup partials of sum(-nlp + H)
        L.fin.target_entropy = h->cfg.target_entropy;
        L.grid = (B + 3) / 4;
        L.flops = 2.0 * B * H1 * Aout;
        L.bytes = 4.0 * B * H1;
        plan.push_back(L);
    }
    plan_alpha_final(h, plan, nm);
    for (size_t i = alpha_first; i < plan.size(); ++i) plan[i].alpha_branch = true;
    for (Launch& L : plan) pack_seeds(L, (int64_t)h->seed_bytes, h->seeds);
}

// one world-model fitting step: gather -> 3 fwd GEMMs -> loss grads -> 2 dX GEMMs -> dW + Adam -> finalize
// the fitting plan of the selected seed (its arena block's pointers).  Folded (h->mfuse, the
// default): the loss and its gradient are model.fwd2's epilogue (mse = 2) and the finalisation is
// one extra workgroup of model.bwd2, so model.adam takes the already-advanced step counter (t_adv);
// the weights are bit-identical to the unfolded chain, the loss statistic sums in another order.
void build_model_plan(sacx_handle* h) {
    std::vector<Launch>& plan = h->mplans[h->sel];
    plan.clear();
    if (!h->cfg.use_expert) return;
    const int S = h->S, A = h->A, mb = h->mb, O = S + 1, ldQ = h->ldQ;
    const int nm = h->nm;
    const NetDims& nmd = h->nd[2];
    const NetDims& nrd = h->nd[3];
    const int Dm = nmd.D(), Dr = h->srn ? nrd.D() : 0;
    const int Lf = std::max(Dm, Dr);          // forward levels 0 .. Lf (a net's head at its own depth)
    // GaussianModel / --separate_reward_nn fits exist only in the folded form (their loss epilogues)
    const bool fuse = h->mfuse != 0 || h->gm || h->srn;
    const int Om = h->Om;             // model-net outputs (S + 1, or S beside a reward net)
    const int nt = (Om + 15) / 16;    // fit-loss partials per row (16-column tiles of model.fwd2)
    const int ldO = (int)r4(O);       // D3 row stride
    const int ntm = (mb + 15) / 16;   // GaussianModel: logstd-gradient partials per column (row tiles)
    // model.bwd2 generated on model.bwd1's operand loads (rowk 7) for narrow heads (S + 1 <= 32)
    const bool bfold = fuse && h->mfuse >= 3 && O <= 32 && h->mtile != 2 && h->unaligned_b && !h->gm && !h->srn &&
                       Dm == 2;
    auto W = [&](const std::string& n) { return h->f(n); };
    auto L_ = [](const std::string& net, int i) { return net + ".l" + std::to_string(i); };
    // hidden-layer buffer i of a chain of D layers: <p>1 (layer 0), <p>2 (the last), <p>m<i>
    auto ch = [&](const std::string& p, int i, int D) -> float* {
        if (i == 0) return W(p + "1");
        if (i == D - 1) return W(p + "2");
        return W(p + "m" + std::to_string(i));
    };
    float *Xf = W("ws.Xf"), *Tf = W("ws.Tf"), *Of = W("ws.Of");
    float *Df3 = W("ws.Df3");
    MGatherArgs mg{};
    mg.replay = W("replay"); mg.cap = h->cap; mg.stride = h->stride; mg.S = S; mg.A = A; mg.mb = mb;
    mg.idx_ring = h->ptr<int32_t>("mfit.idx"); mg.idx_cap = h->mfit_cap; mg.ctl = h->ctl();
    mg.s_mean = W("mnorm.s_mean"); mg.s_den = W("mnorm.s_den"); mg.a_mean = W("mnorm.a_mean");
    mg.a_den = W("mnorm.a_den"); mg.d_mean = W("mnorm.d_mean"); mg.d_den = W("mnorm.d_den"); mg.r_norm = W("mnorm.r");
    mg.X = Xf; mg.ldQ = ldQ; mg.T = Tf; mg.nm = nm;
    mg.clip_d = h->cfg.delta_clip_loss; mg.clip_r = h->cfg.reward_clip_loss;
    // The minibatch rows: pre-gathered (SACX_MPRE, default) -- one k_mgather per block of <= MFIT_PRE steps
    // writes step j's normalised rows / targets into staging slot j before the block's steps, whose
    // launches read slot j (enqueue_fit_step moves their slot-0 pointers); or gathered per step, on
    // model.fwd0's operand loads (rowk 6: 16x16 tiles, whose rows are whole records; the reward nets'
    // layer 0 reads the gathered X, so --separate_reward_nn keeps the gather launch) or by its own launch
    const bool pre = h->mpre != 0;
    float* Xin = pre ? W("mfit.Xs") : Xf;     // what the steps read: slot 0 of the staging, or X / T
    float* Tin = pre ? W("mfit.Ts") : Tf;
    h->mpres[h->sel] = Launch{};
    h->mpres[h->sel].kind = Launch::RNG;      // (none)
    if (pre) {
        Launch L{};
        L.kind = Launch::MGATHER;
        L.name = "model.pregather";
        L.mg = mg;
        L.mg.X = Xin;
        L.mg.T = Tin;
        L.pre_steps = 1;                      // (the block's step count, set at enqueue)
        L.grid = (nm * mb + 3) / 4;
        L.bytes = 4.0 * nm * mb * (2.0 * S + A + 1 + ldQ + O);
        h->mpres[h->sel] = L;
    }
    const bool gfold = !pre && fuse && h->mfuse >= 2 && h->mtile != 2 && h->stride % 4 == 0 && ldQ % 4 == 0 && !h->srn;
    if (!gfold && !pre) {
        Launch L{};
        L.kind = Launch::MGATHER;
        L.name = "model.gather";
        L.mg = mg;
        L.grid = (nm * mb + 3) / 4;
        L.bytes = 4.0 * nm * mb * (2.0 * S + A + 1 + ldQ + O);
        plan.push_back(L);
    }
    // forward levels (f[i]: every net's layer i, the head at its depth), backward steps from the heads
    // (b[t]: the dX through layer D - t of each net of depth D > t), dW + Adam per net
    std::vector<std::vector<GemmProb>> f(Lf + 1), b(Lf);
    std::vector<GemmProb> w, wr;
    for (int k = 0; k < nm; ++k) {
        const std::string n = "m" + std::to_string(k);
        const size_t r0 = (size_t)k * mb;
        for (int i = 0; i <= Dm; ++i) {
            const bool head = i == Dm;
            const float* in = i == 0 ? Xin + r0 * ldQ : ch("ws.Hf", i - 1, Dm) + r0 * nmd.h[i - 1];
            const int K = i == 0 ? S + A : nmd.h[i - 1];
            if (!head) {
                f[i].push_back(prob_fwd(in, i == 0 ? ldQ : K, mb, K, W(L_(n, i)), nmd.h[i],
                                        ch("ws.Hf", i, Dm) + r0 * nmd.h[i], nmd.act[i]));
            } else {
                f[i].push_back(prob_fwd(in, K, mb, K, W(L_(n, i)), Om, fuse ? Df3 + r0 * ldO : Of + r0 * O, ACT_NONE));
                if (fuse) {   // MSEModel / GaussianModel.get_loss as the head's epilogue: C = d loss / d out, partials
                    GemmProb& p = f[i].back();
                    p.ldc = ldO;
                    p.mse = MSE_FIT | (h->gm ? MSE_GAUSS : 0) | (h->lscale ? MSE_SCALE : 0) | (h->srn ? MSE_NOREW : 0);
                    p.se_raw = Tin + r0 * O; p.ldp = O; p.part = W("ws.lf") + r0 * nt;
                    p.grad_scale = 1.f / (float)mb; p.fcoef = h->cfg.reward_loss_coef;   // the reward column's
                    if (h->gm) {
                        p.spe_raw = W(n + ".logstd");
                        p.ppart = W("ws.lgp") + (size_t)k * ntm * S;
                    }
                }
            }
        }
        for (int i = Dm; i >= 1; --i) {
            const bool head = i == Dm;
            GemmProb p = prob_dx(head ? Df3 + r0 * ldO : ch("ws.Df", i, Dm) + r0 * nmd.h[i], mb, head ? Om : nmd.h[i],
                                 W(L_(n, i)), nmd.h[i - 1], ch("ws.Hf", i - 1, Dm) + r0 * nmd.h[i - 1],
                                 ch("ws.Df", i - 1, Dm) + r0 * nmd.h[i - 1], nmd.act[i - 1]);
            if (head) p.lda = ldO;
            if (bfold && i == 1) {   // A = D2 generated from H2, D3 and W2 on load; column tile 0 stores it for model.adam
                p.A = W("ws.Hf2") + r0 * nmd.h[1]; p.wgen = W(L_(n, 2)); p.gen_act = nmd.act[1];
                p.gd = Df3 + r0 * ldO; p.gd_ld = ldO; p.g_o = O; p.gst = W("ws.Df2") + r0 * nmd.h[1]; p.gst_ld = nmd.h[1];
            }
            b[Lf - i - (Lf - Dm)].push_back(p);
        }
        for (int i = 0; i <= Dm; ++i) {
            const bool head = i == Dm;
            const float* X = i == 0 ? Xin + r0 * ldQ : ch("ws.Hf", i - 1, Dm) + r0 * nmd.h[i - 1];
            const int K = i == 0 ? S + A : nmd.h[i - 1];
            w.push_back(prob_dw(X, i == 0 ? ldQ : K, K, mb, head ? Df3 + r0 * ldO : ch("ws.Df", i, Dm) + r0 * nmd.h[i],
                                head ? Om : nmd.h[i], W(L_(n, i)), nullptr, GRP_MODEL));
            if (head) w.back().ldb = ldO;
        }
    }
    if (h->srn) {
        // --separate_reward_nn (base_world_model.py:32-37, :72-74): the reward nets ride in the same
        // launches -- their hidden layers beside the model nets', the 1-wide head with the MSE loss
        // epilogue on the targets' reward column, their dX and (own launch) dW + Adam
        float* Dr3 = W("ws.Drf3");
        for (int k = 0; k < nm; ++k) {
            const std::string n = "r" + std::to_string(k);
            const size_t r0 = (size_t)k * mb;
            for (int i = 0; i <= Dr; ++i) {
                const float* in = i == 0 ? Xin + r0 * ldQ : ch("ws.Hrf", i - 1, Dr) + r0 * nrd.h[i - 1];
                const int K = i == 0 ? S + A : nrd.h[i - 1];
                if (i < Dr) {
                    f[i].push_back(prob_fwd(in, i == 0 ? ldQ : K, mb, K, W(L_(n, i)), nrd.h[i],
                                            ch("ws.Hrf", i, Dr) + r0 * nrd.h[i], nrd.act[i]));
                } else {
                    f[i].push_back(prob_fwd(in, K, mb, K, W(L_(n, i)), 1, Dr3 + r0 * 4, ACT_NONE));
                    GemmProb& p = f[i].back();
                    p.ldc = 4;
                    p.mse = MSE_FIT;                                // N = 1: column 0 is the reward column
                    p.se_raw = Tin + r0 * O + S; p.ldp = O; p.part = W("ws.lf") + (size_t)nm * mb * nt + r0;
                    p.grad_scale = 1.f / (float)mb; p.fcoef = h->cfg.reward_loss_coef;
                }
            }
            for (int i = Dr; i >= 1; --i) {
                const bool head = i == Dr;
                GemmProb p = prob_dx(head ? Dr3 + r0 * 4 : ch("ws.Drf", i, Dr) + r0 * nrd.h[i], mb, head ? 1 : nrd.h[i],
                                     W(L_(n, i)), nrd.h[i - 1], ch("ws.Hrf", i - 1, Dr) + r0 * nrd.h[i - 1],
                                     ch("ws.Drf", i - 1, Dr) + r0 * nrd.h[i - 1], nrd.act[i - 1]);
                if (head) p.lda = 4;
                b[Dr - i].push_back(p);
            }
            for (int i = 0; i <= Dr; ++i) {
                const bool head = i == Dr;
                const float* X = i == 0 ? Xin + r0 * ldQ : ch("ws.Hrf", i - 1, Dr) + r0 * nrd.h[i - 1];
                const int K = i == 0 ? S + A : nrd.h[i - 1];
                wr.push_back(prob_dw(X, i == 0 ? ldQ : K, K, mb, head ? Dr3 + r0 * 4 : ch("ws.Drf", i, Dr) + r0 * nrd.h[i],
                                     head ? 1 : nrd.h[i], W(L_(n, i)), nullptr, GRP_MODEL));
                if (head) wr.back().ldb = 4;
            }
        }
    }
    // the fit's own tile shapes (SACX_MTILE): its 2 x 200 rows want 16x16 forward / dX tiles
    // (832 workgroups at 512 wide, against 224 as 32x32) whatever the update's batch made
    // h->tile32; the dW + Adam launch takes 32x32 tiles when its 16x16 ones exceed one round of
    // residency (HC 2,372 -> 610 tiles), the rule of add_gemm at tile32 = 2.  2: the handle's.
    const int tile32_h = h->tile32;
    if (h->mtile != 2) h->tile32 = 0;
    auto has_head = [](const std::vector<GemmProb>& ps) {
        for (const auto& p : ps)
            if (p.mse) return true;
        return false;
    };
    for (int i = 0; i <= Lf; ++i) {
        const std::string name = "model.fwd" + std::to_string(i);
        const int t32_fit = h->tile32;
        if (i == 0) {
            add_gemm(h, plan, name, f[0], false);    // (<= SACX_MAX_MODELS problems: one launch)
            if (gfold) {
                Launch& F = plan.back();
                if (F.gemm.t32 || F.gemm.dwl) { fprintf(stderr, "sacx: model.fwd0 gather needs 16x16 tiles\n"); abort(); }
                F.gemm.rowk = 6;
                F.gemm.mg = mg;
                F.name = "model.gather+fwd0";
                F.bytes += 4.0 * nm * mb * (2.0 * S + A + 1 + O);
            }
            continue;
        }
        if (!has_head(f[i])) {
            // hidden levels on 32x32 tiles (mt32 bit 2) when not inside the k_fwd2 pair
            if (h->mtile == 1 && (h->mt32 & 2) && !(i == 1 && (gfold || pre) && h->mfwd2 && S + A <= 32)) h->tile32 = 2;
        } else if (i == Lf && h->mtile == 1 && (h->mt32 & 8) && !h->gm && !h->srn) {
            h->tile32 = 2;     // the heads (+ the MSE loss epilogue) on 32x32 tiles (mt32 bit 8; MSE heads only)
        }
        add_gemm_split(h, plan, name, f[i], false);
        h->tile32 = t32_fit;
        // the gathered layer 0 and layer 1 as ONE k_fwd2 launch (SACX_MFWD2, default; K0 = S + A <= 32)
        if (i == 1 && gfold && h->mfwd2) fuse_fwd2(h, plan, "model.gather+fwd01");
        // or, pre-gathered, layer 0 (rowk 9: H0 <= 512, plain A) and layer 1 the same way
        if (i == 1 && pre && h->mfwd2 && h->mtile != 2 && S + A <= 32) {
            Launch& F0 = plan[plan.size() - 2];
            if (F0.kind == Launch::GEMM && F0.gemm.rowk == 0 && !F0.gemm.t32) {
                F0.gemm.rowk = 9;
                if (!fuse_fwd2(h, plan, "model.fwd01")) plan[plan.size() - 2].gemm.rowk = 0;
            }
        }
        if (i == Lf && fuse) plan.back().name = "model.fwd" + std::to_string(i) + "+loss";
    }
    if (!fuse) {
        Launch L{};
        L.kind = Launch::MLOSS;
        L.name = "model.loss";
        L.ml.S = S; L.ml.mb = mb; L.ml.nm = nm; L.ml.T = Tin; L.ml.O = Of; L.ml.D3 = Df3; L.ml.ldD = ldO;
        L.ml.loss_rows = W("ws.lf");
        L.ml.reward_coef = h->cfg.reward_loss_coef;
        L.grid = (nm * mb + 3) / 4;
        L.bytes = 4.0 * nm * mb * O * 3;
        plan.push_back(L);
    }
    MFinalArgs mf{};
    mf.ctl = h->ctl(); mf.loss_rows = W("ws.lf"); mf.mb = mb; mf.nm = nm;
    mf.mstats = W("mstats"); mf.mstats_cap = h->stats_cap; mf.nt = fuse ? nt : 0;
    if (h->srn) mf.nt2 = 1;            // the reward heads' partials follow the model heads' in ws.lf
    if (h->gm) {                       // the logstd gradient and Adam (or its store for the global-norm clip)
        mf.lgpart = W("ws.lgp"); mf.ntm = ntm; mf.S = S; mf.lscale = h->lscale ? 1 : 0;
        mf.gstore = h->cfg.model_max_grad_norm > 0.f ? 1 : 0;
        mf.logstd = W("m0.logstd");
        mf.lstride = nm > 1 ? (int64_t)(h->off_of("m1.logstd") - h->off_of("m0.logstd")) / 4 : 0;
        for (int k = 1; k < nm; ++k)      // (build_layout gives every model the same block)
            if ((int64_t)(h->off_of("m" + std::to_string(k) + ".logstd") - h->off_of("m0.logstd")) / 4 != k * mf.lstride) {
                fprintf(stderr, "sacx: model parameter blocks differ\n");
                abort();
            }
    }
    for (int t = 0; t < Lf; ++t) {
        const std::string name = "model.bwd" + std::to_string(Lf - t);
        if (t == Lf - 1 && bfold) {      // model.bwd2 folded: model.bwd1 generates its A operand
            add_gemm(h, plan, name, b[t], false);
            Launch& B1 = plan.back();
            if (B1.gemm.t32 || B1.gemm.dwl) { fprintf(stderr, "sacx: model.bwd1 generation needs 16x16 tiles\n"); abort(); }
            B1.name = "model.bwd2+bwd1+final";
            B1.gemm.rowk = 7;
            B1.gemm.has_mfinal = 1;
            B1.gemm.mfin = mf;
            for (const GemmProb& q : b[0]) { B1.flops += gemm_flops(q); B1.bytes += gemm_bytes(q); }
            continue;
        }
        if (t == 0 && bfold) continue;   // (in the launch above)
        const int t32_fit = h->tile32;   // the heads' dX (+ k_mfinal's workgroup): mt32 bit 4; the others bit 1
        if (h->mtile == 1 && (h->mt32 & (t == 0 ? 4 : 1))) h->tile32 = 2;
        const size_t first = plan.size();
        add_gemm_split(h, plan, name, b[t], false);
        h->tile32 = t32_fit;
        if (t == 0 && fuse) {
            Launch& B2 = plan[first];
            B2.name += "+final";
            B2.gemm.has_mfinal = 1;
            B2.gemm.mfin = mf;
        }
    }
    if (h->mtile == 1) h->tile32 = 2;
    int n_adam = add_gemm_split(h, plan, "model.adam", w, false);
    for (int j = 0; j < n_adam; ++j) plan[plan.size() - 1 - j].gemm.t_adv = fuse ? 1 : 0;
    if (!wr.empty()) {
        const int nr = add_gemm_split(h, plan, "reward.adam", wr, false);
        for (int j = 0; j < nr; ++j) plan[plan.size() - 1 - j].gemm.t_adv = 1;
        n_adam += nr;
    }
    h->tile32 = tile32_h;
    for (Launch& L : plan)           // GaussianModel fits: the head epilogue has the 16x16 form only
        if (L.kind == Launch::GEMM && L.gemm.t32)
            for (int i = 0; i < L.gemm.nprob; ++i)
                if (L.gemm.probs[i].mse & (MSE_GAUSS | MSE_NOREW)) {
                    fprintf(stderr, "sacx: GaussianModel / reward-net fit heads need 16x16 tiles\n");
                    abort();
                }
    if (h->cfg.model_max_grad_norm > 0.f) {
        // --model_max_grad_norm (mbrl_onpolicy_alg.py:315-317): the dW launches store the
        // gradients (+3 p_stride; GaussianModel's logstd gradient from mfit_final); their global
        // norm gives one scale; Adam applies g * scale over the models' whole contiguous range
        for (int a = 0; a < n_adam; ++a) {
            Launch& G = plan[plan.size() - 1 - a];
            for (int i = 0; i < G.gemm.nprob; ++i) G.gemm.probs[i].epi = EPI_STORE;
            const size_t at = G.name.find(".adam");
            G.name = G.name.substr(0, at) + ".grad" + G.name.substr(at + 5);
        }
        const AdamConsts gadam = adam_consts(h);
        std::string last = L_("m" + std::to_string(nm - 1), Dm);
        if (h->gm) last = "m" + std::to_string(nm - 1) + ".logstd";
        if (h->srn) last = L_("r" + std::to_string(nm - 1), Dr);
        const uint64_t o0 = h->off_of("m0.l0");
        const SegInfo& sl = h->seg(last);
        const int64_t n = (int64_t)((sl.off + (uint64_t)(sl.rows * sl.cols) * 4 - o0) / 4);
        float* P = h->f("m0.l0");
        Launch N{};
        N.kind = Launch::GNORM;
        N.name = "model.gnorm";
        N.gn.g = P + 3 * h->p_stride; N.gn.n = n;
        N.gn.part = W("ws.gnorm"); N.gn.scale_out = W("ws.gnorm") + GNORM_PARTS;
        N.gn.clip = (float)((double)h->cfg.model_max_grad_norm * nm);    // max_norm * self.B
        N.grid = GNORM_PARTS;
        N.bytes = 4.0 * n;
        plan.push_back(N);
        Launch U{};
        U.kind = Launch::APPLY;
        U.name = "model.adam";
        AdamApplyArgs& a = U.ap;
        a.P = P; a.n = n; a.p_stride = h->p_stride; a.group = GRP_MODEL; a.t_off = 0;
        a.grad_scale = 1.f; a.scale_dev = N.gn.scale_out;
        a.ctl = h->ctl(); a.adam = gadam; a.t_adv = fuse ? 1 : 0;
        U.grid = (int)((n + 255) / 256);
        U.bytes = 4.0 * n * 7;
        plan.push_back(U);
    }
    if (!fuse) {
        Launch L{};
        L.kind = Launch::MFINAL;
        L.name = "model.final";
        L.mf = mf;
        L.grid = 1;
        L.block = 64;
        plan.push_back(L);
    }
}

void enqueue(const Launch& L, sacx_handle* h, hipStream_t s) {
    switch (L.kind) {
        case Launch::RNG: launch_rng(L.rng, s); break;
        case Launch::GATHER: launch_gather(L.gather, s); break;
        case Launch::GEMM: launch_gemm(L.gemm, s); break;
        case Launch::AHEAD: launch_actor_head(L.head, L.fin, s); break;
        case Launch::QHEAD: launch_qhead(L.qh, s); break;
        case Launch::ABWD: launch_actor_bwd(L.ab, s); break;
        case Launch::FINAL: launch_alpha_final(L.fin, s); break;
        case Launch::MGATHER: launch_mgather(L.mg, s, L.pre_steps); break;
        case Launch::MLOSS: launch_mloss(L.ml, s); break;
        case Launch::MFINAL: launch_mfinal(L.mf, s); break;
        case Launch::ALLREDUCE:
            if (h->dp_local) break;            // sacx_dp_local_step reduces over the ranks' handles
            if (ncclAllReduce(L.ar_buf, L.ar_buf, (size_t)L.ar_count, ncclFloat32, ncclSum, h->comm, s) != ncclSuccess)
                h->nccl_failed = true;
            break;
        case Launch::APPLY: launch_adam_apply(L.ap, s); break;
        case Launch::AAPPLY: launch_alpha_apply(L.fin, s); break;
        case Launch::GNORM: launch_gnorm(L.gn, s); break;
        case Launch::LNORM: launch_ln(L.ln, s); break;
    }
}

// A fit step's launches as step j of a pre-gathered block (SACX_MPRE): the pointers into slot 0 of the
// staging (the rows mfit.Xs the first layers and the layer-0 dW read, the targets mfit.Ts of the loss)
// moved to slot j
Launch fit_step_launch(const sacx_handle* h, const Launch& L, int j) {
    Launch C = L;
    if (!h->mpre || j == 0) return C;
    const float* x0 = h->f("mfit.Xs");
    const float* t0 = h->f("mfit.Ts");
    const int64_t xs = h->seg("mfit.Xs").cols, ts = h->seg("mfit.Ts").cols;
    auto mv = [&](const float*& p) {
        if (p >= x0 && p < x0 + xs) p += (size_t)j * xs;
        else if (p >= t0 && p < t0 + ts) p += (size_t)j * ts;
    };
    if (C.kind == Launch::GEMM) {
        for (int i = 0; i < C.gemm.nprob; ++i) {
            mv(C.gemm.probs[i].A);
            mv(C.gemm.probs[i].se_raw);
        }
    } else if (C.kind == Launch::MLOSS) {
        mv(C.ml.T);
    }
    return C;
}

// The pre-gather of a block of n fit steps (none without SACX_MPRE)
void enqueue_fit_pre(sacx_handle* h, int n, hipStream_t s) {
    if (!h->mpre || h->mpres[h->sel].kind != Launch::MGATHER) return;
    Launch P = h->mpres[h->sel];
    P.pre_steps = n;
    enqueue(P, h, s);
}

// Rebuilds every bf16 weight shadow from the fp32 weights (all seeds): at each entry point that
// runs the update plans, so that parameter writes from the host reach the bf16 forward tiles
void wbf_refresh(sacx_handle* h, hipStream_t s) {
    if (!h->wbf_live || h->wbf_mats.empty()) return;
    WbfArgs a{};
    for (const auto& m : h->wbf_mats) {
        if (a.nmat == WBF_MAXM) break;
        a.W[a.nmat] = reinterpret_cast<const float*>(h->arena0 + h->off_of(m.name));
        a.S[a.nmat] = reinterpret_cast<uint16_t*>(h->arena0 + h->off_of("wbf." + m.name));
        a.K[a.nmat] = m.K;
        a.N[a.nmat] = m.N;
        ++a.nmat;
    }
    a.sstride = (int64_t)h->seed_bytes;
    a.nseeds = h->seeds;
    launch_wbf_refresh(a, s);
}

// the sampler + gather launches of a slot (the update's inputs)
bool is_prologue(const Launch& L) { return L.kind == Launch::RNG || L.kind == Launch::GATHER; }

void enqueue_step(sacx_handle* h, int slot, bool with_rng, hipStream_t s) {
    if (!with_rng)   // caller-provided randoms: perm of this update
        launch_set_pseq(h->ctl0(), slot, (int64_t)h->seed_bytes, h->seeds, s);
    for (const Launch& L : h->plan[slot]) {
        if (L.kind == Launch::RNG && !with_rng) continue;
        enqueue(L, h, s);
    }
}

// The main-stream launches of update `slot` with the alpha branch (alpha.fwd, alpha.head,
// alpha.final) of the PREVIOUS update (prev_slot >= 0) folded in:
//   alpha.fwd   -> extra problems of this update's actor forward launch(es);
//   alpha.head  -> an extra segment (rows from round4(Ra)) of this update's actor.head;
//   alpha.final -> one extra workgroup of the first GEMM after actor.head (q.fwd).
// Each folded piece computes exactly what it computed standalone (bit-identical results);
// the update's own alpha branch is left out (folded into the next update, or the tail).
// Returns false if the plans do not line up (then the caller keeps the branch separate).
bool merged_body(sacx_handle* h, int slot, int prev_slot, std::vector<Launch>& out) {
    out.clear();
    std::vector<const Launch*> pg;
    const Launch *ph = nullptr, *pf = nullptr, *pln = nullptr;
    if (prev_slot >= 0)
        for (const Launch& L : h->plan[prev_slot]) {
            if (!L.alpha_branch) continue;
            if (L.kind == Launch::GEMM) pg.push_back(&L);
            else if (L.kind == Launch::AHEAD) ph = &L;
            else if (L.kind == Launch::FINAL) pf = &L;
            else if (L.kind == Launch::LNORM) pln = &L;
        }
    size_t gi = 0;
    bool head_done = prev_slot < 0, final_done = prev_slot < 0, ln_done = pln == nullptr;
    bool afin_next = false;    // the split alpha finalisation still has its q.head half to place
    for (const Launch& L : h->plan[slot]) {
        if (is_prologue(L) || L.alpha_branch) continue;
        Launch C = L;
        if (prev_slot >= 0) {
            if (C.kind == Launch::GEMM && !head_done && gi < pg.size() && C.name.rfind("actor.fwd", 0) == 0) {
                if (!merge_gemm(C.gemm, pg[gi]->gemm)) return false;
                C.name += "+alpha";
                ++gi;
            } else if (C.kind == Launch::LNORM && !ln_done && C.ln.mode == 0) {
                // the previous update's alpha rows through the layer norm in the same launch
                C.ln.nrange = 2;
                C.ln.r[2] = pln->ln.r[0];
                C.ln.r[3] = pln->ln.r[1];
                C.grid += pln->grid;
                C.name += "+alpha";
                ln_done = true;
            } else if (!head_done && ph && (C.kind == Launch::AHEAD || (C.kind == Launch::GEMM && C.gemm.rowk == 3))) {
                // the head rows: a standalone actor.head, or the rows folded into q.fwd0
                HeadArgs& a = C.kind == Launch::AHEAD ? C.head : C.gemm.head;
                const HeadSeg& sg = ph->head.seg[0];
                if (a.nseg >= 4) return false;
                const int r0 = (a.total_rows + 3) & ~3;
                HeadSeg m = sg;
                m.r0 = r0;
                m.r1 = r0 + (sg.r1 - sg.r0);
                a.seg[a.nseg++] = m;
                a.total_rows = m.r1;
                a.alpha_mode = 1;
                a.alpha_row0 = r0;
                if (C.kind == Launch::AHEAD) {
                    C.fin = ph->fin;
                } else {
                    C.gemm.hfin = ph->fin;
                    int rb = (a.total_rows + 3) / 4 - C.gemm.head_block0;
                    if (C.gemm.mode == GM_FWD2) {
                        // k_fwd2's head workgroups hold NW / 4 groups of 4 rows; the ticketed alpha
                        // path needs the alpha rows to start a workgroup (its group 0 initialises the
                        // ticket flags and no group of an alpha workgroup may take the early return)
                        if ((r0 / 4 - C.gemm.head_block0) % (SACX_FWD2_HEAD_NW / 4) != 0) return false;
                        rb = (rb + SACX_FWD2_HEAD_NW / 4 - 1) / (SACX_FWD2_HEAD_NW / 4);
                    }
                    C.grid += rb - C.gemm.row_blocks;
                    C.gemm.row_blocks = rb;
                }
                C.name += "+alpha";
                head_done = true;
                if (C.kind == Launch::GEMM && C.gemm.mode == GM_FWD2 && pf) {
                    // k_fwd2 has no later forward launch to take it.  Split (SACX_AFIN, default): its
                    // first alpha block snapshots the finalisation's operands and the next launch's
                    // target rows finish the alpha step; else the last alpha block finalises (ticket)
                    // (qhead_block reads the snapshot unrelocated, and FinalArgs::pre shares its slot with
                    // the data-parallel alpha_g: one seed, no data-parallel ranks)
                    const bool split = h->afin && h->seeds == 1 && h->dp_ranks == 0 && !h->dp_local;
                    C.gemm.has_final = split ? 2 : 1;
                    C.gemm.fin = pf->fin;
                    if (split) {
                        C.gemm.fin.pre = h->ptr<AfinPre>("ws.afin");
                        afin_next = true;
                    } else {
                        C.name += ".final";
                    }
                    final_done = true;
                }
            } else if (afin_next && C.kind == Launch::GEMM && C.gemm.mode == GM_DX && C.gemm.rowk == 1) {
                // q.head+critic.bwd1: every target row block finishes the previous update's alpha step
                C.gemm.fin = pf->fin;
                C.gemm.fin.pre = h->ptr<AfinPre>("ws.afin");
                C.name += "+alpha.final";
                afin_next = false;
            } else if (C.kind == Launch::GEMM && head_done && !final_done && pf &&
                       C.gemm.mode == GM_FWD) {
                C.gemm.has_final = 1;
                C.gemm.fin = pf->fin;
                C.name += "+alpha.final";
                final_done = true;
            }
        }
        out.push_back(C);
    }
    return gi == pg.size() && head_done && final_done && ln_done && !afin_next;
}

// Captured chain of G updates on two streams (see the fork branch below):
//   cs: the updates, alpha branches folded one update later (merged_body) + a tail;
//   rs: sampler + gather, two updates ahead (slot double buffer).
// skip_kind >= 0 leaves that launch kind out (measurement only: sacx_time_graph)
// kt (measurement only, uncached): every k_gemm launch gets its own per-workgroup timestamp
// slots in kt->base, recorded in kt->spans as (offset, workgroups).
struct KTimeMap {
    uint64_t* base = nullptr;
    int64_t cap = 0, used = 0;
    std::vector<std::pair<int64_t, int>> spans;
    std::vector<std::string> names;
    std::vector<char> is_gemm;
    std::vector<std::pair<int, int>> rowspan;   // [first, end) workgroups that run row kernels
    std::vector<std::vector<int>> cls;          // k_fwd2: first workgroup of each problem pair's tiles
    bool rows = false;      // also stamp the row kernels (k_actor_head, k_actor_bwd): dump only
};

// Sampler batches [s, e) of a G-update call: sizes ramp 1, 2, 4, ... up to nbatch, never crossing
// a multiple of nbatch (see get_graph)
std::vector<std::pair<int, int>> sampler_batches(const sacx_handle* h, int G) {
    std::vector<std::pair<int, int>> batches;
    const int nbatch = h->nbatch;
    for (int s0 = 0, ramp = 1; s0 < G; ramp = std::min(nbatch, 2 * ramp)) {
        const int sz = std::min({ramp, nbatch - s0 % nbatch, G - s0});
        batches.push_back({s0, s0 + sz});
        s0 += sz;
    }
    return batches;
}

int get_graph(sacx_handle* h, int G, bool with_rng, hipGraphExec_t* out, int skip_kind = -1,
              KTimeMap* kt = nullptr) {
    auto key = std::make_tuple(G, with_rng ? 1 : 0, skip_kind);
    if (!kt) {
        auto it = h->graphs.find(key);
        if (it != h->graphs.end()) {
            *out = it->second;
            return 0;
        }
    }
    auto emit = [&](const Launch& L, hipStream_t st) {
        const bool timed = kt && (L.kind == Launch::GEMM || (kt->rows && (L.kind == Launch::AHEAD || L.kind == Launch::ABWD)));
        if (timed) {
            Launch C = L;
            // (a k_fwd2 launch finalises alpha in its last alpha block, not in a workgroup of its own)
            const int fin_wg = C.gemm.has_final && C.gemm.mode != GM_FWD2 ? 1 : 0;
            const int nwg1 = L.kind == Launch::GEMM
                                 ? C.gemm.total_tiles + fin_wg + (C.gemm.rowk ? C.gemm.row_blocks : 0)
                                 : (L.kind == Launch::AHEAD ? (C.head.total_rows + 3) / 4 : C.grid);
            const int nwg = nwg1 * h->seeds;   // slots of every seed (seed-major)
            if (kt->used + 2 * nwg <= kt->cap) {
                uint64_t* p = kt->base + kt->used;
                if (L.kind == Launch::GEMM) C.gemm.ktime = p;
                else if (L.kind == Launch::AHEAD) C.head.ktime = p;
                else C.ab.ktime = p;
                kt->spans.push_back({kt->used, nwg});
                kt->names.push_back(C.name);
                kt->is_gemm.push_back(L.kind == Launch::GEMM);
                if (L.kind != Launch::GEMM) kt->rowspan.push_back({0, 0});
                else if (C.gemm.rowk == 3) kt->rowspan.push_back({fin_wg, fin_wg + C.gemm.row_blocks});
                else kt->rowspan.push_back({C.gemm.total_tiles + fin_wg, nwg1});
                std::vector<int> cb;
                if (L.kind == Launch::GEMM && C.gemm.mode == GM_FWD2) {
                    const int nn = C.gemm.nprob / 2, r0 = C.gemm.rowk == 3 ? C.gemm.row_blocks : 0;
                    for (int i = 0; i < nn; ++i) cb.push_back(r0 + C.gemm.probs[nn + i].tile_begin);
                }
                kt->cls.push_back(cb);
                kt->used += 2 * nwg;
            }
            enqueue(C, h, st);
        } else {
            enqueue(L, h, st);
        }
    };
    hipStream_t cs = h->cap_stream, rs = h->rng_stream;
    const int nev = 3 * G + 1;
    for (int i = (int)h->events.size(); i < nev; ++i) {
        hipEvent_t e;
        HIPCHK(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        h->events.push_back(e);
    }
    hipEvent_t* evR = h->events.data();          // inputs of update j ready
    hipEvent_t* evS = h->events.data() + G;      // update j's body done
    hipEvent_t* evF = h->events.data() + 2 * G;  // alpha.final of update j done
    hipEvent_t evFork = h->events[3 * G];
    HIPCHK(h, hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    if (with_rng) {
        // cs: the updates, each with the previous update's alpha branch folded into its first
        //     launches (merged_body), plus the last update's alpha branch as a tail;
        // rs: sampler + gather of update j+2 into slot (j+2)%3 == (j-1)%3, once update j's
        //     actor.head (the last reader of that slot, through the folded alpha rows) has run.
        const bool merge = h->dp_ranks == 0;   // the DP mode keeps each alpha branch as its own launches
        HIPCHK(h, hipEventRecord(evFork, cs));
        HIPCHK(h, hipStreamWaitEvent(rs, evFork, 0));
        // Sampler batches [s, e): one k_rng launch draws updates s..e-1 in stream order and one
        // gather fills their slots s % nslot .. s % nslot + (e - s) - 1 -- consecutive slots (the
        // kernels address slot + u), so a batch never crosses a multiple of nbatch (nslot is
        // one).  Sizes ramp 1, 2, 4, ... up to nbatch so the first update of the graph waits
        // for one update's draws only.  Slot u%nslot is last read through update u's folded
        // alpha rows in update u+1's actor.head, so batch [s, e) is drawn after the actor.head
        // of update e-nslot, and must be done before update s.  When e <= nslot its slots are
        // fresh at graph start: their last reader is update e-1-nslot < 0 of an earlier graph
        // (update 0 folds no alpha rows), complete before this graph starts.
        const std::vector<std::pair<int, int>> batches = sampler_batches(h, G);
        const int nslot = h->nslot;
        for (int b = 0; b < (int)batches.size(); ++b) {
            const int s0 = batches[b].first, n = batches[b].second - s0;
            if ((b + 1 < (int)batches.size() && batches[b + 1].first != batches[b].second) || n < 1 ||
                s0 % nslot + n > nslot)
                return fail(h, "internal: sampler batches");
        }
        auto prologue = [&](int b) {
            const int j0 = batches[b].first, n = batches[b].second - j0;
            for (const Launch& L : h->plan[j0 % nslot]) {
                if (!is_prologue(L)) continue;
                if ((int)L.kind == skip_kind) continue;   // ablation of the sampler (stale randoms)
                Launch C = L;
                if (C.kind == Launch::RNG) {
                    C.rng.reset_seq = (b == 0);
                    C.rng.nupd = n;
                    // the segmented sampler (k_mtj_*) where the chain waits for the draw: the ramp's
                    // batches; the batches drawn ahead stay on k_rng's one CU, which the chain's
                    // launches never miss (the segmented launches take CUs: Humanoid bf16 -2 %)
                    if (b >= h->mtj_ramp) C.rng.jmin = INT32_MAX;
                } else {
                    C.gather.nupd = n;
                }
                enqueue(C, h, b == 0 && h->g_inline0 ? cs : rs);
            }
            return hipEventRecord(evR[b], b == 0 && h->g_inline0 ? cs : rs);
        };
        std::vector<int> batch_of(G, -1), emit_after(batches.size(), -1);
        for (int b = 0; b < (int)batches.size(); ++b) {
            batch_of[batches[b].first] = b;
            emit_after[b] = batches[b].second - nslot;          // <= 0: slots fresh at graph start
        }
        for (int b = 0; b < (int)batches.size(); ++b)
            if (emit_after[b] <= 0) {
                HIPCHK(h, prologue(b));
                emit_after[b] = -1;                             // drawn once: not again after update 0
                // batch 0 on the chain's stream (g_inline0): the side stream's draws continue after it
                if (b == 0 && h->g_inline0) HIPCHK(h, hipStreamWaitEvent(rs, evR[0], 0));
            }
        std::vector<Launch> body;
        for (int j = 0; j < G; ++j) {
            if (batch_of[j] >= 0) HIPCHK(h, hipStreamWaitEvent(cs, evR[batch_of[j]], 0));
            const int slot = j % nslot, prev = j > 0 ? (j - 1) % nslot : -1;
            const bool folded = merge && merged_body(h, slot, prev, body);
            if (!folded) {                    // plain order: previous alpha branch, then this body
                body.clear();
                if (prev >= 0)
                    for (const Launch& L : h->plan[prev])
                        if (L.alpha_branch) body.push_back(L);
                for (const Launch& L : h->plan[slot])
                    if (!is_prologue(L) && !L.alpha_branch) body.push_back(L);
            }
            std::vector<int> due;               // batches whose slots this update's actor.head frees
            for (int b = 0; b < (int)batches.size(); ++b)
                if (emit_after[b] == j) due.push_back(b);
            bool recorded = false;
            bool afin_skipped = false;          // ablation: the split finalisation's snapshot was never taken
            for (const Launch& L : body) {
                if ((int)L.kind == skip_kind) {
                    // ablation: the alpha.final folded into a skipped GEMM still runs
                    if (L.kind == Launch::GEMM && L.gemm.has_final) {
                        FinalArgs f = L.gemm.fin;
                        f.pre = nullptr;                 // (the split form's snapshot: finalise in place)
                        launch_alpha_final(f, cs);
                        afin_skipped = afin_skipped || L.gemm.has_final == 2;
                    }
                    continue;
                }
                if (afin_skipped && L.kind == Launch::GEMM && L.gemm.rowk == 1 && L.gemm.fin.pre != nullptr) {
                    Launch C = L;                        // its q.head half: alpha is already final in place
                    C.gemm.fin.pre = nullptr;
                    afin_skipped = false;
                    emit(C, cs);
                    continue;
                }
                emit(L, cs);
                if (!due.empty() && !recorded && L.frees_slot) {
                    HIPCHK(h, hipEventRecord(evS[j], cs));
                    recorded = true;
                }
            }
            if (!due.empty()) {
                if (!recorded) HIPCHK(h, hipEventRecord(evS[j], cs));
                HIPCHK(h, hipStreamWaitEvent(rs, evS[j], 0));
                for (int b : due) HIPCHK(h, prologue(b));
            }
        }
        for (const Launch& L : h->plan[(G - 1) % nslot])   // tail: the last update's alpha branch
            if (L.alpha_branch && (int)L.kind != skip_kind) emit(L, cs);
        HIPCHK(h, hipEventRecord(evF[0], rs));
        HIPCHK(h, hipStreamWaitEvent(cs, evF[0], 0));    // join the sampler stream
    } else {
        if (skip_kind >= 0) return fail(h, "kernel ablation needs the forked sampler graph");
        for (int j = 0; j < G; ++j) enqueue_step(h, 0, with_rng, cs);
    }
    hipGraph_t graph;
    HIPCHK(h, hipStreamEndCapture(cs, &graph));
    hipGraphExec_t exec;
    HIPCHK(h, hipGraphInstantiateWithFlags(&exec, graph, 0));
    HIPCHK(h, hipGraphDestroy(graph));
    HIPCHK(h, hipGraphUpload(exec, h->stream));   // the first replay does not pay the upload
    if (!kt) h->graphs[key] = exec;
    *out = exec;
    return 0;
}

// The one-update graphs of the drop-in loop's speculative path: gather + update of slot `slot`
// (1 or 2), reading the randoms the speculative k_rng drew there -- not slot 0, so that slot 0
// keeps the randoms of the last update a caller observed: a cancelled draw leaves no trace in it
// -- with the alpha branch of the previous speculative update (slot `prev`, -1: none) folded in
// and the update's own alpha branch left out (deferred to the next one, or to settle()).
int get_spec_graph(sacx_handle* h, int slot, int prev, hipGraphExec_t* out) {
    const auto key = std::make_tuple(-1, 64 * slot + (prev + 1), -1);   // < 0: never a get_graph key
    auto it = h->graphs.find(key);
    if (it != h->graphs.end()) {
        *out = it->second;
        return 0;
    }
    if (h->nslot <= slot || h->plan[slot].empty()) return fail(h, "internal: no spare slot for the speculative draw");
    std::vector<Launch> body;
    if (!merged_body(h, slot, prev, body)) {   // plans that do not fold: the branch, then the body
        std::vector<Launch> own;
        if (!merged_body(h, slot, -1, own)) return fail(h, "internal: speculative update body");
        body.clear();
        for (const Launch& L : h->plan[prev])
            if (L.alpha_branch) body.push_back(L);
        body.insert(body.end(), own.begin(), own.end());
    }
    HIPCHK(h, hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal));
    if (h->cfg.use_expert)                     // plain SAC: the speculative draw gathered too
        for (const Launch& L : h->plan[slot])  // (the draw stamped pseq[slot] itself)
            if (L.kind == Launch::GATHER) enqueue(L, h, h->cap_stream);
    for (const Launch& L : body) enqueue(L, h, h->cap_stream);
    hipGraph_t graph;
    HIPCHK(h, hipStreamEndCapture(h->cap_stream, &graph));
    hipGraphExec_t exec;
    HIPCHK(h, hipGraphInstantiateWithFlags(&exec, graph, 0));
    HIPCHK(h, hipGraphDestroy(graph));
    HIPCHK(h, hipGraphUpload(exec, h->stream));
    h->graphs[key] = exec;
    *out = exec;
    return 0;
}

// Single-stream segments (round 4).  A graph that forks the sampler onto a second stream pays
// two runtime costs the update chain does not: its host launch takes ~0.55 ms for 20 updates
// (0.12-0.31 ms for a single-stream graph of the same chain), and its FIRST replay takes
// ~0.17 ms longer on the device than later ones (a single-stream graph shows no such penalty;
// r04_first_replay_v1.txt, r04_single_stream_v1.txt).  A call of n <= nslot updates draws every
// input at its start anyway (all its slots are fresh), so it needs no dependency from the chain to
// the sampler: the sampler batches run as plain launches on the side stream, and the chain as one
// single-stream graph per batch segment [s, e), each behind its batch's event.  Segment graphs
// carry exactly the fork / join graph's main-stream launches: the previous segment's last alpha
// branch folded into their first update (merged_body), the call's last segment ending with the
// tail; so the results are bit-identical.  Keyed by (first slot, length, folds a previous
// branch, ends the call).
int get_seg_graph(sacx_handle* h, int s0, int n, bool has_prev, bool is_last, hipGraphExec_t* out) {
    const int nslot = h->nslot;
    // (first element -4: get_graph's keys start with G > 0, so a segment never replays a G-update graph)
    const auto key = std::make_tuple(-4, (s0 % nslot) * 1024 + n, (has_prev ? 2 : 0) + (is_last ? 1 : 0));
    auto it = h->graphs.find(key);
    if (it != h->graphs.end()) {
        *out = it->second;
        return 0;
    }
    hipStream_t cs = h->cap_stream;
    HIPCHK(h, hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    std::vector<Launch> body;
    for (int j = s0; j < s0 + n; ++j) {
        const int slot = j % nslot, prev = (j > s0 || has_prev) ? (j - 1 + nslot) % nslot : -1;
        if (!merged_body(h, slot, prev, body)) {
            hipGraph_t g;
            (void)hipStreamEndCapture(cs, &g);
            if (g) (void)hipGraphDestroy(g);
            return fail(h, "internal: segment body");
        }
        for (const Launch& L : body) enqueue(L, h, cs);
    }
    if (is_last)
        for (const Launch& L : h->plan[(s0 + n - 1) % nslot])
            if (L.alpha_branch) enqueue(L, h, cs);
    hipGraph_t graph;
    HIPCHK(h, hipStreamEndCapture(cs, &graph));
    hipGraphExec_t exec;
    HIPCHK(h, hipGraphInstantiateWithFlags(&exec, graph, 0));
    HIPCHK(h, hipGraphDestroy(graph));
    HIPCHK(h, hipGraphUpload(exec, h->stream));
    h->graphs[key] = exec;
    *out = exec;
    return 0;
}

// whether step(n) takes the single-stream segments (SACX_SEGMENTS, default on)
// (2: every call, the mid-call sampler batches behind the end of the segment holding the update
// that frees their slots)
bool use_segments(const sacx_handle* h, int64_t n, int32_t flags) {
    const char* e = std::getenv("SACX_SEGMENTS");
    const int env = e ? std::atoi(e) : 1;
    // n = 1 keeps its fork / join graph: 115 vs 134 us per warm call (r04_segments_by_n_v1.txt;
    // from n = 2 on the segments win, 202 vs 209 us, 1,316 vs 1,375 us at n = 20)
    const int nmin = std::getenv("SACX_SEG_NMIN") ? std::atoi(std::getenv("SACX_SEG_NMIN")) : 2;
    return env != 0 && flags == 0 && h->dp_ranks == 0 && !h->dp_local && n >= nmin &&
           (n <= h->nslot || (env == 2 && n <= (int64_t)1 << 24));
}

// The segments of step(n): every segment graph instantiated (prepare), or also launched (run):
// sampler batches as plain launches on the side stream, each segment behind its batch
// The sampler batches of a segmented call (n <= nslot: every slot fresh, all drawn at the call's
// start).  With the one-workgroup k_rng alone, sizes grow 1, 4, 16, ... (SACX_SEG_GROW, 0: the graphs'
// ramp 1, 2, 4, 8 aligned to nbatch): each batch still lands before its first update (a batch of k
// updates draws in ~1.5 + 11.5 k us against 61 us per update at HC), and the call has fewer segments,
// so fewer cross-stream waits and graph launches (20 updates: 3 segments instead of 6)
std::vector<std::pair<int, int>> segment_batches(const sacx_handle* h, int n) {
    static const int grow = [] { const char* e = std::getenv("SACX_SEG_GROW"); return e ? std::atoi(e) : 4; }();
    if (grow < 2 || h->rng_jump || h->rng_split || n > h->nslot) return sampler_batches(h, n);
    std::vector<std::pair<int, int>> batches;
    for (int s0 = 0, sz = 1; s0 < n; sz *= grow) {
        const int k = std::min(sz, n - s0);
        batches.push_back({s0, s0 + k});
        s0 += k;
    }
    return batches;
}

// SACX_SEG_INLINE0 (default 1): batch 0 of a segmented call drawn on the bound stream
static int seg_inline0() {
    static const int v = [] { const char* e = std::getenv("SACX_SEG_INLINE0"); return e ? std::atoi(e) : 1; }();
    return v;
}

int run_segments(sacx_handle* h, int n, bool run) {
    const auto batches = segment_batches(h, n);
    const int nb = (int)batches.size(), nslot = h->nslot;
    // segment k = batch k; batch b is drawn at the start when its slots are fresh (e <= nslot),
    // else behind the end of the segment holding update e - nslot (the one that frees them)
    std::vector<int> due_seg(nb, -1);
    for (int b = 0, k = 0; b < nb; ++b) {
        const int u = batches[b].second - nslot;
        if (u <= 0) continue;
        while (batches[k].second <= u) ++k;
        due_seg[b] = k;
    }
    std::vector<hipGraphExec_t> gx(nb);
    for (int b = 0; b < nb; ++b)
        if (get_seg_graph(h, batches[b].first, batches[b].second - batches[b].first, b > 0, b + 1 == nb, &gx[b]))
            return -1;
    if (!run) return 0;
    const int nev = 2 * nb + 1;
    for (int i = (int)h->events.size(); i < nev; ++i) {
        hipEvent_t e;
        HIPCHK(h, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        h->events.push_back(e);
    }
    hipEvent_t* evR = h->events.data();          // batch b drawn
    hipEvent_t* evE = h->events.data() + nb;     // segment k done
    hipStream_t rs = h->rng_stream;
    const int first_inline = seg_inline0();
    const int sig = h->seg_sig;
    if (sig && !h->sig_mem[0]) {
        int dev = 0, can = 0;
        HIPCHK(h, hipGetDevice(&dev));
        if (hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev) != hipSuccess || !can) {
            h->seg_sig = 0;
            return run_segments(h, n, run);
        }
        for (int w = 0; w < 2; ++w) {
            HIPCHK(h, hipExtMallocWithFlags((void**)&h->sig_mem[w], sizeof(uint64_t), hipMallocSignalMemory));
            HIPCHK(h, hipStreamWriteValue64(h->stream, h->sig_mem[w], 0, 0));
        }
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    const uint64_t base0 = h->sig_seq[0];
    auto draw = [&](int b, hipStream_t st) {
        const int j0 = batches[b].first, n_b = batches[b].second - j0;
        for (const Launch& L : h->plan[j0 % nslot]) {
            if (!is_prologue(L)) continue;
            Launch C = L;
            if (C.kind == Launch::RNG) {
                C.rng.reset_seq = (b == 0);
                C.rng.nupd = n_b;
            } else {
                C.gather.nupd = n_b;
            }
            enqueue(C, h, st);
        }
        if (sig == 0 || (b == 0 && st == h->stream && sig < 2)) return hipEventRecord(evR[b], st);
        const int w = st == h->stream ? 1 : 0;
        const hipError_t e = hipStreamWriteValue64(st, h->sig_mem[w], h->sig_seq[w] + 1, 0);
        if (e == hipSuccess) ++h->sig_seq[w];   // (the waits count on every queued write)
        return e;
    };
    auto wait_batch = [&](hipStream_t st, int b) {   // st waits for batch b's draw
        if (sig == 0 || (b == 0 && st == rs && sig < 2)) return hipStreamWaitEvent(st, evR[b], 0);
        // batch b's value: batch 0 (bound stream) is the one write of sig_mem[1] this call; side
        // stream batch b the (b - first)-th write of sig_mem[0] after this call's base
        const int w = b == 0 && first_inline ? 1 : 0;
        const uint64_t v = w ? h->sig_seq[1] : base0 + (uint64_t)(b - (first_inline ? 1 : 0)) + 1;
        return hipStreamWaitValue64(st, h->sig_mem[w], v, hipStreamWaitValueGte, ~0ull);
    };
    // the sampler follows the bound stream's earlier work but not this call's k_set_ctl (it writes
    // num_timesteps / ts_increment, which the sampler does not read): sacx_sac_step recorded
    // seg_start before launching it
    // SACX_SEG_INLINE0 (default 1): warm step(20) 1,296 vs 1,320 us, the driver's command +0.3 %
    // (r04_seg_inline0_v1.txt)
    if (first_inline) {
        // batch 0 on the bound stream itself, right before segment 0: no cross-stream hop on the
        // call's critical path; the side stream continues the draws after it
        HIPCHK(h, draw(0, h->stream));
        HIPCHK(h, wait_batch(rs, 0));
    } else {
        HIPCHK(h, hipStreamWaitEvent(rs, h->seg_start, 0));
    }
    for (int b = first_inline ? 1 : 0; b < nb; ++b)
        if (due_seg[b] < 0) HIPCHK(h, draw(b, rs));
    for (int k = 0; k < nb; ++k) {
        if (k > 0 || !first_inline) HIPCHK(h, wait_batch(h->stream, k));
        HIPCHK(h, hipGraphLaunch(gx[k], h->stream));
        bool rec = false;
        for (int b = 0; b < nb; ++b)
            if (due_seg[b] == k) {
                if (!rec) {
                    if (sig >= 2) {     // segment k done, as a write on the bound stream
                        HIPCHK(h, hipStreamWriteValue64(h->stream, h->sig_mem[1], h->sig_seq[1] + 1, 0));
                        ++h->sig_seq[1];
                        HIPCHK(h, hipStreamWaitValue64(rs, h->sig_mem[1], h->sig_seq[1], hipStreamWaitValueGte, ~0ull));
                    } else {
                        HIPCHK(h, hipEventRecord(evE[k], h->stream));
                        HIPCHK(h, hipStreamWaitEvent(rs, evE[k], 0));
                    }
                    rec = true;
                }
                HIPCHK(h, draw(b, rs));
            }
    }
    return 0;
}

// the deferred append, queued now (sacx_handle::app_defer)
// An append whose source rows are the pinned staging buffer: its workgroups (one per seed) bump
// done_host[1] once they have read them, and the next staging reuse polls that count (stage_begin)
// instead of waiting for an event marker recorded behind the launch (SACX_APP_CTR)
static int launch_staged_append(sacx_handle* h, AppendArgs g) {
    if (h->app_ctr) {
        g.done = h->done_dev + 1;
        launch_append(g, h->stream);
        if (hipGetLastError() != hipSuccess) return fail(h, "append launch");
        h->app_seq += (uint32_t)(g.nseeds > 1 ? g.nseeds : 1);
        h->app_ctr_pending = true;
        return 0;
    }
    launch_append(g, h->stream);
    if (hipGetLastError() != hipSuccess || hipEventRecord(h->pin_ev, h->stream) != hipSuccess)
        return fail(h, "append launch");
    h->pin_pending = true;
    return 0;
}

int flush_append(sacx_handle* h) {
    if (!h->app_pending) return 0;
    h->app_pending = false;
    return launch_staged_append(h, h->app_args);
}

// Queues a held append, runs a deferred alpha branch (the tail a one-update graph would have ended
// with), then undoes a queued speculative draw: the state every entry point but act / append / the
// speculative step(1) starts from.
int settle(sacx_handle* h, bool keep_rng_state = false) {
    if (flush_append(h)) return -1;
    h->ctl_known = false;
    if (h->alpha_pending >= 0) {
        const int slot = h->alpha_pending;
        h->alpha_pending = -1;
        for (const Launch& L : h->plan[slot])
            if (L.alpha_branch) enqueue(L, h, h->stream);
        HIPCHK(h, hipGetLastError());
    }
    return spec_cancel(h, keep_rng_state);
}

// The graphs sacx_sac_step(n_steps) replays: n_steps / G full graphs of G updates, then the
// remainder as ONE graph of exactly r updates (each graph pays its own sampler start-up and
// alpha tail, so one remainder graph beats a chain of power-of-two pieces).  Up to
// kMaxRemGraphs distinct remainder sizes are cached; beyond that a new remainder is split
// into cached powers of two.  The returned list is what sacx_sac_step launches and what
// sacx_prepare instantiates ahead of time.
constexpr int kMaxRemGraphs = 24;

int step_graph_list(sacx_handle* h, int64_t n_steps, bool ext, std::vector<std::pair<hipGraphExec_t, int64_t>>* out) {
    out->clear();
    const int G = ext ? 1 : h->graph_steps;
    const int64_t q = n_steps / G;
    int64_t r = n_steps % G;
    if (q > 0) {
        hipGraphExec_t g;
        if (get_graph(h, G, !ext, &g)) return -1;
        out->push_back({g, q});
    }
    if (r == 0) return 0;
    int n_rem = 0;
    for (const auto& kv : h->graphs)
        if (std::get<0>(kv.first) > 0 && std::get<0>(kv.first) != h->graph_steps && std::get<2>(kv.first) < 0) ++n_rem;
    const bool exact = h->graphs.count(std::make_tuple((int)r, ext ? 0 : 1, -1)) > 0 || n_rem < kMaxRemGraphs;
    if (exact) {
        hipGraphExec_t g;
        if (get_graph(h, (int)r, !ext, &g)) return -1;
        out->push_back({g, 1});
        return 0;
    }
    for (int p = 1 << 30; r > 0 && p >= 1; p >>= 1) {
        if (p > r) continue;
        hipGraphExec_t g;
        if (get_graph(h, p, !ext, &g)) return -1;
        out->push_back({g, 1});
        r -= p;
    }
    return 0;
}

}  // namespace

// ============================================================================ C ABI
extern "C" {

int sacx_create(const sacx_config* cfg, sacx_handle** out) {
    g_create_error.clear();
    if (!cfg || !out) {
        g_create_error = "null argument";
        return -1;
    }
    auto bad = [&](const char* m) {
        g_create_error = m;
        return -2;
    };
    if (cfg->abi_version != SACX_ABI_VERSION) return bad("abi_version mismatch");
    if (cfg->seeds < 0 || cfg->seeds > 64) return bad("seeds must be in [0, 64]");
    if (cfg->s_dim <= 0 || cfg->a_dim <= 0 || cfg->a_dim > 32) return bad("s_dim/a_dim out of range (a_dim <= 32)");
    if (cfg->activation < 0 || cfg->activation > 2) return bad("activation must be relu/tanh/elu");
    if (cfg->batch <= 0 || cfg->buffer_capacity <= 0) return bad("batch/buffer_capacity must be positive");
    if (cfg->buffer_capacity >= (int64_t(1) << 31)) return bad("buffer_capacity must be < 2^31");
    if (cfg->num_models < 0 || cfg->num_models > SACX_MAX_MODELS) return bad("num_models must be in [1, 8] (0 -> 2)");
    if (cfg->use_expert) {
        const int nmc = cfg->num_models > 0 ? cfg->num_models : 2;
        if (cfg->expert_batch <= 0) return bad("expert_batch must be positive");
        // the expert term adds model 0's and model 1's rows elementwise (SAC_expert.py:329-332): the
        // first two sections of np.array_split(perm, num_models) must hold the same number of rows
        if (nmc == 2 && (cfg->expert_batch & 1))
            return bad("expert_batch must be even with 2 models (SAC_expert.py:329-332 adds equal halves)");
        if (nmc > 2 && cfg->expert_batch % nmc == 1)
            return bad("expert_batch % num_models == 1: the two array_split sections of the expert term differ in length");
        if (nmc >= 2 && cfg->expert_batch < nmc) return bad("expert_batch < num_models");
        if (cfg->expert_capacity < cfg->expert_batch) return bad("expert_capacity < expert_batch");
        if (cfg->model_activation < 0 || cfg->model_activation > 2) return bad("model activation invalid");
        if (cfg->s_dim + 1 > 512) return bad("s_dim > 511 unsupported by the model MSE head");
    }
    for (int n = 0; n < 4; ++n)
        if (cfg->net_depth[n] < 0 || cfg->net_depth[n] > SACX_MAX_DEPTH) return bad("net_depth must be in [0, 4]");
    if (cfg->act_per_layer)
        for (int n = 0; n < 3; ++n)
            for (int l = 0; l < 2; ++l)
                if (cfg->act_layers[n][l] < 0 || cfg->act_layers[n][l] > 2) return bad("act_layers must be relu/tanh/elu");
    // every net's hidden layers: the ABI-8 lists, or the two of the older fields
    NetDims nd[4];
    {
        const int leg_w[4][2] = {{cfg->hidden[0], cfg->hidden[1]},
                                 {cfg->critic_hidden[0] > 0 ? cfg->critic_hidden[0] : cfg->hidden[0],
                                  cfg->critic_hidden[1] > 0 ? cfg->critic_hidden[1] : cfg->hidden[1]},
                                 {cfg->model_hidden[0], cfg->model_hidden[1]},
                                 {cfg->reward_hidden[0] > 0 ? cfg->reward_hidden[0] : 512,
                                  cfg->reward_hidden[1] > 0 ? cfg->reward_hidden[1] : 512}};
        for (int n = 0; n < 4; ++n) {
            if (cfg->net_depth[n] > 0) {
                for (int l = 0; l < cfg->net_depth[n]; ++l) {
                    nd[n].h.push_back(cfg->net_hidden[n][l]);
                    nd[n].act.push_back(cfg->net_acts[n][l]);
                }
                continue;
            }
            for (int l = 0; l < 2; ++l) {
                nd[n].h.push_back(leg_w[n][l]);
                int a = n == 3 ? cfg->reward_act_layers[l]
                               : cfg->act_per_layer ? cfg->act_layers[n][l] : (n == 2 ? cfg->model_activation : cfg->activation);
                nd[n].act.push_back(a);
            }
        }
        const bool used[4] = {true, true, cfg->use_expert != 0, cfg->use_expert && cfg->separate_reward_nn};
        for (int n = 0; n < 4; ++n) {
            if (!used[n]) continue;
            for (int l = 0; l < nd[n].D(); ++l) {
                if (nd[n].h[l] <= 0 || nd[n].h[l] > 512)
                    return bad("hidden sizes must be in [1, 512] (row kernels hold a row in 8 regs/lane)");
                if (nd[n].act[l] < 0 || nd[n].act[l] > 2) return bad("activations must be relu/tanh/elu");
            }
        }
    }
    if (cfg->actor_gaussian && cfg->actor_std_mult < 0.f) return bad("actor_std_mult must be positive");
    auto* h = new sacx_handle();
    h->cfg = *cfg;
    h->S = cfg->s_dim;
    h->A = cfg->a_dim;
    for (int n = 0; n < 4; ++n) h->nd[n] = nd[n];
    // the first and the last hidden layer of each net (one layer: both the same)
    h->H0 = nd[0].h.front();
    h->H1 = nd[0].h.back();
    h->Hc0 = nd[1].h.front();   // --critic_layers (nn_utils.py:86-138)
    h->Hc1 = nd[1].h.back();
    h->B = cfg->batch;
    h->cap = cfg->buffer_capacity;
    h->aact[0] = nd[0].act.front(); h->aact[1] = nd[0].act.back();
    h->cact[0] = nd[1].act.front(); h->cact[1] = nd[1].act.back();
    h->macts[0] = nd[2].act.front(); h->macts[1] = nd[2].act.back();
    h->Aout = cfg->per_state_std ? 2 * h->A : h->A;
    h->nm = cfg->use_expert ? (cfg->num_models > 0 ? cfg->num_models : 2) : 0;
    h->ne_perm = cfg->use_expert ? cfg->expert_batch : 0;
    // the update's expert rows: every row with one model, else the first two array_split sections
    // (each ceil(ne / nm) rows here: their lengths agree, checked above)
    h->ne = h->nm <= 1 ? h->ne_perm : 2 * ((h->ne_perm + h->nm - 1) / h->nm);
    h->ecap = cfg->use_expert ? cfg->expert_capacity : 0;
    h->Hm0 = cfg->use_expert ? nd[2].h.front() : 0;
    h->Hm1 = cfg->use_expert ? nd[2].h.back() : 0;
    h->gm = cfg->use_expert && cfg->gaussian_model;
    h->lscale = h->gm && cfg->scale_model_loss;
    h->srn = cfg->use_expert && cfg->separate_reward_nn;
    h->Om = h->srn ? h->S : h->S + 1;
    if (h->srn) {
        h->Hr0 = nd[3].h.front();
        h->Hr1 = nd[3].h.back();
        h->racts[0] = nd[3].act.front();
        h->racts[1] = nd[3].act.back();
    }
    // the fused plans are built for two hidden layers per net; any other depth takes the generic
    // plans (SACX_GENERIC=1 forces them at two layers too: their parity test)
    h->deep = nd[0].D() != 2 || nd[1].D() != 2 || (cfg->use_expert && nd[2].D() != 2) || (h->srn && nd[3].D() != 2);
    if (const char* e = std::getenv("SACX_GENERIC")) h->deep = h->deep || std::atoi(e) != 0;
    h->mb = cfg->use_expert ? (cfg->model_batch > 0 ? cfg->model_batch : 200) : 0;
    h->ln = cfg->actor_layer_norm != 0;
    h->ldS = (int)r4(h->S);
    h->ldQ = (int)r4(h->S + h->A);
    h->stride = (int)r4(2 * h->S + h->A + 2);
    h->Ra = 2 * h->B + h->ne;
    h->Rb = h->B + h->ne;
    h->n_norm = (3 * h->B + h->ne) * h->A;
    if (cfg->graph_steps > 0) h->graph_steps = cfg->graph_steps;
    if (h->graph_steps > 256) h->graph_steps = 256;
    if (h->graph_steps > 1 && (h->graph_steps & 1)) h->graph_steps += 1;
    if (cfg->stats_capacity > 0) h->stats_cap = cfg->stats_capacity;
    if (cfg->perm_capacity > 0) h->perm_cap = cfg->perm_capacity;
    if (h->Aout > 64) {
        delete h;
        return bad("action output > 64 unsupported");
    }
    if (const char* e = std::getenv("SACX_WBF")) h->wbf_enabled = std::atoi(e);
    build_layout(h);
    h->seeds = cfg->seeds > 1 ? cfg->seeds : 1;
    h->seed_bytes = h->seeds > 1 ? (h->arena_bytes + 65535) & ~uint64_t(65535) : h->arena_bytes;
    h->plan_seeds = cfg->single_seed_plan ? 1 : h->seeds;
    *out = h;
    return 0;
}

void sacx_destroy(sacx_handle* h) {
    if (!h) return;
    if (h->rng_stream) (void)hipStreamSynchronize(h->rng_stream);
    if (h->act_ev) (void)hipEventDestroy(h->act_ev);
    if (h->seg_start) (void)hipEventDestroy(h->seg_start);
    for (uint64_t* p : h->sig_mem)
        if (p) (void)hipFree(p);
    for (auto& kv : h->graphs) (void)hipGraphExecDestroy(kv.second);
    for (auto& m : h->mgraphs)
        for (auto& kv : m) (void)hipGraphExecDestroy(kv.second);
    for (auto& kv : h->roll_graphs) (void)hipGraphExecDestroy(kv.second);
    for (auto e : h->events) (void)hipEventDestroy(e);
    if (h->pin) (void)hipHostFree(h->pin);
    if (h->done_host) (void)hipHostFree(h->done_host);
    if (h->pin_ev) (void)hipEventDestroy(h->pin_ev);
    if (h->cap_stream) (void)hipStreamDestroy(h->cap_stream);
    if (h->rng_stream) (void)hipStreamDestroy(h->rng_stream);
    if (h->comm) (void)ncclCommDestroy(h->comm);
    delete h;
}

const char* sacx_last_error(const sacx_handle* h) {
    if (!h) return g_create_error.c_str();
    return h->err.c_str();
}

int64_t sacx_arena_bytes(const sacx_handle* h) { return h ? (int64_t)h->total_bytes() : -1; }

int64_t sacx_seed_stride(const sacx_handle* h) { return h ? (int64_t)h->seed_bytes : -1; }

int sacx_seed_select(sacx_handle* h, int32_t seed) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (seed < 0 || seed >= h->seeds) return fail(h, "seed out of range");
    h->sel = seed;
    h->arena = h->arena0 + (uint64_t)seed * h->seed_bytes;
    return 0;
}

int sacx_layout(const sacx_handle* h, sacx_segment* segs, int32_t cap, int32_t* n_out) {
    if (!h || !n_out) return -1;
    *n_out = (int32_t)h->segs.size();
    if (!segs) return 0;
    for (int i = 0; i < (int)h->segs.size() && i < cap; ++i) {
        const SegInfo& s = h->segs[i];
        std::memset(&segs[i], 0, sizeof(sacx_segment));
        std::strncpy(segs[i].name, s.name.c_str(), sizeof(segs[i].name) - 1);
        segs[i].offset = s.off;
        segs[i].rows = s.rows;
        segs[i].cols = s.cols;
        segs[i].dtype = s.dtype;
        segs[i].role = s.role;
    }
    return 0;
}

int sacx_bind(sacx_handle* h, void* arena, uint64_t bytes, void* stream) {
    if (!h) return -1;
    if (!arena || bytes < h->total_bytes()) return fail(h, "arena missing or too small");
    if (((uintptr_t)arena) & 255) return fail(h, "arena must be 256-byte aligned");
    if (h->bound) return fail(h, "handle already bound");
    h->arena = h->arena0 = static_cast<char*>(arena);
    h->sel = 0;
    h->stream = static_cast<hipStream_t>(stream);
    h->probs.clear();
    {   // ws.ones: the B-row scale of unscaled dW problems
        const SegInfo& so = h->seg("ws.ones");
        std::vector<float> ones((size_t)(so.rows * so.cols), 1.0f);
        for (int k = 0; k < h->seeds; ++k)
            HIPCHK(h, hipMemcpy(h->arena0 + (uint64_t)k * h->seed_bytes + so.off, ones.data(), ones.size() * sizeof(float),
                                hipMemcpyHostToDevice));
    }
    if (h->rng_jump) {   // rng.jc: the segmented sampler's jump coefficients
        const SegInfo& sj = h->seg("rng.jc");
        std::vector<int32_t> jc;
        int64_t used = 0;
        try {   // (a C entry point: no exception may leave it -- bad_alloc, or the charpoly search failing)
            jc.resize((size_t)mt_jump_lists_words(h->jsmax - 1, MTJ_CH));
            used = mt_jump_lists(h->jL, h->jsmax - 1, MTJ_CH, jc.data());
        } catch (const std::exception& e) {
            return fail(h, std::string("segmented sampler jump coefficients: ") + e.what());
        }
        for (int k = 0; k < h->seeds; ++k)
            HIPCHK(h, hipMemcpy(h->arena0 + (uint64_t)k * h->seed_bytes + sj.off, jc.data(), (size_t)used * sizeof(int32_t),
                                hipMemcpyHostToDevice));
    }
    // 32x32 forward / dX tiles once the launches are wide: seeds x batch >= 1024 rows (packed
    // seeds; Humanoid B = 1024: SAC-EO +5.6 %, model fit +8 %, SAC +1 %); a handle-level rule, so
    // the launches merged_body folds together always agree.  From 4,096 rows the dW + Adam
    // launches take 32x32 tiles too (tools/t32_dw.sh: Humanoid 4 seeds +3.5 %, 8 seeds +5 %,
    // bf16 4 seeds +8 %, HC 32 seeds +1.9 %; HC 8 / 16 seeds and one Humanoid seed even or worse)
    auto t32_of = [](int64_t rows) { return rows >= 4096 ? 1 : rows >= 1024 ? 2 : 0; };
    h->tile32 = t32_of((int64_t)h->seeds * h->B);
    h->tile32_plan = t32_of((int64_t)h->plan_seeds * h->B);
    if (const char* e = std::getenv("SACX_T32")) h->tile32 = h->tile32_plan = std::atoi(e);
    // dW + Adam over >= 512 batch rows (Humanoid B = 1,024) on k_dwl: LDS-DMA staged 128-B row
    // pieces instead of the fragment-shaped column loads, bit-identical results
    if (const char* e = std::getenv("SACX_DWL")) h->dwl = std::atoi(e);
    if (const char* e = std::getenv("SACX_DW_ROUND")) h->dw_round_tiles = std::atoi(e);
    if (const char* e = std::getenv("SACX_MFUSE")) h->mfuse = std::atoi(e);
    if (const char* e = std::getenv("SACX_MTILE")) h->mtile = std::atoi(e);
    if (const char* e = std::getenv("SACX_MT32")) h->mt32 = std::atoi(e);
    if (const char* e = std::getenv("SACX_UNALIGNED")) h->unaligned_b = std::atoi(e);
    if (const char* e = std::getenv("SACX_FWD2")) h->fwd2 = std::atoi(e);
    if (const char* e = std::getenv("SACX_AFIN")) h->afin = std::atoi(e);
    if (const char* e = std::getenv("SACX_MFWD2")) h->mfwd2 = std::atoi(e);
    if (const char* e = std::getenv("SACX_MPRE")) h->mpre = std::atoi(e);
    if (const char* e = std::getenv("SACX_DWL_NH")) h->dwl_nh = std::atoi(e) == 2 ? 2 : 1;
    // Sampler batch: each batch start is a cross-stream wait on the chain (~1 us of gap), so a
    // cheap sampler takes 8 updates per launch (HC one seed, A/B x2: 13.55k vs 13.38k at 4);
    // an expensive one (Humanoid: 52k normals, 146 us per update) keeps 4, where the graph's
    // ramp and the sampler's lead over the chain favour smaller batches (5.80k vs 5.62k at 8)
    // (16 updates per k_rng launch measured within noise of 8 -- HC 2,000 updates 16.22k / 16.30k against
    // 16.15k / 16.17k, profiles/r06_ab_nbatch_v1.txt -- and slowed the profiled run: 10.2k updates/s
    // and 7.73 us per k_gemm / k_fwd2 launch under rocprofv3 against 16.1k and 6.92 at 8; SACX_NBATCH=16)
    h->nbatch = h->n_norm <= 16384 ? 8 : 4;
    if (const char* e = std::getenv("SACX_NBATCH"))   // (k_rng alone takes batches up to half the ring)
        h->nbatch = std::max(1, std::min(h->rng_jump || h->rng_split ? NBATCH_MAX : NSLOT / 2, std::atoi(e)));
    if (const char* e = std::getenv("SACX_MTJ_RAMP")) h->mtj_ramp = std::atoi(e);
    if (const char* e = std::getenv("SACX_MTJ_UNDER")) h->mtj_under = std::atoi(e);
    while (h->nslot % h->nbatch || h->nslot < 2 * h->nbatch) --h->nbatch;   // the ring holds whole batches
    if (h->dp_ranks > 0) {
        if (h->cfg.use_expert) return fail(h, "data-parallel mode covers plain SAC (use_expert = 0)");
        const int64_t d = (int64_t)(h->off_of("t0.l0") - h->off_of("q0.l0"));
        for (int l = 0; l <= h->nd[1].D(); ++l)
            for (int k = 0; k < 2; ++k)
                if ((int64_t)(h->off_of("t" + std::to_string(k) + ".l" + std::to_string(l)) -
                              h->off_of("q" + std::to_string(k) + ".l" + std::to_string(l))) != d)
                    return fail(h, "internal: target layout is not a fixed shift of the critics");
    }
    // the weight shadows feed the update plans' 32x32 bf16 forward tiles; the Adam epilogues
    // keep them current (not the data-parallel modes, whose Adam runs in k_adam_apply)
    h->wbf_attach = (!h->wbf_mats.empty() || !h->abf_segs.empty()) && h->tile32 > 0 && h->dp_ranks == 0;
    h->wbf_live = h->wbf_attach;
    for (int sl = 0; sl < h->nslot; ++sl) {
        h->abf_written.clear();
        if (h->deep) build_plan_generic(h, sl, sl == 0);
        else build_plan(h, sl, sl == 0);
    }
    h->abf_written.clear();
    h->wbf_attach = false;
    for (int sl = 1; sl < h->nslot; ++sl) {
        if (h->plan[0].size() != h->plan[sl].size()) return fail(h, "internal: slot plans differ");
        for (size_t i = 0; i < h->plan[0].size(); ++i)
            if (h->plan[0][i].kind == Launch::GEMM &&
                (h->plan[0][i].gemm_first != h->plan[sl][i].gemm_first ||
                 h->plan[0][i].gemm_first + h->plan[0][i].gemm.nprob > (int)h->probs.size()))
                return fail(h, "internal: GEMM problem table mismatch");
    }
    h->mplans.assign(h->seeds, {});
    h->mpres.assign(h->seeds, Launch{});
    h->mgraphs.assign(h->seeds, {});
    h->mfit_hosts.assign(h->seeds, 0);
    {
        const int cur = h->probs_cursor;
        build_model_plan(h);                  // seed 0's; the others' on their first model_fit
        h->probs_cursor = cur;
    }
    HIPCHK(h, hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking));
    HIPCHK(h, hipStreamCreateWithFlags(&h->rng_stream, hipStreamNonBlocking));
    HIPCHK(h, hipEventCreateWithFlags(&h->act_ev, hipEventDisableTiming));
    if (const char* e = std::getenv("SACX_SPEC")) h->spec_enabled = std::atoi(e) != 0;
    if (const char* e = std::getenv("SACX_ACT_RNG")) h->act_rng = std::atoi(e) != 0;
    if (const char* e = std::getenv("SACX_ACT_POLL")) h->act_poll = std::atoi(e) != 0;
    h->cur_size_host = 0;
    h->bound = true;
    return 0;
}

int sacx_resync(sacx_handle* h) {
    if (!h || !h->bound) return fail(h, "not bound");
    h->alpha_pending = -1;                   // the restored state is authoritative
    h->ctl_known = false;
    if (spec_cancel(h, true)) return -1;
    Ctl c{};
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(&c, h->ctl(), sizeof(Ctl), hipMemcpyDeviceToHost));
    h->seq_host = c.step_seq;
    h->cur_size_host = c.cur_size;
    h->mfit_hosts[h->sel] = c.mfit_seq;
    return 0;
}

int sacx_dp_unique_id(void* id_out, int32_t cap) {
    if (!id_out || cap < (int32_t)sizeof(ncclUniqueId)) return -1;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -2;
    std::memcpy(id_out, &id, sizeof(id));
    return (int)sizeof(id);
}

int sacx_dp_init(sacx_handle* h, const void* id, int32_t nranks, int32_t rank) {
    if (!h) return -1;
    if (h->bound) return fail(h, "sacx_dp_init must precede sacx_bind");
    if (h->comm) return fail(h, "data-parallel communicator already set");
    if (h->seeds > 1) return fail(h, "data-parallel mode needs seeds = 1");
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(h, "bad data-parallel arguments");
    if (h->cfg.use_expert) return fail(h, "data-parallel mode covers plain SAC (use_expert = 0)");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const ncclResult_t r = ncclCommInitRank(&h->comm, nranks, uid, rank);
    if (r != ncclSuccess) return fail(h, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    h->dp_ranks = nranks;
    h->dp_rank = rank;
    return 0;
}

int sacx_dp_init_local(sacx_handle* h, int32_t nranks, int32_t rank) {
    if (!h) return -1;
    if (h->bound) return fail(h, "sacx_dp_init_local must precede sacx_bind");
    if (h->comm || h->dp_ranks) return fail(h, "data-parallel mode already set");
    if (h->seeds > 1) return fail(h, "data-parallel mode needs seeds = 1");
    if (nranks < 1 || nranks > DP_LOCAL_MAX || rank < 0 || rank >= nranks) return fail(h, "bad data-parallel arguments");
    if (h->cfg.use_expert) return fail(h, "data-parallel mode covers plain SAC (use_expert = 0)");
    h->dp_ranks = nranks;
    h->dp_rank = rank;
    h->dp_local = true;
    return 0;
}

int sacx_dp_local_step(sacx_handle* const* hs, int32_t nranks, int64_t n_steps, int64_t num_timesteps,
                       int32_t ts_increment) {
    if (!hs || nranks < 1 || nranks > DP_LOCAL_MAX) return -1;
    sacx_handle* h0 = hs[0];
    for (int r = 0; r < nranks; ++r) {
        sacx_handle* h = hs[r];
        if (!h || !h->bound) return fail(h0, "rank handle not bound");
        if (!h->dp_local || h->dp_ranks != nranks || h->dp_rank != r)
            return fail(h0, "handles must be ranks 0..n-1 of one sacx_dp_init_local group, in rank order");
        if (h->stream != h0->stream) return fail(h0, "the ranks' handles must be bound to one stream");
    }
    if (n_steps <= 0) return 0;
    hipStream_t s = h0->stream;
    for (int r = 0; r < nranks; ++r)
        launch_set_ctl(hs[r]->ctl0(), num_timesteps, ts_increment, 0, 1, s);
    for (int64_t j = 0; j < n_steps; ++j) {
        std::vector<size_t> pos(nranks, 0);
        for (;;) {
            // every rank up to its next all-reduce (or its end), in rank order, on the one stream
            int at_ar = 0;
            for (int r = 0; r < nranks; ++r) {
                const std::vector<Launch>& pl = hs[r]->plan[0];
                while (pos[r] < pl.size() && pl[pos[r]].kind != Launch::ALLREDUCE) enqueue(pl[pos[r]++], hs[r], s);
                at_ar += pos[r] < pl.size();
            }
            if (at_ar == 0) break;
            if (at_ar != nranks) return fail(h0, "internal: the ranks' plans do not line up");
            DpSumArgs a{};
            a.nranks = nranks;
            a.n = hs[0]->plan[0][pos[0]].ar_count;
            for (int r = 0; r < nranks; ++r) {
                const Launch& L = hs[r]->plan[0][pos[r]];
                if (L.ar_count != a.n) return fail(h0, "internal: all-reduce sizes differ");
                a.buf[r] = L.ar_buf;
                ++pos[r];
            }
            launch_dp_sum(a, s);
        }
    }
    HIPCHK(h0, hipGetLastError());
    for (int r = 0; r < nranks; ++r) hs[r]->seq_host += n_steps;
    return 0;
}

int sacx_buffer_append(sacx_handle* h, const float* s, const float* a, const float* r, const float* sp,
                       const float* d, int64_t n) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (n <= 0) return 0;
    if (!s || !a || !r || !sp || !d) return fail(h, "null row pointer");
    if (flush_append(h)) return -1;           // appends stay in call order
    AppendArgs g{};
    g.replay = h->f("replay"); g.cap = h->cap; g.stride = h->stride; g.S = h->S; g.A = h->A;
    g.s = s; g.a = a; g.r = r; g.sp = sp; g.d = d; g.n = n; g.ctl = h->ctl();
    launch_append(g, h->stream);
    HIPCHK(h, hipGetLastError());
    h->cur_size_host = std::min<int64_t>(h->cur_size_host + n, h->cap);
    ++h->n_appends;
    return 0;
}

// Host-pointer variants for the env loop (one transition / one observation per call).  The
// rows go into one pinned, device-mapped buffer that the kernels read (k_append, the obs
// normaliser) and write (the action head) in place over PCIe: no DMA copy on either side,
// whose fixed cost exceeds the whole transfer at these sizes.
static int stage_alloc(sacx_handle* h) {
    if (!h->pin) {
        HIPCHK(h, hipHostMalloc((void**)&h->pin, sizeof(float) * 2 * STAGE_CAP, hipHostMallocMapped));
        HIPCHK(h, hipHostGetDevicePointer((void**)&h->pin_dev, h->pin, 0));
        HIPCHK(h, hipEventCreateWithFlags(&h->pin_ev, hipEventDisableTiming));
        HIPCHK(h, hipHostMalloc((void**)&h->done_host, 64, hipHostMallocMapped));
        HIPCHK(h, hipHostGetDevicePointer((void**)&h->done_dev, h->done_host, 0));
        __atomic_store_n(h->done_host, 0u, __ATOMIC_RELEASE);
        __atomic_store_n(h->done_host + 1, 0u, __ATOMIC_RELEASE);
        h->done_seq = 0;
    }
    return 0;
}

static inline void cpu_relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
}

// The act_host rows' outputs are on the host once the counter reaches done_seq: spin on it (a
// few us) instead of waiting for the whole stream position (k_act_rng's sampler workgroup, the
// event's own latency).  An act queued behind a long stream prefix (step(G), a model fit) would
// keep spinning, so past ACT_SPIN the stream is waited for instead; a counter still short then
// is an error, and done_seq is resynchronised from the counter so later acts do not wait on it.
static constexpr auto ACT_SPIN = std::chrono::microseconds(2000);   // > one update graph (the drop-in cadence)
static int act_rows_wait(sacx_handle* h) {
    if (!h->act_poll) return hipEventSynchronize(h->act_ev) == hipSuccess ? 0 : fail(h, "act event");
    const uint32_t target = h->done_seq;
    auto reached = [&]() { return (int32_t)(__atomic_load_n(h->done_host, __ATOMIC_ACQUIRE) - target) >= 0; };
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 1; !reached(); ++it) {
        cpu_relax();
        if ((it & 255) == 0 && std::chrono::steady_clock::now() - t0 > ACT_SPIN) {
            const hipError_t e = h->act_ev_live ? hipEventSynchronize(h->act_ev) : hipStreamSynchronize(h->stream);
            if (e != hipSuccess || !reached()) {
                h->done_seq = __atomic_load_n(h->done_host, __ATOMIC_ACQUIRE);
                return fail(h, e != hipSuccess ? "act event" : "act rows finished without their completion count");
            }
            break;
        }
    }
    return 0;
}
// the append half: waits until its last reader (a k_append) has finished
static int stage_begin(sacx_handle* h) {
    if (stage_alloc(h)) return -1;
    if (h->app_ctr_pending) {           // the held append's workgroup has read the rows
        const uint32_t target = h->app_seq;
        auto reached = [&]() { return (int32_t)(__atomic_load_n(h->done_host + 1, __ATOMIC_ACQUIRE) - target) >= 0; };
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t it = 1; !reached(); ++it) {
            cpu_relax();
            if ((it & 255) == 0 && std::chrono::steady_clock::now() - t0 > ACT_SPIN) {
                HIPCHK(h, hipStreamSynchronize(h->stream));
                if (!reached()) return fail(h, "held append finished without its completion count");
                break;
            }
        }
        h->app_ctr_pending = false;
    }
    if (h->pin_pending) HIPCHK(h, hipEventSynchronize(h->pin_ev));   // its last reader has finished
    h->pin_pending = false;
    return 0;
}

int sacx_buffer_append_host(sacx_handle* h, const float* s, const float* a, const float* r, const float* sp,
                            const float* d, int64_t n) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (n <= 0) return 0;
    if (!s || !a || !r || !sp || !d) return fail(h, "null row pointer");
    const int S = h->S, A = h->A;
    const int64_t per = 2 * S + A + 2, chunk = STAGE_CAP / per;
    if (chunk <= 0) return fail(h, "a transition is larger than the pinned staging buffer (use sacx_buffer_append)");
    if (flush_append(h)) return -1;           // (a held one first: appends stay in call order)
    // the drop-in cadence: hold the row for the next act's launch (sacx_handle::app_defer)
    const bool defer = n == 1 && h->app_defer && h->last_step_one && h->seeds == 1 && spec_mode(h) && h->act_rng;
    for (int64_t done = 0; done < n; done += chunk) {
        const int64_t m = std::min(chunk, n - done);
        if (stage_begin(h)) return -1;
        float* p = h->pin;
        std::memcpy(p, s + done * S, sizeof(float) * m * S);
        std::memcpy(p + m * S, a + done * A, sizeof(float) * m * A);
        std::memcpy(p + m * (S + A), r + done, sizeof(float) * m);
        std::memcpy(p + m * (S + A + 1), sp + done * S, sizeof(float) * m * S);
        std::memcpy(p + m * (2 * S + A + 1), d + done, sizeof(float) * m);
        const float* g = h->pin_dev;
        if (defer) {
            AppendArgs& ap = h->app_args;
            ap = AppendArgs{};
            ap.replay = h->f("replay"); ap.cap = h->cap; ap.stride = h->stride; ap.S = S; ap.A = A;
            ap.s = g; ap.a = g + m * S; ap.r = g + m * (S + A); ap.sp = g + m * (S + A + 1); ap.d = g + m * (2 * S + A + 1);
            ap.n = m; ap.ctl = h->ctl();
            h->app_pending = true;
            h->cur_size_host = std::min<int64_t>(h->cur_size_host + m, h->cap);
            ++h->n_appends;
            continue;
        }
        AppendArgs ag{};
        ag.replay = h->f("replay"); ag.cap = h->cap; ag.stride = h->stride; ag.S = S; ag.A = A;
        ag.s = g; ag.a = g + m * S; ag.r = g + m * (S + A); ag.sp = g + m * (S + A + 1); ag.d = g + m * (2 * S + A + 1);
        ag.n = m; ag.ctl = h->ctl();
        if (launch_staged_append(h, ag)) return -1;
        h->cur_size_host = std::min<int64_t>(h->cur_size_host + m, h->cap);
        ++h->n_appends;
    }
    return 0;
}

// The speculative draw (see sacx_handle::spec_live): the sampler launch of slot 1 or 2 for one
// update at the ring's current size, queued on the bound stream; it saves the state it starts
// from into "rng.spec" for spec_cancel.
static int spec_rng_args(sacx_handle* h, RngArgs* out) {
    const int slot = h->alpha_pending == 1 ? 2 : 1;    // not the slot a deferred alpha branch reads
    const Launch* R = nullptr;
    for (const Launch& L : h->plan[slot])
        if (L.kind == Launch::RNG) { R = &L; break; }
    if (!R) return fail(h, "internal: no sampler launch");
    RngArgs r = R->rng;
    // stamps pseq[slot] with the update that follows: step_seq, + 1 while a deferred
    // alpha.final has not counted the previous update yet
    r.reset_seq = h->alpha_pending >= 0 ? 2 : 1;
    h->spec_slot = slot;
    r.nupd = 1;
    r.size_fixed = 0;           // each seed's ring size, read on the device (final until the update)
    r.backup = reinterpret_cast<RngState*>(h->arena0 + h->off_of("rng.spec"));   // seed 0's (relocated per seed)
    *out = r;
    return 0;
}

// after the speculative sampler launch: plain SAC's gather too (SAC-EO's reads the permutation the
// caller pushes before the update), and the draw's bookkeeping
static int spec_after_rng(sacx_handle* h) {
    if (!h->cfg.use_expert)
        for (const Launch& L : h->plan[h->spec_slot])
            if (L.kind == Launch::GATHER) {
                if (!h->spec_polar_live) {
                    enqueue(L, h, h->stream);
                    continue;
                }
                Launch G = L;                  // + the draw's polar transform (sacx_handle::spec_polar)
                G.gather.pairs = h->ptr<uint32_t>("rng.spairs");
                G.gather.pairs_oi = h->ptr<int32_t>("rng.spairs_oi");
                for (const Launch& R : h->plan[h->spec_slot])
                    if (R.kind == Launch::RNG) G.gather.norm = R.rng.out_norm;
                G.gather.n_norm = h->n_norm;
                G.gather.polar_wgs = std::min(16, (h->spcap + 255) / 256);
                enqueue(G, h, h->stream);
            }
    h->spec_polar_live = false;
    HIPCHK(h, hipGetLastError());
    h->spec_live = true;
    h->spec_size = h->cur_size_host;
    h->spec_appends = h->n_appends;
    return 0;
}

static int spec_draw(sacx_handle* h) {
    RngArgs r;
    if (spec_rng_args(h, &r)) return -1;
    launch_rng(r, h->stream);
    return spec_after_rng(h);
}

// k_act_rows' arguments for n <= ACT_ROWS_MAX observation rows of the selected seed
static ActRowArgs act_rows_args(sacx_handle* h, const float* obs, float* noise, float* act_out) {
    ActRowArgs a{};
    a.obs = obs; a.s_mean = h->f("norm.s_mean"); a.s_den = h->f("norm.s_den");
    a.W0 = h->f("actor.l0"); a.W1 = h->f("actor.l1"); a.W3 = h->f("actor.l2"); a.logstd = h->f("actor.logstd");
    a.noise = noise; a.out = act_out;
    a.S = h->S; a.A = h->A; a.Aout = h->Aout; a.H0 = h->H0; a.H1 = h->H1;
    a.act0 = h->aact[0]; a.act1 = h->aact[1];
    a.mode = h->cfg.actor_gaussian ? 2 : 1;
    a.per_state_std = h->cfg.per_state_std;
    a.lim = h->cfg.act_limit;
    if (h->cfg.actor_gaussian) {          // logstd_init (continuous_actors.py:39-44), f32
        const double sm = h->cfg.actor_std_mult > 0.f ? h->cfg.actor_std_mult : 1.0;
        a.logstd_init = (float)(std::log(sm) - (h->cfg.per_state_std ? std::log(std::log(2.0)) : 0.0));
        a.output_norm = h->cfg.actor_output_norm;
    }
    return a;
}
static int actor_act(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out,
                     uint32_t* done);
static bool act_rows_ok(const sacx_handle* h, int64_t n) {
    return n > 0 && n <= ACT_ROWS_MAX && !h->ln && h->nd[0].D() == 2 && h->S <= ACT_ROWS_DIM && h->H0 <= ACT_ROWS_DIM &&
           h->H1 <= ACT_ROWS_DIM && h->Aout <= 64;
}

int sacx_actor_act_host(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (n < 0 || (n > 0 && (!obs || !act_out))) return fail(h, "bad arguments");
    const int S = h->S, A = h->A;
    const int64_t chunk = std::min<int64_t>(ACT_CAP, STAGE_CAP / (S + A));
    if (chunk <= 0) return fail(h, "an observation row is larger than the pinned staging buffer (use sacx_actor_act)");
    const bool spec = h->last_step_one && spec_mode(h) && !h->spec_live && h->cur_size_host > 0;
    for (int64_t done = 0; done < n; done += chunk) {
        const int64_t m = std::min(chunk, n - done);
        if (stage_alloc(h)) return -1;
        float* p = h->pin + STAGE_CAP;          // the act half: its last reader was a synchronous act
        const float* g = h->pin_dev + STAGE_CAP;
        std::memcpy(p, obs + done * S, sizeof(float) * m * S);
        // (one seed's handle only: on a packed handle the act is the selected seed's rows while the
        // draw is every seed's, which spec_draw's own sampler launch covers)
        if (spec && deterministic && h->act_rng && h->seeds == 1 && done + m >= n && act_rows_ok(h, m)) {
            // the drop-in loop's act with the next update's draw beside the rows (k_act_rng)
            RngArgs r;
            if (spec_rng_args(h, &r)) return -1;
            ActRowArgs a = act_rows_args(h, g, nullptr, (float*)g + m * S);
            a.done = h->done_dev;
            const bool app = h->app_pending;  // the held append as one more workgroup: the draw then
            if (app) r.size_fixed = h->cur_size_host;   // takes the ring size from the host
            h->app_pending = false;
            if (h->spec_polar) {
                r.pairs = h->ptr<uint32_t>("rng.spairs");
                r.pairs_oi = h->ptr<int32_t>("rng.spairs_oi");
                r.pcap = h->spcap;
                h->spec_polar_live = true;
            }
            AppendArgs ag = h->app_args;
            if (app && h->app_ctr) {
                ag.done = h->done_dev + 1;
                ++h->app_seq;
                h->app_ctr_pending = true;
            }
            launch_act_rng(a, (int)m, r, h->stream, app ? &ag : nullptr, !h->spec_polar);
            HIPCHK(h, hipGetLastError());
            h->done_seq += (uint32_t)m;
            // no event markers behind the launch: each one held the next kernel back ~7-10 us on the
            // device (r06_dropin_ab_v2.txt).  The host polls the rows' count (act_poll) and the held
            // append's own count (stage_begin)
            h->act_ev_live = !(h->act_poll && h->app_ctr);
            if (h->act_ev_live) HIPCHK(h, hipEventRecord(h->act_ev, h->stream));
            if (app && !h->app_ctr) {
                HIPCHK(h, hipEventRecord(h->pin_ev, h->stream));
                h->pin_pending = true;
            }
            if (spec_after_rng(h)) return -1;
            if (act_rows_wait(h)) return -1;
            std::memcpy(act_out + done * A, p + m * S, sizeof(float) * m * A);
            continue;
        }
        if (flush_append(h)) return -1;
        const bool rows = act_rows_ok(h, m);     // k_act_rows: the host polls the rows' count
        const int rc = actor_act(h, g, m, deterministic, (float*)g + m * S, rows ? h->done_dev : nullptr);
        if (rc) return rc;
        if (rows) h->done_seq += (uint32_t)m;    // only once the launch that counts them is queued
        h->act_ev_live = !(rows && h->act_poll && h->app_ctr);   // (a marker holds the next launch back)
        if (h->act_ev_live) HIPCHK(h, hipEventRecord(h->act_ev, h->stream));
        // the drop-in loop steps next: its randoms are drawn while the host has the action
        if (done + m >= n && spec && spec_draw(h)) return -1;
        if (rows) {
            if (act_rows_wait(h)) return -1;
        } else {
            HIPCHK(h, hipEventSynchronize(h->act_ev));
        }
        std::memcpy(act_out + done * A, p + m * S, sizeof(float) * m * A);
    }
    return 0;
}

// Every seed of a packed handle at once (one launch chain for all): the env loop of K lock-step
// runs (sac_eo.train --runs K) hands over one row per run.  Arrays are [seeds, n, ...].
int sacx_buffer_append_host_seeds(sacx_handle* h, const float* s, const float* a, const float* r, const float* sp,
                                  const float* d, int64_t n) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (flush_append(h)) return -1;
    if (n <= 0) return 0;
    if (!s || !a || !r || !sp || !d) return fail(h, "null row pointer");
    const int S = h->S, A = h->A, K = h->seeds;
    const int64_t tot = (int64_t)K * n;
    if (tot * (2 * S + A + 2) > STAGE_CAP) return fail(h, "rows exceed the pinned staging buffer (append per seed)");
    if (stage_begin(h)) return -1;
    float* p = h->pin;
    std::memcpy(p, s, sizeof(float) * tot * S);
    std::memcpy(p + tot * S, a, sizeof(float) * tot * A);
    std::memcpy(p + tot * (S + A), r, sizeof(float) * tot);
    std::memcpy(p + tot * (S + A + 1), sp, sizeof(float) * tot * S);
    std::memcpy(p + tot * (2 * S + A + 1), d, sizeof(float) * tot);
    const float* g = h->pin_dev;
    AppendArgs ag{};
    ag.replay = h->f0("replay"); ag.cap = h->cap; ag.stride = h->stride; ag.S = S; ag.A = A;
    ag.s = g; ag.a = g + tot * S; ag.r = g + tot * (S + A); ag.sp = g + tot * (S + A + 1); ag.d = g + tot * (2 * S + A + 1);
    ag.n = n; ag.ctl = h->ctl0(); ag.sstride = (int64_t)h->seed_bytes; ag.nseeds = K;
    if (launch_staged_append(h, ag)) return -1;
    h->cur_size_host = std::min<int64_t>(h->cur_size_host + n, h->cap);   // every seed grows alike
    ++h->n_appends;
    return 0;
}

int sacx_actor_act_host_seeds(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (flush_append(h)) return -1;
    if (n <= 0 || !obs || !act_out) return fail(h, "bad arguments");
    const int S = h->S, A = h->A, K = h->seeds;
    if (n > ACT_ROWS_MAX || h->ln || h->nd[0].D() != 2 || S > ACT_ROWS_DIM || h->H0 > ACT_ROWS_DIM ||
        h->H1 > ACT_ROWS_DIM || h->Aout > 64)
        return fail(h, "sacx_actor_act_host_seeds: n <= 16 rows per seed, two hidden layers, no layer norm "
                       "(use per-seed calls)");
    const int64_t tot = (int64_t)K * n;
    if (tot * (S + A) > STAGE_CAP) return fail(h, "rows exceed the pinned staging buffer (act per seed)");
    if (stage_alloc(h)) return -1;
    float* const pa = h->pin + STAGE_CAP;          // the act half (acts are synchronous)
    float* const ga = h->pin_dev + STAGE_CAP;
    std::memcpy(pa, obs, sizeof(float) * tot * S);
    float* noise = deterministic ? nullptr : h->f0("act.noise");
    if (!deterministic && spec_cancel(h)) return -1;   // a draw from the streams: undo the speculative one
    if (!deterministic) {            // each seed's u = np.random.normal(size=(n, A)) from its own stream
        RngArgs r{};
        r.st = reinterpret_cast<RngState*>(h->f0("rng")); r.ctl = h->ctl0();
        r.n_int = 0; r.n_norm = (int32_t)n * A; r.out_idx = nullptr; r.out_norm = noise;
        r.slot = -1; r.reset_seq = 0; r.nupd = 1;
        r.sstride = (int64_t)h->seed_bytes; r.nseeds = K;
        launch_rng(r, h->stream);
    }
    ActRowArgs a{};
    a.obs = ga; a.s_mean = h->f0("norm.s_mean"); a.s_den = h->f0("norm.s_den");
    a.W0 = h->f0("actor.l0"); a.W1 = h->f0("actor.l1"); a.W3 = h->f0("actor.l2"); a.logstd = h->f0("actor.logstd");
    a.noise = noise; a.out = ga + tot * S;
    a.S = S; a.A = A; a.Aout = h->Aout; a.H0 = h->H0; a.H1 = h->H1;
    a.act0 = h->aact[0]; a.act1 = h->aact[1];
    a.mode = h->cfg.actor_gaussian ? 2 : 1;
    a.per_state_std = h->cfg.per_state_std;
    a.lim = h->cfg.act_limit;
    if (h->cfg.actor_gaussian) {
        const double sm = h->cfg.actor_std_mult > 0.f ? h->cfg.actor_std_mult : 1.0;
        a.logstd_init = (float)(std::log(sm) - (h->cfg.per_state_std ? std::log(std::log(2.0)) : 0.0));
        a.output_norm = h->cfg.actor_output_norm;
    }
    a.sstride = (int64_t)h->seed_bytes; a.nseeds = K; a.m = (int32_t)n;
    a.done = h->done_dev;                   // every seed's rows count
    // lock-step drop-in cadence: every seed's next sampler draw, beside the action rows
    // (deterministic: k_act_rng) or queued behind them
    const bool spec = h->last_step_one && spec_mode(h) && !h->spec_live && h->cur_size_host > 0;
    if (spec && deterministic && h->act_rng) {
        RngArgs r;
        if (spec_rng_args(h, &r)) return -1;
        launch_act_rng(a, (int)n, r, h->stream);
        HIPCHK(h, hipGetLastError());
        h->done_seq += (uint32_t)(n * K);
        h->act_ev_live = !(h->act_poll && h->app_ctr);
        if (h->act_ev_live) HIPCHK(h, hipEventRecord(h->act_ev, h->stream));
        if (spec_after_rng(h)) return -1;
    } else {
        launch_act_rows(a, (int)n, h->stream);
        HIPCHK(h, hipGetLastError());
        h->done_seq += (uint32_t)(n * K);
        h->act_ev_live = !(h->act_poll && h->app_ctr);
        if (h->act_ev_live) HIPCHK(h, hipEventRecord(h->act_ev, h->stream));
        if (spec && spec_draw(h)) return -1;
    }
    if (act_rows_wait(h)) return -1;
    std::memcpy(act_out, pa + tot * S, sizeof(float) * tot * A);
    return 0;
}

int sacx_expert_set(sacx_handle* h, const float* s_e, const float* sp_e, int32_t n, float epsilon) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;             // alpha.final reads the epsilon this sets
    if (!h->cfg.use_expert) return fail(h, "handle was created without use_expert");
    if (n != h->ne_perm) return fail(h, "expert rows must equal expert_batch");
    const size_t bytes = sizeof(float) * (size_t)n * h->S;
    HIPCHK(h, hipMemcpyAsync(h->f("expert.s"), s_e, bytes, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(h, hipMemcpyAsync(h->f("expert.sp"), sp_e, bytes, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    Ctl* c = h->ctl();
    const int64_t nn = n;
    HIPCHK(h, hipMemcpy(&c->n_expert, &nn, sizeof(nn), hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy(&c->epsilon, &epsilon, sizeof(float), hipMemcpyHostToDevice));
    return 0;
}

int sacx_perm_push(sacx_handle* h, const int32_t* perms, int64_t n_steps) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (!h->cfg.use_expert) return 0;
    if (n_steps > h->perm_cap) return fail(h, "n_steps exceeds perm_capacity");
    int32_t* ring = h->ptr<int32_t>("perm");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    for (int64_t j = 0; j < n_steps; ++j) {
        const int64_t slot = (h->seq_host + j) % h->perm_cap;
        HIPCHK(h, hipMemcpy(ring + slot * h->ne_perm, perms + j * h->ne_perm, sizeof(int32_t) * h->ne_perm,
                            hipMemcpyHostToDevice));
    }
    return 0;
}

int sacx_rng_seed(sacx_handle* h, uint32_t seed) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h, true)) return -1;
    RngState st{};
    for (int pos = 0; pos < 624; ++pos) {       // init_genrand (seeding.py:12 -> np.random.seed)
        st.key[pos] = seed;
        seed = 1812433253U * (seed ^ (seed >> 30)) + (uint32_t)pos + 1U;
    }
    st.pos = 624;
    st.has_gauss = 0;
    st.gauss = 0.0;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(h->ptr<RngState>("rng"), &st, sizeof(st), hipMemcpyHostToDevice));
    return 0;
}

int sacx_rng_set_state(sacx_handle* h, const uint32_t key[624], int32_t pos, int32_t has_gauss, double gauss) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h, true)) return -1;
    if (pos < 0 || pos > 624) return fail(h, "pos out of range");
    RngState st{};
    std::memcpy(st.key, key, sizeof(st.key));
    st.pos = pos;
    st.has_gauss = has_gauss;
    st.gauss = gauss;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(h->ptr<RngState>("rng"), &st, sizeof(st), hipMemcpyHostToDevice));
    return 0;
}

int sacx_rng_get_state(sacx_handle* h, uint32_t key[624], int32_t* pos, int32_t* has_gauss, double* gauss) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;
    RngState st{};
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(&st, h->ptr<RngState>("rng"), sizeof(st), hipMemcpyDeviceToHost));
    std::memcpy(key, st.key, sizeof(st.key));
    *pos = st.pos;
    *has_gauss = st.has_gauss;
    *gauss = st.gauss;
    return 0;
}

int sacx_sac_step(sacx_handle* h, int64_t n_steps, int64_t num_timesteps, int32_t ts_increment, int32_t flags) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (h->dp_local) return fail(h, "in-process data-parallel ranks step together (sacx_dp_local_step)");
    if (h->cfg.actor_gaussian) return fail(h, "GaussianActor handle: inference only (sacx_actor_act)");
    if (n_steps <= 0) return 0;
    // the drop-in loop's one-update steps: the randoms drawn speculatively after the previous
    // step are valid when the ring now holds the size they assumed (nothing else drew meanwhile:
    // every other consumer of the stream undid the draw)
    if (flush_append(h)) return -1;
    const bool spec_ok = spec_mode(h) && n_steps == 1 && flags == 0;
    const bool use_spec = spec_ok && h->spec_live && h->spec_appends == h->n_appends;
    if (!use_spec && settle(h)) return -1;
    h->last_step_one = spec_ok;
    // a deferred alpha.final (folded into this update) adds ts_increment to num_timesteps before
    // this update reads it
    const int prev = use_spec ? h->alpha_pending : -1;
    const bool segs = !use_spec && !(flags & SACX_STEP_EAGER) && use_segments(h, n_steps, flags);
    if (segs) {
        // (only the side-stream batch 0 waits for it: a marker on the bound stream otherwise costs the
        // call's first launches, r06_ab_seg_sig_v1.txt)
        if (!h->seg_start) HIPCHK(h, hipEventCreateWithFlags(&h->seg_start, hipEventDisableTiming));
        if (!seg_inline0()) HIPCHK(h, hipEventRecord(h->seg_start, h->stream));
    }
    wbf_refresh(h, h->stream);
    const int64_t nts_set = num_timesteps - (prev >= 0 ? ts_increment : 0);
    if (!(use_spec && h->ctl_skip && h->ctl_known && h->ctl_nts == nts_set && h->ctl_inc == ts_increment))
        launch_set_ctl(h->ctl0(), nts_set, ts_increment, (int64_t)h->seed_bytes, h->seeds, h->stream);
    h->ctl_known = false;
    const bool ext = (flags & SACX_STEP_EXTERNAL_RANDOMS) != 0;
    if (use_spec) {
        h->spec_live = false;
        ++h->spec_hits;
        hipGraphExec_t g;                 // gather + update, the randoms already in spec_slot
        if (get_spec_graph(h, h->spec_slot, prev, &g)) return -1;
        HIPCHK(h, hipGraphLaunch(g, h->stream));
        h->alpha_pending = h->spec_slot;
        // the control block after this chain: num_timesteps (the folded alpha.final added
        // ts_increment; this update's own is deferred into the next step)
        h->ctl_known = true;
        h->ctl_nts = num_timesteps;
        h->ctl_inc = ts_increment;
    } else if (flags & SACX_STEP_EAGER) {
        for (int64_t j = 0; j < n_steps; ++j) enqueue_step(h, 0, !ext, h->stream);
        HIPCHK(h, hipGetLastError());
    } else if (segs) {
        if (run_segments(h, (int)n_steps, true)) return -1;
    } else {
        std::vector<std::pair<hipGraphExec_t, int64_t>> gl;
        if (step_graph_list(h, n_steps, ext, &gl)) return -1;
        for (const auto& g : gl)
            for (int64_t i = 0; i < g.second; ++i) HIPCHK(h, hipGraphLaunch(g.first, h->stream));
    }
    h->seq_host += n_steps;
    if (h->nccl_failed) return fail(h, "ncclAllReduce failed");
    return 0;
}

int sacx_prepare(sacx_handle* h, int64_t n_steps, int32_t flags) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;
    if (n_steps <= 0 || (flags & SACX_STEP_EAGER)) return 0;
    if (use_segments(h, n_steps, flags)) {
        if (run_segments(h, (int)n_steps, false)) return -1;
    } else {
        std::vector<std::pair<hipGraphExec_t, int64_t>> gl;
        if (step_graph_list(h, n_steps, (flags & SACX_STEP_EXTERNAL_RANDOMS) != 0, &gl)) return -1;
    }
    if (spec_mode(h) && n_steps == 1 && flags == 0) {
        hipGraphExec_t g;                 // the drop-in loop's speculative path replays these
        for (int slot = 1; slot <= 2; ++slot)
            for (int prev : {-1, 3 - slot})
                if (get_spec_graph(h, slot, prev, &g)) return -1;
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int sacx_model_fit(sacx_handle* h, const int32_t* idx, int64_t n_steps, int32_t flags) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;
    if (!h->cfg.use_expert) return fail(h, "handle was created without use_expert (no world models)");
    if (n_steps <= 0) return 0;
    if (!idx) return fail(h, "null index array");
    const int k = h->sel;                 // packed seeds: the selected seed's models and ring
    if (h->mplans[k].empty()) {
        const int cur = h->probs_cursor;
        build_model_plan(h);
        h->probs_cursor = cur;
    }
    const std::vector<Launch>& mplan = h->mplans[k];
    const int R2 = h->nm * h->mb;
    int32_t* ring = h->ptr<int32_t>("mfit.idx");
    // every step's launches read their minibatch rows from the index ring at ctl->mfit_seq, so a
    // graph of several steps replays them back to back (one graph launch per MFIT_GRAPH steps)
    // (every HIP failure is reported with its error text; the capture is ended and the captured graph
    // destroyed on every exit path, so a failed capture leaves the stream usable for the next fit)
    auto graph_of = [&](int n, hipGraphExec_t* out) -> int {
        auto it = h->mgraphs[k].find(n);
        if (it != h->mgraphs[k].end()) {
            *out = it->second;
            return 0;
        }
        HIPCHK(h, hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal));
        enqueue_fit_pre(h, n, h->cap_stream);     // (n <= MFIT_PRE)
        for (int j = 0; j < n; ++j)
            for (const Launch& L : mplan) enqueue(fit_step_launch(h, L, j), h, h->cap_stream);
        const hipError_t le = hipGetLastError();
        hipGraph_t graph = nullptr;
        const hipError_t ee = hipStreamEndCapture(h->cap_stream, &graph);
        if (le != hipSuccess || ee != hipSuccess) {
            if (graph) (void)hipGraphDestroy(graph);
            return fail(h, std::string("model-fit graph capture: ") + hipGetErrorString(le != hipSuccess ? le : ee));
        }
        hipGraphExec_t ex = nullptr;
        const hipError_t ie = hipGraphInstantiateWithFlags(&ex, graph, 0);
        (void)hipGraphDestroy(graph);
        if (ie != hipSuccess) return fail(h, std::string("model-fit graph instantiate: ") + hipGetErrorString(ie));
        h->mgraphs[k][n] = ex;
        *out = ex;
        return 0;
    };
    for (int64_t done = 0; done < n_steps;) {
        const int64_t chunk = std::min<int64_t>(n_steps - done, h->mfit_cap);
        HIPCHK(h, hipStreamSynchronize(h->stream));   // ring slots of earlier chunks are consumed
        // the chunk's slots are contiguous modulo the ring: at most two copies
        const int64_t s0 = (h->mfit_hosts[k] + done) % h->mfit_cap;
        const int64_t first = std::min<int64_t>(chunk, h->mfit_cap - s0);
        HIPCHK(h, hipMemcpy(ring + s0 * R2, idx + done * R2, sizeof(int32_t) * R2 * first, hipMemcpyHostToDevice));
        if (chunk > first)
            HIPCHK(h, hipMemcpy(ring, idx + (done + first) * R2, sizeof(int32_t) * R2 * (chunk - first),
                                hipMemcpyHostToDevice));
        const char* kdump = std::getenv("SACX_MFIT_KTIME");
        if ((flags & SACX_STEP_EAGER) && kdump) {
            // diagnostics: per-workgroup start / end stamps of every GEMM launch of each step, appended
            // to <file> as one line per launch and step: name, workgroups, span, mean / max workgroup,
            // last-start offset, gap to the previous launch's end (us)
            std::vector<int> nwg;
            int64_t tot = 0;
            for (const Launch& L : mplan) {
                const int n = L.kind == Launch::GEMM ? L.grid + (L.gemm.has_mfinal ? 1 : 0) : 0;
                nwg.push_back(n);
                tot += 2 * n;
            }
            uint64_t* kb = nullptr;
            HIPCHK(h, hipMalloc(&kb, sizeof(uint64_t) * std::max<int64_t>(1, tot)));
            std::vector<uint64_t> host((size_t)std::max<int64_t>(1, tot));
            FILE* f = std::fopen(kdump, "a");
            for (int64_t j = 0; j < chunk; ++j) {
                HIPCHK(h, hipMemsetAsync(kb, 0, sizeof(uint64_t) * std::max<int64_t>(1, tot), h->stream));
                if (j % MFIT_PRE == 0) enqueue_fit_pre(h, (int)std::min<int64_t>(MFIT_PRE, chunk - j), h->stream);
                int64_t o = 0;
                for (size_t i = 0; i < mplan.size(); ++i) {
                    Launch C = fit_step_launch(h, mplan[i], (int)(j % MFIT_PRE));
                    if (nwg[i] > 0) {
                        C.gemm.ktime = kb + o;
                        o += 2 * nwg[i];
                    }
                    enqueue(C, h, h->stream);
                }
                HIPCHK(h, hipStreamSynchronize(h->stream));
                HIPCHK(h, hipMemcpy(host.data(), kb, sizeof(uint64_t) * host.size(), hipMemcpyDeviceToHost));
                o = 0;
                uint64_t prev = 0;
                for (size_t i = 0; f && i < mplan.size(); ++i) {
                    if (nwg[i] == 0) continue;
                    uint64_t lo = UINT64_MAX, hi = 0, ls = 0, wmax = 0;
                    double wsum = 0.0;
                    int cnt = 0;
                    for (int b = 0; b < nwg[i]; ++b) {
                        const uint64_t t0 = host[o + 2 * b], t1 = host[o + 2 * b + 1];
                        if (t0 == 0 || t1 == 0) continue;           // (workgroups that return early stamp nothing)
                        lo = std::min(lo, t0); hi = std::max(hi, t1); ls = std::max(ls, t0);
                        wmax = std::max(wmax, t1 - t0); wsum += (double)(t1 - t0); ++cnt;
                    }
                    std::fprintf(f, "%s,%d,%.2f,%.2f,%.2f,%.2f,%.2f\n", mplan[i].name.c_str(), cnt, (hi - lo) * 0.01,
                                 wsum / std::max(1, cnt) * 0.01, wmax * 0.01, (ls - lo) * 0.01,
                                 prev ? ((double)lo - (double)prev) * 0.01 : 0.0);
                    prev = hi;
                    o += 2 * nwg[i];
                }
            }
            if (f) std::fclose(f);
            (void)hipFree(kb);
        } else if (flags & SACX_STEP_EAGER) {
            for (int64_t j = 0; j < chunk; ++j) {
                if (j % MFIT_PRE == 0) enqueue_fit_pre(h, (int)std::min<int64_t>(MFIT_PRE, chunk - j), h->stream);
                for (const Launch& L : mplan) enqueue(fit_step_launch(h, L, (int)(j % MFIT_PRE)), h, h->stream);
            }
            HIPCHK(h, hipGetLastError());
        } else {
            for (int64_t j = 0; j < chunk;) {
                const int n = chunk - j >= MFIT_GRAPH ? MFIT_GRAPH : chunk - j >= 8 ? 8 : 1;   // (<= MFIT_PRE)
                hipGraphExec_t ex = nullptr;
                if (graph_of(n, &ex)) return -1;
                HIPCHK(h, hipGraphLaunch(ex, h->stream));
                j += n;
            }
        }
        done += chunk;
    }
    h->mfit_hosts[k] += n_steps;
    return 0;
}

int sacx_settle(sacx_handle* h) {
    if (!h || !h->bound) return fail(h, "not bound");
    return settle(h);
}

int sacx_sync(sacx_handle* h) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;           // an observation point: the arena holds no speculative draw
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipGetLastError());
    return 0;
}

int64_t sacx_spec_hits(const sacx_handle* h) { return h ? h->spec_hits : -1; }

static int launch_info(const std::vector<Launch>& plan, sacx_launch_info* out, int32_t cap, int32_t* n_out);

int sacx_plan_info(const sacx_handle* h, sacx_launch_info* out, int32_t cap, int32_t* n_out) {
    if (!h || !n_out) return -1;
    if (!h->bound) {
        *n_out = 0;
        return -1;
    }
    return launch_info(h->plan[0], out, cap, n_out);
}

int sacx_model_plan_info(const sacx_handle* h, sacx_launch_info* out, int32_t cap, int32_t* n_out) {
    if (!h || !n_out) return -1;
    if (!h->bound || h->mplans.empty()) {
        *n_out = 0;
        return h->bound ? 0 : -1;
    }
    return launch_info(h->mplans[h->sel], out, cap, n_out);
}

static int launch_info(const std::vector<Launch>& plan, sacx_launch_info* out, int32_t cap, int32_t* n_out) {
    *n_out = (int32_t)plan.size();
    if (!out) return 0;
    for (int i = 0; i < (int)plan.size() && i < cap; ++i) {
        std::memset(&out[i], 0, sizeof(sacx_launch_info));
        std::strncpy(out[i].name, plan[i].name.c_str(), sizeof(out[i].name) - 1);
        std::strncpy(out[i].kernel, kernel_family(plan[i].kind), sizeof(out[i].kernel) - 1);
        out[i].grid = plan[i].grid;
        out[i].block = plan[i].block;
        out[i].flops = plan[i].flops;
        out[i].bytes = plan[i].bytes;
    }
    return 0;
}

int sacx_profile(sacx_handle* h, int64_t n_steps, double* ms_per_launch, int32_t cap) {
    if (h && h->bound && settle(h)) return -1;
    if (!h || !h->bound) return fail(h, "not bound");
    wbf_refresh(h, h->stream);
    const auto& plan = h->plan[0];
    const int n = (int)plan.size();
    std::vector<hipEvent_t> ev(n + 1);
    for (auto& e : ev) HIPCHK(h, hipEventCreate(&e));
    std::vector<double> acc(n, 0.0);
    for (int64_t s = 0; s < n_steps; ++s) {
        launch_spin(3000.0, h->stream);   // the host queues the whole step while the GPU waits
        HIPCHK(h, hipEventRecord(ev[0], h->stream));
        for (int i = 0; i < n; ++i) {
            enqueue(plan[i], h, h->stream);
            HIPCHK(h, hipEventRecord(ev[i + 1], h->stream));
        }
        HIPCHK(h, hipEventSynchronize(ev[n]));
        for (int i = 0; i < n; ++i) {
            float ms = 0.f;
            HIPCHK(h, hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            acc[i] += ms;
        }
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    h->seq_host += n_steps;
    for (int i = 0; i < n && i < cap; ++i) ms_per_launch[i] = acc[i];
    return 0;
}

// The hidden layers of net `net` (nd: its widths / activations) on m rows of X (row stride ldX, K0
// inputs), alternating between H1b and H2b (layer 0 -> H1b, layer 1 -> H2b, ...); returns the
// buffer holding the last hidden layer.  The actor's --actor_layer_norm puts Dense -> LayerNorm ->
// tanh on layer 0 (nn_utils.py:110-119).  Eager launches on st (or captured by the caller).
static float* net_hidden(sacx_handle* h, const std::string& net, const NetDims& nd, const float* X, int ldX, int K0,
                         int m, float* H1b, float* H2b, hipStream_t st, bool ln = false) {
    const float* in = X;
    int ld = ldX, K = K0;
    float* out = H1b;
    for (int i = 0; i < nd.D(); ++i) {
        out = (i & 1) ? H2b : H1b;
        std::vector<Launch> pl;
        add_gemm(h, pl, net + ".fwd", {prob_fwd(in, ld, m, K, h->f(net + ".l" + std::to_string(i)), nd.h[i], out,
                                                (i == 0 && ln) ? ACT_NONE : nd.act[i])}, false);
        h->probs_cursor -= 1;      // host table bookkeeping of add_gemm (these launches are not in a plan)
        launch_gemm(pl[0].gemm, st);
        if (i == 0 && ln) {
            LNArgs a{};
            a.mode = 0; a.H = nd.h[0]; a.Z = out; a.nrange = 1; a.r[1] = m; a.gamma = h->f("actor.ln");
            launch_ln(a, st);
        }
        in = out;
        ld = K = nd.h[i];
    }
    return out;
}

static float* actor_hidden(sacx_handle* h, const float* X, int ldX, int m, float* H1b, float* H2b, hipStream_t st) {
    return net_hidden(h, "actor", h->nd[0], X, ldX, h->S, m, H1b, H2b, st, h->ln);
}

static int actor_act(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out,
                     uint32_t* done);
int sacx_actor_act(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out) {
    return actor_act(h, obs, n, deterministic, act_out, nullptr);
}
// done: the rows' completion counter (act_host; k_act_rows path only)
static int actor_act(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out,
                     uint32_t* done) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (!deterministic && spec_cancel(h)) return -1;   // a draw from the stream: undo the speculative one
    if (n < 0 || (n > 0 && (!obs || !act_out))) return fail(h, "bad arguments");
    const int S = h->S, A = h->A, H1 = h->H1, ldS = h->ldS;
    auto W = [&](const std::string& nm) { return h->f(nm); };
    if (act_rows_ok(h, n)) {
        // the env loop's few rows: the noise draw, then one workgroup per row (k_act_rows)
        float* noise = deterministic ? nullptr : W("act.noise");
        if (!deterministic) {          // u = np.random.normal(size=(n, A)) from the global stream
            RngArgs r{};
            r.st = h->ptr<RngState>("rng"); r.ctl = h->ctl();
            r.n_int = 0; r.n_norm = (int32_t)n * A; r.out_idx = nullptr; r.out_norm = noise;
            r.slot = -1; r.reset_seq = 0; r.nupd = 1;
            launch_rng(r, h->stream);
        }
        ActRowArgs a = act_rows_args(h, obs, noise, act_out);
        a.done = done;
        launch_act_rows(a, (int)n, h->stream);
        HIPCHK(h, hipGetLastError());
        return 0;
    }
    for (int64_t done = 0; done < n; done += ACT_CAP) {
        const int m = (int)std::min<int64_t>(ACT_CAP, n - done);
        float* noise = deterministic ? nullptr : W("act.noise");
        if (!deterministic) {          // u = np.random.normal(size=(m, A)) from the global stream
            RngArgs r{};
            r.st = h->ptr<RngState>("rng"); r.ctl = h->ctl();
            r.n_int = 0; r.n_norm = m * A; r.out_idx = nullptr; r.out_norm = noise;
            r.slot = -1; r.reset_seq = 0; r.nupd = 1;
            launch_rng(r, h->stream);
        }
        launch_obs_norm(obs + done * S, m, S, W("norm.s_mean"), W("norm.s_den"), W("act.X"), ldS, h->stream);
        HeadArgs a{};
        a.H2 = actor_hidden(h, W("act.X"), ldS, m, W("act.H1"), W("act.H2"), h->stream);
        a.ldh = H1; a.W3 = W(actor_head_name(h)); a.logstd = W("actor.logstd");
        a.H1 = H1; a.A = A; a.Aout = h->Aout; a.S = S; a.ldQ = h->ldQ; a.per_state_std = h->cfg.per_state_std;
        a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
        a.nseg = 1;
        // SquashedGaussianActor.sample (mode 1) or GaussianActor.sample (mode 2)
        a.seg[0] = {0, m, h->cfg.actor_gaussian ? 2 : 1, 0, noise, nullptr, nullptr, act_out + done * A};
        if (h->cfg.actor_gaussian) {          // logstd_init (continuous_actors.py:39-44), f32
            const double sm = h->cfg.actor_std_mult > 0.f ? h->cfg.actor_std_mult : 1.0;
            a.logstd_init = (float)(std::log(sm) - (h->cfg.per_state_std ? std::log(std::log(2.0)) : 0.0));
            a.output_norm = h->cfg.actor_output_norm;
        }
        a.total_rows = m;
        a.cache_row0 = 1 << 30;
        a.alpha_mode = 0;
        FinalArgs f{};
        launch_actor_head(a, f, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

// ---------------------------------------------------------------- reference object methods
// model = true: the world models' normaliser set (MSEModel calls), else the update's (QCritic)
static NetIOArgs netio_base(sacx_handle* h, bool model = false) {
    auto W = [&](const std::string& nm) { return h->f(nm); };
    auto N = [&](const char* x) { return model ? W(mnorm(h, x)) : W(std::string("norm.") + x); };
    NetIOArgs g{};
    g.S = h->S; g.A = h->A;
    g.s_mean = N("s_mean"); g.s_den = N("s_den"); g.a_mean = N("a_mean"); g.a_den = N("a_den");
    g.d_mean = N("d_mean"); g.d_den = N("d_den"); g.r_norm = N("r"); g.ret_den = W("norm.ret_den");
    g.reward_coef = h->cfg.reward_loss_coef;
    return g;
}

int sacx_actor_evaluate(sacx_handle* h, const float* s, int64_t n, float* pi_out, float* nlp_out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;
    if (h->cfg.actor_gaussian) return fail(h, "GaussianActor handle: inference only (sacx_actor_act)");
    if (n < 0 || (n > 0 && (!s || !pi_out || !nlp_out))) return fail(h, "bad arguments");
    const int S = h->S, A = h->A, H1 = h->H1, ldS = h->ldS;
    auto W = [&](const std::string& nm) { return h->f(nm); };
    for (int64_t done = 0; done < n; done += ACT_CAP) {
        const int m = (int)std::min<int64_t>(ACT_CAP, n - done);
        RngArgs r{};                   // u = np.random.normal(size=np.shape(a_mean)) (:351)
        r.st = h->ptr<RngState>("rng"); r.ctl = h->ctl();
        r.n_int = 0; r.n_norm = m * A; r.out_idx = nullptr; r.out_norm = W("act.noise");
        r.slot = -1; r.reset_seq = 0; r.nupd = 1;
        launch_rng(r, h->stream);
        launch_obs_norm(s + done * S, m, S, W("norm.s_mean"), W("norm.s_den"), W("act.X"), ldS, h->stream);
        HeadArgs a{};
        a.H2 = actor_hidden(h, W("act.X"), ldS, m, W("act.H1"), W("act.H2"), h->stream);
        a.ldh = H1; a.W3 = W(actor_head_name(h)); a.logstd = W("actor.logstd");
        a.H1 = H1; a.A = A; a.Aout = h->Aout; a.S = S; a.ldQ = h->ldQ; a.per_state_std = h->cfg.per_state_std;
        a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
        a.nseg = 1;
        a.seg[0] = {0, m, 0, 0, W("act.noise"), nullptr, nlp_out + done, pi_out + done * A};   // mode 0: evaluate
        a.total_rows = m;
        a.cache_row0 = 1 << 30;
        FinalArgs f{};
        launch_actor_head(a, f, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

int sacx_critic_forward(sacx_handle* h, int32_t net, const float* s, const float* a, int64_t n, int32_t value,
                        float* out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;
    if (net < 0 || net > 3) return fail(h, "net must be 0..3 (q0, q1, t0, t1)");
    if (n < 0 || (n > 0 && (!s || !a || !out))) return fail(h, "bad arguments");
    const int S = h->S, A = h->A, H1 = h->Hc1, ldQ = h->ldQ;   // the critics' sizes
    auto W = [&](const std::string& nm) { return h->f(nm); };
    static const char* names[4] = {"q0", "q1", "t0", "t1"};
    const std::string nm = names[net];
    for (int64_t done = 0; done < n; done += ACT_CAP) {
        const int m = (int)std::min<int64_t>(ACT_CAP, n - done);
        NetIOArgs g = netio_base(h);
        g.mode = 0; g.n = m; g.ldX = ldQ; g.s = s + done * S; g.a = a + done * A; g.X = W("act.Xq");
        launch_net_io(g, h->stream);
        float* Hl = net_hidden(h, nm, h->nd[1], W("act.Xq"), ldQ, S + A, m, W("act.H1"), W("act.H2"), h->stream);
        std::vector<Launch> pl;
        add_gemm(h, pl, "critic.head", {prob_fwd(Hl, H1, m, H1, W(nm + ".l" + std::to_string(h->nd[1].D())), 1, W("act.Q"),
                                                 ACT_NONE)}, false);
        launch_gemm(pl[0].gemm, h->stream);
        h->probs_cursor -= 1;
        g.mode = 1; g.O = W("act.Q"); g.ldO = 1; g.value = value ? 1 : 0; g.out0 = out + done;
        launch_net_io(g, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

// The world model's GEMM launches on the m rows of roll.Xm (stream st): the model net roll.Xm ->
// M1 -> M2 -> roll.O [m, S+1] (its Om columns), and with --separate_reward_nn the reward net
// (base_world_model.py:72-74) in the same launches into roll.O's reward column.  Model k's rows
// start at row k * rstride of M1 / M2 / O / R1 / R2 (nk models on the same inputs: the diagnostics)
static void model_gemms(sacx_handle* h, const std::vector<int>& models, int m, int64_t rstride, hipStream_t st,
                        const char* tag) {
    const int S = h->S, A = h->A, ldQ = h->ldQ, O = S + 1;
    auto W = [&](const std::string& nm) { return h->f(nm); };
    const NetDims& nmd = h->nd[2];
    const NetDims& nrd = h->nd[3];
    const int Dm = nmd.D(), Dr = h->srn ? nrd.D() : 0, Lf = std::max(Dm, Dr);
    // the hidden layers alternate between the two buffers of each net (layer 0 -> M1 / R1, layer 1 ->
    // M2 / R2, ...): their row stride is the layer's width, so model i's rows start at i * rstride * width
    auto hb = [&](const char* b1, const char* b2, int i, int w, size_t mi) {
        return W((i & 1) ? b2 : b1) + mi * rstride * w;
    };
    std::vector<std::vector<GemmProb>> lv(Lf + 1);
    for (size_t mi = 0; mi < models.size(); ++mi) {
        const std::string mn = "m" + std::to_string(models[mi]);
        float* Oo = W("roll.O") + mi * rstride * O;
        for (int i = 0; i <= Dm; ++i) {
            const float* in = i == 0 ? W("roll.Xm") : hb("roll.M1", "roll.M2", i - 1, nmd.h[i - 1], mi);
            const int K = i == 0 ? S + A : nmd.h[i - 1];
            if (i < Dm) {
                lv[i].push_back(prob_fwd(in, i == 0 ? ldQ : K, m, K, W(mn + ".l" + std::to_string(i)), nmd.h[i],
                                         hb("roll.M1", "roll.M2", i, nmd.h[i], mi), nmd.act[i]));
            } else {
                lv[i].push_back(prob_fwd(in, K, m, K, W(mn + ".l" + std::to_string(i)), h->Om, Oo, ACT_NONE));
                lv[i].back().ldc = O;
            }
        }
        if (h->srn) {     // the reward net into roll.O's reward column (base_world_model.py:72-74)
            const std::string rn = "r" + std::to_string(models[mi]);
            for (int i = 0; i <= Dr; ++i) {
                const float* in = i == 0 ? W("roll.Xm") : hb("roll.R1", "roll.R2", i - 1, nrd.h[i - 1], mi);
                const int K = i == 0 ? S + A : nrd.h[i - 1];
                if (i < Dr) {
                    lv[i].push_back(prob_fwd(in, i == 0 ? ldQ : K, m, K, W(rn + ".l" + std::to_string(i)), nrd.h[i],
                                             hb("roll.R1", "roll.R2", i, nrd.h[i], mi), nrd.act[i]));
                } else {
                    lv[i].push_back(prob_fwd(in, K, m, K, W(rn + ".l" + std::to_string(i)), 1, Oo + S, ACT_NONE));
                    lv[i].back().ldc = O;
                }
            }
        }
    }
    std::vector<Launch> pl;
    const std::string t(tag);
    int np = 0;
    for (int i = 0; i <= Lf; ++i) {
        add_gemm_split(h, pl, t + ".fwd" + std::to_string(i), lv[i], false);
        np += (int)lv[i].size();
    }
    for (auto& L : pl) launch_gemm(L.gemm, st);
    h->probs_cursor -= np;   // add_gemm's table (not a plan)
}

// the model net on rows [c0, c0 + m) of (s, a): roll.Xm -> roll.M1 -> roll.M2 -> roll.O
static void model_net_chunk(sacx_handle* h, int32_t model, const float* s, const float* a, int m) {
    NetIOArgs g = netio_base(h, true);
    g.mode = 0; g.n = m; g.ldX = h->ldQ; g.s = s; g.a = a; g.X = h->f("roll.Xm");
    launch_net_io(g, h->stream);
    model_gemms(h, {model}, m, 0, h->stream, "model");
}

// GaussianModel noise (continuous_models.py:40, :61): np.random.normal(size=(m, S)) from the device
// stream into roll.mnoise (+ offset rows)
static void model_noise_draw(sacx_handle* h, int64_t rows, int64_t row0, hipStream_t st) {
    RngArgs r{};
    r.st = h->ptr<RngState>("rng"); r.ctl = h->ctl();
    r.n_int = 0; r.n_norm = (int32_t)(rows * h->S); r.out_idx = nullptr;
    r.out_norm = h->f("roll.mnoise") + row0 * h->S;
    r.slot = -1; r.reset_seq = 0; r.nupd = 1;
    launch_rng(r, st);
}

int sacx_model_sample(sacx_handle* h, int32_t model, const float* s, const float* a, int64_t n,
                      int32_t stochastic, float delta_clip, float reward_clip, float* pred_out, float* sp_out,
                      float* r_out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;
    if (!h->cfg.use_expert) return fail(h, "the world models exist only with use_expert");
    if (model < 0 || model >= h->nm) return fail(h, "model index out of range (num_models)");
    if (n < 0 || (n > 0 && (!s || !a))) return fail(h, "bad arguments");
    const int S = h->S;
    const bool noisy = stochastic && h->gm;
    for (int64_t done = 0; done < n; done += ROLL_CAP) {
        const int m = (int)std::min<int64_t>(ROLL_CAP, n - done);
        model_net_chunk(h, model, s + done * S, a + done * h->A, m);
        if (noisy) model_noise_draw(h, m, 0, h->stream);   // chunks in row order: one draw of (n, S)
        NetIOArgs g = netio_base(h, true);
        g.mode = 2; g.n = m; g.s = s + done * S; g.O = h->f("roll.O"); g.ldO = S + 1;
        g.clip_d = delta_clip; g.clip_r = reward_clip;
        g.out0 = pred_out ? pred_out + done * (S + 1) : nullptr;
        g.out1 = sp_out ? sp_out + done * S : nullptr;
        g.out2 = r_out ? r_out + done : nullptr;
        if (noisy) {
            g.mlogstd = h->f("m" + std::to_string(model) + ".logstd");
            g.mnoise = h->f("roll.mnoise");
        }
        launch_net_io(g, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

int sacx_model_forward(sacx_handle* h, int32_t model, const float* s, const float* a, int64_t n, float delta_clip,
                       float reward_clip, float* pred_out, float* sp_out, float* r_out) {
    return sacx_model_sample(h, model, s, a, n, 0, delta_clip, reward_clip, pred_out, sp_out, r_out);
}

int sacx_model_loss(sacx_handle* h, int32_t model, const float* s, const float* sp, const float* a, const float* r,
                    int64_t n, float delta_clip_loss, float reward_clip_loss, float* loss_out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (settle(h)) return -1;
    if (!h->cfg.use_expert) return fail(h, "the world models exist only with use_expert");
    if (model < 0 || model >= h->nm) return fail(h, "model index out of range (num_models)");
    if (n <= 0 || !s || !sp || !a || !r || !loss_out) return fail(h, "bad arguments");
    const int S = h->S, A = h->A;
    for (int64_t done = 0; done < n; done += ROLL_CAP) {
        const int m = (int)std::min<int64_t>(ROLL_CAP, n - done);
        model_net_chunk(h, model, s + done * S, a + done * A, m);      // _forward(s, a, clip=False)
        NetIOArgs g = netio_base(h, true);
        g.mode = 3; g.n = m; g.s = s + done * S; g.sp = sp + done * S; g.r = r + done;
        g.O = h->f("roll.O"); g.ldO = S + 1;
        g.clip_d = delta_clip_loss; g.clip_r = reward_clip_loss;
        g.out0 = h->f("roll.noise");           // running sum (workspace scalar)
        g.out1 = loss_out;
        if (h->gm) {                           // GaussianModel.get_loss (continuous_models.py:101-131)
            g.mlogstd = h->f("m" + std::to_string(model) + ".logstd");
            g.lscale = h->lscale ? 1 : 0;
        }
        g.first = done == 0; g.last = done + m >= n; g.n_total = n;
        launch_net_io(g, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

// the launches of one rollout call on stream st (eager, or captured by sacx_rollout)
static void enqueue_rollout(sacx_handle* h, int32_t model, const float* s_init, int64_t n, int32_t horizon,
                     int32_t deterministic, float delta_clip, float reward_clip, float* s_out, float* a_out,
                     float* r_out, float* sp_out, uint8_t* d_out, hipStream_t st) {
    const int S = h->S, A = h->A, H1 = h->H1, ldS = h->ldS, ldQ = h->ldQ;
    auto W = [&](const std::string& nm) { return h->f(nm); };
    const std::string mn = "m" + std::to_string(model);
    // steps outer, chunks inner: each step draws normal(size=(n, A)) in row order, exactly the
    // reference's one draw per step (samplers.py:92) however the rows are chunked
    for (int t = 0; t < horizon; ++t) {
        for (int64_t c0 = 0; c0 < n; c0 += ROLL_CAP) {
            const int m = (int)std::min<int64_t>(ROLL_CAP, n - c0);
            RollArgs ra{};
            ra.n = m; ra.S = S; ra.A = A; ra.H = horizon; ra.t = t; ra.ldS = ldS; ra.ldQ = ldQ;
            ra.s_init = s_init + c0 * S;
            ra.s_out = s_out + c0 * horizon * S; ra.a_out = a_out + c0 * horizon * A;
            ra.r_out = r_out + c0 * horizon; ra.sp_out = sp_out + c0 * horizon * S; ra.d_out = d_out + c0 * horizon;
            ra.O = W("roll.O"); ra.a_raw = W("roll.A"); ra.X = W("roll.X"); ra.Xm = W("roll.Xm");
            ra.s_mean = W("norm.s_mean"); ra.s_den = W("norm.s_den");          // the actor's
            ra.ms_mean = W("mnorm.s_mean"); ra.ms_den = W("mnorm.s_den");      // the model's
            ra.d_mean = W("mnorm.d_mean"); ra.d_den = W("mnorm.d_den"); ra.r_norm = W("mnorm.r");
            ra.clip_d = delta_clip; ra.clip_r = reward_clip;
            if (h->gm) {               // GaussianModel.step: exp(logstd) * u (continuous_models.py:38-41)
                ra.mlogstd = W(mn + ".logstd");
                ra.mnoise = W("roll.mnoise");
            }
            ra.mode = 0;
            launch_roll(ra, st);
            float* noise = deterministic ? nullptr : W("roll.noise");
            if (!deterministic) {      // actor.sample: u = np.random.normal(size=(m, A))
                RngArgs r{};
                r.st = h->ptr<RngState>("rng"); r.ctl = h->ctl();
                r.n_int = 0; r.n_norm = m * A; r.out_idx = nullptr; r.out_norm = noise;
                r.slot = -1; r.reset_seq = 0; r.nupd = 1;
                launch_rng(r, st);
            }
            HeadArgs a{};
            a.H2 = actor_hidden(h, W("roll.X"), ldS, m, W("roll.H1"), W("roll.H2"), st);
            a.ldh = H1; a.W3 = W(actor_head_name(h)); a.logstd = W("actor.logstd");
            a.H1 = H1; a.A = A; a.Aout = h->Aout; a.S = S; a.ldQ = ldQ; a.per_state_std = h->cfg.per_state_std;
            a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
            a.ma_mean = W("mnorm.a_mean"); a.ma_den = W("mnorm.a_den");
            a.nseg = 1;
            // sample(): raw action to roll.A, normalised clip(a) (= a: |lim tanh| <= lim) into
            // the action columns of the model input
            a.seg[0] = {0, m, 1, 0, noise, W("roll.Xm"), nullptr, W("roll.A")};
            a.total_rows = m;
            a.cache_row0 = 1 << 30;
            a.alpha_mode = 0;
            FinalArgs f{};
            launch_actor_head(a, f, st);
            model_gemms(h, {model}, m, 0, st, "roll.m");
            if (h->gm) model_noise_draw(h, m, 0, st);    // after the actor's draw (samplers.py:93-95)
            ra.mode = 1;
            launch_roll(ra, st);
        }
    }
}

int sacx_rollout(sacx_handle* h, int32_t model, const float* s_init, int64_t n, int32_t horizon,
                 int32_t deterministic, float delta_clip, float reward_clip, float* s_out, float* a_out,
                 float* r_out, float* sp_out, uint8_t* d_out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (!h->cfg.use_expert) return fail(h, "rollout needs the world models (use_expert)");
    if (model < 0 || model >= h->nm) return fail(h, "model index out of range (num_models)");
    if (n < 0 || horizon < 0) return fail(h, "bad arguments");
    if (n == 0 || horizon == 0) return 0;
    if (!s_init || !s_out || !a_out || !r_out || !sp_out || !d_out) return fail(h, "null output");
    if (h->gm && n > ROLL_CAP)   // one step's draws: the actor's (n, A), then the model's (n, S)
        return fail(h, "GaussianModel rollout: at most 4096 trajectories per call (the draws of a step interleave)");
    if (settle(h)) return -1;
    // one captured graph per (model, shape, clips, pointers): the Python host keeps its
    // staging / output buffers per shape, so repeated calls replay (SACX_ROLL_GRAPH=0: eager)
    const char* rg = std::getenv("SACX_ROLL_GRAPH");
    if (rg && std::atoi(rg) == 0) {
        enqueue_rollout(h, model, s_init, n, horizon, deterministic, delta_clip, reward_clip, s_out, a_out, r_out,
                        sp_out, d_out, h->stream);
        HIPCHK(h, hipGetLastError());
        return 0;
    }
    RollKey key{model, h->sel, n, horizon, deterministic, delta_clip, reward_clip, {s_init, s_out, a_out, r_out, sp_out, d_out}};
    hipGraphExec_t ge = nullptr;
    for (auto& kv : h->roll_graphs)
        if (std::memcmp(&kv.first, &key, sizeof(RollKey)) == 0) ge = kv.second;
    if (!ge) {
        HIPCHK(h, hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal));
        enqueue_rollout(h, model, s_init, n, horizon, deterministic, delta_clip, reward_clip, s_out, a_out, r_out,
                        sp_out, d_out, h->cap_stream);
        hipGraph_t g;
        HIPCHK(h, hipStreamEndCapture(h->cap_stream, &g));
        const hipError_t e = hipGraphInstantiateWithFlags(&ge, g, 0);
        (void)hipGraphDestroy(g);
        if (e != hipSuccess) return fail(h, std::string("rollout graph: ") + hipGetErrorString(e));
        if (h->roll_graphs.size() >= 4) {          // a few shapes live at once; drop the oldest
            (void)hipGraphExecDestroy(h->roll_graphs.front().second);
            h->roll_graphs.erase(h->roll_graphs.begin());
        }
        h->roll_graphs.push_back({key, ge});
    }
    HIPCHK(h, hipGraphLaunch(ge, h->stream));
    return 0;
}

int sacx_expert_diag(sacx_handle* h, const float* s_e, const float* a_e, const float* sp_e, int32_t n,
                     int32_t flags, float delta_clip, float* out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (!h->cfg.use_expert) return fail(h, "expert diagnostics need the world models (use_expert)");
    if (n <= 0 || n > 2048) return fail(h, "expert rows must be in [1, 2048]");
    const bool disc = (flags & SACX_DIAG_DISC) != 0, ea = (flags & SACX_DIAG_EXPERT_ACTIONS) != 0;
    if (disc && h->nm < 2) return fail(h, "_calc_disc compares two world models (num_models >= 2)");
    if (!s_e || !sp_e || !out || (ea && !a_e) || (!disc && !a_e)) return fail(h, "null argument");
    if (settle(h)) return -1;
    const int S = h->S, A = h->A, H1 = h->H1, ldS = h->ldS, ldQ = h->ldQ;
    auto W = [&](const std::string& nm) { return h->f(nm); };
    DiagArgs d{};
    d.n = n; d.S = S; d.A = A; d.ldS = ldS; d.ldQ = ldQ;
    d.s_e = s_e; d.a_e = a_e; d.sp_e = sp_e; d.O = W("roll.O"); d.X = W("roll.X"); d.Xm = W("roll.Xm");
    d.s_mean = W("norm.s_mean"); d.s_den = W("norm.s_den");                 // the actor's
    d.ms_mean = W("mnorm.s_mean"); d.ms_den = W("mnorm.s_den");             // the models'
    d.a_mean = W("mnorm.a_mean"); d.a_den = W("mnorm.a_den");
    d.d_mean = W("mnorm.d_mean"); d.d_den = W("mnorm.d_den"); d.clip_d = delta_clip; d.out = out;
    // every model on the same n input rows: model k's rows land at [k n, (k+1) n)
    // (one model: its MSE twice, the mean is exact); _calc_disc reads models 0 and 1
    std::vector<int> all;
    for (int k = 0; k < std::max(2, h->nm); ++k) all.push_back(h->nm > 1 ? k : 0);
    d.nmod = (int)all.size();
    auto models = [&](bool two) {
        model_gemms(h, two ? std::vector<int>{0, 1} : all, n, n, h->stream, "diag.m");
    };
    // actor.sample(s_e, deterministic=False) (continuous_actors.py:270-306) into the action columns
    auto counterfactual = [&]() {
        RngArgs r{};
        r.st = h->ptr<RngState>("rng"); r.ctl = h->ctl();
        r.n_int = 0; r.n_norm = n * A; r.out_idx = nullptr; r.out_norm = W("roll.noise");
        r.slot = -1; r.reset_seq = 0; r.nupd = 1;
        launch_rng(r, h->stream);
        HeadArgs a{};
        a.H2 = actor_hidden(h, W("roll.X"), ldS, n, W("roll.H1"), W("roll.H2"), h->stream);
        a.ldh = H1; a.W3 = W(actor_head_name(h)); a.logstd = W("actor.logstd");
        a.H1 = H1; a.A = A; a.Aout = h->Aout; a.S = S; a.ldQ = ldQ; a.per_state_std = h->cfg.per_state_std;
        a.lim = h->cfg.act_limit; a.a_mean = W("norm.a_mean"); a.a_den = W("norm.a_den");
        a.ma_mean = W("mnorm.a_mean"); a.ma_den = W("mnorm.a_den");
        a.nseg = 1;
        a.seg[0] = {0, n, 1, 0, W("roll.noise"), W("roll.Xm"), nullptr, W("roll.A")};
        a.total_rows = n;
        a.cache_row0 = 1 << 30;
        FinalArgs f{};
        launch_actor_head(a, f, h->stream);
    };
    d.mode = 0;
    d.a_e = (disc && !ea) ? nullptr : a_e;
    launch_diag(d, h->stream);
    if (disc) {                      // _calc_disc (SAC_expert.py:427-460)
        if (!ea) counterfactual();
        models(true);
        if (h->gm) {                 // model.sample(deterministic=False): (n, S) for every model in order
            model_noise_draw(h, (int64_t)h->nm * n, 0, h->stream);
            d.mlogstd[0] = W("m0.logstd");
            d.mlogstd[1] = W("m1.logstd");
            d.mnoise = W("roll.mnoise");
        }
        d.mode = 3;
        launch_diag(d, h->stream);
    } else {                         // SAC_expert.py:579-608
        models(false);
        d.mode = 1;
        launch_diag(d, h->stream);
        if (!ea) {
            counterfactual();
            models(false);
        }
        d.mode = 2;                  // use_expert_actions: the counterfactual MSE is the data MSE
        launch_diag(d, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return 0;
}

int sacx_time_kernels(sacx_handle* h, const char* kernel, int32_t n_replays, double* avg_us, double* us_per_update,
                      int64_t* n_launches) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (!kernel || std::strcmp(kernel, "k_gemm") != 0) return fail(h, "only k_gemm carries timestamps");
    if (settle(h)) return -1;
    wbf_refresh(h, h->stream);
    if (!avg_us || n_replays <= 0) return fail(h, "bad arguments");
    const int G = h->graph_steps;
    KTimeMap kt;
    kt.cap = (int64_t)G * 16 * 4096 * 2 * h->seeds;    // generous: <= 16 GEMM launches x 4096 WGs per update
    kt.rows = std::getenv("SACX_KTIME_DUMP") != nullptr;
    HIPCHK(h, hipMalloc(&kt.base, kt.cap * sizeof(uint64_t)));
    hipGraphExec_t g = nullptr;
    int rc = get_graph(h, G, true, &g, -1, &kt);
    double sum = 0.0;
    int64_t cnt = 0;
    std::vector<uint64_t> host((size_t)kt.used);
    for (int r = 0; rc == 0 && r < n_replays; ++r) {
        if (hipGraphLaunch(g, h->stream) != hipSuccess || hipStreamSynchronize(h->stream) != hipSuccess ||
            hipMemcpy(host.data(), kt.base, host.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) {
            rc = fail(h, "timing replay failed");
            break;
        }
        // diagnostics: SACX_KTIME_DUMP=<file> appends one line per launch of the last replay:
        // name, span, mean / max workgroup duration, last-start offset, gap to the previous end (us)
        FILE* dump = nullptr;
        if (r == n_replays - 1)
            if (const char* path = std::getenv("SACX_KTIME_DUMP")) dump = std::fopen(path, "a");
        uint64_t prev_hi = 0;
        for (size_t si = 0; si < kt.spans.size(); ++si) {
            const auto& sp = kt.spans[si];
            uint64_t lo = UINT64_MAX, hi = 0, last_start = 0, wmax = 0, rmax = 0;
            double wsum = 0.0, rsum = 0.0;
            const int rb0 = kt.rowspan[si].first, rb1 = kt.rowspan[si].second;
            const int nt = sp.second - (rb1 - rb0) * h->seeds;
            const int per = sp.second / h->seeds;     // workgroups per seed (seed-major slots)
            for (int b = 0; b < sp.second; ++b) {
                const uint64_t t0 = host[sp.first + 2 * b], t1 = host[sp.first + 2 * b + 1];
                lo = std::min(lo, t0);
                hi = std::max(hi, t1);
                last_start = std::max(last_start, t0);
                const int bx = b % per;
                if (bx < rb0 || bx >= rb1) {
                    wmax = std::max(wmax, t1 - t0);
                    wsum += (double)(t1 - t0);
                } else {
                    rmax = std::max(rmax, t1 - t0);
                    rsum += (double)(t1 - t0);
                }
            }
            if (kt.is_gemm[si]) {
                sum += (double)(hi - lo) * 0.01;         // 100 MHz ticks -> us
                ++cnt;
            }
            if (dump)
                std::fprintf(dump, "%s,%d,%.2f,%.2f,%.2f,%.2f,%.2f,%.2f,%.2f\n", kt.names[si].c_str(), sp.second,
                             (hi - lo) * 0.01, wsum / std::max(1, nt) * 0.01, wmax * 0.01, (last_start - lo) * 0.01,
                             prev_hi ? ((double)lo - (double)prev_hi) * 0.01 : 0.0,
                             rb1 > rb0 ? rsum / ((rb1 - rb0) * h->seeds) * 0.01 : 0.0, rmax * 0.01);
            prev_hi = hi;
        }
        if (dump) std::fclose(dump);
        // SACX_KTIME_CLASSES=<file>: k_fwd2 launches' workgroups by problem pair (mean / max us)
        if (const char* path = std::getenv("SACX_KTIME_CLASSES"); path && r == n_replays - 1 && h->seeds == 1) {
            if (FILE* f = std::fopen(path, "a")) {
                for (size_t si = 0; si < kt.spans.size(); ++si) {
                    const auto& cb = kt.cls[si];
                    if (cb.empty()) continue;
                    const auto& sp = kt.spans[si];
                    std::fprintf(f, "%s", kt.names[si].c_str());
                    for (size_t c = 0; c < cb.size(); ++c) {
                        const int b0 = cb[c], b1 = c + 1 < cb.size() ? cb[c + 1] : sp.second;
                        double su = 0.0, mx = 0.0;
                        for (int b = b0; b < b1; ++b) {
                            const double d = (double)(host[sp.first + 2 * b + 1] - host[sp.first + 2 * b]) * 0.01;
                            su += d;
                            mx = std::max(mx, d);
                        }
                        std::fprintf(f, ",p%zu:%d:%.2f:%.2f", c, b1 - b0, su / std::max(1, b1 - b0), mx);
                    }
                    std::fprintf(f, "\n");
                }
                std::fclose(f);
            }
        }
    }
    if (g) (void)hipGraphExecDestroy(g);
    (void)hipFree(kt.base);
    if (rc) return rc;
    h->seq_host += (int64_t)n_replays * G;
    *avg_us = cnt ? sum / cnt : 0.0;
    if (us_per_update) *us_per_update = sum / ((double)n_replays * G);
    if (n_launches) *n_launches = cnt / n_replays;
    return 0;
}

int sacx_time_graph(sacx_handle* h, int64_t n_replays, const char* skip_kernel, double* ms_out) {
    if (!h || !h->bound) return fail(h, "not bound");
    if (!ms_out || n_replays <= 0) return fail(h, "bad arguments");
    if (settle(h)) return -1;
    wbf_refresh(h, h->stream);
    int skip = -1;
    if (skip_kernel && skip_kernel[0]) {
        for (int k = Launch::RNG; k <= Launch::MFINAL; ++k)
            if (std::strcmp(kernel_family((Launch::Kind)k), skip_kernel) == 0) skip = k;
        if (skip < 0 || skip == Launch::GATHER) return fail(h, "unknown or non-removable kernel family");
    }
    hipGraphExec_t g;
    if (get_graph(h, h->graph_steps, true, &g, skip)) return -1;
    hipEvent_t e0, e1;
    HIPCHK(h, hipEventCreate(&e0));
    HIPCHK(h, hipEventCreate(&e1));
    HIPCHK(h, hipGraphLaunch(g, h->stream));   // warm
    HIPCHK(h, hipEventRecord(e0, h->stream));
    for (int64_t i = 0; i < n_replays; ++i) HIPCHK(h, hipGraphLaunch(g, h->stream));
    HIPCHK(h, hipEventRecord(e1, h->stream));
    HIPCHK(h, hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(h, hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *ms_out = ms;
    h->seq_host += (n_replays + 1) * h->graph_steps;
    return 0;
}

}  // extern "C"
