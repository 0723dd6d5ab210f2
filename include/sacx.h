/*
 * sacx.h -- C ABI of libsacx, the MI355X-native SAC / SAC-EO update engine.
 *
 * The reference (noc-lab/sac-expert, TensorFlow-eager Python) has no FFI: its
 * hot path sits behind duck-typed Python objects.  This ABI is the boundary a
 * binding (ctypes here) calls in place of the reference
 * functions named next to each entry.  Everything is plain C: opaque handle,
 * plain pointers and sizes, int status codes (0 = OK, < 0 = error, message in
 * sacx_last_error).  No torch types cross the boundary.
 *
 * Memory model: the caller allocates ONE device arena (any allocator, e.g. a
 * torch uint8 CUDA tensor), binds it with sacx_bind(), and addresses named
 * tensors inside it through the segment table (sacx_layout).  Weights use the
 * Keras (in, out) row-major layout with the bias stored as one extra row
 * (W_ext = [W ; b]), so reference get_weights()/set_weights() lists map onto
 * views (sac_eo/common/nn_utils.py:59-76).  Every call is asynchronous on the
 * bound HIP stream unless stated otherwise.  A handle is not re-entrant; use
 * one handle per learner (per GPU / per seed), or one handle of packed seeds.
 *
 * Packed seeds (cfg.seeds = K > 1): the handle holds K independent learners --
 * the reference's --runs (sac_eo/train.py:118-152), each with its own weights,
 * optimiser state, replay ring and RNG stream -- in K equal arena blocks
 * sacx_seed_stride() bytes apart, each laid out as sacx_layout() describes.
 * sacx_sac_step advances all K in the same kernel launches (grid z = seed).
 * The data-path and RNG calls (append, expert rows, permutations, RNG state,
 * actor_act, rollout, expert_diag, model_fit, resync) address the seed chosen with
 * sacx_seed_select (default 0); the *_seeds forms address every seed at once.
 * The data-parallel mode needs K = 1.
 */
#ifndef SACX_H
#define SACX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SACX_ABI_VERSION 8
#define SACX_MAX_DEPTH 4    /* hidden layers per net (create_nn's layers list, nn_utils.py:100-138) */
#define SACX_MAX_MODELS 8   /* --num_models */

typedef struct sacx_handle sacx_handle;

enum sacx_activation { SACX_ACT_RELU = 0, SACX_ACT_TANH = 1, SACX_ACT_ELU = 2 };
enum sacx_dtype { SACX_F32 = 0, SACX_I32 = 1, SACX_I64 = 2, SACX_U32 = 3, SACX_F64 = 4 };
enum sacx_role { SACX_ROLE_WORK = 0, SACX_ROLE_PARAM = 1, SACX_ROLE_TARGET = 2, SACX_ROLE_STATE = 3 };

/* Flags for sacx_sac_step. */
#define SACX_STEP_EXTERNAL_RANDOMS 1  /* skip the device sampler: caller filled slot0.idx / slot0.noise */
#define SACX_STEP_EAGER 2             /* launch kernels directly instead of replaying a hipGraph */
/* floats in the pinned staging buffer of each half (append / act) of the *_host entry points:
   one append_host_seeds call takes seeds*n*(2S+A+2) <= this, act_host_seeds seeds*n*(S+A) */
#define SACX_STAGE_FLOATS 65536

/* Hyper-parameters; names follow sac_eo/common/train_parser.py. */
typedef struct sacx_config {
    int32_t abi_version;        /* = SACX_ABI_VERSION */
    int32_t s_dim;              /* observation dim (HalfCheetah 17, Humanoid 376) */
    int32_t a_dim;              /* action dim (6, 17) */
    int32_t hidden[2];          /* --actor_layers / --critic_layers (same for both) */
    int32_t activation;         /* --actor_activations / --critic_activations */
    int32_t batch;              /* --sac_batch_size */
    int64_t buffer_capacity;    /* --env_buffer_size (ring capacity, rows) */
    int32_t per_state_std;      /* --actor_per_state_std */
    int32_t use_expert;         /* alg_type sac_imit (SAC-EO expert regulariser) */
    int32_t expert_capacity;    /* --expert_buffer_size */
    int32_t expert_batch;       /* rows of expert data per update (even) */
    int32_t model_hidden[2];    /* --model_layers */
    int32_t model_activation;   /* --model_activations */
    int32_t model_batch;        /* --model_batch_size */
    int32_t target_update_int;  /* --target_update_int */
    int32_t graph_steps;        /* updates per captured hipGraph (0 -> 128, max 256) */
    int32_t stats_capacity;     /* rows of the per-update statistics ring (0 -> 4096) */
    int32_t perm_capacity;      /* per-update expert permutations held on device (0 -> 4096) */
    float gamma;                /* --gamma */
    float tau;                  /* --soft_tau */
    float lr_q;                 /* --q_crit_lr */
    float lr_pi;                /* --mbpo_actor_lr */
    float lr_alpha;             /* --mbpo_alpha_lr */
    float lr_model;             /* --model_lr */
    float init_temperature;     /* --init_temperature (alpha var = log of it) */
    float target_entropy;       /* -len(action) (SAC_expert.py:46) */
    float act_limit;            /* action_space.high (continuous_actors.py:252) */
    float epsilon;              /* --epsilon (expert weight) */
    float reward_loss_coef;     /* --reward_loss_coef */
    int32_t gemm_bf16;          /* 1: the MLP GEMMs take bf16 operands (rounded on load) with fp32
                                   accumulation, fp32 master weights / Adam (config C5); 0: fp32 */
    int32_t seeds;              /* independent learners packed in this handle (0/1 = one; <= 64) */
    /* --- ABI 4 --- */
    int32_t actor_gaussian;     /* 0: SquashedGaussianActor (SAC, continuous_actors.py:237-379); 1: GaussianActor
                                   (:9-123), inference only (sacx_actor_act) -- an expert imported from a log
                                   (sac_eo/train.py:65-86 builds it without actor_squash) */
    float actor_std_mult;       /* --actor_std_mult (GaussianActor.logstd_init; 0 -> 1) */
    int32_t actor_output_norm;  /* --actor_output_norm (GaussianActor mean normalisation) */
    int32_t actor_layer_norm;   /* --actor_layer_norm: Dense -> LayerNormalization -> tanh on layer 0
                                   (nn_utils.py:110-119) */
    int32_t num_models;         /* --num_models for SAC-EO: 1 .. SACX_MAX_MODELS world models (0 -> 2); all are
                                   fitted in one model-Adam step, the expert term uses the first two sections of
                                   array_split(perm, num_models) (SAC_expert.py:297-336) */
    float model_max_grad_norm;  /* --model_max_grad_norm: clip_by_global_norm(grads, max_norm * num_models)
                                   of the model fit (mbrl_onpolicy_alg.py:315-317); <= 0: None */
    float delta_clip_loss;      /* --delta_clip_loss of MSEModel.get_loss in the model fit; <= 0: None */
    float reward_clip_loss;     /* --reward_clip_loss of MSEModel.get_loss in the model fit; <= 0: None */
    int32_t act_per_layer;      /* 1: act_layers below give each hidden layer's activation; 0: `activation`
                                   (actor, critics) and `model_activation` for every hidden layer */
    int32_t act_layers[3][2];   /* [actor | critics | world models][hidden layer 0, 1]: a sacx_activation
                                   value; the --actor_activations / --critic_activations / --model_activations
                                   lists of nn_utils.py:5-22 */
    /* --- ABI 5 --- */
    float delta_clip_pred;      /* --delta_clip_pred: MSEModel.sample clips the normalised delta prediction
                                   (base_world_model.py:80-82) in the SAC-EO expert term; <= 0: None */
    /* --- ABI 6 --- */
    int32_t single_seed_plan;   /* packed seeds: 1 = every seed sums as a one-seed handle does (the
                                   one-seed plan's head folds and fused heads; 32x32 workgroup tiles, which
                                   accumulate exactly as 16x16 ones, still by the packed row count), so
                                   each is bit-identical to its one-seed run (sac_eo.train --runs in
                                   lock-step); 0 = the packed plan (separate heads from 4 seeds: faster) */
    /* --- ABI 7 --- */
    int32_t gaussian_model;     /* --gaussian_model: GaussianModel world models (init_world_models.py:13-16):
                                   a trainable logstd [1, S] per model after its net (segment m<k>.logstd,
                                   continuous_models.py:24-27), the Gaussian NLL fit loss (:101-131), and
                                   exp(logstd) * u noise in sample(deterministic=False) / step (:36-70) */
    int32_t scale_model_loss;   /* --scale_model_loss: GaussianModel's loss times the stop-gradient
                                   mean(exp(logstd)^2) (:122-127) */
    int32_t separate_reward_nn; /* --separate_reward_nn (base_world_model.py:32-37): the model net has S
                                   outputs and a reward net r<k> ([S+A] -> reward_hidden -> 1) predicts
                                   the reward (:72-74), fitted in the same step */
    int32_t reward_hidden[2];   /* --reward_layers (2 hidden layers; 0 -> 512) */
    int32_t reward_act_layers[2]; /* --reward_activations per hidden layer (sacx_activation) */
    int32_t critic_hidden[2];   /* --critic_layers when they differ from --actor_layers (0: = hidden) */
    /* --- ABI 8 --- */
    int32_t net_depth[4];       /* hidden layers of [actor | critics | world models | reward nets]: 0 -> the two of
                                   hidden / critic_hidden / model_hidden / reward_hidden (and their activations);
                                   1..SACX_MAX_DEPTH -> net_hidden / net_acts below give every layer (the
                                   --actor_layers / --critic_layers / --model_layers / --reward_layers lists,
                                   train_parser.py:56-57, :107-108, of any length).  Any net not of 2 layers runs
                                   the generic launch plan (unfused, every layer its own GEMM problem) */
    int32_t net_hidden[4][SACX_MAX_DEPTH];   /* widths, [1, 512] */
    int32_t net_acts[4][SACX_MAX_DEPTH];     /* per-layer sacx_activation */
} sacx_config;

typedef struct sacx_segment {
    char name[48];
    uint64_t offset;            /* bytes from arena base */
    int64_t rows;
    int64_t cols;
    int32_t dtype;              /* enum sacx_dtype */
    int32_t role;               /* enum sacx_role */
} sacx_segment;

typedef struct sacx_launch_info {
    char name[32];              /* stage name, e.g. "critic.dW+adam" */
    char kernel[32];            /* kernel symbol family, e.g. "k_gemm" */
    int32_t grid;               /* workgroups */
    int32_t block;              /* threads per workgroup */
    double flops;               /* algorithmic FLOPs of the launch (unpadded shapes) */
    double bytes;               /* algorithmic HBM/L2 bytes of the launch */
} sacx_launch_info;

/* Statistics row written per update into the stats ring (float32 x 8). */
enum sacx_stat { SACX_STAT_Q1_LOSS = 0, SACX_STAT_Q2_LOSS, SACX_STAT_P_LOSS, SACX_STAT_ALPHA_LOSS,
                 SACX_STAT_ALPHA, SACX_STAT_MSE_LOSS, SACX_STAT_NLP_MEAN, SACX_STAT_STEP };

/* --- lifecycle ------------------------------------------------------------ */
/* Replaces the construction done by init_actor / init_critics / init_alg
 * (sac_eo/actors/init_actor.py:8-30, sac_eo/critics/init_critic.py:5-38,
 * sac_eo/algs/init_alg.py:9-34): validates the config, computes the layout. */
int sacx_create(const sacx_config* cfg, sacx_handle** out);
void sacx_destroy(sacx_handle* h);
const char* sacx_last_error(const sacx_handle* h);   /* NULL handle: error of the last failed create */
int64_t sacx_arena_bytes(const sacx_handle* h);   /* all seeds */
/* Bytes between consecutive seeds' arena blocks (packed seeds; = the arena size for one). */
int64_t sacx_seed_stride(const sacx_handle* h);
/* Packed seeds: the seed (0 <= seed < cfg.seeds) that the per-seed calls address. */
int sacx_seed_select(sacx_handle* h, int32_t seed);
int sacx_layout(const sacx_handle* h, sacx_segment* segs, int32_t cap, int32_t* n_out);
/* Binds the caller-owned arena (>= sacx_arena_bytes, 256-B aligned) and the HIP
 * stream (hipStream_t as void*, NULL = default stream); builds the launch plan.
 * The caller zero-fills the arena and writes weights / normalisers / RNG state
 * through the segment views before the first step. */
int sacx_bind(sacx_handle* h, void* arena, uint64_t bytes, void* stream);

/* --- data path ------------------------------------------------------------ */
/* TrajectoryBuffer.add (sac_eo/common/buffers.py:41-71): appends n rows at the
 * ring head with FIFO truncation to buffer_capacity.  Device pointers, rows of
 * s[n,S], a[n,A], r[n], sp[n,S], d[n] (0/1 as float). */
int sacx_buffer_append(sacx_handle* h, const float* s, const float* a, const float* r,
                       const float* sp, const float* d, int64_t n);
/* expert_reg of _expert_preprocess (sac_eo/algs/SAC_expert.py:375-424): the
 * expert rows (device pointers s_e[n,S], sp_e[n,S]) used by every following
 * update, and the regulariser weight epsilon. */
int sacx_expert_set(sacx_handle* h, const float* s_e, const float* sp_e, int32_t n, float epsilon);
/* Host array perms[n_steps, expert_batch]: the self.rng.shuffle permutations
 * (sac_eo/algs/SAC_expert.py:301-303) for the next n_steps updates. */
int sacx_perm_push(sacx_handle* h, const int32_t* perms, int64_t n_steps);

/* --- RNG (the reference's global NumPy legacy MT19937 stream) ------------- */
/* np.random.seed / RandomState.set_state / get_state (sac_eo/common/seeding.py:12).
 * set/get are synchronous with respect to the bound stream. */
int sacx_rng_seed(sacx_handle* h, uint32_t seed);
int sacx_rng_set_state(sacx_handle* h, const uint32_t key[624], int32_t pos, int32_t has_gauss, double gauss);
int sacx_rng_get_state(sacx_handle* h, uint32_t key[624], int32_t* pos, int32_t* has_gauss, double* gauss);

/* --- the hot path ---------------------------------------------------------- */
/* n_steps x SAC_exp._update / SAC._update (sac_eo/algs/SAC_expert.py:463-477,
 * sac_eo/algs/SAC.py:236-250): sample + gather, twin-Q target, Q1/Q2 Adam,
 * actor (+ expert term) Adam, alpha Adam + clamp, Polyak.  ts_increment is
 * added to num_timesteps after every update (1 = SAC_exp.train, 0 = repeated
 * updates at one env step as in SAC.train). */
int sacx_sac_step(sacx_handle* h, int64_t n_steps, int64_t num_timesteps, int32_t ts_increment,
                  int32_t flags);
/* Captures, instantiates and uploads every hipGraph that sacx_sac_step(h, n_steps, ..., flags)
 * will replay (n_steps / graph_steps full graphs + one graph of the remainder), without
 * running an update, so a following sacx_sac_step(n_steps) launches only cached graphs.
 * (No reference counterpart: TF-eager has no capture step.)  Synchronous. */
int sacx_prepare(sacx_handle* h, int64_t n_steps, int32_t flags);
/* n_steps x _apply_model_grads (sac_eo/algs/mbrl_onpolicy_alg.py:301-319) as
 * called by SAC_exp._update_models (sac_eo/algs/SAC_expert.py:519-550): each
 * step fits both world models on their own minibatch and applies one Keras
 * Adam over all model variables.  idx: host array [n_steps, 2, model_batch]
 * of replay-logical row indices (the caller's np.random.shuffle minibatches
 * of model_data, mapped into the replay ring).  Per-step summed loss goes to
 * the "mstats" ring.  Requires use_expert. */
int sacx_model_fit(sacx_handle* h, const int32_t* idx, int64_t n_steps, int32_t flags);
/* SquashedGaussianActor.sample (sac_eo/actors/continuous_actors.py:270-306) on n device
 * rows obs[n,S] -> act_out[n,A] (device): normalise, MLP, a = act_limit*tanh(mu + std*u).
 * deterministic != 0: u = 0 and the RNG is untouched (the reference draws nothing);
 * otherwise u = np.random.normal(size=(n,A)) from the device copy of the global stream,
 * in the order the reference would draw it.  Behaviour-policy inference for the env loop. */
int sacx_actor_act(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out);

/* --- host-pointer forms for the env loop (SAC_exp.train, sac_eo/algs/SAC_expert.py:585-605:
 * one host observation -> actor.sample -> env.step -> buffer.add per timestep) -------------- */
/* sacx_buffer_append with HOST rows: packed into a library-owned pinned, device-mapped buffer
 * that k_append reads in place (no DMA copy; chunked above 64 Ki floats).  Asynchronous: returns
 * once the rows are packed, so the caller's arrays may be reused immediately. */
int sacx_buffer_append_host(sacx_handle* h, const float* s, const float* a, const float* r,
                            const float* sp, const float* d, int64_t n);
/* sacx_actor_act with HOST obs[n,S] in and HOST act_out[n,A] out, through the same mapped
 * buffer (the normaliser reads obs and the head writes actions in place).  Synchronous: waits
 * for the action kernel (and so for any update queued before it) before returning the actions.
 * Drop-in cadence (SAC_expert.py:779-797: sample, _update, env.step, add): after a one-update
 * sacx_sac_step it also queues the next update's sampler draw behind the action kernel (for the
 * ring as it is now), which the next sacx_sac_step(h, 1, ...) uses when the ring still has that
 * size; that step then also runs the previous update's alpha branch, folded into its launches. */
int sacx_actor_act_host(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out);
/* Both for EVERY seed of a packed handle in one launch chain: K runs of the reference's
 * --runs (sac_eo/train.py:118-152) stepping their env loops in lock-step hand over n rows each.
 * Arrays are [seeds, n, ...] in seed order; each seed appends to its own ring / acts with its
 * own actor, normaliser and RNG stream (as sacx_seed_select + the calls above would, seed by
 * seed).  act: n <= 16 rows per seed, no --actor_layer_norm. */
int sacx_buffer_append_host_seeds(sacx_handle* h, const float* s, const float* a, const float* r,
                                  const float* sp, const float* d, int64_t n);
int sacx_actor_act_host_seeds(sacx_handle* h, const float* obs, int64_t n, int32_t deterministic, float* act_out);

/* --- the reference objects' standalone network calls (device rows in, device rows out) -- */
/* SquashedGaussianActor.evaluate (sac_eo/actors/continuous_actors.py:327-379) on s[n,S]:
 * u = np.random.normal(size=(n, A)) from the device copy of the global stream, x = mu + std*u,
 * pi_out[n,A] = act_limit*tanh(x), nlp_out[n] = neglogp_adjusted. */
int sacx_actor_evaluate(sacx_handle* h, const float* s, int64_t n, float* pi_out, float* nlp_out);
/* QCritic._forward / value (sac_eo/critics/critics.py:84-103) of net 0 / 1 (q_critics) or
 * 2 / 3 (q_targets) on s[n,S], a[n,A]: out[n] = the [n,1] net output (value = 0), or that
 * times max(ret_rms.std, 1e-8) (value = 1). */
int sacx_critic_forward(sacx_handle* h, int32_t net, const float* s, const float* a, int64_t n, int32_t value,
                        float* out);
/* BaseWorldModel._forward + MSEModel.sample / step (sac_eo/models/base_world_model.py:65-87,
 * sac_eo/models/continuous_models.py:225-254) of world model `model` on s[n,S], a[n,A].
 * delta_clip / reward_clip > 0: --delta_clip_pred / --reward_clip_pred.  Outputs (each
 * nullable): pred_out[n,S+1] = [delta_n | r_n] after the clips, sp_out[n,S] = s +
 * delta_rms.denormalize(delta_n) (sample), r_out[n] = r_rms.denormalize(r_n) (step).
 * Requires use_expert. */
int sacx_model_forward(sacx_handle* h, int32_t model, const float* s, const float* a, int64_t n, float delta_clip,
                       float reward_clip, float* pred_out, float* sp_out, float* r_out);
/* sacx_model_forward with GaussianModel's noise (continuous_models.py:36-70, ABI 7): stochastic != 0
 * on a gaussian_model handle draws u = np.random.normal(size=(n, S)) from the device stream and
 * adds exp(logstd) * u to the clipped delta_n before sp_out (GaussianModel.sample(deterministic=False)
 * and .step); pred_out stays the mean.  stochastic = 0, or an MSEModel handle: sacx_model_forward. */
int sacx_model_sample(sacx_handle* h, int32_t model, const float* s, const float* a, int64_t n,
                      int32_t stochastic, float delta_clip, float reward_clip, float* pred_out, float* sp_out,
                      float* r_out);
/* MSEModel.get_loss (continuous_models.py:280-302) of world model `model` on s, sp [n,S],
 * a [n,A], r [n]: loss_out[0] = mean_i 0.5||clip(norm(sp-s)) - delta_pred||^2 +
 * reward_loss_coef * 0.5 (clip(norm(r)) - r_pred)^2, the clips > 0 being --delta_clip_loss /
 * --reward_clip_loss; on a gaussian_model handle GaussianModel.get_loss (:101-131), the delta
 * term 0.5 sum_j (((norm(sp-s) - delta_pred) / e^l)^2 + 2 l + log 2 pi) (x mean(e^{2l}) with
 * scale_model_loss).  loss_out is device memory.  Requires use_expert. */
int sacx_model_loss(sacx_handle* h, int32_t model, const float* s, const float* sp, const float* a, const float* r,
                    int64_t n, float delta_clip_loss, float reward_clip_loss, float* loss_out);
/* batch_simtrajectory_sampler (sac_eo/common/samplers.py:73-122) with world model `model`
 * as the environment (MSEModel.reset / step, sac_eo/models/continuous_models.py:225-258)
 * and the actor's sample() (continuous_actors.py:270-306), all on the device.
 * s_init[n,S] (device) -> s_out[n,H,S], a_out[n,H,A], r_out[n,H], sp_out[n,H,S], d_out[n,H]
 * (uint8; always 0: MSEModel.step never terminates).  Per step t: a = sample(s_t) drawing
 * np.random.normal(size=(n, A)) from the device stream (nothing when deterministic);
 * (delta_n, r_n) = model([norm s_t, norm clip(a)]), clipped to +-delta_clip / +-reward_clip
 * when > 0 (--delta_clip_pred / --reward_clip_pred); a GaussianModel (ABI 7) then draws
 * normal(size=(n, S)) and adds exp(logstd) * u (GaussianModel.step, :36-54; n <= 4096);
 * s_{t+1} = s_t + delta_n*den + mean.  Requires use_expert (the models exist only then). */
int sacx_rollout(sacx_handle* h, int32_t model, const float* s_init, int64_t n, int32_t horizon,
                 int32_t deterministic, float delta_clip, float reward_clip, float* s_out, float* a_out,
                 float* r_out, float* sp_out, uint8_t* d_out);
/* Expert diagnostics on the device, n <= 2048 expert rows (device).
 * flags = 0: model_MSE_on_expert_data and _counterfactual_action (SAC_expert.py:579-608):
 *   out[0] = mean over the nm models of mean_i 0.5||model.sample(s_e, a_e) - sp_e||^2,
 *   out[1] = the same with a = actor.sample(s_e, deterministic=False) (draws n*A normals
 *   from the device stream), out[2 .. 2+nm) / out[2+nm .. 2+2nm) = per model (nm = 1: model 0
 *   twice).  n * max(nm, 2) <= 4096.
 * flags & SACX_DIAG_DISC: _calc_disc (:427-460): s_disc_i = ||sp_pred0 - sp_pred1||_2 on
 *   (s_e, counterfactual a); out[0] = sum, out[1] = max, out[2] = median, out[3 + i] = ratio.
 *   The models sample with deterministic=False: GaussianModels draw normal(size=(n, S)) each,
 *   every model in order (only models 0 and 1 enter the distance), after the counterfactual
 *   action's draw (:437, :446).
 * flags & SACX_DIAG_EXPERT_ACTIONS (use_expert_actions): a_e replaces the counterfactual
 *   action (no draw; out[1] = out[0]).  delta_clip > 0: --delta_clip_pred.  out: device, >= 2 + 2
 *   max(nm, 2) floats (3 + n with DISC).  The adaptive epsilon of :383-418 is scalar host arithmetic. */
enum { SACX_DIAG_DISC = 1, SACX_DIAG_EXPERT_ACTIONS = 2 };
int sacx_expert_diag(sacx_handle* h, const float* s_e, const float* a_e, const float* sp_e, int32_t n,
                     int32_t flags, float delta_clip, float* out);
int sacx_sync(sacx_handle* h);
/* Brings the arena to the state the calls so far define, without waiting: runs an alpha branch
 * the drop-in loop's one-update steps deferred (its alpha Adam, stats row and counters; see
 * sacx_actor_act_host) and undoes a speculative sampler draw.  Every entry point but act, append
 * and the speculative step does this itself; a caller that reads or writes the arena directly
 * (segment views) calls it first.  sacx_sync = sacx_settle + a wait for the bound stream. */
int sacx_settle(sacx_handle* h);

/* After the caller restored the arena's PARAM / TARGET / STATE segments (a resume
 * snapshot, sac_eo Engine.load_state): re-reads the host mirrors of the device counters
 * (update and model-fit sequence numbers that place host-pushed permutations / indices). */
int sacx_resync(sacx_handle* h);

/* --- data-parallel mode (config C4: one learner over k GPUs) --------------------
 * Not in the reference (its --runs are independent learners, sac_eo/train.py:118-152):
 * each rank samples its local batch from its own buffer and stream; the critic, actor
 * (+logstd) and alpha gradients are summed over the ranks by RCCL inside the update
 * graph (three all-reduces per update: 2*P_q, P_a + A, 1 floats) and every rank applies
 * the same Keras Adam with gradient/k, so weights stay identical when they start so.
 * With batch = B/k this is the B-row update of SAC.py:236-250 (the losses are means).
 * sacx_dp_unique_id: on one rank, fills id_out (cap >= 128 bytes), returns its size.
 * sacx_dp_init: on every rank after sacx_create, before sacx_bind, on the rank's device.
 * Plain SAC only (use_expert = 0). */
int sacx_dp_unique_id(void* id_out, int32_t cap);
int sacx_dp_init(sacx_handle* h, const void* id, int32_t nranks, int32_t rank);
/* The same protocol with the ranks as handles of ONE process (<= 8, no RCCL): sacx_dp_init_local
 * on each (before sacx_bind; all bound to one stream), then sacx_dp_local_step(handles in rank
 * order, ...) runs n_steps updates of every rank eagerly, interleaved at the all-reduce points,
 * where one kernel sums the ranks' gradient ranges in rank order and writes the sum back to each
 * (ncclAllReduce(sum)'s result; with two ranks bit for bit).  The reduce is the only difference
 * from the RCCL mode: the plans, local-gradient stores and Adam apply launches are the same. */
int sacx_dp_init_local(sacx_handle* h, int32_t nranks, int32_t rank);
int sacx_dp_local_step(sacx_handle* const* handles, int32_t nranks, int64_t n_steps, int64_t num_timesteps,
                       int32_t ts_increment);

/* --- measurement ----------------------------------------------------------- */
/* One-update sacx_sac_step calls that replayed the sampler-less graph on randoms drawn
 * speculatively by the preceding sacx_actor_act_host (the drop-in loop's cadence act -> step ->
 * append of SAC_expert.py:779-797); the other steps drew their own.  -1 for a NULL handle. */
int64_t sacx_spec_hits(const sacx_handle* h);
int sacx_plan_info(const sacx_handle* h, sacx_launch_info* out, int32_t cap, int32_t* n_out);
/* The launches of one world-model fitting step (sacx_model_fit) of the selected seed, as
 * sacx_plan_info (use_expert handles; *n_out = 0 before the first sacx_model_fit builds them). */
int sacx_model_plan_info(const sacx_handle* h, sacx_launch_info* out, int32_t cap, int32_t* n_out);
/* Runs n_steps updates eagerly with a HIP event around every launch on the
 * bound stream and returns the summed device milliseconds per launch index
 * (array of length n_launches from sacx_plan_info).  Each step is queued
 * behind a ~3 ms device-side wait so the deltas are back-to-back device time,
 * not host launch latency.  Synchronous. */
int sacx_profile(sacx_handle* h, int64_t n_steps, double* ms_per_launch, int32_t cap);

/* Replays the captured update graph (graph_steps updates, device sampler) n_replays
 * times between two HIP events on the bound stream and returns the elapsed ms.
 * skip_kernel names a kernel family (sacx_launch_info.kernel, e.g. "k_gemm") whose
 * launches are left out of the graph: the difference of the two timings is that
 * family's in-pipeline time.  With a family skipped the updates are meaningless and
 * the state must be discarded (measurement only).  Synchronous. */
int sacx_time_graph(sacx_handle* h, int64_t n_replays, const char* skip_kernel, double* ms_out);
/* Replays a copy of the update graph in which every launch of `kernel` (only "k_gemm")
 * records per-workgroup start/end device ticks (s_memrealtime, 100 MHz) into its own
 * slots; returns the mean launch span (first workgroup start .. last workgroup end) in
 * us, the summed span per update and the launches per graph replay.  The replays are
 * real updates.  Synchronous. */
int sacx_time_kernels(sacx_handle* h, const char* kernel, int32_t n_replays, double* avg_us, double* us_per_update,
                      int64_t* n_launches);

#ifdef __cplusplus
}
#endif
#endif /* SACX_H */
