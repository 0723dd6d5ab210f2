"""CPU oracle for the SAC / SAC-EO update hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``sac-expert_amd/``)
may import this module; only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` use it, and only as the checker / the
timed CPU port.

What it is
----------
A NumPy restatement of the reference's TensorFlow-eager update math, written
from the reference sources (all citations relative to noc-lab/sac-expert):

* replay sampling / gather          sac_eo/common/buffers.py:126-144
* normaliser                        sac_eo/common/normalizer.py:26-58
* Keras Dense MLP                   sac_eo/common/nn_utils.py:59-138
* squashed Gaussian evaluate/sample sac_eo/actors/continuous_actors.py:270-379
* Q critic _forward / value         sac_eo/critics/critics.py:84-103
* twin-Q target                     sac_eo/algs/SAC_expert.py:211-229
* critic update                     sac_eo/algs/SAC_expert.py:232-259
* actor (+ expert term) and alpha   sac_eo/algs/SAC_expert.py:262-356 (SAC.py:178-217)
* Polyak sync                       sac_eo/algs/SAC_expert.py:362-373
* one gradient step                 sac_eo/algs/SAC_expert.py:463-477 (SAC.py:236-250)
* world-model sample / loss         sac_eo/models/continuous_models.py:244-302 (MSEModel),
                                    :7-131 (GaussianModel), base_world_model.py:25-87
                                    (--separate_reward_nn reward net)
* model-fit step                    sac_eo/algs/mbrl_onpolicy_alg.py:301-319
* Keras Adam (legacy OptimizerV2, epsilon-hat form, eps=1e-7)

Backward passes are written in closed form (the reference uses
tf.GradientTape); ``tests/test_oracle.py`` checks them against torch autograd
in fp64 on the same forward formulas.

Precision modes: ``np.float64`` (reference-quality arithmetic) and
``np.float32`` (op-by-op emulation of the TF fp32 graph: every elementwise op
rounds to fp32, constants are cast the way TF casts python / numpy scalars).

Parity status: the random streams are pinned bit-exactly against NumPy's own
legacy ``RandomState`` (the reference's RNG; see oracle/mt19937.c and
tests/golden/).  The floating-point math is *parity unpinned* against the
reference itself: TensorFlow is not installable in this image and the
reference ships no tests or golden numbers for this path.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Sequence

import numpy as np

LOG_STD_MIN = -5.0   # continuous_actors.py:250
LOG_STD_MAX = 2.0    # continuous_actors.py:251


# ---------------------------------------------------------------------------
# configuration / state containers
# ---------------------------------------------------------------------------
@dataclasses.dataclass
class Config:
    S: int = 17
    A: int = 6
    hidden: Sequence[int] = (256, 256)
    act: str = "relu"
    B: int = 256
    gamma: float = 0.995          # train_parser.py:160
    tau: float = 5e-3             # train_parser.py:326
    lr_q: float = 3e-4            # train_parser.py:310
    lr_pi: float = 1e-4           # train_parser.py:312
    lr_alpha: float = 1e-4        # train_parser.py:314
    init_temperature: float = 0.1  # train_parser.py:308
    act_limit: float = 1.0
    per_state_std: bool = False
    layer_norm: bool = False      # --actor_layer_norm: Dense -> LayerNorm -> tanh (nn_utils.py:110-119)
    # --critic_layers when they differ from --actor_layers (`hidden`); None: `hidden`
    critic_hidden: Optional[Sequence[int]] = None
    # per-hidden-layer activations (nn_utils.py:5-22); None: `act` for every layer
    actor_acts: Optional[Sequence[str]] = None
    critic_acts: Optional[Sequence[str]] = None
    # SAC-EO
    epsilon: float = 1e-3         # train_parser.py:280
    model_hidden: Sequence[int] = (512, 512)
    model_act: str = "relu"
    lr_model: float = 1e-3
    reward_loss_coef: float = 1.0
    delta_clip_pred: float = 0.0  # --delta_clip_pred (base_world_model.py:80-82); 0: None
    # --gaussian_model (init_world_models.py:13-16): GaussianModel, a trainable logstd (1, S) per
    # model (continuous_models.py:24-27), the Gaussian NLL fit loss (:101-131) with the optional
    # --scale_model_loss stop-gradient scale mean(exp(logstd)^2) (:122-127), noise in sample / step
    gaussian_model: bool = False
    scale_model_loss: bool = False
    # --separate_reward_nn (base_world_model.py:32-37): the model net predicts the S delta columns,
    # a second net [S+A] -> reward_hidden -> 1 the reward (:72-74)
    separate_reward_nn: bool = False
    reward_hidden: Sequence[int] = (512, 512)
    reward_act: str = "relu"

    # SAC-EO world models (--num_models): all are fitted, the expert term uses models 0 and 1
    num_models: int = 2

    @property
    def aacts(self):
        return tuple(self.actor_acts) if self.actor_acts else (self.act,) * len(self.hidden)

    @property
    def cacts(self):
        return tuple(self.critic_acts) if self.critic_acts else (self.act,) * len(self.chidden)

    @property
    def chidden(self):
        return tuple(self.critic_hidden) if self.critic_hidden else tuple(self.hidden)

    @property
    def target_entropy(self) -> float:
        return -float(self.A)     # SAC_expert.py:46


@dataclasses.dataclass
class Normalizers:
    """(x - mean) / max(std, 1e-8) per normalizer.py:26-41 ('den' = max(std,1e-8))."""
    s_mean: np.ndarray
    s_den: np.ndarray
    a_mean: np.ndarray
    a_den: np.ndarray
    d_mean: np.ndarray
    d_den: np.ndarray
    r_mean: float = 0.0
    r_den: float = 1.0
    ret_den: float = 1.0

    @staticmethod
    def identity(S: int, A: int) -> "Normalizers":
        z = np.zeros
        o = np.ones
        return Normalizers(z(S, np.float32), o(S, np.float32), z(A, np.float32),
                           o(A, np.float32), z(S, np.float32), o(S, np.float32))

    def cast(self, dt):
        c = lambda x: np.asarray(x, dtype=dt)
        return Normalizers(c(self.s_mean), c(self.s_den), c(self.a_mean), c(self.a_den),
                           c(self.d_mean), c(self.d_den), c(self.r_mean), c(self.r_den),
                           c(self.ret_den))


@dataclasses.dataclass
class AdamState:
    t: int
    m: List[np.ndarray]
    v: List[np.ndarray]

    @staticmethod
    def zeros_like(params: List[np.ndarray]) -> "AdamState":
        return AdamState(0, [np.zeros_like(p) for p in params], [np.zeros_like(p) for p in params])


@dataclasses.dataclass
class SACState:
    """Keras weight-list layout [W0(in,out), b0, W1, b1, W2, b2] per net
    (pinned by the reference's pickled logs); the actor's global
    logstd (1,A) variable is kept separately (continuous_actors.py:56-58)."""
    actor: List[np.ndarray]
    logstd: np.ndarray
    q: List[List[np.ndarray]]
    q_targ: List[List[np.ndarray]]
    alpha: np.ndarray
    opt_actor: AdamState
    opt_q: List[AdamState]
    opt_alpha: AdamState
    models: Optional[List[List[np.ndarray]]] = None
    opt_model: Optional[AdamState] = None
    # GaussianModel's logstd variable (1, S) per model (continuous_models.py:24-25)
    model_logstd: Optional[List[np.ndarray]] = None
    # --separate_reward_nn: the reward net's Keras weight list per model (base_world_model.py:36-37)
    reward_nets: Optional[List[List[np.ndarray]]] = None

    def copy(self) -> "SACState":
        cp = lambda L: [x.copy() for x in L]
        cpo = lambda o: AdamState(o.t, cp(o.m), cp(o.v))
        return SACState(cp(self.actor), self.logstd.copy(), [cp(x) for x in self.q],
                        [cp(x) for x in self.q_targ], self.alpha.copy(), cpo(self.opt_actor),
                        [cpo(o) for o in self.opt_q], cpo(self.opt_alpha),
                        None if self.models is None else [cp(x) for x in self.models],
                        None if self.opt_model is None else cpo(self.opt_model),
                        None if self.model_logstd is None else cp(self.model_logstd),
                        None if self.reward_nets is None else [cp(x) for x in self.reward_nets])

    def astype(self, dt) -> "SACState":
        c = lambda L: [np.asarray(x, dtype=dt).copy() for x in L]
        co = lambda o: AdamState(o.t, c(o.m), c(o.v))
        return SACState(c(self.actor), np.asarray(self.logstd, dt).copy(), [c(x) for x in self.q],
                        [c(x) for x in self.q_targ], np.asarray(self.alpha, dt).copy(),
                        co(self.opt_actor), [co(o) for o in self.opt_q], co(self.opt_alpha),
                        None if self.models is None else [c(x) for x in self.models],
                        None if self.opt_model is None else co(self.opt_model),
                        None if self.model_logstd is None else c(self.model_logstd),
                        None if self.reward_nets is None else [c(x) for x in self.reward_nets])

    def model_vars(self, k: int) -> List[np.ndarray]:
        """model.trainable (continuous_models.py:27-32, :216-221): the model net's variables,
        GaussianModel's logstd, then the separate reward net's -- the model optimiser's order
        (mbrl_onpolicy_alg.py:28-30 concatenates them over the models)."""
        out = list(self.models[k])
        if self.model_logstd is not None:
            out.append(self.model_logstd[k])
        if self.reward_nets is not None:
            out += self.reward_nets[k]
        return out

    def model_all_vars(self) -> List[np.ndarray]:
        return [w for k in range(len(self.models)) for w in self.model_vars(k)]


# ---------------------------------------------------------------------------
# initialisation (orthogonal, nn_utils.py:24-57; TF's RNG is not reproducible,
# so parity tests inject these weights identically into oracle and device)
# ---------------------------------------------------------------------------
def orthogonal(rng: np.random.RandomState, shape, gain: float) -> np.ndarray:
    rows, cols = int(np.prod(shape[:-1])), int(shape[-1])
    flat = (rows, cols) if rows >= cols else (cols, rows)
    a = rng.normal(size=flat)
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    if rows < cols:
        q = q.T
    return (gain * q).reshape(shape).astype(np.float32)


def init_mlp(rng, in_dim: int, out_dim: int, hidden: Sequence[int], gain_final: float,
             bias_scale: float = 0.0) -> List[np.ndarray]:
    dims = [in_dim] + list(hidden) + [out_dim]
    params = []
    for l in range(len(dims) - 1):
        g = math.sqrt(2.0) if l < len(dims) - 2 else gain_final
        params.append(orthogonal(rng, (dims[l], dims[l + 1]), g))
        params.append((bias_scale * rng.normal(size=dims[l + 1])).astype(np.float32))
    return params


def init_state(cfg: Config, seed: int = 1, with_models: bool = False,
               bias_scale: float = 0.0, actor_gain: float = 0.01, critic_gain: float = 1.0,
               model_gain: float = 0.01, model_std_mult: float = 1.0, reward_gain: float = 0.01) -> SACState:
    rng = np.random.RandomState(seed)
    out_a = 2 * cfg.A if cfg.per_state_std else cfg.A
    actor = init_mlp(rng, cfg.S, out_a, cfg.hidden, actor_gain, bias_scale)
    if cfg.layer_norm:            # gamma, beta after b0 (perturbed from 1 / 0 so the test sees them)
        H0 = cfg.hidden[0]
        actor = actor[:2] + [(1.0 + 0.1 * rng.normal(size=H0)).astype(np.float32),
                             (0.1 * rng.normal(size=H0)).astype(np.float32)] + actor[2:]
    q = [init_mlp(rng, cfg.S + cfg.A, 1, cfg.chidden, critic_gain, bias_scale) for _ in range(2)]
    q_targ = [[w.copy() for w in net] for net in q]         # init_critic.py:34-35
    logstd = np.zeros((1, cfg.A), np.float32)
    alpha = np.asarray(np.log(cfg.init_temperature), np.float32)  # SAC_expert.py:106
    st = SACState(actor, logstd, q, q_targ, alpha,
                  AdamState.zeros_like(actor + [logstd]),
                  [AdamState.zeros_like(n) for n in q], AdamState.zeros_like([alpha]))
    if with_models:
        om = cfg.S if cfg.separate_reward_nn else cfg.S + 1
        st.models = [init_mlp(rng, cfg.S + cfg.A, om, cfg.model_hidden, model_gain, bias_scale)
                     for _ in range(max(2, cfg.num_models))]
        if cfg.gaussian_model:           # np.ones((1, s_dim)) * np.log(std_mult) (continuous_models.py:24)
            # (perturbed from the uniform init so that the tests see a per-column logstd)
            st.model_logstd = [(np.ones((1, cfg.S)) * np.log(model_std_mult)
                                + 0.05 * rng.normal(size=(1, cfg.S))).astype(np.float32)
                               for _ in range(max(2, cfg.num_models))]
        if cfg.separate_reward_nn:
            st.reward_nets = [init_mlp(rng, cfg.S + cfg.A, 1, cfg.reward_hidden, reward_gain, bias_scale)
                              for _ in range(max(2, cfg.num_models))]
        st.opt_model = AdamState.zeros_like(st.model_all_vars())
    return st


# ---------------------------------------------------------------------------
# elementwise pieces (TF semantics)
# ---------------------------------------------------------------------------
def _F(dt, x):
    return np.asarray(x, dtype=dt)


def act_fwd(z, kind):
    if kind == "relu":
        return np.maximum(z, 0)
    if kind == "tanh":
        return np.tanh(z)
    if kind == "elu":            # TF: features<0 ? exp(x)-1 : x
        return np.where(z < 0, np.exp(np.minimum(z, 0)) - 1, z).astype(z.dtype)
    raise ValueError(kind)


def act_grad(h, kind):
    """Derivative expressed through the layer OUTPUT (TF ReluGrad / TanhGrad /
    EluGrad all take the activation output)."""
    one = np.ones((), h.dtype)
    if kind == "relu":
        return (h > 0).astype(h.dtype)
    if kind == "tanh":
        return one - h * h
    if kind == "elu":
        return np.where(h < 0, h + one, one).astype(h.dtype)
    raise ValueError(kind)


def softplus(x):
    # TF softplus_op.h: x > -thr ? x : (x < thr ? exp(x) : log1p(exp(x)))
    thr = x.dtype.type(np.log(np.finfo(x.dtype).eps) + 2.0)      # < 0
    xc = np.clip(x, thr, -thr)
    out = np.where(x > -thr, x, np.where(x < thr, np.exp(np.minimum(x, thr)), np.log1p(np.exp(xc))))
    return out.astype(x.dtype)


# ---------------------------------------------------------------------------
# MLP (Keras Dense: y = act(x @ W + b))
# ---------------------------------------------------------------------------
# Summation order of the fp32 forward products.  Every order is a faithful fp32 execution of
# the reference's Dense layers (TF's kernels fix none of them); tests/test_gpu_schedule.py runs
# the fp32 oracle under each to get the envelope of the drift a faithful fp32 run has from fp64.
MATMUL_ORDERS = ("default", "reversed", "split4")
MATMUL_ORDER = "default"


def matmul(h, w):
    if h.dtype != np.float32 or MATMUL_ORDER == "default":
        return h @ w
    if MATMUL_ORDER == "reversed":                   # k accumulated from the last row of w
        return np.ascontiguousarray(h[:, ::-1]) @ np.ascontiguousarray(w[::-1])
    if MATMUL_ORDER == "split4":                     # four k slabs, summed pairwise (k_gemm's 4 waves)
        c = (w.shape[0] + 3) // 4
        p = [h[:, i * c:(i + 1) * c] @ w[i * c:(i + 1) * c] for i in range(4)]
        return (p[0] + p[1]) + (p[2] + p[3])
    raise ValueError(MATMUL_ORDER)


def mlp_forward(params, x, act):
    hs = []
    h = x
    nl = len(params) // 2
    out = None
    for l in range(nl):
        z = matmul(h, params[2 * l]) + params[2 * l + 1]
        if l < nl - 1:
            h = act_fwd(z, act[l] if isinstance(act, (list, tuple)) else act)
            hs.append(h)
        else:
            out = z
    return out, hs


def mlp_backward(params, x, hs, dout, act, need_dx=False, need_dw=True):
    nl = len(params) // 2
    grads = [None] * len(params)
    d = dout
    dx = None
    for l in reversed(range(nl)):
        inp = x if l == 0 else hs[l - 1]
        if need_dw:
            grads[2 * l] = inp.T @ d
            grads[2 * l + 1] = d.sum(axis=0)
        if l > 0:
            d = (d @ params[2 * l].T) * act_grad(hs[l - 1], act[l - 1] if isinstance(act, (list, tuple)) else act)
        elif need_dx:
            dx = d @ params[0].T
    return grads, dx


# ---------------------------------------------------------------------------
# the actor's MLP: create_nn with layer_norm (nn_utils.py:108-119) puts Keras
# LayerNormalization (epsilon 1e-3, gamma, beta) and tanh after the first Dense; its weight
# list is [W0, b0, gamma, beta, W1, b1, W2, b2].  hs = [H1, H2] (+ [xhat, rstd] with the norm).
# ---------------------------------------------------------------------------
LN_EPS = 1e-3


def actor_forward(params, x, cfg):
    if not cfg.layer_norm:
        return mlp_forward(params, x, cfg.aacts)
    dt = x.dtype.type
    z = x @ params[0] + params[1]
    mu = z.mean(-1, keepdims=True)
    d = z - mu
    rstd = _F(dt, 1) / np.sqrt((d * d).mean(-1, keepdims=True) + _F(dt, LN_EPS))
    xh = d * rstd
    h1 = np.tanh(params[2] * xh + params[3])
    out, hs = mlp_forward(params[4:], h1, cfg.aacts[1:])
    return out, [h1] + hs + [xh, rstd]


def actor_backward(params, x, hs, dout, cfg):
    """Gradients of the actor weight list (same order as params)."""
    if not cfg.layer_norm:
        return mlp_backward(params, x, hs, dout, cfg.aacts)[0]
    h1, rest, xh, rstd = hs[0], hs[1:-2], hs[-2], hs[-1]
    g_rest, dh1 = mlp_backward(params[4:], h1, rest, dout, cfg.aacts[1:], need_dx=True)
    one = np.ones((), h1.dtype)
    dy = dh1 * (one - h1 * h1)
    gg = dy * params[2]
    dz = rstd * ((gg - gg.mean(-1, keepdims=True)) - xh * (gg * xh).mean(-1, keepdims=True))
    return [x.T @ dz, dz.sum(axis=0), (dy * xh).sum(axis=0), dy.sum(axis=0)] + g_rest


# ---------------------------------------------------------------------------
# squashed Gaussian head (continuous_actors.py:270-379)
# ---------------------------------------------------------------------------
@dataclasses.dataclass
class HeadCache:
    x: np.ndarray
    t: np.ndarray
    std: np.ndarray
    u: np.ndarray
    mask: np.ndarray      # d clip/d logstd_raw (TF clip_by_value: pass inside [min,max] incl.)


def split_head(out, logstd_var, cfg: Config):
    if cfg.per_state_std:
        return out[:, :cfg.A], out[:, cfg.A:]       # no softplus (:334-336)
    return out, np.broadcast_to(logstd_var, out.shape)


def head_evaluate(mu, logstd_raw, u, lim, dt):
    """evaluate(): returns (pi, neglogp_adjusted, cache).  u is the N(0,1)
    draw already cast to the compute dtype (TF casts numpy f64 -> f32)."""
    l = np.clip(logstd_raw, _F(dt, LOG_STD_MIN), _F(dt, LOG_STD_MAX)).astype(dt)
    std = np.exp(l)
    x = mu + std * u
    z = (x - mu) / np.exp(l)
    vec = z * z + _F(dt, 2) * l + _F(dt, np.log(_F(dt, 2 * np.pi)))
    nlp = _F(dt, 0.5) * vec.sum(axis=-1)
    corr = _F(dt, 2.0) * (_F(dt, np.log(2.0)) - x - softplus(_F(dt, -2.0) * x))
    nlp_adj = nlp + corr.sum(axis=-1)
    t = np.tanh(x)
    pi = _F(dt, lim) * t
    mask = ((logstd_raw >= LOG_STD_MIN) & (logstd_raw <= LOG_STD_MAX)).astype(dt)
    return pi, nlp_adj, HeadCache(x, t, std, u, mask)


def head_sample(mu, logstd_raw, u, lim, dt):
    """sample(deterministic=False) (continuous_actors.py:270-306)."""
    l = np.clip(logstd_raw, _F(dt, LOG_STD_MIN), _F(dt, LOG_STD_MAX)).astype(dt)
    std = np.exp(l)
    x = mu + std * u
    t = np.tanh(x)
    mask = ((logstd_raw >= LOG_STD_MIN) & (logstd_raw <= LOG_STD_MAX)).astype(dt)
    return _F(dt, lim) * t, HeadCache(x, t, std, u, mask)


def head_backward(g_pi, c, cache: HeadCache, lim, dt):
    """Closed-form gradient of pi (and, for evaluate, of neglogp_adjusted with
    per-row weight c) w.r.t. mu and the unclipped logstd."""
    one = _F(dt, 1)
    gx = g_pi * _F(dt, lim) * (one - cache.t * cache.t)
    if c is not None:
        gx = gx - _F(dt, 2) * c[:, None] * cache.t
    dmu = gx
    dl = gx * cache.std * cache.u
    if c is not None:
        dl = dl + c[:, None]
    dl = dl * cache.mask
    return dmu, dl


# ---------------------------------------------------------------------------
# Keras Adam (legacy OptimizerV2 / ResourceApplyAdam) and NumPy Polyak
# ---------------------------------------------------------------------------
def adam_step(params: List[np.ndarray], grads: List[np.ndarray], opt: AdamState, lr: float, dt):
    opt.t += 1
    b1, b2, eps = _F(dt, 0.9), _F(dt, 0.999), _F(dt, 1e-7)
    tt = _F(dt, opt.t)
    b1p = np.power(b1, tt)
    b2p = np.power(b2, tt)
    one = _F(dt, 1)
    alpha_t = _F(dt, lr) * np.sqrt(one - b2p) / (one - b1p)
    for i, (p, g) in enumerate(zip(params, grads)):
        m, v = opt.m[i], opt.v[i]
        m += (g - m) * (one - b1)
        v += (g * g - v) * (one - b2)
        p -= (m * alpha_t) / (np.sqrt(v) + eps)


def polyak(targ: List[np.ndarray], src: List[np.ndarray], tau: float, dt):
    """SAC_expert.py:362-373 -- two fp32 roundings then an add, no FMA."""
    c1, c2 = _F(dt, 1.0 - tau), _F(dt, tau)
    for t, s in zip(targ, src):
        t[...] = t * c1 + s * c2


# ---------------------------------------------------------------------------
# one SAC / SAC-EO gradient step
# ---------------------------------------------------------------------------
@dataclasses.dataclass
class Expert:
    s1: np.ndarray
    sp1: np.ndarray
    s2: np.ndarray
    sp2: np.ndarray
    noise1: np.ndarray
    noise2: np.ndarray
    epsilon: float


def _norm(x, mean, den):
    return (x - mean) / den


def sac_update(st: SACState, cfg: Config, nrm: Normalizers, batch, noise_t, noise_pi, noise_alpha,
               expert: Optional[Expert] = None, do_polyak: bool = True, keep: Optional[dict] = None,
               grad_hook=None, mnrm: Optional[Normalizers] = None):
    """One ``_update`` (SAC_expert.py:463-477 / SAC.py:236-250), in place on
    ``st``.  ``batch`` = (s, a, sp, r, d) raw rows; noises are (n, A) arrays.
    Returns the step statistics.  ``keep`` (optional dict) receives the
    intermediates used by the stage-level GPU parity tests.  ``grad_hook(name, grads)``
    (optional) maps each optimiser's gradient list before its Adam ("q0", "q1", "actor",
    "alpha"): the data-parallel mode's all-reduce / ranks (include/sacx.h sacx_dp_init).
    ``mnrm``: the world models' normaliser (SAC_expert.py:139-144, --only_model_normalizer);
    None: the shared ``nrm`` (the reference's default)."""
    hook = grad_hook if grad_hook is not None else (lambda name, g: g)
    dt = st.alpha.dtype.type
    F = lambda x: _F(dt, x)
    nrm = nrm.cast(dt)
    mnrm = nrm if mnrm is None else mnrm.cast(dt)
    s, a, sp, r, d = [np.asarray(x, dt) for x in batch]
    n1, n2, n3 = [np.asarray(x, dt) for x in (noise_t, noise_pi, noise_alpha)]
    B, S = s.shape
    lim = cfg.act_limit
    alpha = st.alpha.copy()
    actor_all = st.actor
    stats = {}

    # ---------------- target (_get_Q_target, SAC_expert.py:211-229)
    sp_n = _norm(sp, nrm.s_mean, nrm.s_den)
    out_t, hs_t = actor_forward(actor_all, sp_n, cfg)
    mu_t, ls_t = split_head(out_t, st.logstd, cfg)
    a_t, nlp_t, _ = head_evaluate(mu_t, ls_t, n1, lim, dt)
    xq_t = np.concatenate([sp_n, _norm(a_t, nrm.a_mean, nrm.a_den)], axis=1)
    qt = [mlp_forward(net, xq_t, cfg.cacts)[0][:, 0] * nrm.ret_den for net in st.q_targ]
    next_value = np.minimum(qt[0], qt[1]) + alpha * nlp_t
    y = r + F(cfg.gamma) * ((F(1) - d) * next_value)
    if keep is not None:
        keep.update(sp_n=sp_n, actor_h_t=hs_t, mu_t=mu_t, a_t=a_t, nlp_t=nlp_t, qt=qt, y=y)

    # ---------------- critic (_update_critic, :232-259)
    s_n = _norm(s, nrm.s_mean, nrm.s_den)
    xq = np.concatenate([s_n, _norm(a, nrm.a_mean, nrm.a_den)], axis=1)
    for k in range(2):
        q, hs = mlp_forward(st.q[k], xq, cfg.cacts)
        e = q[:, 0] - y
        stats["q%d_loss" % (k + 1)] = float(np.mean(F(0.5) * e * e))
        dq = (e * F(1.0 / B))[:, None]
        grads, _ = mlp_backward(st.q[k], xq, hs, dq, cfg.cacts)
        if keep is not None:
            keep["q%d_h" % k] = hs
            keep["q%d_out" % k] = q[:, 0]
            keep["q%d_grads" % k] = grads
        adam_step(st.q[k], hook("q%d" % k, grads), st.opt_q[k], cfg.lr_q, dt)

    # ---------------- actor (_update_actor_and_alpha, :262-338)
    out_p, hs_p = actor_forward(actor_all, s_n, cfg)
    mu_p, ls_p = split_head(out_p, st.logstd, cfg)
    a_p, nlp_p, cache_p = head_evaluate(mu_p, ls_p, n2, lim, dt)
    xq_p = np.concatenate([s_n, _norm(a_p, nrm.a_mean, nrm.a_den)], axis=1)
    fq = [mlp_forward(net, xq_p, cfg.cacts) for net in st.q]
    q1p, q2p = fq[0][0][:, 0], fq[1][0][:, 0]
    minq = np.minimum(q1p, q2p)
    p_loss = np.mean(-alpha * nlp_p - minq)
    w_sac = F(1.0 - expert.epsilon) if expert is not None else F(1)
    # d p / d minQ_i = -1/B, split on ties (TF _MinOrMaxGrad)
    gmin = -w_sac * F(1.0 / B)
    sel1 = np.where(q1p < q2p, F(1), np.where(q1p == q2p, F(0.5), F(0)))
    sel2 = np.where(q2p < q1p, F(1), np.where(q1p == q2p, F(0.5), F(0)))
    dxa = None
    for k, sel in enumerate((sel1, sel2)):
        _, dx = mlp_backward(st.q[k], xq_p, fq[k][1], (gmin * sel)[:, None], cfg.cacts,
                             need_dx=True, need_dw=False)
        part = dx[:, S:] / nrm.a_den
        dxa = part if dxa is None else dxa + part
    c = np.full(B, -w_sac * alpha * F(1.0 / B), dt)
    dmu, dl = head_backward(dxa, c, cache_p, lim, dt)
    rows_x = [s_n]
    rows_h = [hs_p]
    rows_dmu = [dmu]
    rows_dl = [dl]
    mse = None
    if expert is not None:
        eps = F(expert.epsilon)
        # 2 models: the permuted halves (:301-335); 1 model (expert.s2 None): every expert row
        # through model 0 (:290-296)
        halves = [(expert.s1, expert.sp1, expert.noise1)]
        if expert.s2 is not None:
            halves.append((expert.s2, expert.sp2, expert.noise2))
        diffs = []
        caches = []
        for k, (se, spe, ne) in enumerate(halves):
            se, spe, ne = np.asarray(se, dt), np.asarray(spe, dt), np.asarray(ne, dt)
            se_n = _norm(se, nrm.s_mean, nrm.s_den)
            out_e, hs_e = actor_forward(actor_all, se_n, cfg)
            mu_e, ls_e = split_head(out_e, st.logstd, cfg)
            ca, cache_e = head_sample(mu_e, ls_e, ne, lim, dt)
            # the model normalises its own inputs (MSEModel.sample -> _forward, base_world_model.py:67-69)
            xm = np.concatenate([_norm(se, mnrm.s_mean, mnrm.s_den), _norm(ca, mnrm.a_mean, mnrm.a_den)], axis=1)
            om, hsm = mlp_forward(st.models[k], xm, cfg.model_act)
            dn = om[:, :S]
            dpass = np.ones_like(dn)
            if cfg.delta_clip_pred:
                # MSEModel.sample -> _forward(clip=True): tf.clip_by_value, whose gradient is zero
                # outside [-c, c] and passes at the bounds (TF _ClipByValueGrad)
                c = F(cfg.delta_clip_pred)
                dpass = ((dn >= -c) & (dn <= c)).astype(dt)
                dn = np.minimum(np.maximum(dn, -c), c)
            sp_hat = se + (dn * mnrm.d_den + mnrm.d_mean)
            diffs.append(spe - sp_hat)
            caches.append((se_n, hs_e, cache_e, xm, hsm, spe, sp_hat, dpass))
        if len(diffs) == 2:
            dl_e = F(0.5) * ((diffs[0] ** 2).sum(-1) + (diffs[1] ** 2).sum(-1))
        else:
            dl_e = F(0.5) * (diffs[0] ** 2).sum(-1)
        mse = np.mean(dl_e)
        p_loss = (F(1) - eps) * p_loss + eps * mse
        ne_half = diffs[0].shape[0]
        for k, (se_n, hs_e, cache_e, xm, hsm, spe, sp_hat, dpass) in enumerate(caches):
            dsp = -eps * F(1.0 / ne_half) * diffs[k]
            dout = np.zeros((ne_half, om.shape[1]), dt)        # S + 1, or S with the separate reward net
            dout[:, :S] = dsp * mnrm.d_den * dpass
            if keep is not None:
                keep["clip_frac%d" % k] = float(1.0 - dpass.mean())
            _, dxm = mlp_backward(st.models[k], xm, hsm, dout, cfg.model_act,
                                  need_dx=True, need_dw=False)
            dca = dxm[:, S:] / mnrm.a_den
            dmu_e, dl_ee = head_backward(dca, None, cache_e, lim, dt)
            rows_x.append(se_n)
            rows_h.append(hs_e)
            rows_dmu.append(dmu_e)
            rows_dl.append(dl_ee)
        stats["mse_loss"] = float(mse)
    X = np.concatenate(rows_x, 0)
    Hs = [np.concatenate([h[l] for h in rows_h], 0) for l in range(len(rows_h[0]))]
    DMU = np.concatenate(rows_dmu, 0)
    DL = np.concatenate(rows_dl, 0)
    if cfg.per_state_std:
        dout_a = np.concatenate([DMU, DL], axis=1)
        g_logstd = np.zeros_like(st.logstd)
    else:
        dout_a = DMU
        g_logstd = DL.sum(axis=0, keepdims=True)
    grads_a = actor_backward(actor_all, X, Hs, dout_a, cfg)
    if keep is not None:
        keep.update(actor_h_p=hs_p, mu_p=mu_p, a_p=a_p, nlp_p=nlp_p, q1p=q1p, q2p=q2p,
                    dxa=dxa, dmu=DMU, dl=DL, actor_grads=grads_a, g_logstd=g_logstd)
    stats["p_loss"] = float(p_loss)
    adam_step(st.actor + [st.logstd], hook("actor", grads_a + [g_logstd]), st.opt_actor, cfg.lr_pi, dt)

    # ---------------- alpha (:340-348)
    out_3, _ = actor_forward(st.actor, s_n, cfg)
    mu_3, ls_3 = split_head(out_3, st.logstd, cfg)
    _, nlp_3, _ = head_evaluate(mu_3, ls_3, n3, lim, dt)
    m_ent = np.mean(-nlp_3 + F(cfg.target_entropy))
    stats["alpha_loss"] = float(-alpha * m_ent)
    g_alpha = np.asarray(-m_ent, dt)
    # a 0-d ARRAY, updated in place by adam_step (a NumPy scalar would be rebound, not updated)
    al = [np.array(st.alpha, dtype=dt)]
    adam_step(al, hook("alpha", [g_alpha]), st.opt_alpha, cfg.lr_alpha, dt)
    st.alpha = np.array(np.maximum(al[0], F(1e-5)), dtype=dt)
    stats["alpha"] = float(st.alpha)
    if keep is not None:
        keep.update(nlp_3=nlp_3, g_alpha=g_alpha)

    # ---------------- Polyak (:362-373)
    if do_polyak:
        for k in range(2):
            polyak(st.q_targ[k], st.q[k], cfg.tau, dt)
    return stats


# ---------------------------------------------------------------------------
# world model: loss and one fitting step (continuous_models.py:280-302,
# mbrl_onpolicy_alg.py:301-319)
# ---------------------------------------------------------------------------
def model_predict(st: SACState, cfg: Config, k: int, xm):
    """BaseWorldModel._forward before its clips (base_world_model.py:65-78): the model net's delta
    columns and the reward -- its last column, or the separate reward net's output (:72-74).
    Returns (delta_n [n, S], r_n [n], (out, hs, rout, rhs)) with the caches of both nets."""
    out, hs = mlp_forward(st.models[k], xm, cfg.model_act)
    if cfg.separate_reward_nn:
        ro, rhs = mlp_forward(st.reward_nets[k], xm, cfg.reward_act)
        return out[:, :cfg.S], ro[:, 0], (out, hs, ro, rhs)
    return out[:, :cfg.S], out[:, cfg.S], (out, hs, None, None)


def model_entropy(st: SACState, cfg: Config, k: int) -> float:
    """model.entropy's per-row value (logged as model_ent, SAC_expert.py:486-490): GaussianModel
    0.5 sum(2 logstd + log 2 pi + 1) (continuous_models.py:162-166); MSEModel 0 (:321-323)."""
    if not cfg.gaussian_model:
        return 0.0
    dt = st.alpha.dtype.type
    l = np.asarray(st.model_logstd[k], dt)
    return float(_F(dt, 0.5) * np.sum(_F(dt, 2) * l + _F(dt, np.log(np.float32(2 * np.pi))) + _F(dt, 1)))


def model_fit_step(st: SACState, cfg: Config, nrm: Normalizers, batches, max_grad_norm=None,
                   delta_clip_loss=0.0, reward_clip_loss=0.0):
    """``batches`` = [(s, a, sp, r)] per model (independent minibatches,
    SAC_expert.py:519-543; one entry per world model).  Sum of the per-model mean losses
    (get_loss with the optional target clips: MSEModel continuous_models.py:280-302, GaussianModel
    :101-131 -- 0.5 sum_j (((dn - mu) / e^l)^2 + 2 l + log 2 pi), times the stop-gradient
    mean(e^{2l}) with --scale_model_loss, plus reward_loss_coef * 0.5 (rn - r_pred)^2, the reward from
    the separate reward net with --separate_reward_nn), the optional
    clip_by_global_norm(grads, max_grad_norm * num_models) (mbrl_onpolicy_alg.py:315-317,
    TF clip_ops: scale = clip * min(1 / norm, 1 / clip)), one Adam over all model variables in
    model.trainable order (SACState.model_vars).  Returns the summed loss."""
    dt = st.alpha.dtype.type
    F = lambda x: _F(dt, x)
    nrm = nrm.cast(dt)
    S = cfg.S
    grads_all = []
    loss_all = F(0)
    for k, (s, a, sp, r) in enumerate(batches):
        s, a, sp, r = [np.asarray(x, dt) for x in (s, a, sp, r)]
        n = s.shape[0]
        xm = np.concatenate([_norm(s, nrm.s_mean, nrm.s_den), _norm(a, nrm.a_mean, nrm.a_den)], 1)
        dpred, rpred, (out, hs, ro, rhs) = model_predict(st, cfg, k, xm)
        dn = ((sp - s) - nrm.d_mean) / nrm.d_den
        rn = (r - nrm.r_mean) / nrm.r_den
        if delta_clip_loss:
            dn = np.clip(dn, -F(delta_clip_loss), F(delta_clip_loss))
        if reward_clip_loss:
            rn = np.clip(rn, -F(reward_clip_loss), F(reward_clip_loss))
        ed = dn - dpred
        er = rn - rpred
        g_l = None
        if cfg.gaussian_model:
            l = np.asarray(st.model_logstd[k], dt)
            e = np.exp(l)
            q = ed / e
            dscale = np.mean(e * e) if cfg.scale_model_loss else F(1)     # tf.stop_gradient (:122-127)
            nlp = F(0.5) * (q * q + F(2) * l + F(np.log(np.float32(2 * np.pi)))).sum(-1)
            per = dscale * nlp + F(cfg.reward_loss_coef) * (F(0.5) * er * er)
            dd = -(q / e) * (dscale * F(1.0 / n))
            g_l = ((F(1) - q * q) * (dscale * F(1.0 / n))).sum(axis=0, keepdims=True)
        else:
            per = F(0.5) * (ed * ed).sum(-1) + F(cfg.reward_loss_coef) * (F(0.5) * er * er)
            dd = -ed * F(1.0 / n)
        dr = -er * F(cfg.reward_loss_coef / n)
        loss_all = loss_all + np.mean(per)
        dout = np.zeros_like(out)
        dout[:, :S] = dd
        if not cfg.separate_reward_nn:
            dout[:, S] = dr
        g, _ = mlp_backward(st.models[k], xm, hs, dout, cfg.model_act)
        grads_all += g
        if g_l is not None:
            grads_all.append(g_l)
        if cfg.separate_reward_nn:
            gr, _ = mlp_backward(st.reward_nets[k], xm, rhs, dr[:, None], cfg.reward_act)
            grads_all += gr
    nm = len(batches)
    if max_grad_norm:
        clip = F(max_grad_norm * nm)
        norm = np.sqrt(sum(np.sum(g * g) for g in grads_all)).astype(dt)
        scale = clip * np.minimum(F(1) / norm, F(1) / clip)
        grads_all = [g * scale for g in grads_all]
    params = [w for k in range(nm) for w in st.model_vars(k)]
    adam_step(params, grads_all, st.opt_model, cfg.lr_model, dt)
    return float(loss_all)


def _model_noise(st, cfg, k, dn, u):
    """GaussianModel.sample / step (continuous_models.py:36-70): delta_n + exp(logstd) * u, u the
    global stream's normal(size=shape(delta_n)) cast to f32 (None: deterministic / MSEModel)."""
    if u is None or not cfg.gaussian_model:
        return dn
    dt = dn.dtype.type
    return dn + np.exp(np.asarray(st.model_logstd[k], dt)) * np.asarray(u, dt)


# ---------------------------------------------------------------------------
# world-model rollout (F2): batch_simtrajectory_sampler (samplers.py:73-122) with an
# MSEModel as the environment (continuous_models.py:225-258)
# ---------------------------------------------------------------------------
def rollout(st: SACState, cfg: Config, nrm: Normalizers, s_init, horizon: int, k: int, rs=None,
            deterministic: bool = False, delta_clip: float = 0.0, reward_clip: float = 0.0,
            mnrm: Optional[Normalizers] = None):
    """Returns (s, a, r, sp, d) of shapes [n,H,S], [n,H,A], [n,H], [n,H,S], [n,H].

    Per step (samplers.py:89-116): a = actor.sample(s) (continuous_actors.py:270-306,
    u = rs.normal(size=(n, A)) cast to f32, none when deterministic); env.step(actor.clip(a))
    = MSEModel.step: (delta_n, r_n) = _forward(s, clip(a)) with the optional prediction clips
    (base_world_model.py:65-87), s <- s + delta_rms.denormalize(delta_n), r =
    r_rms.denormalize(r_n), d = (ones_like(r) == 0) = False; the last step stores
    d = terminated (all False).  A GaussianModel adds exp(logstd) * u to delta_n (u =
    rs.normal(size=(n, S)) after the actor's draw, continuous_models.py:36-54).  ``mnrm``: the
    model's normaliser (None: ``nrm``)."""
    dt = st.alpha.dtype.type
    F = lambda x: _F(dt, x)
    nrm = nrm.cast(dt)
    mnrm = nrm if mnrm is None else mnrm.cast(dt)
    S, A = cfg.S, cfg.A
    s = np.asarray(s_init, dt).reshape(-1, S)
    n = s.shape[0]
    out = dict(s=[], a=[], r=[], sp=[], d=[])
    lim = F(cfg.act_limit)
    for _ in range(horizon):
        x = _norm(s, nrm.s_mean, nrm.s_den)
        o, _ = actor_forward(st.actor, x, cfg)
        mu, lraw = split_head(o, st.logstd, cfg)
        u = np.zeros_like(mu) if deterministic else f32_noise(rs.normal(size=mu.shape)).astype(dt)
        a, _ = head_sample(mu, lraw, u, cfg.act_limit, dt)
        ac = np.clip(a, -lim, lim)                                # actor.clip (continuous_actors.py:125)
        xm = np.concatenate([_norm(s, mnrm.s_mean, mnrm.s_den), _norm(ac, mnrm.a_mean, mnrm.a_den)], 1)
        dn, rn, _ = model_predict(st, cfg, k, xm)
        if delta_clip:
            dn = np.clip(dn, -F(delta_clip), F(delta_clip))
        if reward_clip:
            rn = np.clip(rn, -F(reward_clip), F(reward_clip))
        if cfg.gaussian_model:        # GaussianModel.step (continuous_models.py:36-54): always noisy
            dn = _model_noise(st, cfg, k, dn, f32_noise(rs.normal(size=dn.shape)))
        sp = s + (dn * mnrm.d_den + mnrm.d_mean)
        r = rn * mnrm.r_den + mnrm.r_mean
        for key, v in (("s", s), ("a", a), ("r", r), ("sp", sp), ("d", np.zeros(n, bool))):
            out[key].append(v)
        s = sp
    return tuple(np.stack(out[key], axis=1) for key in ("s", "a", "r", "sp", "d"))


# ---------------------------------------------------------------------------
# expert diagnostics (A17 / F3): SAC_expert.py:579-608 and _calc_disc :427-460
# ---------------------------------------------------------------------------
def _model_sample(st, cfg, nrm, k, s, a, delta_clip=0.0, rs=None):
    """MSEModel.sample (continuous_models.py:244-254) / GaussianModel.sample (:56-70) with
    _forward(clip=True); ``rs``: deterministic=False (a GaussianModel draws normal(size=(n, S)))."""
    dt = st.alpha.dtype.type
    xm = np.concatenate([_norm(s, nrm.s_mean, nrm.s_den), _norm(a, nrm.a_mean, nrm.a_den)], 1)
    dn, _, _ = model_predict(st, cfg, k, xm)
    if delta_clip:
        dn = np.clip(dn, -_F(dt, delta_clip), _F(dt, delta_clip))
    if rs is not None and cfg.gaussian_model:
        dn = _model_noise(st, cfg, k, dn, f32_noise(rs.normal(size=dn.shape)))
    return s + (dn * nrm.d_den + nrm.d_mean)


def _actor_sample(st, cfg, nrm, s, rs):
    dt = st.alpha.dtype.type
    o, _ = actor_forward(st.actor, _norm(s, nrm.s_mean, nrm.s_den), cfg)
    mu, lraw = split_head(o, st.logstd, cfg)
    u = f32_noise(rs.normal(size=mu.shape)).astype(dt)
    return head_sample(mu, lraw, u, cfg.act_limit, dt)[0]


def expert_mse_diag(st, cfg, nrm, s_e, a_e, sp_e, rs=None, use_expert_actions=False, delta_clip=0.0, mnrm=None):
    """(model_MSE_on_expert_data, model_MSE_on_expert_counterfactual_action): per model
    mean_i 0.5 ||model.sample(s_e, a) - sp_e||^2, averaged over the models; a = a_e, then
    a = actor.sample(s_e, deterministic=False) (one normal(size=(n, A)) draw) unless
    use_expert_actions.  ``mnrm``: the models' normaliser (None: ``nrm``, the actor's)."""
    dt = st.alpha.dtype.type
    nrm = nrm.cast(dt)
    mnrm = nrm if mnrm is None else mnrm.cast(dt)
    s_e, a_e, sp_e = [np.asarray(x, dt) for x in (s_e, a_e, sp_e)]
    nmod = len(st.models)

    def mse(a):
        per = [np.mean(_F(dt, 0.5) * ((_model_sample(st, cfg, mnrm, k, s_e, a, delta_clip) - sp_e) ** 2).sum(-1))
               for k in range(nmod)]
        return float(np.mean(per)), per
    m_data, per_data = mse(a_e)
    if use_expert_actions:
        return m_data, m_data, per_data, per_data
    m_cf, per_cf = mse(_actor_sample(st, cfg, nrm, s_e, rs))
    return m_data, m_cf, per_data, per_cf


def calc_disc(st, cfg, nrm, s_e, a_e, rs=None, use_expert_actions=False, delta_clip=0.0, mnrm=None):
    """_calc_disc: (disc_ratio, max_disc, median_disc, s_disc_total) of the two models'
    predictions on (s_e, a) with a = a_e or a fresh actor.sample(s_e) (tf_clip: a no-op); the
    models sample with deterministic=False (SAC_expert.py:437, :446: a GaussianModel draws its
    noise, model 0 then model 1, after the actor's)."""
    dt = st.alpha.dtype.type
    nrm = nrm.cast(dt)
    mnrm = nrm if mnrm is None else mnrm.cast(dt)
    s_e = np.asarray(s_e, dt)
    a = np.asarray(a_e, dt) if use_expert_actions else _actor_sample(st, cfg, nrm, s_e, rs)
    p0 = _model_sample(st, cfg, mnrm, 0, s_e, a, delta_clip, rs=rs)
    diff = p0 - _model_sample(st, cfg, mnrm, 1, s_e, a, delta_clip, rs=rs)
    for k in range(2, len(st.models)):          # every model samples (and draws); sp_pred[0] - sp_pred[1]
        _model_sample(st, cfg, mnrm, k, s_e, a, delta_clip, rs=rs)
    s_disc = np.sqrt((diff * diff).sum(axis=1))
    tot = np.sum(s_disc)
    return s_disc / tot, float(np.max(s_disc)), float(np.median(s_disc)), float(tot)


# ---------------------------------------------------------------------------
# the reference objects' standalone network calls (the methods a caller
# of the actor / critic / model objects uses)
# ---------------------------------------------------------------------------
def actor_evaluate(st, cfg, nrm, s, rs):
    """SquashedGaussianActor.evaluate (continuous_actors.py:327-379): (pi, neglogp_adjusted)
    with u = rs.normal(size=(n, A)) cast to f32."""
    dt = st.alpha.dtype.type
    nrm = nrm.cast(dt)
    o, _ = actor_forward(st.actor, _norm(np.asarray(s, dt), nrm.s_mean, nrm.s_den), cfg)
    mu, lraw = split_head(o, st.logstd, cfg)
    u = f32_noise(rs.normal(size=mu.shape)).astype(dt)
    pi, nlp, _ = head_evaluate(mu, lraw, u, cfg.act_limit, dt)
    return pi, nlp


def gaussian_actor_sample(params, logstd_var, cfg, nrm, s, u, std_mult=1.0, output_norm=False):
    """GaussianActor.sample (continuous_actors.py:74-123): mean (optionally output-normalised),
    logstd = log(softplus(out_std)) (per_state_std) or the variable, + logstd_init, floored at
    log(1e-3); a = mean + exp(logstd) * u (u = 0: deterministic).  No squash."""
    dt = params[0].dtype.type
    nrm = nrm.cast(dt)
    out, _ = mlp_forward(params, _norm(np.asarray(s, dt), nrm.s_mean, nrm.s_den), cfg.aacts)
    A = cfg.A
    if cfg.per_state_std:
        mean, l = out[:, :A], np.log(softplus(out[:, A:]))
        init = np.float32(np.log(std_mult) - np.log(np.log(2)))
    else:
        mean, l = out, np.broadcast_to(np.asarray(logstd_var, dt), out.shape)
        init = np.float32(np.log(std_mult))
    l = np.maximum(l + _F(dt, init), _F(dt, np.log(np.float32(1e-3))))
    if output_norm:
        mean = mean / np.maximum(np.mean(np.abs(mean), axis=-1, keepdims=True), _F(dt, 1.0))
    return mean + np.exp(l) * np.asarray(u, dt)


def critic_forward(params, cfg, nrm, s, a, value=False):
    """QCritic._forward ([n, 1]) / value (squeeze * max(ret std, 1e-8)) (critics.py:84-103)."""
    dt = params[0].dtype.type
    nrm = nrm.cast(dt)
    x = np.concatenate([_norm(np.asarray(s, dt), nrm.s_mean, nrm.s_den),
                        _norm(np.asarray(a, dt), nrm.a_mean, nrm.a_den)], 1)
    out, _ = mlp_forward(params, x, cfg.cacts)
    return out[:, 0] * _F(dt, nrm.ret_den) if value else out


def model_forward(st, cfg, nrm, k, s, a, delta_clip=0.0, reward_clip=0.0, noise=None):
    """BaseWorldModel._forward with the prediction clips (base_world_model.py:65-87) and what
    MSEModel.sample / step make of it (continuous_models.py:225-254): (pred [n, S+1] after the
    clips, sp = s + delta_rms.denormalize(delta_n), r = r_rms.denormalize(r_n)).  ``noise`` [n, S]:
    GaussianModel.sample(deterministic=False) / step (:36-70), exp(logstd) * u added to delta_n
    after the clips (pred stays the mean)."""
    dt = st.alpha.dtype.type
    nrm = nrm.cast(dt)
    s, a = np.asarray(s, dt), np.asarray(a, dt)
    xm = np.concatenate([_norm(s, nrm.s_mean, nrm.s_den), _norm(a, nrm.a_mean, nrm.a_den)], 1)
    dn, rn, _ = model_predict(st, cfg, k, xm)
    dn, rn = dn.copy(), rn.copy()
    if delta_clip:
        dn = np.clip(dn, -_F(dt, delta_clip), _F(dt, delta_clip))
    if reward_clip:
        rn = np.clip(rn, -_F(dt, reward_clip), _F(dt, reward_clip))
    dns = _model_noise(st, cfg, k, dn, None if noise is None else f32_noise(noise))
    return (np.concatenate([dn, rn[:, None]], 1), s + (dns * nrm.d_den + nrm.d_mean), rn * nrm.r_den + nrm.r_mean)


def model_loss(st, cfg, nrm, k, s, sp, a, r, delta_clip_loss=0.0, reward_clip_loss=0.0):
    """MSEModel.get_loss (continuous_models.py:280-302) / GaussianModel.get_loss (:101-131):
    _forward(clip=False), the loss clips on the normalised targets, mean over rows."""
    dt = st.alpha.dtype.type
    nrm = nrm.cast(dt)
    s, sp, a, r = [np.asarray(x, dt) for x in (s, sp, a, r)]
    pred, _, _ = model_forward(st, cfg, nrm, k, s, a)
    dn = ((sp - s) - nrm.d_mean) / nrm.d_den
    if delta_clip_loss:
        dn = np.clip(dn, -_F(dt, delta_clip_loss), _F(dt, delta_clip_loss))
    rn = (r - nrm.r_mean) / nrm.r_den
    if reward_clip_loss:
        rn = np.clip(rn, -_F(dt, reward_clip_loss), _F(dt, reward_clip_loss))
    ed = dn - pred[:, :cfg.S]
    if cfg.gaussian_model:
        l = np.asarray(st.model_logstd[k], dt)
        e = np.exp(l)
        q = ed / e
        dscale = np.mean(e * e) if cfg.scale_model_loss else _F(dt, 1)
        dl = dscale * (_F(dt, 0.5) * (q * q + _F(dt, 2) * l + _F(dt, np.log(np.float32(2 * np.pi)))).sum(-1))
    else:
        dl = _F(dt, 0.5) * (ed ** 2).sum(-1)
    per = dl + _F(dt, cfg.reward_loss_coef) * (_F(dt, 0.5) * (rn - pred[:, cfg.S]) ** 2)
    return float(np.mean(per))


# ---------------------------------------------------------------------------
# RNG consumption in the reference's order ("RNG consumption
# order"): the global legacy NumPy stream feeds the sampler and every noise
# draw; the expert split uses the algorithm's Generator (base_onpolicy_alg.py:109).
# ---------------------------------------------------------------------------
def draw_step_randoms(rs, cur_size: int, B: int, A: int, n_expert: int = 0, gen=None, n_models: int = 2):
    idx = rs.randint(cur_size, size=B)                          # buffers.py:136
    n1 = rs.normal(size=(B, A))                                 # target evaluate(sp)
    n2 = rs.normal(size=(B, A))                                 # actor evaluate(s)
    out = {"idx": idx, "noise_t": n1, "noise_pi": n2}
    if n_expert and n_models == 1:                              # SAC_expert.py:290-291: no shuffle
        out["sections"] = [np.arange(n_expert)]
        out["noise_e1"] = rs.normal(size=(n_expert, A))         # sample(s_expert)
        out["noise_e2"] = None
    elif n_expert:
        perm = np.arange(n_expert)
        gen.shuffle(perm)                                       # SAC_expert.py:301-303
        sec = np.array_split(perm, n_models)                    # the expert term takes sections 0 and 1
        out["perm"] = perm
        out["sections"] = sec
        out["noise_e1"] = rs.normal(size=(len(sec[0]), A))      # sample(s_expert_one)
        out["noise_e2"] = rs.normal(size=(len(sec[1]), A))      # sample(s_expert_two)
    out["noise_alpha"] = rs.normal(size=(B, A))                 # alpha evaluate(s)
    return out


def gather(buf, idx):
    """buffers.py:137-141: rows s, a, sp, r, d at idx (logical order)."""
    return buf["s"][idx], buf["a"][idx], buf["sp"][idx], buf["r"][idx], buf["d"][idx]


def f32_noise(x):
    """TF converts the float64 numpy draw to float32 (round to nearest)."""
    return np.asarray(x, np.float64).astype(np.float32)
