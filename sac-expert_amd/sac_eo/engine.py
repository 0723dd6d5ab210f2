"""Device engine: one libsacx handle + its HBM arena, viewed as torch tensors.

PyTorch-ROCm is plumbing here: it allocates the arena, supplies the HIP
stream and gives named views for setting weights / reading results.  All
update arithmetic runs in the hand-written gfx950 kernels behind the C ABI.
"""
from __future__ import annotations

import ctypes
import os
import dataclasses
import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _native as N

_TORCH_DT = {0: torch.float32, 1: torch.int32, 2: torch.int64, 3: torch.int32, 4: torch.float64}
_ESZ = {0: 4, 1: 4, 2: 8, 3: 4, 4: 8}

# ctl field indices (int64 slots, see csrc/sacx_internal.h struct Ctl)
CTL = {"t_sac": 0, "t_model": 1, "num_timesteps": 2, "ts_increment": 3, "cur_size": 4, "start": 5,
       "step_seq": 6, "n_expert": 7, "mfit_seq": 14, "rng_seq": 15, "pseq0": 16, "pseq1": 17, "pseq2": 18}


@dataclasses.dataclass
class EngineConfig:
    s_dim: int
    a_dim: int
    hidden: Sequence[int] = (256, 256)       # --actor_layers (and the critics' unless critic_hidden); 1-4 layers
    activation: str = "relu"
    critic_hidden: Optional[Sequence[int]] = None   # --critic_layers when they differ from the actor's
    batch: int = 256
    buffer_capacity: int = 1_000_000
    per_state_std: bool = False
    use_expert: bool = False
    expert_capacity: int = 20
    expert_batch: int = 20
    model_hidden: Sequence[int] = (512, 512)
    model_activation: str = "relu"
    model_batch: int = 200
    target_update_int: int = 1
    graph_steps: int = 128
    stats_capacity: int = 4096
    perm_capacity: int = 4096
    gamma: float = 0.995
    tau: float = 5e-3
    lr_q: float = 3e-4
    lr_pi: float = 1e-4
    lr_alpha: float = 1e-4
    lr_model: float = 1e-3
    init_temperature: float = 0.1
    target_entropy: Optional[float] = None
    act_limit: float = 1.0
    epsilon: float = 1e-3
    reward_loss_coef: float = 1.0
    gemm_bf16: bool = False     # config C5: bf16 MFMA operands, fp32 accumulate / master weights
    seeds: int = 1              # independent learners packed in one handle (one launch chain for all)
    single_seed_plan: bool = False  # packed seeds run the one-seed plan: each seed bit-identical to its own run
    actor_gaussian: bool = False    # GaussianActor (no squash): inference only (an imported expert)
    actor_std_mult: float = 1.0
    actor_output_norm: bool = False
    actor_layer_norm: bool = False  # Dense -> LayerNorm -> tanh on the actor's layer 0
    num_models: int = 2             # SAC-EO world models (1 .. 8; the expert term uses models 0 and 1)
    model_max_grad_norm: float = 0.0    # <= 0: None
    delta_clip_loss: float = 0.0        # <= 0: None
    reward_clip_loss: float = 0.0       # <= 0: None
    delta_clip_pred: float = 0.0        # the expert term's MSEModel.sample clip; <= 0: None
    # per-layer activations (the reference's --actor_activations / --critic_activations /
    # --model_activations lists); None: `activation` / `model_activation` for every layer
    actor_activations: Optional[Sequence[str]] = None
    critic_activations: Optional[Sequence[str]] = None
    model_activations: Optional[Sequence[str]] = None
    # world-model variants (ABI 7): --gaussian_model (GaussianModel: a trainable logstd per model,
    # the Gaussian NLL fit, noise in sample / step), --scale_model_loss, --separate_reward_nn (a
    # reward net of reward_hidden beside each model net)
    gaussian_model: bool = False
    scale_model_loss: bool = False
    separate_reward_nn: bool = False
    reward_hidden: Sequence[int] = (512, 512)
    reward_activations: Optional[Sequence[str]] = None

    @staticmethod
    def _acts(lst, dflt: str, depth: int, what: str) -> List[str]:
        """create_activations (nn_utils.py:5-22): one name for every layer, or one per layer."""
        lst = list(lst) if lst is not None else [dflt]
        lst = lst * depth if len(lst) == 1 else lst
        if len(lst) != depth:                               # create_nn's assert (nn_utils.py:106-107)
            raise ValueError(f"{what}: activations must be list of length len(layers) ({depth})")
        return lst

    def nets(self):
        """[(hidden widths, activation names)] of the actor, the critics, the world models and the
        reward nets (create_nn's layers / activations lists, nn_utils.py:86-138)."""
        hid = [tuple(self.hidden), tuple(self.critic_hidden if self.critic_hidden is not None else self.hidden),
               tuple(self.model_hidden), tuple(self.reward_hidden)]
        acts = [self._acts(self.actor_activations, self.activation, len(hid[0]), "actor"),
                self._acts(self.critic_activations, self.activation, len(hid[1]), "critic"),
                self._acts(self.model_activations, self.model_activation, len(hid[2]), "model"),
                self._acts(self.reward_activations, "relu", len(hid[3]), "reward")]
        return list(zip(hid, acts))

    def to_c(self) -> N.Config:
        c = N.Config()
        c.abi_version = N.SACX_ABI_VERSION
        c.s_dim, c.a_dim = int(self.s_dim), int(self.a_dim)
        nets = self.nets()
        for n, (hid, acts) in enumerate(nets):
            if not 1 <= len(hid) <= N.MAX_DEPTH:
                raise NotImplementedError(f"the device nets run 1 to {N.MAX_DEPTH} hidden layers (got {list(hid)})")
            # ABI 8: every layer of every net (the legacy two-layer fields below stay filled as well)
            c.net_depth[n] = len(hid)
            for l, (w, a) in enumerate(zip(hid, acts)):
                c.net_hidden[n][l] = int(w)
                c.net_acts[n][l] = N.ACT[a]
        two = lambda x: (list(x) + list(x))[:2]             # the legacy fields of a net (any depth: unused)
        c.hidden[0], c.hidden[1] = [int(x) for x in two(self.hidden)]
        if self.critic_hidden is not None:
            c.critic_hidden[0], c.critic_hidden[1] = [int(x) for x in two(self.critic_hidden)]
        c.activation = N.ACT[self.activation]
        c.batch = int(self.batch)
        c.buffer_capacity = int(self.buffer_capacity)
        c.per_state_std = int(bool(self.per_state_std))
        c.use_expert = int(bool(self.use_expert))
        c.expert_capacity = int(self.expert_capacity)
        c.expert_batch = int(self.expert_batch)
        c.model_hidden[0], c.model_hidden[1] = [int(x) for x in two(self.model_hidden)]
        c.model_activation = N.ACT[self.model_activation]
        c.model_batch = int(self.model_batch)
        c.target_update_int = int(self.target_update_int)
        c.graph_steps = int(self.graph_steps)
        c.stats_capacity = int(self.stats_capacity)
        c.perm_capacity = int(self.perm_capacity)
        c.gamma, c.tau = self.gamma, self.tau
        c.lr_q, c.lr_pi, c.lr_alpha, c.lr_model = self.lr_q, self.lr_pi, self.lr_alpha, self.lr_model
        c.init_temperature = self.init_temperature
        c.target_entropy = float(-self.a_dim if self.target_entropy is None else self.target_entropy)
        c.act_limit = self.act_limit
        c.epsilon = self.epsilon
        c.reward_loss_coef = self.reward_loss_coef
        c.gemm_bf16 = int(bool(self.gemm_bf16))
        c.seeds = int(self.seeds)
        c.single_seed_plan = int(bool(self.single_seed_plan))
        c.actor_gaussian = int(bool(self.actor_gaussian))
        c.actor_std_mult = float(self.actor_std_mult)
        c.actor_output_norm = int(bool(self.actor_output_norm))
        c.actor_layer_norm = int(bool(self.actor_layer_norm))
        if not 1 <= int(self.num_models) <= N.MAX_MODELS:
            raise ValueError(f"num_models must be in [1, {N.MAX_MODELS}]")
        c.num_models = int(self.num_models)
        c.model_max_grad_norm = float(self.model_max_grad_norm or 0.0)
        c.delta_clip_loss = float(self.delta_clip_loss or 0.0)
        c.reward_clip_loss = float(self.reward_clip_loss or 0.0)
        c.delta_clip_pred = float(self.delta_clip_pred or 0.0)
        c.act_per_layer = 1
        for n in range(3):
            a2 = two(nets[n][1])
            c.act_layers[n][0], c.act_layers[n][1] = N.ACT[a2[0]], N.ACT[a2[1]]
        c.gaussian_model = int(bool(self.gaussian_model))
        c.scale_model_loss = int(bool(self.scale_model_loss))
        c.separate_reward_nn = int(bool(self.separate_reward_nn))
        if self.separate_reward_nn:
            c.reward_hidden[0], c.reward_hidden[1] = [int(x) for x in two(self.reward_hidden)]
            a2 = two(nets[3][1])
            c.reward_act_layers[0], c.reward_act_layers[1] = N.ACT[a2[0]], N.ACT[a2[1]]
        return c


class Engine:
    """One SAC / SAC-EO learner on one GPU (one handle, one arena) -- or, with
    ``cfg.seeds = K``, K independent learners (the reference's ``--runs``) packed into one
    handle: ``step`` advances all of them in the same launches, and every per-seed method
    (weights, normalisers, RNG, replay, stats, snapshot) addresses the seed chosen with
    ``select_seed``."""

    NETS = ("actor", "q0", "q1", "t0", "t1", "m0", "m1")

    def __init__(self, cfg: EngineConfig, device: Optional[torch.device] = None, stream=None, dp=None,
                 dp_local=None):
        """dp = (unique_id bytes, nranks, rank): data-parallel mode (sacx_dp_init), the
        gradients of the local batch ``cfg.batch`` are summed over the ranks by RCCL.
        dp_local = (nranks, rank): the same protocol over handles of this process
        (sacx_dp_init_local; the ranks step together through Engine.dp_local_step)."""
        if not torch.cuda.is_available():
            raise RuntimeError("sac_eo.engine needs a ROCm GPU (no CPU fallback)")
        self.cfg = cfg
        self.lib = N.lib()
        self.device = torch.device(device or "cuda")
        h = ctypes.c_void_p()
        c = cfg.to_c()
        N.check(self.lib.sacx_create(ctypes.byref(c), ctypes.byref(h)), None, "sacx_create")
        self.h = h
        total = int(self.lib.sacx_arena_bytes(h))
        self.seeds = max(1, int(cfg.seeds))
        self.seed_stride = int(self.lib.sacx_seed_stride(h))
        self._raw = torch.zeros(total + 256, dtype=torch.uint8, device=self.device)
        off = (-self._raw.data_ptr()) % 256
        self.arena_all = self._raw[off: off + total]
        n = ctypes.c_int32()
        self.lib.sacx_layout(h, None, 0, ctypes.byref(n))
        segs = (N.Segment * n.value)()
        self.lib.sacx_layout(h, segs, n.value, ctypes.byref(n))
        self.segments: Dict[str, dict] = {}
        for s in segs:
            self.segments[s.name.decode()] = dict(offset=int(s.offset), rows=int(s.rows), cols=int(s.cols),
                                                  dtype=N.DTYPES[s.dtype], role=int(s.role), code=int(s.dtype))
        # per seed: its arena block and the named views into it
        self.nbytes = total if self.seeds == 1 else self.seed_stride
        self._arenas, self._views = [], []
        for k in range(self.seeds):
            a = self.arena_all[k * self.seed_stride: k * self.seed_stride + self.nbytes]
            views = {}
            for name, d in self.segments.items():
                nb = d["rows"] * d["cols"] * _ESZ[d["code"]]
                views[name] = a[d["offset"]: d["offset"] + nb].view(_TORCH_DT[d["code"]]).view(d["rows"], d["cols"])
            self._arenas.append(a)
            self._views.append(views)
        self.seed_index = 0
        self.arena = self._arenas[0]
        self._v: Dict[str, torch.Tensor] = self._views[0]
        self._bound = False
        with torch.cuda.device(self.device):
            self.stream = stream if stream is not None else torch.cuda.current_stream(self.device)
            if dp is not None:
                uid, nranks, rank = dp
                buf = ctypes.create_string_buffer(bytes(uid), len(uid))
                N.check(self.lib.sacx_dp_init(h, buf, int(nranks), int(rank)), h, "sacx_dp_init")
            if dp_local is not None:
                N.check(self.lib.sacx_dp_init_local(h, int(dp_local[0]), int(dp_local[1])), h, "sacx_dp_init_local")
        self.dp = dp
        self.dp_local = dp_local
        N.check(self.lib.sacx_bind(h, ctypes.c_void_p(self.arena_all.data_ptr()), total,
                                   ctypes.c_void_p(self.stream.cuda_stream)), h, "sacx_bind")
        self._bound = True
        for k in range(self.seeds):
            self.select_seed(k)
            self._init_state()
        self.select_seed(0)

    def select_seed(self, k: int):
        """Packed seeds: the seed the per-seed methods (and libsacx's per-seed calls) address."""
        k = int(k)
        N.check(self.lib.sacx_seed_select(self.h, k), self.h, "seed_select")
        self.seed_index = k
        self.arena = self._arenas[k]
        self._v = self._views[k]

    @property
    def v(self) -> Dict[str, torch.Tensor]:
        """The segment views of the selected seed.  Reading or writing them is an observation
        point: a deferred alpha branch runs and a speculative draw is undone first (sacx_settle;
        a no-op unless the drop-in loop's one-update steps left one)."""
        if getattr(self, "h", None) is not None and getattr(self, "_bound", False):
            N.check(self.lib.sacx_settle(self.h), self.h, "settle")
        return self._v

    @staticmethod
    def dp_local_step(engines: Sequence["Engine"], n: int = 1, num_timesteps: int = 0, ts_increment: int = 1):
        """n updates of every in-process data-parallel rank (sacx_dp_local_step); ``engines`` in
        rank order, all on one stream."""
        lib = N.lib()
        hs = (ctypes.c_void_p * len(engines))(*[e.h.value for e in engines])
        N.check(lib.sacx_dp_local_step(hs, len(engines), int(n), int(num_timesteps), int(ts_increment)),
                engines[0].h, "dp_local_step")

    @staticmethod
    def dp_unique_id() -> bytes:
        """A fresh RCCL unique id (sacx_dp_unique_id) for Engine(dp=(id, nranks, rank))."""
        lib = N.lib()
        buf = ctypes.create_string_buffer(256)
        n = lib.sacx_dp_unique_id(buf, 256)
        if n <= 0:
            raise RuntimeError("sacx_dp_unique_id failed")
        return buf.raw[:n]

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "h", None) is not None:
            self.sync()
            self.lib.sacx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _init_state(self):
        cfg = self.cfg
        v = self.v
        for k in ("norm.s_den", "norm.a_den", "norm.d_den", "norm.ret_den"):
            v[k].fill_(1.0)
        v["norm.r"][0, 1] = 1.0
        if "mnorm.r" in v:                       # the world models' normaliser set (SAC-EO)
            for k in ("mnorm.s_den", "mnorm.a_den", "mnorm.d_den"):
                v[k].fill_(1.0)
            v["mnorm.r"][0, 1] = 1.0
        v["alpha"].fill_(float(np.float32(np.log(cfg.init_temperature))))   # SAC_expert.py:106
        if cfg.actor_layer_norm:
            v["actor.ln"][0].fill_(1.0)                                      # gamma = 1, beta = 0
        self.rng_seed(0)

    # ------------------------------------------------------------------ weights
    def _layers(self, net: str) -> List[torch.Tensor]:
        """The Dense layers l0 .. l<D> of `net` (D hidden layers, then the output head)."""
        out = []
        while f"{net}.l{len(out)}" in self._v:
            out.append(self.v[f"{net}.l{len(out)}"])
        return out

    def set_net(self, net: str, weights: Sequence[np.ndarray]):
        """Keras get_weights() list [W0, b0, W1, b1, W2, b2] -> W_ext views; the actor with
        actor_layer_norm has [W0, b0, gamma, beta, W1, ...] (nn_utils.py:110-119)."""
        weights = list(weights)
        if net == "actor" and self.cfg.actor_layer_norm:
            gb = np.stack([np.asarray(weights[2], np.float32).reshape(-1), np.asarray(weights[3], np.float32).reshape(-1)])
            self.v["actor.ln"].copy_(torch.as_tensor(gb))
            weights = weights[:2] + weights[4:]
        for i, t in enumerate(self._layers(net)):
            W = torch.as_tensor(np.asarray(weights[2 * i], np.float32))
            b = torch.as_tensor(np.asarray(weights[2 * i + 1], np.float32)).reshape(1, -1)
            if tuple(W.shape) != (t.shape[0] - 1, t.shape[1]):
                raise ValueError(f"{net}.l{i}: expected {(t.shape[0] - 1, t.shape[1])}, got {tuple(W.shape)}")
            t.copy_(torch.cat([W, b], 0).to(self.device))

    def get_net(self, net: str) -> List[np.ndarray]:
        out = []
        for t in self._layers(net):
            a = t.detach().cpu().numpy()
            out += [a[:-1].copy(), a[-1].copy()]
        if net == "actor" and self.cfg.actor_layer_norm:
            gb = self.v["actor.ln"].cpu().numpy()
            out = out[:2] + [gb[0].copy(), gb[1].copy()] + out[2:]
        return out

    def set_logstd(self, logstd):
        self.v["actor.logstd"].copy_(torch.as_tensor(np.asarray(logstd, np.float32).reshape(1, -1)))

    def set_model_logstd(self, model: int, logstd):
        """GaussianModel's logstd variable [1, S] of world model `model` (continuous_models.py:24-25)."""
        self.v[f"m{int(model)}.logstd"].copy_(torch.as_tensor(np.asarray(logstd, np.float32).reshape(1, -1)))

    def get_model_logstd(self, model: int) -> np.ndarray:
        return self.v[f"m{int(model)}.logstd"].detach().cpu().numpy().copy()

    def set_alpha(self, alpha: float):
        self.v["alpha"].fill_(float(np.float32(alpha)))

    def alpha(self) -> float:
        return float(self.v["alpha"].item())

    def set_normalizers(self, s_mean, s_den, a_mean, a_den, d_mean=None, d_den=None,
                        r_mean=0.0, r_den=1.0, ret_den=1.0, which: str = "all"):
        """Values of RunningNormalizer.normalize: mean and max(std, 1e-8) (normalizer.py:26-41).

        which = "main": the set the actor and critics use (norm.*); "model": the world models'
        set (mnorm.*, SAC-EO; SAC_expert.py:139-144 gives the models their own normaliser with
        --only_model_normalizer); "all": both (the reference's shared normaliser)."""
        if which not in ("all", "main", "model"):
            raise ValueError("which must be 'all', 'main' or 'model'")
        v = self.v
        S, A = self.cfg.s_dim, self.cfg.a_dim
        put = lambda k, x, n: v[k].copy_(torch.as_tensor(np.array(x, np.float32).reshape(1, n)))
        pres = (["norm."] if which != "model" else []) + (["mnorm."] if which != "main" and "mnorm.r" in v else [])
        for p in pres:
            put(p + "s_mean", s_mean, S)
            put(p + "s_den", s_den, S)
            put(p + "a_mean", a_mean, A)
            put(p + "a_den", a_den, A)
            put(p + "d_mean", np.zeros(S) if d_mean is None else d_mean, S)
            put(p + "d_den", np.ones(S) if d_den is None else d_den, S)
            v[p + "r"].copy_(torch.tensor([[np.float32(r_mean), np.float32(r_den)]]))
        if which != "model":
            v["norm.ret_den"].fill_(float(np.float32(ret_den)))

    def reset_optimizers(self):
        self.v["adam_m"].zero_()
        self.v["adam_v"].zero_()
        self.v["ctl"][0, CTL["t_sac"]] = 0

    # ------------------------------------------------------------------ RNG (global NumPy stream)
    def rng_seed(self, seed: int):
        N.check(self.lib.sacx_rng_seed(self.h, ctypes.c_uint32(int(seed) & 0xFFFFFFFF)), self.h, "rng_seed")

    def rng_set_state(self, state):
        """Accepts np.random.get_state() / RandomState.get_state()."""
        _, key, pos, has_gauss, gauss = state[:5]
        key = np.ascontiguousarray(key, dtype=np.uint32)
        N.check(self.lib.sacx_rng_set_state(self.h, key.ctypes.data, int(pos), int(has_gauss), float(gauss)),
                self.h, "rng_set_state")

    def rng_get_state(self):
        key = np.zeros(624, np.uint32)
        pos, hg, g = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_double()
        N.check(self.lib.sacx_rng_get_state(self.h, key.ctypes.data, ctypes.byref(pos), ctypes.byref(hg),
                                            ctypes.byref(g)), self.h, "rng_get_state")
        return ("MT19937", key, pos.value, hg.value, g.value)

    # ------------------------------------------------------------------ data
    def _dev(self, x, shape) -> torch.Tensor:
        t = torch.as_tensor(x, dtype=torch.float32, device=self.device).reshape(shape).contiguous()
        return t

    @staticmethod
    def _is_host(x) -> bool:
        return not (torch.is_tensor(x) and x.is_cuda)

    @staticmethod
    def _host_f32(x, shape) -> np.ndarray:
        xv = x.detach().cpu().numpy() if torch.is_tensor(x) else x
        return np.ascontiguousarray(np.asarray(xv, dtype=np.float32).reshape(shape))

    def append(self, s, a, r, sp, d):
        """TrajectoryBuffer.add (buffers.py:41-71) into the device ring."""
        n = int(np.shape(r)[0]) if not torch.is_tensor(r) else int(r.shape[0])
        S, A = self.cfg.s_dim, self.cfg.a_dim
        if all(self._is_host(x) for x in (s, a, r, sp, d)):
            # env-loop transitions: one pinned staging copy inside the library
            hs = [self._host_f32(s, (n, S)), self._host_f32(a, (n, A)), self._host_f32(r, (n,)),
                  self._host_f32(sp, (n, S)), self._host_f32(d, (n,))]
            N.check(self.lib.sacx_buffer_append_host(self.h, *[x.ctypes.data for x in hs], n),
                    self.h, "buffer_append_host")
            return n
        ts = [self._dev(s, (n, S)), self._dev(a, (n, A)), self._dev(r, (n,)), self._dev(sp, (n, S)),
              self._dev(d, (n,))]
        N.check(self.lib.sacx_buffer_append(self.h, *[ctypes.c_void_p(t.data_ptr()) for t in ts], n),
                self.h, "buffer_append")
        self._keep = ts   # keep sources alive until the stream consumes them
        return n

    def set_expert(self, s_e, sp_e, epsilon: float):
        n = int(np.shape(s_e)[0])
        S = self.cfg.s_dim
        a, b = self._dev(s_e, (n, S)), self._dev(sp_e, (n, S))
        N.check(self.lib.sacx_expert_set(self.h, ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()),
                                         n, float(epsilon)), self.h, "expert_set")

    def push_perms(self, perms: np.ndarray):
        perms = np.ascontiguousarray(perms, dtype=np.int32)
        N.check(self.lib.sacx_perm_push(self.h, perms.ctypes.data, int(perms.shape[0])), self.h, "perm_push")

    def act(self, obs, deterministic: bool = True) -> "torch.Tensor":
        """SquashedGaussianActor.sample (continuous_actors.py:270-306) on the device:
        obs [n, S] or [S] -> actions [n, A] (a CUDA tensor; [A] for a single row).
        deterministic=False draws u from the device copy of the global NumPy stream."""
        single = np.ndim(obs) == 1 if not torch.is_tensor(obs) else obs.dim() == 1
        S, A = self.cfg.s_dim, self.cfg.a_dim
        o = self._dev(obs, (-1, S))
        n = int(o.shape[0])
        out = torch.empty((n, A), dtype=torch.float32, device=self.device)
        N.check(self.lib.sacx_actor_act(self.h, ctypes.c_void_p(o.data_ptr()), n, int(bool(deterministic)),
                                        ctypes.c_void_p(out.data_ptr())), self.h, "actor_act")
        self._keep_act = o
        return out[0] if single else out

    def act_host(self, obs, deterministic: bool = True) -> np.ndarray:
        """SquashedGaussianActor.sample for the env loop: host obs [n, S] or [S] -> host actions
        [n, A] ([A] for one row), as the reference hands env.step a NumPy action
        (sac_eo/algs/SAC_expert.py:585-605).  One pinned copy each way inside the library."""
        S, A = self.cfg.s_dim, self.cfg.a_dim
        single = np.ndim(obs) == 1 if not torch.is_tensor(obs) else obs.dim() == 1
        o = self._host_f32(obs, (-1, S))
        out = np.empty((o.shape[0], A), dtype=np.float32)
        N.check(self.lib.sacx_actor_act_host(self.h, o.ctypes.data, int(o.shape[0]), int(bool(deterministic)),
                                             out.ctypes.data), self.h, "actor_act_host")
        return out[0] if single else out

    def act_host_seeds(self, obs, deterministic: bool = True) -> np.ndarray:
        """act_host for EVERY seed of a packed handle in one launch chain: obs [seeds, n, S]
        (or [seeds, S]) -> actions [seeds, n, A] (or [seeds, A]); each seed draws from its own
        stream (sacx_actor_act_host_seeds).  Actors the one-launch rows kernel does not cover
        (layer norm, other than two hidden layers) act seed by seed."""
        S, A, K = self.cfg.s_dim, self.cfg.a_dim, self.seeds
        o = np.ascontiguousarray(np.asarray(obs, np.float32))
        one = o.ndim == 2
        o = o.reshape(K, -1, S)
        out = np.empty((K, o.shape[1], A), dtype=np.float32)
        if self.cfg.actor_layer_norm or len(self.cfg.hidden) != 2 or o.shape[1] > 16:
            sel = self.seed_index
            for k in range(K):
                self.select_seed(k)
                out[k] = self.act_host(o[k], deterministic)
            self.select_seed(sel)
            return out[:, 0] if one else out
        N.check(self.lib.sacx_actor_act_host_seeds(self.h, o.ctypes.data, int(o.shape[1]), int(bool(deterministic)),
                                                   out.ctypes.data), self.h, "actor_act_host_seeds")
        return out[:, 0] if one else out

    def append_host_seeds(self, s, a, r, sp, d) -> int:
        """append for EVERY seed of a packed handle (sacx_buffer_append_host_seeds): arrays
        [seeds, n, ...]; returns n."""
        S, A, K = self.cfg.s_dim, self.cfg.a_dim, self.seeds
        r = np.asarray(r, np.float32).reshape(K, -1)
        n = r.shape[1]
        hs = [self._host_f32(s, (K, n, S)), self._host_f32(a, (K, n, A)), np.ascontiguousarray(r),
              self._host_f32(sp, (K, n, S)), self._host_f32(d, (K, n))]
        N.check(self.lib.sacx_buffer_append_host_seeds(self.h, *[x.ctypes.data for x in hs], n),
                self.h, "buffer_append_host_seeds")
        return n

    def evaluate(self, s):
        """SquashedGaussianActor.evaluate (continuous_actors.py:327-379) on the device:
        s [n, S] -> (pi [n, A], neglogp [n]) CUDA tensors; draws normal(size=(n, A)) from the
        device copy of the global NumPy stream."""
        S, A = self.cfg.s_dim, self.cfg.a_dim
        x = self._dev(s, (-1, S))
        n = int(x.shape[0])
        pi = torch.empty((n, A), dtype=torch.float32, device=self.device)
        nlp = torch.empty((n,), dtype=torch.float32, device=self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        N.check(self.lib.sacx_actor_evaluate(self.h, p(x), n, p(pi), p(nlp)), self.h, "actor_evaluate")
        self._keep_eval = x
        return pi, nlp

    def critic_forward(self, net: str, s, a, value: bool = False):
        """QCritic._forward (value=False: [n, 1]) / value (value=True: [n], x ret sigma)
        (critics.py:84-103) of net q0 / q1 / t0 / t1 on the device."""
        S, A = self.cfg.s_dim, self.cfg.a_dim
        x, u = self._dev(s, (-1, S)), self._dev(a, (-1, A))
        n = int(x.shape[0])
        if int(u.shape[0]) != n:
            raise ValueError("s and a need the same number of rows")
        out = torch.empty((n,), dtype=torch.float32, device=self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        N.check(self.lib.sacx_critic_forward(self.h, ("q0", "q1", "t0", "t1").index(net), p(x), p(u), n,
                                             int(bool(value)), p(out)), self.h, "critic_forward")
        self._keep_q = (x, u)
        return out if value else out.reshape(n, 1)

    def model_forward(self, model: int, s, a, delta_clip: float = 0.0, reward_clip: float = 0.0,
                      stochastic: bool = False):
        """BaseWorldModel._forward + MSEModel.sample / step (base_world_model.py:65-87,
        continuous_models.py:225-254): -> (pred [n, S+1] = [delta_n | r_n] after the clips,
        sp [n, S] = s + denormalised delta, r [n] = denormalised reward).  stochastic on a
        gaussian_model engine: GaussianModel.sample(deterministic=False) / step (:36-70), sp from
        delta_n + exp(logstd) * u with u = normal(size=(n, S)) from the device stream."""
        S, A = self.cfg.s_dim, self.cfg.a_dim
        x, u = self._dev(s, (-1, S)), self._dev(a, (-1, A))
        n = int(x.shape[0])
        kw = dict(dtype=torch.float32, device=self.device)
        pred, sp, r = torch.empty((n, S + 1), **kw), torch.empty((n, S), **kw), torch.empty((n,), **kw)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        N.check(self.lib.sacx_model_sample(self.h, int(model), p(x), p(u), n, int(bool(stochastic)),
                                           float(delta_clip or 0.0), float(reward_clip or 0.0), p(pred), p(sp), p(r)),
                self.h, "model_forward")
        self._keep_m = (x, u)
        return pred, sp, r

    def model_loss(self, model: int, s, sp, a, r, delta_clip_loss: float = 0.0, reward_clip_loss: float = 0.0):
        """MSEModel.get_loss (continuous_models.py:280-302) / GaussianModel.get_loss (:101-131) on
        the device -> float."""
        S, A = self.cfg.s_dim, self.cfg.a_dim
        x, y, u = self._dev(s, (-1, S)), self._dev(sp, (-1, S)), self._dev(a, (-1, A))
        n = int(x.shape[0])
        rr = self._dev(r, (n,))
        out = torch.empty((1,), dtype=torch.float32, device=self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        N.check(self.lib.sacx_model_loss(self.h, int(model), p(x), p(y), p(u), p(rr), n, float(delta_clip_loss or 0.0),
                                         float(reward_clip_loss or 0.0), p(out)), self.h, "model_loss")
        return float(out.item())

    def rollout(self, model: int, s_init, horizon: int, deterministic: bool = False,
                delta_clip: float = 0.0, reward_clip: float = 0.0):
        """batch_simtrajectory_sampler (samplers.py:73-122) with world model `model` as the
        environment: s_init [n, S] -> (s, a, r, sp, d) of shapes [n,H,S], [n,H,A], [n,H],
        [n,H,S], [n,H] (CUDA tensors, d bool).  Draws the actor's noise from the device copy
        of the global NumPy stream, one normal(size=(n, A)) per step."""
        S, A = self.cfg.s_dim, self.cfg.a_dim
        src = self._dev(s_init, (-1, S))
        n, H = int(src.shape[0]), int(horizon)
        # staging + outputs kept per shape: stable pointers let libsacx replay its captured
        # rollout graph; the caller gets copies
        if not hasattr(self, "_roll_bufs"):
            self._roll_bufs = {}
        bufs = self._roll_bufs.get((n, H))
        if bufs is None:
            kw = dict(dtype=torch.float32, device=self.device)
            bufs = (torch.empty((n, S), **kw), torch.empty((n, H, S), **kw), torch.empty((n, H, A), **kw),
                    torch.empty((n, H), **kw), torch.empty((n, H, S), **kw),
                    torch.empty((n, H), dtype=torch.uint8, device=self.device))
            if len(self._roll_bufs) >= 4:
                self._roll_bufs.pop(next(iter(self._roll_bufs)))
            self._roll_bufs[(n, H)] = bufs
        s0, s, a, r, sp, d = bufs
        with torch.cuda.stream(self.stream):
            s0.copy_(src)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        N.check(self.lib.sacx_rollout(self.h, int(model), p(s0), n, H, int(bool(deterministic)),
                                      float(delta_clip or 0.0), float(reward_clip or 0.0),
                                      p(s), p(a), p(r), p(sp), p(d)), self.h, "rollout")
        with torch.cuda.stream(self.stream):
            return s.clone(), a.clone(), r.clone(), sp.clone(), d.bool()

    def expert_diag(self, s_e, a_e, sp_e, disc: bool = False, use_expert_actions: bool = False,
                    delta_clip: float = 0.0) -> dict:
        """Expert diagnostics on the device (sacx_expert_diag): the model MSE on expert data and
        on counterfactual actions (SAC_expert.py:579-608) or, with disc, _calc_disc (:427-460)."""
        S, A = self.cfg.s_dim, self.cfg.a_dim
        s0, sp0 = self._dev(s_e, (-1, S)), self._dev(sp_e, (-1, S))
        n = int(s0.shape[0])
        a0 = self._dev(a_e, (n, A)) if a_e is not None else None
        nmod = max(2, int(self.cfg.num_models or 2))       # every model (one model: twice)
        out = torch.zeros(3 + n if disc else 2 + 2 * nmod, dtype=torch.float32, device=self.device)
        flags = (N.DIAG_DISC if disc else 0) | (N.DIAG_EXPERT_ACTIONS if use_expert_actions else 0)
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        N.check(self.lib.sacx_expert_diag(self.h, p(s0), p(a0), p(sp0), n, flags, float(delta_clip or 0.0),
                                          p(out)), self.h, "expert_diag")
        o = out.cpu().numpy()
        if disc:
            return dict(s_disc_total=float(o[0]), max_disc=float(o[1]), median_disc=float(o[2]),
                        disc_ratio=o[3:].copy())
        return dict(mse_expert_data=float(o[0]), mse_counterfactual=float(o[1]),
                    mse_expert_data_per_model=o[2:2 + nmod].copy(),
                    mse_counterfactual_per_model=o[2 + nmod:2 + 2 * nmod].copy())

    # ------------------------------------------------------------------ snapshot (F4)
    def _state_ranges(self):
        """Merged byte ranges of every PARAM / TARGET / STATE segment (aliases fold in)."""
        iv = sorted((d["offset"], d["offset"] + int(self.v[n].numel() * self.v[n].element_size()))
                    for n, d in self.segments.items() if d["role"] != N.ROLE_WORK)
        out = []
        for a, b in iv:
            if out and a <= out[-1][1]:
                out[-1][1] = max(out[-1][1], b)
            else:
                out.append([a, b])
        return out

    def _layout_sig(self):
        return [[n, d["offset"], d["rows"], d["cols"], d["role"]] for n, d in sorted(self.segments.items())]

    def save_state(self, path: str):
        """Full-state snapshot (the reference keeps only final weights and logs,
        base_onpolicy_alg.py:351-374): weights, targets, alpha, Adam moments, normalisers,
        counters, the device RNG stream, replay ring, expert rows, permutation and stats
        rings -- every non-workspace segment, byte for byte, of every seed of the handle
        (packed seeds: one ``seed<k>`` directory each).  Resuming continues the run
        bit-identically (tests/test_gpu_engine.py)."""
        import json
        os.makedirs(path, exist_ok=True)
        self.sync()
        ranges = self._state_ranges()
        for k in range(self.seeds):
            d = path if self.seeds == 1 else os.path.join(path, f"seed{k}")
            os.makedirs(d, exist_ok=True)
            for a, b in ranges:
                np.save(os.path.join(d, f"range_{a}.npy"), self._arenas[k][a:b].cpu().numpy())
        with open(os.path.join(path, "meta.json"), "w") as fh:
            json.dump({"arena_bytes": self.nbytes, "ranges": ranges, "layout": self._layout_sig(),
                       "seeds": self.seeds, "format": "sacx-state-1"}, fh)

    def load_state(self, path: str):
        """Restores a save_state snapshot into this engine (same configuration, same seeds)."""
        import json
        with open(os.path.join(path, "meta.json")) as fh:
            meta = json.load(fh)
        if meta.get("format") != "sacx-state-1" or meta["arena_bytes"] != self.nbytes or \
                meta["layout"] != self._layout_sig() or int(meta.get("seeds", 1)) != self.seeds:
            raise ValueError("snapshot layout does not match this engine's configuration")
        self.sync()
        for k in range(self.seeds):
            d = path if self.seeds == 1 else os.path.join(path, f"seed{k}")
            for a, b in meta["ranges"]:
                src = np.load(os.path.join(d, f"range_{a}.npy"))
                if src.shape != (b - a,):
                    raise ValueError("snapshot range size mismatch")
                self._arenas[k][a:b].copy_(torch.from_numpy(src).to(self.device))
        self.sync()
        sel = self.seed_index
        for k in range(self.seeds):            # host mirrors of the counters (every seed steps together)
            self.select_seed(k)
            N.check(self.lib.sacx_resync(self.h), self.h, "resync")
        self.select_seed(sel)

    # ------------------------------------------------------------------ hot path
    def step(self, n: int = 1, num_timesteps: int = 0, ts_increment: int = 1, external: bool = False,
             eager: bool = False):
        flags = (N.STEP_EXTERNAL_RANDOMS if external else 0) | (N.STEP_EAGER if eager else 0)
        N.check(self.lib.sacx_sac_step(self.h, int(n), int(num_timesteps), int(ts_increment), flags),
                self.h, "sac_step")

    def prepare(self, n: int, external: bool = False) -> float:
        """Instantiates every hipGraph a following ``step(n)`` replays (sacx_prepare) without
        running an update; returns the host seconds it took (graph capture + instantiate)."""
        import time
        t0 = time.perf_counter()
        N.check(self.lib.sacx_prepare(self.h, int(n), N.STEP_EXTERNAL_RANDOMS if external else 0),
                self.h, "prepare")
        return time.perf_counter() - t0

    def model_fit(self, idx: np.ndarray, eager: bool = False):
        """``idx[n, num_models, model_batch]``: replay-logical rows of each model's minibatch per
        step (SAC_expert.py:519-543 -> _apply_model_grads)."""
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        nm = int(self.cfg.num_models or 2)
        if idx.ndim != 3 or idx.shape[1] != nm or idx.shape[2] != self.cfg.model_batch:
            raise ValueError(f"idx must be [n, {nm}, {self.cfg.model_batch}]")
        N.check(self.lib.sacx_model_fit(self.h, idx.ctypes.data, int(idx.shape[0]), N.STEP_EAGER if eager else 0),
                self.h, "model_fit")

    def model_stats(self, n_last: int) -> np.ndarray:
        """Summed model loss of the last n_last fitting steps, oldest first."""
        seq = self.ctl()["mfit_seq"]
        cap = self.cfg.stats_capacity
        st = self.v["mstats"].cpu().numpy()
        return st[[(seq - n_last + i) % cap for i in range(n_last)], 0]

    def reset_model_optimizer(self):
        """--reset_model_optimizer (SAC_expert.py:553-555): a fresh Keras Adam for the models, so
        no slot survives for ANY model trainable -- the model nets m<k>.l*, GaussianModel's
        m<k>.logstd and the separate reward nets r<k>.l* (build_layout keeps them one contiguous
        parameter range, the model optimiser's variable list)."""
        lo, hi = None, None
        for name, d in self.segments.items():
            if d["role"] != N.ROLE_PARAM or not (name[:1] in ("m", "r") and name[1:2].isdigit()):
                continue
            o = d["offset"] // 4
            lo = o if lo is None else min(lo, o)
            hi = max(hi or 0, o + d["rows"] * d["cols"])
        if lo is not None:
            self.v["adam_m"][0, lo:hi] = 0
            self.v["adam_v"][0, lo:hi] = 0
        self.v["ctl"][0, CTL["t_model"]] = 0

    def sync(self):
        N.check(self.lib.sacx_sync(self.h), self.h, "sync")

    def spec_hits(self) -> int:
        """One-update steps that ran on randoms drawn speculatively by the preceding act_host."""
        return int(self.lib.sacx_spec_hits(self.h))

    def seed_view(self, k: int) -> "SeedView":
        """The per-seed face of a packed handle for one learner's host code (SeedView)."""
        return SeedView(self, k)

    def ctl(self) -> Dict[str, int]:
        c = self.v["ctl"][0].cpu().numpy()
        return {k: int(c[i]) for k, i in CTL.items()}

    def stats(self, n_last: int) -> np.ndarray:
        """Last n_last rows of the per-update statistics ring, oldest first."""
        seq = self.ctl()["step_seq"]
        cap = self.cfg.stats_capacity
        st = self.v["stats"].cpu().numpy()
        idx = [(seq - n_last + i) % cap for i in range(n_last)]
        return st[idx]

    # ------------------------------------------------------------------ measurement
    def plan_info(self) -> List[dict]:
        n = ctypes.c_int32()
        self.lib.sacx_plan_info(self.h, None, 0, ctypes.byref(n))
        arr = (N.LaunchInfo * n.value)()
        N.check(self.lib.sacx_plan_info(self.h, arr, n.value, ctypes.byref(n)), self.h, "plan_info")
        return [dict(name=a.name.decode(), kernel=a.kernel.decode(), grid=a.grid, block=a.block,
                     flops=a.flops, bytes=a.bytes) for a in arr]

    def model_plan_info(self) -> List[dict]:
        """The launches of one world-model fitting step of the selected seed (after a model_fit)."""
        n = ctypes.c_int32()
        self.lib.sacx_model_plan_info(self.h, None, 0, ctypes.byref(n))
        arr = (N.LaunchInfo * n.value)()
        N.check(self.lib.sacx_model_plan_info(self.h, arr, n.value, ctypes.byref(n)), self.h, "model_plan_info")
        return [dict(name=a.name.decode(), kernel=a.kernel.decode(), grid=a.grid, block=a.block,
                     flops=a.flops, bytes=a.bytes) for a in arr]

    def time_graph(self, n_replays: int, skip_kernel: str = None) -> float:
        """ms per update of graph replays (HIP events); skip_kernel leaves a kernel family
        out (the state is meaningless afterwards)."""
        ms = ctypes.c_double(0.0)
        arg = skip_kernel.encode() if skip_kernel else None
        N.check(self.lib.sacx_time_graph(self.h, int(n_replays), arg, ctypes.byref(ms)), self.h, "time_graph")
        return ms.value / (n_replays * self.cfg.graph_steps)

    def time_kernels(self, kernel: str = "k_gemm", n_replays: int = 3):
        """(mean launch span us, summed span us per update, launches per graph) of `kernel`,
        from per-workgroup device timestamps inside a replay of the update graph."""
        a, u, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        N.check(self.lib.sacx_time_kernels(self.h, kernel.encode(), int(n_replays), ctypes.byref(a),
                                           ctypes.byref(u), ctypes.byref(n)), self.h, "time_kernels")
        return a.value, u.value, int(n.value)

    def profile(self, n_steps: int) -> np.ndarray:
        k = len(self.plan_info())
        out = (ctypes.c_double * k)()
        N.check(self.lib.sacx_profile(self.h, int(n_steps), out, k), self.h, "profile")
        return np.array(list(out)) / n_steps


class SeedView:
    """One seed of a packed Engine, seen as an Engine of its own by a learner's host code
    (an algorithm, its actor / critic / model objects): every per-seed method selects the
    seed first and ``v`` is the seed's views.  ``step`` / ``prepare`` advance every seed of
    the handle, so they belong to the lock-step driver (sac_eo.algs.lockstep), not to a view."""

    _SHARED = ("step", "prepare", "close", "time_graph", "time_kernels", "profile", "plan_info")

    def __init__(self, engine: Engine, k: int):
        self._eng, self._k = engine, int(k)

    @property
    def v(self):
        eng = self._eng
        if getattr(eng, "h", None) is not None and getattr(eng, "_bound", False):   # an observation point
            N.check(eng.lib.sacx_settle(eng.h), eng.h, "settle")
        return eng._views[self._k]

    @property
    def seed_index(self):
        return self._k

    def __getattr__(self, name):
        if name in SeedView._SHARED:
            raise AttributeError(f"SeedView.{name}: advances every seed of the packed handle (use the lock-step driver)")
        attr = getattr(self._eng, name)
        if callable(attr):
            def call(*a, **kw):
                self._eng.select_seed(self._k)
                return attr(*a, **kw)
            return call
        return attr
