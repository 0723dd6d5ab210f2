"""CPU oracle of the reference's TRAINING LOOPS: ``SAC_exp.train`` and ``SAC.train``.

TEST INFRASTRUCTURE ONLY (like ``sac_oracle.py``): nothing in the product path imports
this module; ``tests/`` drive it beside the device loop (``sac_eo.algs``) on the same
synthetic environment, initial weights and seeds, and compare every logged loss and the
global NumPy stream at every episode boundary.

It restates, on top of ``sac_oracle`` (one update, one model-fit step, the diagnostics):

* ``TrajectoryBuffer.add`` FIFO + ``get_offmodel_info`` sampling  sac_eo/common/buffers.py:41-71, :126-144
* ``RunningNormalizer.update`` / ``RunningNormalizers.update_rms``  sac_eo/common/normalizer.py:60-89, :149-159
  (``discounted_sum`` = scipy ``lfilter``, float64: buffer_utils.py:8-9)
* ``trajectory_sampler``                                           sac_eo/common/samplers.py:3-70
* ``SquashedGaussianActor.sample`` (behaviour policy)              sac_eo/actors/continuous_actors.py:270-306
* ``SAC_exp``: ``_collect_expert_data`` :156-207, ``_update`` :463-477 (the expert permutation of
  :301-303 from the algorithm's Generator), ``_update_models`` :480-621 (epoch shuffles from the
  global stream, model-fit steps, expert MSE diagnostics), ``_expert_preprocess`` :375-424,
  ``_collect_env_data`` :625-683, ``train`` :685-824 (the per-episode normaliser refresh :740-746,
  ``--only_model_normalizer`` :53-54 / :139-144 / :646-650)
* ``SAC.train`` :254-385 (G updates at one ``num_timesteps`` every ``real_step_mod`` steps).

The environment objects are passed in (they are the test's synthetic gym-style envs, whose
randomness is their own, never the global stream).  Every draw from the global stream
(``np.random``) goes through ``self.rs`` in the reference's order.

Parity status: as ``sac_oracle`` (float path parity-unpinned against TensorFlow; the
random streams are NumPy's own).
"""
from __future__ import annotations

import copy
from typing import List, Optional

import numpy as np

import sac_oracle as O


# ---------------------------------------------------------------------------- normalisers
class RunningNorm:
    """RunningNormalizer (normalizer.py:5-123)."""

    def __init__(self, dim):
        self.dim = dim
        self.t_last = 0
        if dim == 1:
            self.mean, self.var, self.std = 0.0, 0.0, 1.0
        else:
            self.mean = np.zeros(dim, np.float32)
            self.var = np.zeros(dim, np.float32)
            self.std = np.ones(dim, np.float32)

    def update(self, data):                              # :60-89
        std_norm = np.maximum(self.std, 1e-8)
        var_norm = np.square(std_norm)
        data_norm = data / std_norm
        t_batch = data_norm.shape[0]
        m_b = data_norm.mean(axis=0)
        s_b = np.sum(np.square(data_norm - m_b), axis=0)
        t = t_batch + self.t_last
        self.var = ((var_norm * s_b + self.var * np.maximum(1, self.t_last - 1)
                     + (t_batch / t) * self.t_last * var_norm * np.square(m_b - self.mean / std_norm))
                    / np.maximum(1, t - 1))
        self.mean = (t_batch * m_b * std_norm + self.t_last * self.mean) / t
        self.mean = self.mean.astype("float32")
        self.var = self.var.astype("float32")
        self.std = np.ones_like(self.var) if t == 1 else np.sqrt(self.var)
        self.t_last = t

    def instantiate(self, t, mean, var, ignore=None):    # :104-114
        self.t_last, self.mean, self.var = t, mean, var
        if t == 0:
            self.__init__(self.dim)
        elif t == 1:
            self.std = np.abs(self.mean)
        else:
            self.std = np.sqrt(self.var)

    def den(self):
        return np.maximum(self.std, 1e-8)


def discounted_sum(x, rate):
    """buffer_utils.discounted_sum: lfilter([1], [1, -rate], x[::-1])[::-1], float64."""
    x = np.asarray(x, np.float64)
    y = np.zeros_like(x)
    acc = 0.0
    for t in range(len(x) - 1, -1, -1):
        acc = x[t] + float(rate) * acc
        y[t] = acc
    return y


class RunningNorms:
    """RunningNormalizers (normalizer.py:126-190)."""

    def __init__(self, S, A, gamma, init_rms_stats=None):
        self.gamma = gamma
        self.s_rms, self.a_rms, self.r_rms = RunningNorm(S), RunningNorm(A), RunningNorm(1)
        self.delta_rms, self.ret_rms = RunningNorm(S), RunningNorm(1)
        if init_rms_stats is not None:
            for k in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms"):
                getattr(self, k).instantiate(**init_rms_stats[k])

    def update_rms(self, s, a, r, sp):                   # :149-159
        self.s_rms.update(s)
        self.a_rms.update(a)
        self.r_rms.update(r)
        self.delta_rms.update(sp - s)
        self.ret_rms.update(discounted_sum(r, self.gamma))

    def as_oracle(self, S, A) -> O.Normalizers:
        f = lambda x, n: np.broadcast_to(np.asarray(x, np.float32), (n,)).copy()
        sc = lambda x: np.float32(np.asarray(x).reshape(-1)[0])
        return O.Normalizers(f(self.s_rms.mean, S), f(self.s_rms.den(), S), f(self.a_rms.mean, A),
                             f(self.a_rms.den(), A), f(self.delta_rms.mean, S), f(self.delta_rms.den(), S),
                             sc(self.r_rms.mean), sc(self.r_rms.den()), sc(self.ret_rms.den()))


# ---------------------------------------------------------------------------- replay buffer
class Buffer:
    """TrajectoryBuffer (buffers.py:5-71): rows in add order, FIFO-truncated to buffer_size."""

    def __init__(self, S, A, buffer_size=None):
        self.size = buffer_size
        self.s = np.empty((0, S), np.float32)
        self.a = np.empty((0, A), np.float32)
        self.r = np.empty((0,), np.float32)
        self.sp = np.empty((0, S), np.float32)
        self.d = np.empty((0,))
        self.steps_total = 0

    def add(self, s, a, r, sp, d):
        self.s = np.concatenate((self.s, s))
        self.a = np.concatenate((self.a, a))
        self.r = np.concatenate((self.r, r))
        self.sp = np.concatenate((self.sp, sp))
        self.d = np.concatenate((self.d, d))
        if self.size and len(self.r) > self.size:
            self.s, self.a, self.r = self.s[-self.size:], self.a[-self.size:], self.r[-self.size:]
            self.sp, self.d = self.sp[-self.size:], self.d[-self.size:]
        self.steps_total += len(r)

    @property
    def current_size(self):
        return len(self.r)


# ---------------------------------------------------------------------------- the loop
class LoopOracle:
    """``SAC_exp`` (alg_type 'sac_imit') or ``SAC`` (alg_type 'sac') on the CPU.

    ``st``: the initial learner state (oracle SACState; its dtype is the arithmetic's);
    ``expert``: (params list, logstd) of the squashed expert actor (sac_imit);
    ``k``: the algorithm kwargs the device loop gets (the reference's flag names);
    ``rs_state``: the global NumPy stream at the algorithm's start (np.random.get_state());
    ``alg_seed``: the Generator seed of the expert permutations."""

    def __init__(self, alg_type, cfg: O.Config, st: O.SACState, env, env_expert, expert, k: dict,
                 rs_state, alg_seed, init_rms_stats=None, max_episode_steps=1000):
        self.alg_type = alg_type
        self.eo = alg_type == "sac_imit"
        self.cfg, self.st = cfg, st
        self.dt = st.alpha.dtype.type
        self.env, self.env_expert = env, env_expert
        self.expert = expert
        self.k = dict(k)
        self.S, self.A = cfg.S, cfg.A
        self.rs = np.random.RandomState()
        self.rs.set_state(rs_state)
        self.gen = np.random.default_rng(alg_seed)                 # base_onpolicy_alg.py:108-109
        g = k["gamma"]
        self.normalizer = RunningNorms(self.S, self.A, g, init_rms_stats)
        self.model_normalizer = RunningNorms(self.S, self.A, g, init_rms_stats)
        self.env_data = Buffer(self.S, self.A, k.get("env_buffer_size"))
        self.model_data = Buffer(self.S, self.A, int(k.get("model_buffer_size") or 1e5))
        self.new_traj: List[tuple] = []
        self.max_episode_steps = max_episode_steps
        self.update_stats: List[dict] = []      # one per update: q1, q2, p, alpha losses, epsilon
        self.episode_rng: List[tuple] = []      # the global stream at each episode start (before the hooks)
        self.diag: List[tuple] = []             # (MSE on expert data, on counterfactual actions) per episode
        self.model_losses: List[float] = []
        self.fit_last: List[float] = []          # the last model-fit step's loss of each episode's fit
        self.eps = float(k.get("epsilon", 1e-3))
        self.s_expert = self.sp_expert = self.a_expert = None
        # TrajectoryCorruptor (corruptor.py:3-30, base_onpolicy_alg.py:52): its own default_rng(0)
        self.s_noise_std = float(k.get("s_noise_std") or 0.0)
        self.s_noise_type = k.get("s_noise_type", "all")
        self.s_noise_rng = np.random.default_rng(0)

    # ---------------------------------------------------------------- pieces
    def _nrm(self):
        return self.normalizer.as_oracle(self.S, self.A)

    def _mnrm(self):
        m = self.model_normalizer if self.k.get("only_model_normalizer") else self.normalizer
        return m.as_oracle(self.S, self.A)

    def _sample(self, params, logstd, s, deterministic, nrm):
        """SquashedGaussianActor.sample on one row (float32 result, as TF returns it)."""
        dt = self.dt
        n = nrm.cast(dt)
        x = ((np.asarray(s, dt) - n.s_mean) / n.s_den)[None]
        out, _ = O.actor_forward(params, x, self.cfg)            # (Dense -> LayerNorm -> tanh with the norm)
        mu, lraw = O.split_head(out, np.asarray(logstd, dt), self.cfg)
        u = np.zeros_like(mu) if deterministic else O.f32_noise(self.rs.normal(size=mu.shape)).astype(dt)
        a, _ = O.head_sample(mu, lraw, u, self.cfg.act_limit, dt)
        return np.asarray(a[0], np.float32)

    def _trajectory(self, env, params, logstd, horizon, deterministic, nrm):
        """trajectory_sampler (samplers.py:3-70) with eval=True."""
        s_t, a_t, r_t, sp_t, d_t, J = [], [], [], [], [], 0.0
        s = env.reset()
        for t in range(horizon):
            a = self._sample(params, logstd, s, deterministic, nrm)
            s_true, r, d, _ = env.step(np.clip(a, -self.cfg.act_limit, self.cfg.act_limit))
            sp = s_true
            if self.s_noise_std > 0.0:                         # corrupt_samples (corruptor.py:23-30)
                u = self.s_noise_rng.normal(size=np.shape(s_true)).astype("float32")
                sp = s_true + u * np.sqrt(self.normalizer.delta_rms.var) * self.s_noise_std
            J += r
            if t == horizon - 1:
                d = False
            s_t.append(s); a_t.append(a); r_t.append(r); sp_t.append(sp); d_t.append(d)
            s = sp if self.s_noise_type == "all" else s_true   # samplers.py:35-43
            if d:
                break
        return (np.array(s_t, np.float32), np.array(a_t, np.float32), np.array(r_t, np.float32),
                np.array(sp_t, np.float32), np.array(d_t), J)

    def _add(self, s, a, r, sp, d):
        self.env_data.add(s, a, r, sp, d)
        if self.eo:
            self.model_data.add(s, a, r, sp, d)

    def _collect_expert_data(self):                             # SAC_expert.py:156-207
        n_exp = int(self.k.get("expert_buffer_size") or 20)
        horizon = int(self.k.get("env_horizon", 1000))
        ex_params, ex_logstd = self.expert
        ident = RunningNorms(self.S, self.A, self.k["gamma"]).as_oracle(self.S, self.A)
        buf = Buffer(self.S, self.A, n_exp)
        cur = 0
        while cur < n_exp:
            hz = min(n_exp - cur, horizon)
            s, a, r, sp, d, _ = self._trajectory(self.env_expert, ex_params, ex_logstd, hz, True, ident)
            buf.add(s, a, r, sp, d)
            cur = buf.steps_total
        self.s_expert, self.a_expert, self.sp_expert = buf.s, buf.a, buf.sp

    def _collect_env_data(self):                                # SAC_expert.py:625-683 (base :115-172)
        k = self.k
        batch = int(k.get("env_batch_size_init", 5000))
        horizon = int(k.get("env_horizon", 1000))
        start = self.env_data.steps_total
        cur = 0
        while cur < batch:
            hz = min(batch - cur, horizon)
            s, a, r, sp, d, _ = self._trajectory(self.env, self.st.actor, self.st.logstd, hz, False, self._nrm())
            if k.get("update_normalizers"):
                (self.model_normalizer if k.get("only_model_normalizer") else self.normalizer).update_rms(s, a, r, sp)
            self._add(s, a, r, sp, d)
            cur = self.env_data.steps_total - start
        return self.env_data.steps_total - start

    def _update(self, num_timesteps):
        """SAC_exp._update (:463-477) / SAC._update (SAC.py:236-250)."""
        cfg, st, rs = self.cfg, self.st, self.rs
        B, A = cfg.B, cfg.A
        idx = rs.randint(self.env_data.current_size, size=B)                 # buffers.py:136
        batch = (self.env_data.s[idx], self.env_data.a[idx], self.env_data.sp[idx], self.env_data.r[idx],
                 self.env_data.d[idx])
        n_t = O.f32_noise(rs.normal(size=(B, A)))
        n_pi = O.f32_noise(rs.normal(size=(B, A)))
        ex = None
        if self.eo:
            s_e, sp_e = self.s_e_cur, self.sp_e_cur
            if self.k.get("num_models", 2) == 1:
                ex = O.Expert(s_e, sp_e, None, None, O.f32_noise(rs.normal(size=(len(s_e), A))), None, self.eps)
            else:
                perm = np.arange(len(s_e))
                self.gen.shuffle(perm)                                       # :301-303
                sec = np.array_split(perm, int(self.k.get("num_models", 2)))    # sections 0 and 1 (:303-309)
                n1 = O.f32_noise(rs.normal(size=(len(sec[0]), A)))
                n2 = O.f32_noise(rs.normal(size=(len(sec[1]), A)))
                ex = O.Expert(s_e[sec[0]], sp_e[sec[0]], s_e[sec[1]], sp_e[sec[1]], n1, n2, self.eps)
        n_al = O.f32_noise(rs.normal(size=(B, A)))
        tui = int(self.k.get("target_update_int", 1))
        out = O.sac_update(st, cfg, self._nrm(), batch, n_t, n_pi, n_al, expert=ex,
                           do_polyak=(num_timesteps % tui == 0), mnrm=self._mnrm() if self.eo else None)
        out["epsilon"] = self.eps
        self.update_stats.append(out)

    def _update_models(self):                                   # SAC_expert.py:480-621
        k, rs = self.k, self.rs
        md = self.model_data
        n = md.current_size
        ms, ma, msp, mr = md.s, md.a, md.sp, md.r
        ratio = float(k.get("model_holdout_ratio") or 0.0)
        if ratio > 0.0:                                         # :492-513: fit the shuffled head
            n = int(md.current_size * (1 - ratio))
            rows = np.arange(md.current_size)
            rs.shuffle(rows)
            rows = rows[:n]
            ms, ma, msp, mr = ms[rows], ma[rows], msp[rows], mr[rows]
        mb = int(k.get("model_batch_size", 200))
        nm = int(k.get("num_models", 2))
        max_upd = k.get("model_max_updates", 1e5)
        mnrm = self._mnrm()
        num_updates = 0
        for ep in range(int(k.get("model_num_epochs", 10))):
            idx = np.arange(n)
            if k.get("model_batch_shuffle", True):
                idx = np.tile(idx, (nm, 1))
                for row in idx:
                    rs.shuffle(row)
            else:
                rs.shuffle(idx)
                idx = np.tile(idx, (nm, 1))
            sections = np.arange(0, n, mb)[1:]
            batches = np.array_split(idx, sections, axis=1)
            if n % mb != 0:
                batches = batches[:-1]
            for bi in batches:
                parts = [(ms[bi[j]], ma[bi[j]], msp[bi[j]], mr[bi[j]]) for j in range(nm)]
                self.model_losses.append(O.model_fit_step(
                    self.st, self.cfg, mnrm, parts, max_grad_norm=k.get("model_max_grad_norm"),
                    delta_clip_loss=k.get("delta_clip_loss") or 0.0, reward_clip_loss=k.get("reward_clip_loss") or 0.0))
                num_updates += 1
                if num_updates >= max_upd:
                    break
            if num_updates >= max_upd:
                break
        self.fit_last.append(self.model_losses[-1] if self.model_losses else float("nan"))
        if k.get("reset_model_optimizer"):
            self.st.opt_model = O.AdamState.zeros_like(self.st.opt_model.m)
        dc = k.get("delta_clip_pred") or 0.0
        m_data, m_cf, _, _ = O.expert_mse_diag(self.st, self.cfg, self._nrm(), self.s_expert, self.a_expert,
                                               self.sp_expert, rs=rs, use_expert_actions=bool(k.get("use_expert_actions")),
                                               delta_clip=dc, mnrm=mnrm)
        self.diag.append((m_data, m_cf))

    def _expert_preprocess(self):                               # :375-424 (default epsilon)
        self.eps = float(self.k.get("epsilon", 1e-3))
        s_e, sp_e = self.s_expert, self.sp_expert
        ebs = self.k.get("expert_batch_size")
        if ebs:
            pick = self.rs.randint(len(s_e), size=int(ebs))                  # buffers.py:116-122
            s_e, sp_e = s_e[pick], sp_e[pick]
        self.s_e_cur, self.sp_e_cur = s_e, sp_e

    def _episode_hook(self, episode):                           # :740-746 / SAC.py:309-315
        if self.k.get("update_normalizers") and episode > 0 and self.new_traj:
            s, a, r, sp = (np.concatenate([t[i] for t in self.new_traj]) for i in range(4))
            if self.k.get("only_model_normalizer"):
                self.model_normalizer.update_rms(s, a, r, sp)
            else:
                self.normalizer.update_rms(s, a, r, sp)
                self.model_normalizer.update_rms(s, a, r, sp)
        self.new_traj = []

    # ---------------------------------------------------------------- train
    def train(self, total_timesteps):
        k = self.k
        if self.eo:
            self._collect_expert_data()
        num_timesteps = self._collect_env_data()
        episode_step, episode, done = 0, 0, True
        G, mod = int(k.get("mbpo_G", 3)), int(k.get("real_step_mod", 3))
        obs = None
        while num_timesteps < total_timesteps:
            if done:
                self.episode_rng.append(copy.deepcopy(self.rs.get_state()))
                self._episode_hook(episode)
                obs = self.env.reset()
                done, episode_step = False, 0
                episode += 1
                if self.eo:
                    self._update_models()
                    self._expert_preprocess()
            a = self._sample(self.st.actor, self.st.logstd, obs, not k.get("random_act", False), self._nrm())
            if self.eo:
                self._update(num_timesteps)
            elif episode_step % mod == 0:
                for _ in range(G):
                    self._update(num_timesteps)
            next_obs, r, done, _ = self.env.step(np.clip(a, -self.cfg.act_limit, self.cfg.act_limit))
            d_nm = False if episode_step + 1 == self.max_episode_steps else done
            row = (obs[None].astype(np.float32), a[None], np.array([r], np.float32), next_obs[None].astype(np.float32),
                   np.array([float(d_nm)]))
            self._add(*row)
            if k.get("update_normalizers"):          # new_traj.add(np.array([r])): float64 rewards
                self.new_traj.append(row[:2] + (np.array([r], np.float64), row[3]))
            obs = next_obs
            episode_step += 1
            num_timesteps += 1
        self.episode_rng.append(copy.deepcopy(self.rs.get_state()))
        return self
