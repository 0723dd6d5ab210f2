"""Shared host side of SAC / SAC_exp: builds the device engine from the reference's
actor / critic / model objects and kwargs, owns the env loop bookkeeping.

The gradient step itself is ``Engine.step`` -> ``sacx_sac_step`` (HIP kernels, HBM
resident state).  The global NumPy stream is shared between host and device: the
device keeps the live copy (updates, stochastic actions); host code that draws from
``np.random`` (model-minibatch shuffles) runs inside ``self._host_rng()``, which
pulls the device state into NumPy and pushes it back afterwards, so draws happen in
the reference's order."""
import contextlib
import dataclasses
import time

import numpy as np

from ..common.corruptor import TrajectoryCorruptor
from ..common.logger import Logger
from ..common.normalizer import RunningNormalizers
from ..common.samplers import trajectory_sampler
from ..engine import Engine, EngineConfig


class SACBase:
    use_expert = False

    def __init__(self, idx, env, env_eval, actor, critics, q_targets, q_critics, models, alg_kwargs,
                 mf_update_kwargs):
        self.idx = idx
        self.env, self.env_eval = env, env_eval
        self.actor, self.critics, self.q_targets, self.q_critics = actor, critics, q_targets, q_critics
        self.models = models
        # packed runs (sac_eo.train --runs K, lock-step): (shared packed Engine or None, seed, K);
        # popped so it never reaches the logged params
        self._pack = alg_kwargs.pop("_pack", None)
        self.s_dim = int(np.prod(env.observation_space.shape))
        self.a_dim = int(np.prod(env.action_space.shape))
        self._setup(alg_kwargs)
        self.logger = Logger()
        self.rng = np.random.default_rng(self.alg_seed)            # base_onpolicy_alg.py:108-109
        self.normalizer = RunningNormalizers(self.s_dim, self.a_dim, self.gamma, self.init_rms_stats)
        # the world models' own normaliser (SAC.py:51-52, SAC_expert.py:53-54): used by the models
        # only with --only_model_normalizer (:139-144), updated by the collection and episode hooks
        self.model_normalizer = RunningNormalizers(self.s_dim, self.a_dim, self.gamma, self.init_rms_stats)
        self._new_traj = []                 # the episode's transitions (new_traj, SAC_expert.py:49-51)
        # --s_noise_std / --s_noise_type (base_onpolicy_alg.py:52): applied to every collected
        # trajectory (samplers.py:35-43), its variance read from self.normalizer (set in _set_rms)
        self.corruptor = TrajectoryCorruptor(self.s_noise_std, self.s_noise_type)
        self.corruptor.set_rms(self.normalizer)
        self.last_eval = 0
        self.engine = self._build_engine(alg_kwargs)
        self.steps_total = 0
        self.traj_total = 0
        self.checkpoint_name = f"{self.checkpoint_file}_{idx}"

    # ------------------------------------------------------------------ setup
    def _setup(self, k):
        self.gamma = k["gamma"]
        self.alg_seed = k.get("alg_seed")
        self.init_rms_stats = k.get("init_rms_stats")
        self.total_timesteps = int(k.get("total_timesteps", 0) or 0)
        self.env_buffer_size = k.get("env_buffer_size")
        self.model_buffer_size = int(k.get("model_buffer_size") or 1e5)
        self.checkpoint_file = k.get("checkpoint_file", "TEMPLOG")
        self.save_path = k.get("save_path", "./logs")
        self.save_freq, self.eval_freq = k.get("save_freq"), k.get("eval_freq")
        self.eval_num_traj = k.get("eval_num_traj", 5)
        self.env_horizon = k.get("env_horizon", 1000)
        self.env_batch_type = k.get("env_batch_type", "steps")
        self.env_batch_size_init = k.get("env_batch_size_init", 5000)
        self.env_batch_size = k.get("env_batch_size", 3000)
        self.init_temperature = k["init_temperature"]
        self.mbpo_lr, self.mbpo_actor_lr, self.mbpo_alpha_lr = k["q_crit_lr"], k["mbpo_actor_lr"], k["mbpo_alpha_lr"]
        self.G = k.get("mbpo_G", 3)
        self.sac_batch_size = k["sac_batch_size"]
        self.soft_tau = k["soft_tau"]
        self.target_update_int = k["target_update_int"]
        self.repeat_after_real_steps = k.get("real_step_mod", 3)
        self.random_act = k.get("random_act", False)
        self.update_normalizers = k.get("update_normalizers", False)
        self.only_model_normalizer = k.get("only_model_normalizer", False)
        self.model_lr = k.get("model_lr", 1e-3)
        self.model_num_epochs = k.get("model_num_epochs", 10)
        self.model_batch_size = k.get("model_batch_size", 200)
        self.model_max_updates = k.get("model_max_updates", 1e5)
        self.model_max_grad_norm = k.get("model_max_grad_norm")
        self.model_batch_shuffle = k.get("model_batch_shuffle", True)
        self.reset_model_optimizer = k.get("reset_model_optimizer", False)
        self.epsilon = k.get("epsilon", 1e-3)
        self.s_noise_std = float(k.get("s_noise_std") or 0.0)
        self.s_noise_type = k.get("s_noise_type", "all")
        self.model_holdout_ratio = float(k.get("model_holdout_ratio") or 0.0)
        self.expert_buffer_size = int(k.get("expert_buffer_size") or 20)
        self.expert_batch_size = k.get("expert_batch_size")
        self._max_episode_steps = 1000

    def _capacity(self):
        if self.env_buffer_size:
            return int(self.env_buffer_size)
        # the reference's buffer is unbounded when env_buffer_size is None
        return max(1, self.total_timesteps + self.env_batch_size_init + self.env_horizon)

    def _build_engine(self, k):
        cfg = self._engine_config(k)
        if self._pack is None:
            eng = Engine(cfg)
        else:                                  # one seed of a packed handle (sac_eo.algs.lockstep)
            shared, seed, n = self._pack
            # every seed on the one-seed plan: each run bit-identical to its serial run
            pcfg = dataclasses.replace(cfg, seeds=int(n), single_seed_plan=True)
            if shared is None:
                shared = Engine(pcfg)
            elif shared.cfg != pcfg:
                raise ValueError("packed runs need one configuration (shapes and hyper-parameters)")
            eng = shared.seed_view(seed)
        self.actor._bind(eng, "actor")
        for i, q in enumerate(self.q_critics):
            q._bind(eng, f"q{i}")
        for i, t in enumerate(self.q_targets):
            t._bind(eng, f"t{i}")
        if self.use_expert:
            for i, m in enumerate(self.models):
                m._bind(eng, f"m{i}")
        self._push_normalizers(eng)
        eng.rng_set_state(np.random.get_state())       # adopt the global stream
        return eng

    def _engine_config(self, k):
        if not getattr(self.actor, "squash", False):
            raise ValueError("SAC trains the squashed Gaussian actor (--actor_squash)")
        # --actor_layers / --critic_layers / --model_layers / --reward_layers of any length up to 4
        # (create_nn, nn_utils.py:100-138); other than two, the engine runs its generic plans
        hidden, chidden = self.actor.layers, self.q_critics[0].layers
        cfg = EngineConfig(
            s_dim=self.s_dim, a_dim=self.a_dim, hidden=tuple(hidden), activation=self.actor.activation,
            critic_hidden=tuple(chidden),
            batch=int(self.sac_batch_size), buffer_capacity=self._capacity(), per_state_std=self.actor.per_state_std,
            use_expert=self.use_expert, expert_capacity=self.expert_buffer_size,
            expert_batch=int(self.expert_batch_size or self.expert_buffer_size),
            model_hidden=tuple(self.models[0].layers) if self.use_expert else (512, 512),
            model_activation=self.models[0].activation if self.use_expert else "relu",
            actor_activations=self.actor.activations, critic_activations=self.q_critics[0].activations,
            model_activations=self.models[0].activations if self.use_expert else None,
            model_batch=int(self.model_batch_size), target_update_int=int(self.target_update_int),
            graph_steps=1, gamma=self.gamma, tau=self.soft_tau, lr_q=self.mbpo_lr, lr_pi=self.mbpo_actor_lr,
            lr_alpha=self.mbpo_alpha_lr, lr_model=self.model_lr, init_temperature=self.init_temperature,
            target_entropy=-float(self.a_dim), act_limit=float(np.max(self.actor.act_limit)),
            epsilon=float(self.epsilon),
            reward_loss_coef=self.models[0].reward_loss_coef if self.use_expert else 1.0,
            num_models=len(self.models) if self.use_expert else 2, actor_layer_norm=self.actor.layer_norm,
            model_max_grad_norm=float(self.model_max_grad_norm or 0.0),
            delta_clip_loss=float(self.models[0].delta_clip_loss or 0.0) if self.use_expert else 0.0,
            reward_clip_loss=float(self.models[0].reward_clip_loss or 0.0) if self.use_expert else 0.0,
            delta_clip_pred=float(self.models[0].delta_clip_pred or 0.0) if self.use_expert else 0.0)
        if self.use_expert:
            m = self.models[0]
            cfg.gaussian_model = bool(getattr(m, "gaussian", False))
            cfg.scale_model_loss = bool(m.scale_model_loss) and cfg.gaussian_model   # GaussianModel only (:122-127)
            cfg.separate_reward_nn = bool(m.separate_reward_nn)
            if cfg.separate_reward_nn:
                cfg.reward_hidden = tuple(m.reward_layers)
                cfg.reward_activations = tuple(m.reward_activations)
        return cfg

    # ------------------------------------------------------------------ RNG sharing
    @contextlib.contextmanager
    def _host_rng(self):
        np.random.set_state(self.engine.rng_get_state())
        try:
            yield
        finally:
            self.engine.rng_set_state(np.random.get_state())

    # ------------------------------------------------------------------ normalisers
    def _models_normalizer(self):
        """The normaliser the world models use (SAC_expert.py:139-144)."""
        return self.model_normalizer if self.only_model_normalizer else self.normalizer

    def _push_normalizers(self, eng=None):
        """The device copies: norm.* from the shared normaliser, mnorm.* from the models' one."""
        eng = eng if eng is not None else self.engine
        self.normalizer.push_to(eng, which="main")
        if self.use_expert:
            self._models_normalizer().push_to(eng, which="model")

    def _set_rms(self):
        for obj in [self.actor] + list(self.q_critics) + list(self.q_targets):
            obj.set_rms(self.normalizer)
        self.corruptor.set_rms(self.normalizer)          # base_onpolicy_alg.py:204
        for m in (self.models or []) if self.use_expert else []:
            m.set_rms(self._models_normalizer())
        self._push_normalizers()

    def _update_rms_traj(self, s, a, r, sp, episode_hook=False):
        """RunningNormalizers.update_rms on a trajectory: _collect_env_data (SAC_expert.py:646-650)
        updates one normaliser; the per-episode hook (:740-746, SAC.py:309-315) updates the
        shared normaliser and the models' (or only the models' with --only_model_normalizer)."""
        if self.only_model_normalizer:
            self.model_normalizer.update_rms(s, a, r, sp)
        else:
            self.normalizer.update_rms(s, a, r, sp)
            if episode_hook:
                self.model_normalizer.update_rms(s, a, r, sp)
        self._push_normalizers()

    def _episode_normalizer_update(self, episode):
        """At an episode boundary (done, episode > 0): the episode's transitions into the
        normalisers (new_traj.get_model_info(): s, a, r, sp in add order), then new_traj.reset()."""
        if self.update_normalizers and episode > 0 and self._new_traj:
            s, a, r, sp = (np.concatenate([t[i] for t in self._new_traj]) for i in range(4))
            self._update_rms_traj(s, a, r, sp, episode_hook=True)
        self._new_traj = []

    # ------------------------------------------------------------------ data

    def _add(self, s, a, r, sp, d, track_episode=False):
        rows = self._add_rows(s, a, r, sp, d)
        self._added(rows, self.engine.append(*rows[:5]), track_episode)

    @staticmethod
    def _add_rows(s, a, r, sp, d):
        return tuple(np.asarray(x, np.float32) for x in (s, a, r, sp, d)) + (np.asarray(r, np.float64),)

    def _added(self, rows, n, track_episode):
        self.steps_total += n
        if track_episode and self.update_normalizers:
            # new_traj.add (SAC_expert.py:799-801): np.array([r]) keeps the env's float64 reward,
            # which r_rms.update then merges in float64
            s, a, _, sp, _, r64 = rows
            self._new_traj.append((s, a, r64, sp))

    # ------------------------------------------------------------------ the env loop as requests
    # The train loops are generators that yield the three requests of a timestep -- ("act", obs,
    # deterministic), ("update", n, num_timesteps, ts_increment), ("add", rows) -- and do everything
    # else (episode hooks, model fits, logging, checkpoints) themselves.  train() serves them one by
    # one on this learner's engine; sac_eo.algs.lockstep serves K learners of one packed handle with
    # one launch chain per request (the reference's --runs, sac_eo/train.py:118-152).
    def train(self, total_timesteps, params):
        return self._drive(self._train_loop(total_timesteps, params))

    def _drive(self, loop):
        """Serves a request generator on this learner's engine; returns its value."""
        try:
            req = next(loop)
            while True:
                req = loop.send(self._serve(req))
        except StopIteration as stop:
            return stop.value

    def _serve(self, req):
        kind = req[0]
        if kind == "act":
            return self.engine.act_host(np.asarray(req[1], np.float32), deterministic=req[2])
        if kind == "update":
            self.engine.step(req[1], num_timesteps=req[2], ts_increment=req[3])
            return None
        if kind == "add":
            return self.engine.append(*req[1][:5])
        raise ValueError(kind)

    def _pre_update(self, n):
        """Host work ahead of n updates (SAC_exp: the expert permutations)."""

    def _post_update(self, n):
        """Host bookkeeping after n updates (SAC_exp: the per-update log)."""

    def _collect_env_data(self, num_timesteps, update_normalizers=True, only_model_normalizer=False):
        """SAC_expert.py:625-684: rollouts of the stochastic actor until the batch is full."""
        return self._drive(self._collect_env_data_steps(num_timesteps, update_normalizers, only_model_normalizer))

    def _trajectory_steps(self, env, horizon, deterministic=False):
        """trajectory_sampler(env, actor, horizon, eval=True, corruptor=self.corruptor)
        (samplers.py:3-70) with the actor's sample() as an "act" request per step."""
        s_t, a_t, r_t, sp_t, d_t, J = [], [], [], [], [], 0.0
        s = env.reset()
        for t in range(horizon):
            a = yield ("act", s, deterministic)
            s_true, r, d, _ = env.step(self.actor.clip(a))
            sp, s_next = self.corruptor.store_and_next(s_true)
            J += r
            if t == horizon - 1:
                d = False
            s_t.append(s); a_t.append(a); r_t.append(r); sp_t.append(sp); d_t.append(d)
            s = s_next
            if d:
                break
        return (np.array(s_t, np.float32), np.array(a_t, np.float32), np.array(r_t, np.float32),
                np.array(sp_t, np.float32), np.array(d_t), J)

    def _collect_env_data_steps(self, num_timesteps, update_normalizers=True, only_model_normalizer=False):
        t0 = time.time()
        batch_size = self.env_batch_size_init if num_timesteps == 0 else self.env_batch_size
        steps_start, J_all, cur = self.steps_total, [], 0
        while cur < batch_size:
            horizon = min(batch_size - cur, self.env_horizon) if self.env_batch_type == "steps" else self.env_horizon
            s, a, r, sp, d, J = yield from self._trajectory_steps(self.env, horizon)
            if update_normalizers:
                if only_model_normalizer:
                    self.model_normalizer.update_rms(s, a, r, sp)
                else:
                    self.normalizer.update_rms(s, a, r, sp)
                self._push_normalizers()
            self._add(s, a, r, sp, d)
            self.traj_total += 1
            if horizon == self.env_horizon:
                J_all.append(J)
            cur = self.steps_total - steps_start if self.env_batch_type == "steps" else cur + 1
        steps_new = self.steps_total - steps_start
        self.current_reward = float(np.mean(J_all)) if J_all else float("nan")
        self.logger.log_train({"J_tot": self.current_reward, "steps": steps_new, "traj": 1,
                               "time_env_data": time.time() - t0})
        return steps_new

    def _evaluate(self, num_timesteps):
        """base_onpolicy_alg.py:174-197: eval_num_traj deterministic rollouts in env_eval."""
        t0 = time.time()
        J = []
        for _ in range(self.eval_num_traj):
            *_, Jt = trajectory_sampler(self.env_eval, self.actor, self.env_horizon, eval=True, deterministic=True)
            J.append(Jt)
        self.logger.log_train({"J_tot_eval": float(np.mean(J)), "steps_eval": num_timesteps - self.last_eval,
                               "time_eval": time.time() - t0})
        self.last_eval = num_timesteps

    def _eval_points(self, total_timesteps):
        """SAC_expert.py:707-714: None without --eval_freq."""
        if self.eval_freq is None:
            return None
        return np.concatenate((np.arange(0, total_timesteps, self.eval_freq)[1:], [total_timesteps]))

    # ------------------------------------------------------------------ update
    def _update(self, num_timesteps, expert_reg=None, ts_increment=1):
        """One gradient step (SAC_expert.py:463-477 / SAC.py:236-250) on this learner's engine."""
        self._pre_update(1)
        self.engine.step(1, num_timesteps=num_timesteps, ts_increment=ts_increment)
        self._post_update(1)

    def _dump_stats(self):
        """The reference's final dict (base_onpolicy_alg.py:351-364, mbrl_onpolicy_alg.py:321-329):
        actor weights, the (V) critics' weights, rms stats, model / reward weights -- plus the
        Q critics, targets and alpha the reference never saves."""
        final = {"actor_weights": self.actor.get_weights(),
                 "critic_weights": [c.get_weights() for c in self.critics],
                 "rms_stats": self.normalizer.get_rms_stats(),
                 "q_critic_weights": [q.get_weights() for q in self.q_critics],
                 "q_target_weights": [t.get_weights() for t in self.q_targets],
                 "alpha": self.engine.alpha()}
        if self.use_expert:
            final["model_weights"] = [m.get_weights() for m in self.models]
            final["reward_weights"] = [m.get_reward_weights() for m in self.models]   # mbrl_onpolicy_alg.py:326-327
        return final

    def _dump_and_save(self, params):
        """base_onpolicy_alg.py:366-374: params + final into the logger, appended to the run's
        checkpoint file, logger reset."""
        self.logger.log_params(params)
        self.logger.log_final(self._dump_stats())
        self.logger.dump_and_save(self.save_path, self.checkpoint_name)
        self.logger.reset()

    def _checkpoints(self, total_timesteps):
        if self.save_freq is None:
            return np.array([total_timesteps])
        return np.concatenate((np.arange(0, total_timesteps, self.save_freq)[1:], [total_timesteps]))
