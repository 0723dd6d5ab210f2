"""SAC_exp — SAC-EO (reference ``sac_eo/algs/SAC_expert.py``).

* ``_update`` (``:463-477``): one device gradient step; the expert term's
  ``self.rng.shuffle`` permutation (``:301-303``) is drawn here on the host from the
  same Generator and handed to the device (``sacx_perm_push``).
* ``_update_models`` (``:480-552``): the epoch / minibatch loop with the reference's
  ``np.random.shuffle`` draws (under ``_host_rng``), each minibatch pair fitted on the
  device (``sacx_model_fit``).  The expert-MSE diagnostics of ``:579-608`` and the
  model discrepancy of ``_calc_disc`` (``:427-460``) run on the device
  (``sacx_expert_diag``), drawing the reference's counterfactual actions from the
  device stream; the adaptive epsilon of ``_expert_preprocess`` (``:383-418``) is the
  reference's scalar arithmetic on those results.
* ``_collect_expert_data`` (``:156-208``): rollouts of the expert actor (its own
  inference-only engine) in ``env_expert``.
"""
import time

import numpy as np

from ..common.normalizer import RunningNormalizers
from ..common.samplers import trajectory_sampler
from ..engine import Engine, EngineConfig
from .base import SACBase


class SAC_exp(SACBase):
    use_expert = True

    def __init__(self, idx, env, env_eval, env_expert, actor, expert, init_expert_rms_stats, v_critic, q_targets,
                 q_critics, models, alg_kwargs, mf_update_kwargs):
        if not 1 <= len(models) <= 8:
            # every model is fitted (mbrl_onpolicy_alg.py:305-319); the expert term uses the first two
            # array_split sections and models 0 / 1 (SAC_expert.py:297-336)
            raise ValueError("SAC-EO runs 1 to 8 world models on the device")
        super().__init__(idx, env, env_eval, actor, v_critic, q_targets, q_critics, models, alg_kwargs,
                         mf_update_kwargs)
        if self.env_buffer_size:
            # the world models fit the last model_buffer_size rows of the replay ring; a smaller ring
            # would have dropped some of them by the time the run holds that many rows.  Collection
            # overshoots total_timesteps by up to one trajectory, so the bound is the one an unbounded
            # ring is sized by (base.py _capacity)
            most = self.total_timesteps + self.env_batch_size_init + self.env_horizon
            if int(self.env_buffer_size) < min(self.model_buffer_size, most):
                raise NotImplementedError(
                    f"--model_buffer_size {self.model_buffer_size} larger than --env_buffer_size "
                    f"{int(self.env_buffer_size)} for a run of {most} steps (the model data is the replay ring's tail)")
        self.env_expert = env_expert
        self.expert = expert
        self.expert_normalizer = RunningNormalizers(self.s_dim, self.a_dim, self.gamma, init_expert_rms_stats)
        self.use_expert_actions = alg_kwargs.get("use_expert_actions", False)
        self.scale_epsilon_by_true_MSE = alg_kwargs.get("scale_epsilon_by_true_MSE", False)
        self.scale_max_disc = alg_kwargs.get("scale_max_disc", False)
        self.scale_median_disc = alg_kwargs.get("scale_median_disc", False)
        self.scale_total_disc = alg_kwargs.get("scale_total_disc", False)
        self.min_mult = alg_kwargs.get("min_mult", False)
        self.exp_mult = alg_kwargs.get("exp_mult", False)
        self.mult_coeff = alg_kwargs.get("mult_coeff", 1.0)
        self.delta_clip_pred = (mf_update_kwargs or {}).get("delta_clip_pred") or alg_kwargs.get("delta_clip_pred")
        self.model_MSE_on_expert_data = []
        self._eps_log, self._eps_cur = [], float(self.epsilon)
        self._perm_queue = None        # expert permutations drawn ahead and pushed, not yet used
        self.model_MSE_on_expert_counterfactual_action = []
        self._expert_engine = None
        self.s_expert = self.a_expert = self.sp_expert = None

    # ------------------------------------------------------------------ expert
    def _expert_engine_for(self):
        if self._expert_engine is None:
            ex = self.expert
            # an imported expert is the reference's plain GaussianActor (train.py:65-86)
            cfg = EngineConfig(s_dim=self.s_dim, a_dim=self.a_dim, hidden=tuple(ex.layers), activation=ex.activation,
                               batch=1, buffer_capacity=1, per_state_std=ex.per_state_std, graph_steps=1,
                               act_limit=float(np.max(ex.act_limit)), actor_gaussian=not ex.squash,
                               actor_std_mult=float(ex.std_mult), actor_output_norm=ex.output_norm,
                               actor_layer_norm=ex.layer_norm, actor_activations=ex.activations)
            self._expert_engine = Engine(cfg)
            ex._bind(self._expert_engine, "actor")
            self.expert_normalizer.push_to(self._expert_engine)
        return self._expert_engine

    def _set_rms(self):
        super()._set_rms()
        self.expert.set_rms(self.expert_normalizer)

    def _collect_expert_data(self):
        t0 = time.time()
        self._expert_engine_for()
        s_all, a_all, sp_all, J_all, cur = [], [], [], [], 0
        while cur < self.expert_buffer_size:
            horizon = min(self.expert_buffer_size - cur, self.env_horizon)
            s, a, r, sp, d, J = trajectory_sampler(self.env_expert, self.expert, horizon, eval=True,
                                                   deterministic=True, corruptor=self.corruptor)
            s_all.append(s)
            a_all.append(a)
            sp_all.append(sp)
            cur += len(r)
            if horizon == self.env_horizon:
                J_all.append(J)
        self.s_expert = np.concatenate(s_all)[-self.expert_buffer_size:]
        self.a_expert = np.concatenate(a_all)[-self.expert_buffer_size:]
        self.sp_expert = np.concatenate(sp_all)[-self.expert_buffer_size:]
        self.expert_reward = float(np.mean(J_all)) if J_all else float("nan")
        self.logger.log_train({"expert_J_tot": self.expert_reward, "expert_steps": cur,
                               "expert_time": time.time() - t0})

    def _diag(self, disc: bool):
        return self.engine.expert_diag(self.s_expert, self.a_expert, self.sp_expert, disc=disc,
                                       use_expert_actions=self.use_expert_actions,
                                       delta_clip=self.delta_clip_pred or 0.0)

    def _expert_preprocess(self):
        """:375-424: epsilon_coef (adaptive variants on the device diagnostics), then the
        expert rows (a random batch of them with expert_batch_size)."""
        eps = self.epsilon
        if self.scale_epsilon_by_true_MSE and self.model_MSE_on_expert_counterfactual_action:
            eps = 1.0 / (self.epsilon * self.model_MSE_on_expert_counterfactual_action[-1] + 1.0)
            cur = self.current_reward
            if cur > 0:
                if self.min_mult:
                    eps = eps * (-min(self.mult_coeff * (cur / self.expert_reward) - 1, 0))
                if self.exp_mult:
                    eps = eps * np.exp(-self.mult_coeff * cur / self.expert_reward)
        elif self.scale_max_disc or self.scale_median_disc or self.scale_total_disc:
            d = self._diag(disc=True)
            x = d["max_disc"] if self.scale_max_disc else (d["median_disc"] if self.scale_median_disc
                                                           else d["s_disc_total"])
            eps = 1.0 / (self.epsilon * x + 1.0)
        s_e, sp_e = self.s_expert, self.sp_expert
        if self.expert_batch_size:
            with self._host_rng():               # get_model_info(batch_size), buffers.py:116-122
                pick = np.random.randint(len(s_e), size=int(self.expert_batch_size))
            s_e, sp_e = s_e[pick], sp_e[pick]
        self.engine.set_expert(s_e, sp_e, eps)
        self._eps_cur = float(eps)
        return (s_e, None, sp_e, eps, self.use_expert_actions)

    def _flush_update_logs(self):
        """The per-update log of _update_actor_and_alpha (SAC_expert.py:351-356): alpha_loss,
        p_loss, epsilon -- read back from the device statistics ring (q1 / q2 losses too,
        which the reference computes but does not log)."""
        n = len(self._eps_log)
        if n == 0:
            return
        st = self.engine.stats(n)
        for i in range(n):
            self.logger.log_train({"alpha_loss": np.float32(st[i, 3]), "p_loss": np.float32(st[i, 2]),
                                   "epsilon": self._eps_log[i], "q1_loss": np.float32(st[i, 0]),
                                   "q2_loss": np.float32(st[i, 1])})
        self._eps_log = []

    def _dump_and_save(self, params):
        self._flush_update_logs()
        super()._dump_and_save(params)

    # ------------------------------------------------------------------ update
    _PERM_AHEAD = 256

    def _pre_update(self, n):
        """The self.rng.shuffle permutation of each update (SAC_expert.py:301-303; one model: no
        shuffle).  self.rng is used for nothing else, so they are drawn ahead in the same order,
        _PERM_AHEAD at a time, and pushed into the device ring in one copy."""
        if len(self.models) < 2:
            return
        q = self._perm_queue
        have = 0 if q is None else q.shape[0]
        if have < n:
            m = max(n - have, min(self._PERM_AHEAD, self.engine.cfg.perm_capacity - have))
            new = np.tile(np.arange(self.engine.cfg.expert_batch), (m, 1))
            for row in new:
                self.rng.shuffle(row)
            q = new if q is None else np.concatenate([q, new])
            self.engine.push_perms(q)           # the ring slots of the next len(q) updates
        self._perm_queue = q[n:]

    def _post_update(self, n):
        for _ in range(n):
            self._eps_log.append(self._eps_cur)
            if len(self._eps_log) >= self.engine.cfg.stats_capacity:
                self._flush_update_logs()        # the device ring is full (epsilon is constant within an episode)

    def _update_models(self):
        """:480-552: optional holdout split (a global-stream shuffle of the model rows, the fit on
        the first int(n·(1−ratio)) of them, :492-513), then the epoch / minibatch index draws
        (:519-550), fitted on the device."""
        t0 = time.time()
        n_model = min(self.steps_total, self.model_buffer_size)   # model_data = last rows of the env data
        if n_model > int(self.engine.ctl()["cur_size"]):
            # model_data would hold rows the (smaller) replay ring already dropped (checked at setup)
            raise NotImplementedError("--model_buffer_size larger than --env_buffer_size")
        if n_model == 0:
            return
        base = int(self.engine.ctl()["cur_size"]) - n_model
        # model_ent: mean of model.entropy over the model data, taken BEFORE the epoch loop
        # (SAC_expert.py:486-490, logged at :615) -- a constant per row (GaussianModel: 0.5 sum(2 logstd
        # + log 2 pi + 1) of the pre-fit logstd, continuous_models.py:162-166; MSEModel 0)
        ent = np.array([np.float32(m.entropy(self.s_expert[:1], None)[0]) for m in self.models], np.float32)
        batches = []
        num_updates = 0
        with self._host_rng():
            rows = None                                # model-data row of each training index
            n_train = n_model
            if self.model_holdout_ratio > 0.0:
                n_train = int(n_model * (1 - self.model_holdout_ratio))
                rows = np.arange(n_model)
                np.random.shuffle(rows)
                rows = rows[:n_train]
            for ep in range(self.model_num_epochs):
                idx = np.arange(n_train)
                nm = len(self.models)                 # self.B (SAC_expert.py:61)
                if self.model_batch_shuffle:
                    idx = np.tile(idx, (nm, 1))
                    for row in idx:
                        np.random.shuffle(row)
                else:
                    np.random.shuffle(idx)
                    idx = np.tile(idx, (nm, 1))
                sections = np.arange(0, n_train, self.model_batch_size)[1:]
                parts = np.array_split(idx, sections, axis=1)
                if n_train % self.model_batch_size != 0:
                    parts = parts[:-1]
                for p in parts:
                    batches.append(p if rows is None else rows[p])
                    num_updates += 1
                    if num_updates >= self.model_max_updates:
                        break
                if num_updates >= self.model_max_updates:
                    break
        if batches:
            self.engine.model_fit((np.stack(batches) + base).astype(np.int32))
        if self.reset_model_optimizer:
            self.engine.reset_model_optimizer()
        # model MSE on the expert data and on counterfactual actions (SAC_expert.py:579-608)
        d = self._diag(disc=False)
        self.model_MSE_on_expert_data.append(d["mse_expert_data"])
        self.model_MSE_on_expert_counterfactual_action.append(d["mse_counterfactual"])
        self.logger.log_train({"model_MSE_on_expert_data": d["mse_expert_data"],
                               "model_MSE_on_expert_counterfactual_action": d["mse_counterfactual"],
                               "model_ent": ent,
                               "time_model_fit": time.time() - t0, "model_loss_epochs": ep + 1,
                               "model_updates": num_updates,
                               "model_loss_last": float(self.engine.model_stats(1)[0].sum())})

    # ------------------------------------------------------------------ loop
    def _train_loop(self, total_timesteps, params):
        """SAC_expert.py:685-824 (a generator of env-loop requests, see SACBase.train)."""
        self._set_rms()
        self._collect_expert_data()
        checkpoints = self._checkpoints(total_timesteps)
        eval_points = self._eval_points(total_timesteps)
        ck = ev = 0
        num_timesteps = 0
        if eval_points is not None:
            self._evaluate(num_timesteps)
        num_timesteps += yield from self._collect_env_data_steps(num_timesteps, self.update_normalizers,
                                                                 self.only_model_normalizer)
        episode_step, episode, episode_reward, done = 0, 0, 0.0, True
        t_episode = time.time()
        obs, expert_reg = None, None
        while num_timesteps < total_timesteps:
            if done:
                self._flush_update_logs()            # before epsilon can change
                self._episode_normalizer_update(episode)      # :740-746
                if episode > 0:
                    self.logger.log_train({"J_tot": episode_reward, "steps": episode_step, "traj": 1,
                                           "time_env_data": time.time() - t_episode})
                obs = self.env.reset()
                done, episode_reward, episode_step = False, 0.0, 0
                episode += 1
                self._update_models()
                expert_reg = self._expert_preprocess()
                t_episode = time.time()
            a = yield ("act", obs, not self.random_act)
            self._pre_update(1)                      # _update(num_timesteps, expert_reg), :780
            yield ("update", 1, num_timesteps, 1)
            self._post_update(1)
            next_obs, r, done, _ = self.env.step(self.actor.clip(a))
            done_no_max = False if episode_step + 1 == self._max_episode_steps else done
            episode_reward += r
            rows = self._add_rows(obs[None], a[None], [r], next_obs[None], [float(done_no_max)])
            self._added(rows, (yield ("add", rows)), True)
            obs = next_obs
            episode_step += 1
            num_timesteps += 1
            if eval_points is not None and num_timesteps >= eval_points[ev]:
                self._evaluate(num_timesteps)
                ev = min(ev + 1, len(eval_points) - 1)
            if num_timesteps >= checkpoints[ck]:
                self._dump_and_save(params)
                ck = min(ck + 1, len(checkpoints) - 1)
        self._dump_and_save(params)
        return self.checkpoint_name
