"""SAC (reference ``sac_eo/algs/SAC.py``): the train loop of ``:253-390``; every
``_update`` (``:236-250``) is one device gradient step (``sacx_sac_step``)."""
import time

import numpy as np

from .base import SACBase


class SAC(SACBase):
    use_expert = False

    def _train_loop(self, total_timesteps, params):
        """SAC.py:254-385 (a generator of env-loop requests, see SACBase.train)."""
        self._set_rms()
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
        obs = None
        while num_timesteps < total_timesteps:
            if done:
                self._episode_normalizer_update(episode)      # :309-315
                if episode > 0:
                    self.logger.log_train({"J_tot": episode_reward, "steps": episode_step, "traj": 1,
                                           "time_env_data": time.time() - t_episode})
                obs = self.env.reset()
                done, episode_reward, episode_step = False, 0.0, 0
                episode += 1
                t_episode = time.time()
            a = yield ("act", obs, not self.random_act)
            if episode_step % int(self.repeat_after_real_steps) == 0:
                # G updates at one env step: num_timesteps unchanged (ts_increment 0)
                self._pre_update(self.G)
                yield ("update", int(self.G), num_timesteps, 0)
                self._post_update(self.G)
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
