"""A CPU stand-in for sac_eo.engine.Engine, for the host-logic tests only (no GPU here).

It keeps the weights the algorithms bind, consumes the global NumPy stream in the device
engine's order (sampler: randint + normals per update; stochastic actions; counterfactual
actions of the diagnostics) and returns deterministic stand-in numbers, so the training loops,
their RNG hand-offs, the per-episode hooks, checkpointing and the lock-step driver run end to
end on the CPU.  It computes no SAC arithmetic (the GPU tests do, against the oracle)."""
import dataclasses

import numpy as np
import torch


class FakeEngine:
    def __init__(self, cfg, *a, **k):
        self.cfg = cfg
        self.seeds = max(1, int(cfg.seeds))
        self._k = 0
        self._st = [self._new_seed() for _ in range(self.seeds)]
        self.calls = []

    def _new_seed(self):
        cfg = self.cfg
        return dict(nets={}, rs=np.random.RandomState(0), rows=0, seq=0, nts=0, mseq=0, alpha=np.log(cfg.init_temperature),
                    v={"actor.logstd": torch.zeros(1, cfg.a_dim)}, norms={}, expert=None, perms=[])

    @property
    def S(self):
        return self._st[self._k]

    @property
    def v(self):
        return self.S["v"]

    @property
    def segments(self):
        out = {f"{n}.l{i}": {} for n in ("actor", "q0", "q1", "t0", "t1") for i in range(3)}
        if self.cfg.use_expert:
            for m in range(int(self.cfg.num_models or 2)):
                out.update({f"m{m}.l{i}": {} for i in range(3)})
        return out

    # ------------------------------------------------------------------ seeds
    def select_seed(self, k):
        self._k = int(k)

    def seed_view(self, k):
        from sac_eo.engine import SeedView
        return SeedView(self, k)

    @property
    def _views(self):
        return [s["v"] for s in self._st]

    # ------------------------------------------------------------------ state
    def set_net(self, net, w):
        self.S["nets"][net] = [np.array(x, np.float32) for x in w]

    def get_net(self, net):
        return [x.copy() for x in self.S["nets"][net]]

    def set_logstd(self, l):
        self.S["v"]["actor.logstd"] = torch.as_tensor(np.asarray(l, np.float32).reshape(1, -1))

    def set_alpha(self, a):
        self.S["alpha"] = float(a)

    def alpha(self):
        return float(self.S["alpha"])

    def set_normalizers(self, *a, which="all", **k):
        self.S["norms"][which] = a

    def rng_set_state(self, state):
        self.S["rs"].set_state(state)

    def rng_get_state(self):
        return self.S["rs"].get_state()

    # ------------------------------------------------------------------ data / acting
    def _act(self, obs, deterministic):
        obs = np.asarray(obs, np.float32).reshape(-1, self.cfg.s_dim)
        mu = np.tanh(obs[:, :1] * 0.1 + np.zeros((obs.shape[0], self.cfg.a_dim), np.float32))
        if not deterministic:
            mu = np.tanh(mu + np.float32(0.1) * self.S["rs"].normal(size=mu.shape).astype(np.float32))
        return mu.astype(np.float32)

    def act(self, obs, deterministic=True):
        single = np.ndim(obs) == 1
        out = torch.as_tensor(self._act(obs, deterministic))
        return out[0] if single else out

    def act_host(self, obs, deterministic=True):
        single = np.ndim(obs) == 1
        out = self._act(obs, deterministic)
        return out[0] if single else out

    def act_host_seeds(self, obs, deterministic=True):
        self.calls.append("act_seeds")
        out = []
        for k in range(self.seeds):
            self._k = k
            out.append(self._act(np.asarray(obs)[k], deterministic))
        return np.stack(out)

    def append(self, s, a, r, sp, d):
        n = int(np.shape(r)[0])
        self.S["rows"] = min(self.S["rows"] + n, int(self.cfg.buffer_capacity))
        return n

    def append_host_seeds(self, s, a, r, sp, d):
        self.calls.append("append_seeds")
        n = int(np.asarray(r).reshape(self.seeds, -1).shape[1])
        for k in range(self.seeds):
            self._k = k
            self.append(None, None, np.zeros(n), None, None)
        return n

    def set_expert(self, s_e, sp_e, eps):
        self.S["expert"] = (np.asarray(s_e).shape, float(eps))

    def push_perms(self, perms):
        self.S["perms"] = [np.asarray(p) for p in perms]

    # ------------------------------------------------------------------ updates
    def step(self, n=1, num_timesteps=0, ts_increment=1, **k):
        self.calls.append(("step", n, num_timesteps, ts_increment))
        cfg = self.cfg
        for st in self._st:
            for i in range(n):
                st["rs"].randint(max(st["rows"], 1), size=cfg.batch)
                for _ in range(2):
                    st["rs"].normal(size=(cfg.batch, cfg.a_dim))
                if cfg.use_expert:
                    st["rs"].normal(size=(cfg.expert_batch, cfg.a_dim))
                st["rs"].normal(size=(cfg.batch, cfg.a_dim))
                st["seq"] += 1
            st["nts"] = num_timesteps + n * ts_increment

    def stats(self, n):
        s = self.S["seq"]
        return np.array([[0.5, 0.5, 1.0, 1e-5, 1e-5, 0.0, 3.0, float(i)] for i in range(s - n, s)], np.float32)

    def ctl(self):
        return {"step_seq": self.S["seq"], "cur_size": self.S["rows"], "num_timesteps": self.S["nts"],
                "mfit_seq": self.S["mseq"]}

    def model_fit(self, idx, eager=False):
        self.S["mseq"] += int(np.asarray(idx).shape[0])

    def model_stats(self, n):
        return np.ones(n, np.float32)

    def reset_model_optimizer(self):
        pass

    def expert_diag(self, s_e, a_e, sp_e, disc=False, use_expert_actions=False, delta_clip=0.0):
        if not use_expert_actions:
            self.S["rs"].normal(size=(np.shape(s_e)[0], self.cfg.a_dim))
        if disc:
            n = np.shape(s_e)[0]
            return dict(s_disc_total=1.0, max_disc=0.1, median_disc=0.05, disc_ratio=np.full(n, 1.0 / n))
        return dict(mse_expert_data=0.25, mse_counterfactual=0.5, mse_expert_data_per_model=np.zeros(2),
                    mse_counterfactual_per_model=np.zeros(2))

    def sync(self):
        pass

    def close(self):
        pass


def install(monkeypatch):
    """Routes every Engine the algorithms build (sac_eo.algs.*, the expert engine) to FakeEngine."""
    import sac_eo.algs.base as base
    import sac_eo.algs.SAC_expert as sx
    monkeypatch.setattr(base, "Engine", FakeEngine)
    monkeypatch.setattr(sx, "Engine", FakeEngine)
