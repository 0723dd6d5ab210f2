"""Duck-typed NumPy stand-ins for a gym env, an actor and a world model, used to drive the
reference's own samplers (tests/golden/make_ref_fixtures.py) and the build's (tests) on the
same inputs.  They are test objects with the interface the samplers call
(``env.reset/step``, ``actor.sample(...).numpy()``, ``actor.clip``), not restatements of any
reference code.  Nothing here imports ``sac_eo``."""
import numpy as np


class _T:
    """What ``actor.sample`` returns in the reference: an object with ``.numpy()``."""

    def __init__(self, x):
        self.x = x

    def numpy(self):
        return self.x


class DuckActor:
    """a = tanh(s W) (+ e^logstd u with u from the GLOBAL np.random stream when stochastic)."""

    def __init__(self, S, A, seed=0, logstd=-0.5):
        rs = np.random.RandomState(seed)
        self.W = (rs.normal(size=(S, A)) * 0.3).astype(np.float32)
        self.sig = np.float32(np.exp(logstd))

    def sample(self, s, deterministic=False):
        mu = np.tanh(np.asarray(s, np.float32) @ self.W)
        if deterministic:
            return _T(mu)
        u = np.random.normal(size=mu.shape).astype(np.float32)
        return _T(mu + self.sig * u)

    def clip(self, a):
        return np.clip(a, -1.0, 1.0)


class DuckEnv:
    """float64 observations, python-float rewards, terminates when |s[0]| > thresh or after
    ``term_at`` steps; its own RandomState (the env's seeded stream)."""

    def __init__(self, S, A, seed=0, thresh=2.5, term_at=None):
        self.rs = np.random.RandomState(seed)
        self.M = self.rs.normal(size=(S, A)) * 0.4
        self.S, self.thresh, self.term_at = S, thresh, term_at
        self.s, self.t = None, 0

    def reset(self, s_init=None):
        self.s = self.rs.normal(size=self.S) if s_init is None else np.array(s_init, np.float64)
        self.t = 0
        return self.s.copy()

    def step(self, a):
        self.t += 1
        self.s = 0.9 * self.s + self.M @ np.asarray(a, np.float64) + 0.3 * self.rs.normal(size=self.S)
        r = float(-0.01 * np.sum(self.s ** 2) + np.sum(a))
        d = bool(abs(self.s[0]) > self.thresh or (self.term_at is not None and self.t >= self.term_at))
        return self.s.copy(), r, d, {}


class OracleActor:
    """actor.sample of the build's oracle (the SquashedGaussianActor head on oracle weights),
    with the noise from the GLOBAL np.random stream: u = f32(normal(size=(n, A)))."""

    def __init__(self, O, st, cfg, nrm):
        self.O, self.st, self.cfg, self.nrm = O, st, cfg, nrm

    def sample(self, s, deterministic=False):
        O, st, cfg = self.O, self.st, self.cfg
        dt = st.alpha.dtype.type
        nrm = self.nrm.cast(dt)
        x = O._norm(np.asarray(s, dt), nrm.s_mean, nrm.s_den)
        o, _ = O.actor_forward(st.actor, x, cfg)
        mu, lraw = O.split_head(o, st.logstd, cfg)
        u = np.zeros_like(mu) if deterministic else O.f32_noise(np.random.normal(size=mu.shape)).astype(dt)
        return _T(O.head_sample(mu, lraw, u, cfg.act_limit, dt)[0])

    def clip(self, a):
        lim = self.O._F(self.st.alpha.dtype.type, self.cfg.act_limit)
        return np.clip(a, -lim, lim)


class OracleModelEnv:
    """MSEModel.reset / step on oracle weights (world model k): s' = s + denorm(delta),
    r = denorm(r_n), d = False; batched over rows."""

    def __init__(self, O, st, cfg, nrm, k=0):
        self.O, self.st, self.cfg, self.nrm, self.k = O, st, cfg, nrm, k
        self.s = None

    def reset(self, s_init):
        self.s = np.array(s_init, self.st.alpha.dtype.type)
        return self.s

    def step(self, a):
        O, st, cfg = self.O, self.st, self.cfg
        dt = st.alpha.dtype.type
        nrm = self.nrm.cast(dt)
        S = cfg.S
        xm = np.concatenate([O._norm(self.s, nrm.s_mean, nrm.s_den), O._norm(a, nrm.a_mean, nrm.a_den)], 1)
        pred, _ = O.mlp_forward(st.models[self.k], xm, cfg.model_act)
        sp = self.s + (pred[:, :S] * nrm.d_den + nrm.d_mean)
        r = pred[:, S] * nrm.r_den + nrm.r_mean
        self.s = sp
        return sp, r, np.zeros(len(r), bool), {}


def fill_run_log(Logger, rs, idx, n_upd):
    """One run's log the way the reference's algs fill it (base_onpolicy_alg.py:351-374)."""
    lg = Logger()
    params = {"setup_kwargs": {"idx": idx, "seed": 0, "runs_start": 0, "import_path": "./logs", "import_file": None,
                               "import_idx": None, "import_all": False},
              "env_kwargs": {"env_type": "gym", "env_name": "HalfCheetah-v3", "task_name": None},
              "actor_kwargs": {"actor_layers": [8, 8], "actor_activations": ["tanh"], "actor_gain": 0.01,
                               "actor_squash": True, "actor_adversary_prob": None},
              "critic_kwargs": {"critic_layers": [8, 8], "critic_activations": ["tanh"], "num_models": 2},
              "model_kwargs": {"model_layers": [16, 16], "num_models": 2, "gaussian_model": False},
              "model_setup_kwargs": {"separate_reward_nn": False, "reward_loss_coef": 1.0},
              "alg_kwargs": {"gamma": 0.995, "sac_batch_size": 256, "init_rms_stats": None},
              "mf_update_kwargs": {"adv_center": True}}
    for _ in range(n_upd):
        lg.log_train({"alpha_loss": np.float32(rs.normal()), "p_loss": np.float32(rs.normal()),
                      "epsilon": 1e-3})
    lg.log_train({"J_tot": float(rs.normal()), "steps": 1000, "traj": 1, "time_env_data": 0.5})
    lg.log_train_ensemble([{"model_loss": rs.normal()}, {"model_loss": rs.normal()}])
    lg.log_params(params)
    w = [rs.normal(size=(3, 8)).astype(np.float32), np.zeros(8, np.float32),
         rs.normal(size=(8, 2)).astype(np.float32), np.zeros(2, np.float32), np.zeros((1, 2), np.float32)]
    stats = {k: {"t": 12 + idx, "mean": rs.normal(size=3).astype(np.float32),
                 "var": rs.uniform(0.5, 2, size=3).astype(np.float32)}
             for k in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms")}
    lg.log_final({"actor_weights": w, "critic_weights": [[x.copy() for x in w]], "rms_stats": stats,
                  "model_weights": [[x * 2 for x in w]], "reward_weights": [None]})
    return lg
