"""Running normalisers (reference ``sac_eo/common/normalizer.py:5-190``), host side.

The device engine needs only the derived (mean, max(std, 1e-8)) vectors; these
classes keep the reference's update rule and stats format so logged ``rms_stats``
and ``init_rms_stats`` dicts carry over."""
import numpy as np


def discounted_sum(x, rate):
    """buffer_utils.discounted_sum (buffer_utils.py:8-9): y_t = x_t + rate * y_{t+1}, in
    float64 as scipy.signal.lfilter returns it (its direct form computes the same products and
    sums), so ret_rms merges the float64 returns the reference's does."""
    x = np.asarray(x, dtype=np.float64)
    y = np.zeros_like(x)
    acc = 0.0
    rate = float(rate)
    for t in range(len(x) - 1, -1, -1):
        acc = x[t] + rate * acc
        y[t] = acc
    return y


class RunningNormalizer:
    def __init__(self, dim):
        self.dim = dim
        self.reset()

    def reset(self):
        self.t_last = 0
        if self.dim == 1:
            self.mean, self.var, self.std = 0.0, 0.0, 1.0
        else:
            self.mean = np.zeros(self.dim, np.float32)
            self.var = np.zeros(self.dim, np.float32)
            self.std = np.ones(self.dim, np.float32)

    def normalize(self, data, center=True):
        return (data - self.mean) / np.maximum(self.std, 1e-8) if center else data / np.maximum(self.std, 1e-8)

    def denormalize(self, data_norm, center=True):
        return data_norm * np.maximum(self.std, 1e-8) + (self.mean if center else 0.0)

    def update(self, data):
        """normalizer.py:60-90 (batch merge in the normalised frame)."""
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
        self.mean = np.asarray(self.mean).astype("float32")
        self.var = np.asarray(self.var).astype("float32")
        self.std = np.ones_like(self.var) if t == 1 else np.sqrt(self.var)
        self.t_last = t

    def instantiate(self, t, mean, var, ignore=None):
        self.t_last, self.mean, self.var = t, mean, var
        if self.t_last == 0:
            self.reset()
        elif self.t_last == 1:
            self.std = np.abs(self.mean)
        else:
            self.std = np.sqrt(self.var)

    def get_stats(self):
        return {"t": self.t_last, "mean": self.mean, "var": self.var}

    def den(self):
        return np.maximum(self.std, 1e-8)


class RunningNormalizers:
    def __init__(self, s_dim, a_dim, gamma, init_rms_stats=None):
        self.gamma = gamma
        self.s_rms = RunningNormalizer(s_dim)
        self.a_rms = RunningNormalizer(a_dim)
        self.r_rms = RunningNormalizer(1)
        self.delta_rms = RunningNormalizer(s_dim)
        self.ret_rms = RunningNormalizer(1)
        self.set_rms_stats(init_rms_stats)

    def update_rms(self, s_traj, a_traj, r_traj, sp_traj):
        self.s_rms.update(s_traj)
        self.a_rms.update(a_traj)
        self.r_rms.update(r_traj)
        self.delta_rms.update(sp_traj - s_traj)
        self.ret_rms.update(discounted_sum(r_traj, self.gamma))

    def get_rms(self):
        return self.s_rms, self.a_rms, self.r_rms, self.delta_rms, self.ret_rms

    def set_rms_stats(self, init_rms_stats):
        if init_rms_stats is not None:
            for k in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms"):
                getattr(self, k).instantiate(**init_rms_stats[k])

    def get_rms_stats(self):
        return {k: getattr(self, k).get_stats() for k in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms")}

    def push_to(self, engine, which: str = "all"):
        """Writes the derived vectors the kernels use into the engine (which: "all", "main" =
        the actor's / critics' set, "model" = the world models' set; Engine.set_normalizers)."""
        f = lambda x, n: np.broadcast_to(np.asarray(x, np.float32), (n,))
        S, A = engine.cfg.s_dim, engine.cfg.a_dim
        engine.set_normalizers(f(self.s_rms.mean, S), f(self.s_rms.den(), S), f(self.a_rms.mean, A),
                               f(self.a_rms.den(), A), f(self.delta_rms.mean, S), f(self.delta_rms.den(), S),
                               float(np.asarray(self.r_rms.mean).reshape(-1)[0]),
                               float(np.asarray(self.r_rms.den()).reshape(-1)[0]),
                               float(np.asarray(self.ret_rms.den()).reshape(-1)[0]), which=which)
