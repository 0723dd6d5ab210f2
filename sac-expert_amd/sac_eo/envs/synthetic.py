"""Synthetic continuous-control environment with gym 0.2x semantics."""
import numpy as np

# obs_dim, act_dim of the reference's tasks (MuJoCo v3 / classic control)
ENV_SPECS = {
    "HalfCheetah-v3": (17, 6), "Walker2d-v3": (17, 6), "Hopper-v3": (11, 3), "Ant-v3": (111, 8),
    "Humanoid-v3": (376, 17), "Swimmer-v3": (8, 2), "Pendulum-v1": (3, 1),
}


class Box:
    """gym.spaces.Box subset: shape, low, high, sample()."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = dtype
        self.low = np.broadcast_to(np.asarray(low, dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype), self.shape).copy()
        self.np_random = np.random.RandomState(0)

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)

    def sample(self):
        return self.np_random.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high)


class SyntheticEnv:
    """s' = 0.9 s + 0.5 tanh(W_s s + W_a a) + noise, r = s'_0 - 0.1 |a|^2 (a cheetah-like
    'forward velocity' minus control cost).  Its randomness comes from its own
    RandomState (``seed``), never from the global NumPy stream, like a MuJoCo env."""

    def __init__(self, name="HalfCheetah-v3", obs_dim=None, act_dim=None, max_episode_steps=1000,
                 terminate=False):
        s, a = ENV_SPECS.get(name, (obs_dim, act_dim))
        if obs_dim is not None:
            s, a = obs_dim, act_dim
        if s is None:
            raise ValueError(f"unknown environment {name!r}; known: {sorted(ENV_SPECS)}")
        self.name = name
        self.observation_space = Box(-np.inf, np.inf, (s,))
        self.action_space = Box(-1.0, 1.0, (a,))           # gym.wrappers.RescaleAction(env, -1, 1)
        self._max_episode_steps = max_episode_steps
        self.terminate = terminate
        g = np.random.RandomState(12345 + s * 131 + a)     # fixed dynamics per task shape
        self._Ws = (g.normal(size=(s, s)) / np.sqrt(s)).astype(np.float32)
        self._Wa = (g.normal(size=(a, s)) / np.sqrt(a)).astype(np.float32)
        self.np_random = np.random.RandomState(0)
        self._s = None
        self._t = 0

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        self.action_space.seed(seed)
        return [seed]

    def reset(self, s_init=None):
        s = self.observation_space.shape[0]
        self._s = (np.asarray(s_init, np.float32) if s_init is not None
                   else (0.1 * self.np_random.normal(size=s)).astype(np.float32))
        self._t = 0
        return self._s.copy()

    def step(self, a):
        a = np.clip(np.asarray(a, np.float32).reshape(self.action_space.shape), -1.0, 1.0)
        s = self._s
        sp = 0.9 * s + 0.5 * np.tanh(s @ self._Ws + a @ self._Wa) \
            + 0.01 * self.np_random.normal(size=s.shape)
        sp = sp.astype(np.float32)
        r = float(sp[0] - 0.1 * np.sum(a * a))
        self._t += 1
        done = bool(self.terminate and np.abs(sp).max() > 10.0) or self._t >= self._max_episode_steps
        self._s = sp
        return sp.copy(), r, done, {}


def init_env(env_type="gym", env_name="HalfCheetah-v3", task_name=None):
    """sac_eo/envs/init_env (gym path): RescaleAction(-1, 1) shapes of the named task."""
    if env_type not in ("gym", "synthetic"):
        raise ValueError(f"env_type {env_type!r} is not available here (gym-style synthetic only)")
    return SyntheticEnv(env_name)
