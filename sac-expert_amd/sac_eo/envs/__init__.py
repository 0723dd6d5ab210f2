"""Environments.  gym / MuJoCo are not installed in this image, so ``init_env`` returns
a synthetic gym-style environment with the reference task's observation and action
shapes (obs/act dims of HalfCheetah-v3, Walker2d-v3, Humanoid-v3, ...): the SAC update
path only sees rows of (s, a, r, sp, d), so these exercise it end to end.  Any object
with the gym 0.2x API (``reset() -> obs``, ``step(a) -> (obs, r, done, info)``,
``seed``, ``observation_space`` / ``action_space`` with ``shape``/``low``/``high``) works."""
from .synthetic import ENV_SPECS, Box, SyntheticEnv, init_env

__all__ = ["ENV_SPECS", "Box", "SyntheticEnv", "init_env"]
