"""Seeding, as the reference does it.

``derive_seeds`` restates the per-run seed derivation of ``main`` in the reference's
``sac_eo/train.py:108-118``: five ``SeedSequence`` streams (setup, sim, eval, expert,
algorithm) spawned from ``--seed``, each sliced to ``[runs_start, runs_start + runs)``.
``init_seeds`` follows ``sac_eo/common/seeding.py:7-15`` without TensorFlow; the
device engine adopts the resulting NumPy stream through ``Engine.rng_set_state``.

In the reference the last ``np.random.seed`` before training is
``init_seeds(exp_seed, env_expert)`` (``sac_eo/train.py:95-97``), so the global stream
the gradient steps draw from starts at the run's *expert* seed.
"""
import os
import random

import numpy as np

SEED_KINDS = ("setup", "sim", "eval", "expert", "algorithm")


def derive_seeds(seed: int, runs: int = 1, runs_start: int = 0) -> dict:
    """{kind: np.ndarray[runs] of uint32} for kinds setup/sim/eval/expert/algorithm."""
    base = np.random.SeedSequence(seed).generate_state(5)
    return {kind: np.random.SeedSequence(base[i]).generate_state(runs + runs_start)[runs_start:]
            for i, kind in enumerate(SEED_KINDS)}


def init_seeds(seed, env=None):
    """np.random / random / PYTHONHASHSEED (and env.seed when given)."""
    seed = int(seed)
    if env is not None and hasattr(env, "seed"):
        env.seed(seed)
    np.random.seed(seed)
    random.seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
