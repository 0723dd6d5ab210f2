"""State corruption of collected transitions (reference ``sac_eo/common/corruptor.py:3-30``).

``--s_noise_std`` > 0 adds ``u * sqrt(delta_rms.var) * s_noise_std`` to every observation the
env returns during ``trajectory_sampler`` collection, ``u`` drawn from the corruptor's own
``default_rng(0)`` (never the global stream the device shares).  ``--s_noise_type all``
continues the rollout from the corrupted state, ``next`` only stores it as ``sp``.  The
variance is read live from the normaliser handed to ``set_rms`` (``base_onpolicy_alg.py:204``),
so with the default (never updated) normalisers the noise is zero but the stream still
advances.  Host-side: it touches env observations before they reach the device ring."""
import numpy as np


class TrajectoryCorruptor:
    def __init__(self, s_noise_std=0.0, s_noise_type="all"):
        self.s_noise_std = s_noise_std
        self.s_noise_rng = np.random.default_rng(0)
        self.s_noise_type = s_noise_type
        self.delta_rms = None

    def set_rms(self, normalizer):
        self.delta_rms = normalizer.get_rms()[3]

    def corrupt_samples(self, sp):
        if self.s_noise_std > 0.0:
            u = self.s_noise_rng.normal(size=np.shape(sp)).astype("float32")
            sp = sp + u * np.sqrt(self.delta_rms.var) * self.s_noise_std
        return sp

    def store_and_next(self, s_true):
        """(the state stored as sp, the state the rollout continues from): samplers.py:35-43."""
        s_store = self.corrupt_samples(s_true)
        return s_store, (s_store if self.s_noise_type == "all" else s_true)
