"""QCritic / VCritic weight holders (reference ``sac_eo/critics/critics.py:60-111``).

The critics are evaluated inside the fused update (``k_gemm`` + ``k_qhead``); once an
algorithm binds them, ``get_weights``/``set_weights`` read and write the engine's
arena (Keras order ``[W0, b0, W1, b1, W2, b2]``)."""
import numpy as np

from ..nets import create_nn_weights


class _Critic:
    def __init__(self, in_dim, out_dim, layers, activations, gain, rng=None):
        self.layers = list(layers)
        self.activation = list(activations)[0]
        self.gain = gain
        rng = rng if rng is not None else np.random.default_rng(np.random.randint(2 ** 31))
        self._w = create_nn_weights(rng, in_dim, out_dim, self.layers, gain)
        self._engine = None
        self._net = None

    def _bind(self, engine, net):
        engine.set_net(net, self._w)
        self._engine, self._net = engine, net

    @property
    def trainable(self):
        return self.get_weights()

    def get_weights(self):
        return self._engine.get_net(self._net) if self._engine is not None else [x.copy() for x in self._w]

    def set_weights(self, weights):
        self._w = [np.asarray(x, np.float32) for x in weights]
        if self._engine is not None:
            self._engine.set_net(self._net, self._w)

    def set_rms(self, normalizer):
        self.s_rms, self.a_rms, _, _, self.ret_rms = normalizer.get_rms()

    def _forward(self, s, a):
        raise NotImplementedError("critics are evaluated inside the fused device update (sacx_sac_step)")

    value = _forward


class QCritic(_Critic):
    def __init__(self, env, layers, activations, gain, rng=None):
        s = int(np.prod(env.observation_space.shape))
        a = int(np.prod(env.action_space.shape))
        super().__init__(s + a, 1, layers, activations, gain, rng)


class VCritic(_Critic):
    """State-value critic of the on-policy path; kept so init_critics returns the same tuple."""

    def __init__(self, env, layers, activations, gain, rng=None):
        super().__init__(int(np.prod(env.observation_space.shape)), 1, layers, activations, gain, rng)
