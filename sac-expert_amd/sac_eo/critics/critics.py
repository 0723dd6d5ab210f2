"""QCritic / VCritic (reference ``sac_eo/critics/critics.py:6-111``).

Inside the fused update the critics run as ``k_gemm`` launches + ``qhead`` rows.  Once an
algorithm binds a critic to its engine (``q0`` / ``q1`` for the q_critics, ``t0`` / ``t1``
for the q_targets), ``get_weights``/``set_weights`` read and write the engine's arena
(Keras order ``[W0, b0, W1, b1, W2, b2]``) and ``_forward`` / ``value`` run on the GPU
(``sacx_critic_forward``).  There is no CPU execution path."""
import numpy as np

from ..actors.continuous_actors import _as_out

from ..nets import create_nn_weights


class _Critic:
    def __init__(self, in_dim, out_dim, layers, activations, gain, rng=None):
        self.layers = list(layers)
        self.activations = list(activations)
        self.activation = self.activations[0]
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

    def _require(self):
        if self._engine is None:
            raise RuntimeError("critic is not bound to a device engine (build the algorithm first)")
        return self._engine


class QCritic(_Critic):
    def __init__(self, env, layers, activations, gain, rng=None):
        s = int(np.prod(env.observation_space.shape))
        a = int(np.prod(env.action_space.shape))
        super().__init__(s + a, 1, layers, activations, gain, rng)

    def _forward(self, s, a):
        """Net output [n, 1] on [s_rms.normalize(s), a_rms.normalize(a)] (critics.py:84-94)."""
        return _as_out(self._require().critic_forward(self._net, np.asarray(s, np.float32),
                                                      np.asarray(a, np.float32)).cpu().numpy())

    def value(self, s, a):
        """squeeze(_forward(s, a), -1) * max(ret_rms.std, 1e-8) (critics.py:96-103)."""
        return _as_out(self._require().critic_forward(self._net, np.asarray(s, np.float32),
                                                      np.asarray(a, np.float32), value=True).cpu().numpy())


class VCritic(_Critic):
    """State-value critic of the on-policy path (critics.py:6-57); kept so init_critics returns
    the same tuple.  SAC never evaluates it (the on-policy path is out of scope), so it has
    weights but no device network."""

    def __init__(self, env, layers, activations, gain, rng=None):
        super().__init__(int(np.prod(env.observation_space.shape)), 1, layers, activations, gain, rng)
