"""GaussianActor / SquashedGaussianActor (reference ``sac_eo/actors/continuous_actors.py:9-379``).

Each holds the actor's hyper-parameters and, until an algorithm binds it, its weights in
the Keras ``get_weights()`` order ``[W0, b0, W1, b1, W2, b2] (+ logstd (1, A))``.  Once
bound (``_bind``), the weights live in the engine's HBM arena: get/set go through the
engine and ``sample`` / ``evaluate`` run on the GPU (``sacx_actor_act``,
``sacx_actor_evaluate``).  There is no CPU execution path.

The SAC learner is the squashed actor.  The plain GaussianActor is what the reference builds
for an expert imported from a log (``sac_eo/train.py:65-86`` drops ``actor_squash``): its
device engine is created with ``actor_gaussian`` and serves ``sample`` only.
"""
import numpy as np

from ..nets import create_nn_weights


class _Out(np.ndarray):
    """ndarray with the ``.numpy()`` the reference calls on TF tensors."""

    def numpy(self):
        return np.asarray(self)


def _as_out(x):
    return np.asarray(x).view(_Out)


class GaussianActor:
    squash = False

    def __init__(self, env, layers, activations, gain, init_type, layer_norm, std_mult=1.0, per_state_std=False,
                 output_norm=False, rng=None):
        self.s_dim = int(np.prod(env.observation_space.shape))
        self.a_dim = int(np.prod(env.action_space.shape))
        self.layers = list(layers)
        self.activations = list(activations)          # one name for all layers, or one per layer
        self.activation = self.activations[0]
        self.layer_norm = bool(layer_norm)
        # SquashedGaussianActor.sample / evaluate (continuous_actors.py:270-379) never call
        # _output_normalization, so the flag changes nothing on the squashed actor's SAC path; it is
        # kept as an attribute and acts only on GaussianActor (its _forward, :97-98)
        self.output_norm = bool(output_norm)
        self.gain, self.init_type = gain, init_type
        self.per_state_std = bool(per_state_std)
        self.std_mult = std_mult
        self.act_low = np.asarray(env.action_space.low, np.float32)
        self.act_high = np.asarray(env.action_space.high, np.float32)
        self.act_limit = self.act_high
        self.min_log_std, self.max_log_std = -5, 2
        out_dim = 2 * self.a_dim if self.per_state_std else self.a_dim
        rng = rng if rng is not None else np.random.default_rng(np.random.randint(2 ** 31))
        self._w = create_nn_weights(rng, self.s_dim, out_dim, self.layers, gain, self.layer_norm)
        self._logstd = np.zeros((1, self.a_dim), np.float32)     # tf.Variable(zeros), :56-58
        self._engine = None
        self._net = None

    # ------------------------------------------------------------------ binding
    def _bind(self, engine, net="actor", with_logstd=True):
        """Moves the weights into ``engine`` (net name) and serves them from there."""
        engine.set_net(net, self._w)
        if with_logstd and not self.per_state_std:
            engine.set_logstd(self._logstd)
        self._engine, self._net = engine, net

    @property
    def trainable(self):
        return self.get_weights()

    def get_weights(self):
        if self._engine is not None:
            w = self._engine.get_net(self._net)
            if not self.per_state_std:
                w.append(self._engine.v["actor.logstd"].cpu().numpy().copy())
            return w
        return [x.copy() for x in self._w] + ([] if self.per_state_std else [self._logstd.copy()])

    def set_weights(self, weights):
        weights = [np.asarray(x, np.float32) for x in weights]
        nw = len(self._w)
        self._w = weights[:nw]
        if not self.per_state_std and len(weights) > nw:
            self._logstd = weights[nw].reshape(1, -1)
        if self._engine is not None:
            self._engine.set_net(self._net, self._w)
            if not self.per_state_std:
                self._engine.set_logstd(self._logstd)

    def set_rms(self, normalizer):
        self.s_rms = normalizer.get_rms()[0]

    # ------------------------------------------------------------------ acting
    def sample(self, s, deterministic=False):
        """On the GPU: mu + std * u (GaussianActor, :103-123) or act_limit * tanh(mu + std * u)
        (SquashedGaussianActor, :270-306); u from the global NumPy stream's device copy unless
        deterministic."""
        if self._engine is None:
            raise RuntimeError("actor is not bound to a device engine (build the algorithm first)")
        out = self._engine.act(np.asarray(s, np.float32), deterministic=deterministic)
        return _as_out(out.cpu().numpy())

    def clip(self, a):
        # np.clip (continuous_actors.py's tf.clip_by_value on host arrays); minimum / maximum
        # give the same values without np.clip's per-call dispatch cost in the env loop
        return np.minimum(np.maximum(a, self.act_low), self.act_high)

    def tf_clip(self, a):
        return self.clip(a)


class SquashedGaussianActor(GaussianActor):
    squash = True

    def evaluate(self, s):
        """(pi_action, neglogp_adjusted) of continuous_actors.py:327-379 on the GPU
        (sacx_actor_evaluate): u = np.random.normal(size=(n, A)) from the device copy of the
        global stream, x = mu + std * u, pi = act_limit * tanh(x).  One row (s of shape
        [1, S] or [S]) gives pi [A] and a scalar neglogp, as the reference's squeeze does."""
        if self._engine is None:
            raise RuntimeError("actor is not bound to a device engine (build the algorithm first)")
        x = np.asarray(s, np.float32)
        pi, nlp = self._engine.evaluate(x.reshape(-1, self.s_dim))
        pi, nlp = pi.cpu().numpy(), nlp.cpu().numpy()
        if pi.shape[0] == 1:
            pi, nlp = pi[0], nlp[0]
        return _as_out(pi), _as_out(nlp)
