"""MSEModel and GaussianModel (reference ``sac_eo/models/continuous_models.py:7-349`` over
``sac_eo/models/base_world_model.py:7-138``).

Predicts [normalised delta-s | normalised r] from [norm s | norm a] -- the reward as the model
net's last column, or with ``--separate_reward_nn`` from a second net of ``reward_layers``
(base_world_model.py:32-37, :72-74).  GaussianModel adds a trainable ``logstd`` [1, S]
(continuous_models.py:24-27): its ``sample(deterministic=False)`` and ``step`` add
``exp(logstd) * u`` to the normalised delta (u from the global NumPy stream), and its fit loss is the
Gaussian negative log-likelihood (:101-131).  Fitted on the device by ``sacx_model_fit`` and used by
the SAC-EO expert term inside the update.  Once an algorithm binds the model to its engine (``m0`` /
``m1``, reward net ``r0`` / ``r1``, ``m<k>.logstd``), ``get_weights`` / ``set_weights`` go through the
engine's arena and ``_forward`` / ``sample`` / ``step`` / ``get_loss`` run on the GPU
(``sacx_model_sample``, ``sacx_model_loss``).  There is no CPU execution path."""
import numpy as np

from ..actors.continuous_actors import _as_out
from ..nets import create_nn_weights

_LOG2PI_F32 = float(np.log(np.float32(2 * np.pi), dtype=np.float32))   # tf.math.log(2*np.pi) in float32


class BaseWorldModel:
    """base_world_model.py:7-138: the model net (and the optional reward net) as Keras weight
    lists until bound to a device engine."""
    gaussian = False

    def __init__(self, env, layers, activations, gain, reward_layers, reward_activations, reward_gain,
                 model_setup_kwargs, rng=None):
        self.s_dim = int(np.prod(env.observation_space.shape))
        self.a_dim = int(np.prod(env.action_space.shape))
        k = model_setup_kwargs
        self.separate_reward_nn = bool(k.get("separate_reward_nn", False))
        self.reward_loss_coef = k.get("reward_loss_coef", 1.0)
        self.scale_model_loss = bool(k.get("scale_model_loss", False))
        # base_world_model.py:54-58 (None = off)
        self.delta_clip_loss = k.get("delta_clip_loss")
        self.reward_clip_loss = k.get("reward_clip_loss")
        self.delta_clip_pred = k.get("delta_clip_pred")
        self.reward_clip_pred = k.get("reward_clip_pred")
        self.layers = list(layers)
        self.activations = list(activations)
        self.activation = self.activations[0]
        self.reward_layers = list(reward_layers)
        self.reward_activations = list(reward_activations)
        rng = rng if rng is not None else np.random.default_rng(np.random.randint(2 ** 31))
        in_dim = self.s_dim + self.a_dim
        out_dim = self.s_dim if self.separate_reward_nn else self.s_dim + 1      # :32-41
        self._w = create_nn_weights(rng, in_dim, out_dim, self.layers, gain)
        self._rw = create_nn_weights(rng, in_dim, 1, self.reward_layers, reward_gain) if self.separate_reward_nn \
            else None
        self._engine = None
        self._net = None
        self.s = None

    # ------------------------------------------------------------------ binding / weights
    def _bind(self, engine, net):
        engine.set_net(net, self._w)
        if self._rw is not None:
            engine.set_net("r" + net[1:], self._rw)
        self._engine, self._net = engine, net

    def _require(self):
        if self._engine is None:
            raise RuntimeError("model is not bound to a device engine (build the algorithm first)")
        return self._engine, int(self._net[1])

    def _nn_weights(self):
        return self._engine.get_net(self._net) if self._engine is not None else [x.copy() for x in self._w]

    def _set_nn_weights(self, weights):
        self._w = [np.asarray(x, np.float32) for x in weights]
        if self._engine is not None:
            self._engine.set_net(self._net, self._w)

    def get_reward_weights(self):
        """base_world_model.py:123-128: the reward net's weights, None without it."""
        if not self.separate_reward_nn:
            return None
        return self._engine.get_net("r" + self._net[1:]) if self._engine is not None else [x.copy() for x in self._rw]

    def set_reward_weights(self, weights):
        """base_world_model.py:130-133."""
        if self.separate_reward_nn and weights is not None:
            self._rw = [np.asarray(x, np.float32) for x in weights]
            if self._engine is not None:
                self._engine.set_net("r" + self._net[1:], self._rw)

    @property
    def trainable(self):
        """model.trainable (continuous_models.py:27-32, :216-221): model net, logstd, reward net."""
        out = self.get_weights()
        return out + (self.get_reward_weights() or [])

    def _unflat(self, weights, from_flat, increment):
        cur = self.get_weights()
        if from_flat:
            flat = np.asarray(weights, np.float32).ravel()
            out, o = [], 0
            for x in cur:
                out.append(flat[o:o + x.size].reshape(x.shape))
                o += x.size
            weights = out
        weights = [np.asarray(x, np.float32) for x in weights]
        if increment:
            weights = [x + y for x, y in zip(weights, cur)]
        return weights

    def set_rms(self, normalizer):
        self.s_rms, self.a_rms, self.r_rms, self.delta_rms, _ = normalizer.get_rms()

    # ------------------------------------------------------------------ network calls (device)
    def _rows(self, s, a):
        s2 = np.asarray(s, np.float32).reshape(-1, self.s_dim)
        a2 = np.asarray(a, np.float32).reshape(-1, self.a_dim)
        return s2, a2

    def _forward(self, s, a, clip=True):
        """(delta_n [n, S], r_n [n]) with the prediction clips when clip
        (base_world_model.py:65-87)."""
        eng, k = self._require()
        s2, a2 = self._rows(s, a)
        dc = (self.delta_clip_pred or 0.0) if clip else 0.0
        rc = (self.reward_clip_pred or 0.0) if clip else 0.0
        pred, _, _ = eng.model_forward(k, s2, a2, dc, rc)
        pred = pred.cpu().numpy()
        return _as_out(pred[:, :-1]), _as_out(pred[:, -1])

    def _sample(self, s, a, stochastic):
        eng, k = self._require()
        s2, a2 = self._rows(s, a)
        _, sp, _ = eng.model_forward(k, s2, a2, self.delta_clip_pred or 0.0, self.reward_clip_pred or 0.0,
                                     stochastic=stochastic)
        sp = sp.cpu().numpy()
        return _as_out(sp.reshape(np.shape(s)) if np.ndim(s) == 1 else sp)

    def reset(self, s):
        """continuous_models.py:72-75 / :256-259."""
        self.s = s
        return s

    def seed(self, seed):
        raise NotImplementedError          # continuous_models.py:77-79 / :261-263

    def _step(self, a, stochastic):
        eng, k = self._require()
        s2, a2 = self._rows(self.s, a)
        _, sp, r = eng.model_forward(k, s2, a2, self.delta_clip_pred or 0.0, self.reward_clip_pred or 0.0,
                                     stochastic=stochastic)
        sp, r = sp.cpu().numpy(), r.cpu().numpy()
        if sp.shape[0] == 1:                 # tf.squeeze of one row
            sp, r = sp[0] if np.ndim(self.s) == 1 else sp, r[0]
        self.s = sp
        d = np.zeros(np.shape(r), bool) if np.ndim(r) else False
        return self.s, r, d, {}

    def get_loss(self, s, sp, a, r):
        """MSEModel.get_loss (continuous_models.py:280-302) / GaussianModel.get_loss (:101-131) with
        the optional loss clips, on the device."""
        eng, k = self._require()
        s2, a2 = self._rows(s, a)
        sp2 = np.asarray(sp, np.float32).reshape(-1, self.s_dim)
        r2 = np.asarray(r, np.float32).reshape(-1)
        return eng.model_loss(k, s2, sp2, a2, r2, self.delta_clip_loss or 0.0, self.reward_clip_loss or 0.0)


class MSEModel(BaseWorldModel):
    """continuous_models.py:205-349."""

    def get_weights(self):
        return self._nn_weights()

    def set_weights(self, weights, from_flat=False, increment=False):
        """continuous_models.py:269-278: a weight list, or a flat vector (from_flat), optionally
        added to the current weights (increment)."""
        self._set_nn_weights(self._unflat(weights, from_flat, increment))

    def sample(self, s, a, deterministic=True):
        """s + delta_rms.denormalize(delta_n) (continuous_models.py:244-254; deterministic ignored)."""
        return self._sample(s, a, False)

    def step(self, a):
        """continuous_models.py:225-242: s <- s + denormalised delta; r denormalised; d False."""
        return self._step(a, False)

    def entropy(self, s, a):
        """continuous_models.py:321-323: zeros (logging placeholder)."""
        return np.zeros(np.asarray(s, np.float32).reshape(-1, self.s_dim).shape[0], np.float32)


class GaussianModel(BaseWorldModel):
    """continuous_models.py:7-201: a trainable diagonal logstd [1, S], initialised to
    log(std_mult) (:24-25), trained with the model net by the model optimiser."""
    gaussian = True

    def __init__(self, env, layers, activations, gain, reward_layers, reward_activations, reward_gain,
                 model_setup_kwargs, std_mult, rng=None):
        super().__init__(env, layers, activations, gain, reward_layers, reward_activations, reward_gain,
                         model_setup_kwargs, rng)
        self._logstd = (np.ones((1, self.s_dim)) * np.log(std_mult)).astype(np.float32)

    def _bind(self, engine, net):
        super()._bind(engine, net)
        engine.set_model_logstd(int(net[1]), self._logstd)

    def _get_logstd(self):
        return self._engine.get_model_logstd(int(self._net[1])) if self._engine is not None else self._logstd.copy()

    def get_weights(self):
        """continuous_models.py:81-84: the model net's weights + [logstd]."""
        return self._nn_weights() + [self._get_logstd()]

    def set_weights(self, weights, from_flat=False, increment=False):
        """continuous_models.py:86-99."""
        w = self._unflat(weights, from_flat, increment)
        self._set_nn_weights(w[:-1])
        self._logstd = np.asarray(w[-1], np.float32).reshape(1, self.s_dim)
        if self._engine is not None:
            self._engine.set_model_logstd(int(self._net[1]), self._logstd)

    def sample(self, s, a, deterministic=False):
        """continuous_models.py:56-70: delta_n (+ exp(logstd) * u unless deterministic, u =
        np.random.normal(size=(n, S)) from the device stream), then s + denormalised delta."""
        return self._sample(s, a, not deterministic)

    def step(self, a):
        """continuous_models.py:36-54: always noisy."""
        return self._step(a, True)

    def entropy(self, s, a):
        """continuous_models.py:162-166: 0.5 sum(2 logstd + log 2 pi + 1) per row."""
        l = self._get_logstd().astype(np.float32)
        ent = np.float32(0.5) * np.sum(np.float32(2) * l + np.float32(_LOG2PI_F32) + np.float32(1), dtype=np.float32)
        return np.full(np.asarray(s, np.float32).reshape(-1, self.s_dim).shape[0], ent, np.float32)
