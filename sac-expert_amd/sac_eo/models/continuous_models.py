"""MSEModel (reference ``sac_eo/models/continuous_models.py:205-319`` over
``sac_eo/models/base_world_model.py:7-138``).

Predicts [normalised delta-s | normalised r] from [norm s | norm a].  Fitted on the device
by ``sacx_model_fit`` and used by the SAC-EO expert term inside the update.  Once an
algorithm binds the model to its engine (``m0`` / ``m1``), ``get_weights`` /
``set_weights`` go through the engine's arena and ``_forward`` / ``sample`` / ``step`` /
``get_loss`` run on the GPU (``sacx_model_forward``, ``sacx_model_loss``).  There is no
CPU execution path."""
import numpy as np

from ..actors.continuous_actors import _as_out
from ..nets import create_nn_weights


class MSEModel:
    def __init__(self, env, layers, activations, gain, reward_layers, reward_activations, reward_gain,
                 model_setup_kwargs, rng=None):
        self.s_dim = int(np.prod(env.observation_space.shape))
        self.a_dim = int(np.prod(env.action_space.shape))
        k = model_setup_kwargs
        if k.get("separate_reward_nn"):
            raise NotImplementedError("separate_reward_nn is not built (off by default)")
        self.separate_reward_nn = False
        self.reward_loss_coef = k.get("reward_loss_coef", 1.0)
        self.scale_model_loss = k.get("scale_model_loss", False)
        # base_world_model.py:54-58 (None = off)
        self.delta_clip_loss = k.get("delta_clip_loss")
        self.reward_clip_loss = k.get("reward_clip_loss")
        self.delta_clip_pred = k.get("delta_clip_pred")
        self.reward_clip_pred = k.get("reward_clip_pred")
        self.layers = list(layers)
        self.activations = list(activations)
        self.activation = self.activations[0]
        rng = rng if rng is not None else np.random.default_rng(np.random.randint(2 ** 31))
        self._w = create_nn_weights(rng, self.s_dim + self.a_dim, self.s_dim + 1, self.layers, gain)
        self._engine = None
        self._net = None
        self.s = None

    def _bind(self, engine, net):
        engine.set_net(net, self._w)
        self._engine, self._net = engine, net

    def _require(self):
        if self._engine is None:
            raise RuntimeError("model is not bound to a device engine (build the algorithm first)")
        return self._engine, int(self._net[1])

    @property
    def trainable(self):
        return self.get_weights()

    def get_weights(self):
        return self._engine.get_net(self._net) if self._engine is not None else [x.copy() for x in self._w]

    def set_weights(self, weights, from_flat=False, increment=False):
        """continuous_models.py:269-278: a weight list, or a flat vector (from_flat), optionally
        added to the current weights (increment)."""
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
        self._w = weights
        if self._engine is not None:
            self._engine.set_net(self._net, self._w)

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

    def sample(self, s, a, deterministic=True):
        """s + delta_rms.denormalize(delta_n) (continuous_models.py:244-254)."""
        eng, k = self._require()
        s2, a2 = self._rows(s, a)
        _, sp, _ = eng.model_forward(k, s2, a2, self.delta_clip_pred or 0.0, self.reward_clip_pred or 0.0)
        sp = sp.cpu().numpy()
        return _as_out(sp.reshape(np.shape(s)) if np.ndim(s) == 1 else sp)

    def reset(self, s):
        """continuous_models.py:256-259."""
        self.s = s
        return s

    def step(self, a):
        """continuous_models.py:225-242: s <- s + denormalised delta; r denormalised; d False."""
        eng, k = self._require()
        s2, a2 = self._rows(self.s, a)
        _, sp, r = eng.model_forward(k, s2, a2, self.delta_clip_pred or 0.0, self.reward_clip_pred or 0.0)
        sp, r = sp.cpu().numpy(), r.cpu().numpy()
        if sp.shape[0] == 1:                 # tf.squeeze of one row
            sp, r = sp[0] if np.ndim(self.s) == 1 else sp, r[0]
        self.s = sp
        d = np.zeros(np.shape(r), bool) if np.ndim(r) else False
        return self.s, r, d, {}

    def get_loss(self, s, sp, a, r):
        """mean_i 0.5||norm(sp - s) - delta_pred||^2 + reward_loss_coef * 0.5 (norm(r) - r_pred)^2
        with the optional loss clips (continuous_models.py:280-302)."""
        eng, k = self._require()
        s2, a2 = self._rows(s, a)
        sp2 = np.asarray(sp, np.float32).reshape(-1, self.s_dim)
        r2 = np.asarray(r, np.float32).reshape(-1)
        return eng.model_loss(k, s2, sp2, a2, r2, self.delta_clip_loss or 0.0, self.reward_clip_loss or 0.0)
