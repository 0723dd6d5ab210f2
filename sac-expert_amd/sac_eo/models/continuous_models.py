"""MSEModel weight holder (reference ``sac_eo/models/continuous_models.py:205-319``).

Predicts [normalised delta-s | normalised r] from [norm s | norm a]; fitted on the
device by ``sacx_model_fit`` and used by the SAC-EO expert term inside the update."""
import numpy as np

from ..nets import create_nn_weights


class MSEModel:
    def __init__(self, env, layers, activations, gain, reward_layers, reward_activations, reward_gain,
                 model_setup_kwargs, rng=None):
        s = int(np.prod(env.observation_space.shape))
        a = int(np.prod(env.action_space.shape))
        if model_setup_kwargs.get("separate_reward_nn"):
            raise NotImplementedError("separate_reward_nn is not built (off by default)")
        for k in ("delta_clip_loss", "reward_clip_loss", "delta_clip_pred", "reward_clip_pred"):
            if model_setup_kwargs.get(k) is not None:
                raise NotImplementedError(f"{k} is not built (None by default)")
        self.layers = list(layers)
        self.activation = list(activations)[0]
        self.reward_loss_coef = model_setup_kwargs.get("reward_loss_coef", 1.0)
        rng = rng if rng is not None else np.random.default_rng(np.random.randint(2 ** 31))
        self._w = create_nn_weights(rng, s + a, s + 1, self.layers, gain)
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
        self.s_rms, self.a_rms, self.r_rms, self.delta_rms, _ = normalizer.get_rms()
