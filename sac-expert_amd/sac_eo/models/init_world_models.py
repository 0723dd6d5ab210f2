"""init_world_models (reference ``sac_eo/models/init_world_models.py:5-29``)."""
from .continuous_models import GaussianModel, MSEModel


def init_world_models(env, model_layers, model_activations, model_gain, model_std_mult, model_weights,
                      reward_layers, reward_activations, reward_gain, reward_weights, num_models, gaussian_model,
                      model_setup_kwargs, **unused):
    models = []
    for idx in range(num_models):
        if gaussian_model:
            m = GaussianModel(env, model_layers, model_activations, model_gain, reward_layers, reward_activations,
                              reward_gain, model_setup_kwargs, model_std_mult)
        else:
            m = MSEModel(env, model_layers, model_activations, model_gain, reward_layers, reward_activations,
                         reward_gain, model_setup_kwargs)
        if model_weights is not None:
            m.set_weights(model_weights[idx])
        if reward_weights is not None:
            m.set_reward_weights(reward_weights[idx])
        models.append(m)
    return models
