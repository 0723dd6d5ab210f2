"""init_critics (reference ``sac_eo/critics/init_critic.py:5-38``)."""
from .critics import QCritic, VCritic


def init_critics(env, critic_layers, critic_activations, critic_gain, critic_weights, num_models, critic_ensemble,
                 critic_init_type, critic_layer_norm, **unused):
    """Returns (critics, q_targets, q_critics); the targets start as copies of the critics.
    critic_init_type / critic_layer_norm are accepted and ignored, as in the reference
    (init_critic.py:5-6, critics.py:74 never pass them on)."""
    num_critics = num_models if critic_ensemble else 1
    critics = []
    for idx in range(num_critics):
        c = VCritic(env, critic_layers, critic_activations, critic_gain)
        if critic_weights is not None:
            c.set_weights(critic_weights[idx])
        critics.append(c)
    q_critics = [QCritic(env, critic_layers, critic_activations, critic_gain) for _ in range(2)]
    q_targets = [QCritic(env, critic_layers, critic_activations, critic_gain) for _ in range(2)]
    for t, q in zip(q_targets, q_critics):
        t.set_weights(q.get_weights())
    return critics, q_targets, q_critics
