"""init_actor (reference ``sac_eo/actors/init_actor.py:8-30``)."""
from .continuous_actors import GaussianActor, SquashedGaussianActor


def init_actor(env, actor_layers, actor_activations, actor_gain, actor_std_mult, actor_init_type, actor_layer_norm,
               actor_weights, actor_per_state_std=False, actor_squash=False, actor_output_norm=False, **unused):
    """Builds the actor: the squashed Gaussian with ``actor_squash`` (the SAC learner), else the
    plain Gaussian (an imported expert: inference only).  The SoftMax actor (Discrete spaces)
    belongs to the on-policy path, which is out of scope here."""
    if not hasattr(env.action_space, "low"):
        raise TypeError("Only Box action spaces are supported by the SAC path")
    cls = SquashedGaussianActor if actor_squash else GaussianActor
    actor = cls(env, actor_layers, actor_activations, actor_gain, actor_init_type, actor_layer_norm, actor_std_mult,
                actor_per_state_std, actor_output_norm)
    if actor_weights is not None:
        actor.set_weights(actor_weights)
    return actor
