from .continuous_actors import GaussianActor, SquashedGaussianActor
from .init_actor import init_actor

__all__ = ["GaussianActor", "SquashedGaussianActor", "init_actor"]
