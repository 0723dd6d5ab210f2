from .continuous_actors import SquashedGaussianActor
from .init_actor import init_actor

__all__ = ["SquashedGaussianActor", "init_actor"]
