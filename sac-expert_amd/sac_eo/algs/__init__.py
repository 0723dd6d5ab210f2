from .init_alg import init_alg
from .SAC import SAC
from .SAC_expert import SAC_exp

__all__ = ["init_alg", "SAC", "SAC_exp"]
