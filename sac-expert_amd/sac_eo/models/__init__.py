from .continuous_models import GaussianModel, MSEModel
from .init_world_models import init_world_models

__all__ = ["GaussianModel", "MSEModel", "init_world_models"]
