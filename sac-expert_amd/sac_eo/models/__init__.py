from .continuous_models import MSEModel
from .init_world_models import init_world_models

__all__ = ["MSEModel", "init_world_models"]
