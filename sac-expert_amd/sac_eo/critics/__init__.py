from .critics import QCritic, VCritic
from .init_critic import init_critics

__all__ = ["QCritic", "VCritic", "init_critics"]
