"""Import shim: ``python -m sac_eo.train`` / ``import sac_eo`` from the repo root
resolve to the package in sac-expert_amd/sac_eo."""
import os as _os

_real = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), "sac-expert_amd", "sac_eo")
__path__ = [_real]
with open(_os.path.join(_real, "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(_real, "__init__.py"), "exec"))
