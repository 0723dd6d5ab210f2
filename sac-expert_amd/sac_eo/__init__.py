"""sac_eo -- MI355X-native SAC / SAC-EO (noc-lab/sac-expert API, HIP engine).

The reference's entry point and construction API are mirrored by the
sub-packages (actors, critics, models, algs, train); the update itself runs in
libsacx (sac-expert_amd/csrc) through ``sac_eo.engine``.
"""
__all__ = ["engine"]
