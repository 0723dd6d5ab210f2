"""Host-side helpers mirroring sac_eo/common of the reference (parser, seeding, replicas)."""
