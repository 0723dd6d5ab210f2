"""Host-side weight containers mirroring sac_eo/common/nn_utils.py:86-138.

Keras Dense weights are (in, out) kernels plus a bias; ``create_nn`` builds
in -> hidden... -> out with Orthogonal(sqrt 2) hidden initialisers and
Orthogonal(gain) on the final layer, zero biases (nn_utils.py:24-57).  TF's
initializer RNG cannot be reproduced without TF, so the same algorithm (QR of
a Gaussian matrix, sign-corrected) runs on a NumPy generator seeded from the
run's setup seed.
"""
from __future__ import annotations

import math
from typing import List, Sequence

import numpy as np


def orthogonal(rng: np.random.Generator, shape, gain: float) -> np.ndarray:
    rows, cols = int(np.prod(shape[:-1])), int(shape[-1])
    flat = (rows, cols) if rows >= cols else (cols, rows)
    a = rng.standard_normal(flat)
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    if rows < cols:
        q = q.T
    return (gain * q).reshape(shape).astype(np.float32)


def create_nn_weights(rng: np.random.Generator, in_dim: int, out_dim: int, layers: Sequence[int],
                      gain: float, layer_norm: bool = False) -> List[np.ndarray]:
    """Keras get_weights() list [W0, b0, ..., W_L, b_L] of create_nn(...); with layer_norm the
    LayerNormalization's [gamma (ones), beta (zeros)] follow b0 (nn_utils.py:110-119)."""
    dims = [in_dim] + list(layers) + [out_dim]
    out = []
    for l in range(len(dims) - 1):
        g = math.sqrt(2.0) if l < len(dims) - 2 else gain
        out.append(orthogonal(rng, (dims[l], dims[l + 1]), g))
        out.append(np.zeros(dims[l + 1], np.float32))
        if l == 0 and layer_norm:
            out += [np.ones(dims[1], np.float32), np.zeros(dims[1], np.float32)]
    return out
