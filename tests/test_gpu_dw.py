"""dW + Adam tilings: the 16x16 k_gemm tiles, 32x32 tiles for launches past one round of
residency (SACX_DW_ROUND) and k_dwl (LDS-DMA staged rows, SACX_DWL; 32x16 or 32x32 tiles,
SACX_DWL_NH) keep gemm_core's
summation order, so a learner ends bit-identical whichever the plan takes (stats, every
parameter / Adam / target value).  B = 128 runs k_dwl's short path (2 slabs per wave, fewer
than its stages); B = 1024 its steady-state pipeline."""
import numpy as np
import pytest

from helpers import load_learner, make_learner

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant", ["dwl32x16", "dwl32x32", "round"])
@pytest.mark.parametrize("B", [128, 1024])
@pytest.mark.parametrize("bf16", [False, True])
@pytest.mark.parametrize("use_expert", [False, True])
def test_dw_tilings_bit_identical(monkeypatch, variant, B, bf16, use_expert):
    from sac_eo.engine import Engine, EngineConfig
    n, N, eps = 11, 5000, 0.1
    monkeypatch.setenv("SACX_FUSE_HEAD", "0")       # critic.adam without rows riding along (k_dwl takes it)
    _, st, buf, nrm, ex = make_learner(act="relu", B=B, N=N, seed=3, use_expert=use_expert, epsilon=eps)

    def run(env):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        e = Engine(EngineConfig(s_dim=17, a_dim=6, activation="relu", batch=B, buffer_capacity=N,
                                use_expert=use_expert, expert_capacity=20, expert_batch=20, graph_steps=8,
                                epsilon=eps, gemm_bf16=bf16))
        for k in env:
            monkeypatch.delenv(k)
        load_learner(e, st, buf, nrm, ex, eps)
        e.rng_set_state(np.random.RandomState(77).get_state())
        if use_expert:
            rs = np.random.RandomState(78)
            e.push_perms(np.stack([rs.permutation(20) for _ in range(n)]))
        e.step(n)
        e.sync()
        out = (e.stats(n).copy(), e.v["params"].cpu().numpy().copy(), e.v["adam_m"].cpu().numpy().copy(),
               e.v["adam_v"].cpu().numpy().copy())     # params holds the target nets too
        e.close()
        return out

    ref = run({"SACX_DWL": "0", "SACX_DW_ROUND": "100000000"})
    if variant.startswith("dwl"):
        got = run({"SACX_DWL": "2", "SACX_DWL_NH": "1" if variant == "dwl32x16" else "2"})
    else:
        got = run({"SACX_DWL": "0", "SACX_DW_ROUND": "1"})
    assert np.all(np.isfinite(ref[0]))
    for i, (a, b) in enumerate(zip(got, ref)):
        assert np.array_equal(a, b), (variant, i, int(np.sum(a != b)))
