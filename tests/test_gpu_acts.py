"""Per-net, per-layer hidden activations on the device (the reference's
--actor_activations / --critic_activations lists, nn_utils.py:5-22 create_activations): the
actor and the critics may differ, and each hidden layer may differ from the other.  One update
per stage and a 60-update graph trajectory vs the oracle, graph == eager bit for bit."""
import numpy as np
import pytest

import sac_oracle as O
from helpers import make_pair, oracle_step

pytestmark = pytest.mark.gpu

CASES = [(("tanh", "relu"), ("relu", "elu"), False), (("elu", "elu"), ("tanh", "relu"), True),
         (("relu", "tanh"), ("relu", "relu"), True)]


@pytest.mark.parametrize("actor_acts,critic_acts,layer_norm", CASES)
def test_mixed_activations(gpu_available, actor_acts, critic_acts, layer_norm):
    B, steps = 128, 60
    outs = []
    for eager in (False, True):
        eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=29, use_expert=True, done_p=0.01,
                                                    graph_steps=128, actor_acts=actor_acts, critic_acts=critic_acts,
                                                    layer_norm=layer_norm, normalizers="random")
        N = buf["r"].shape[0]
        rs = np.random.RandomState(97)
        gen = np.random.default_rng(98)
        eng.rng_set_state(rs.get_state())
        Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20, gen=gen) for _ in range(steps)]
        eng.push_perms(np.stack([R["perm"] for R in Rs]))
        eng.step(steps, eager=eager)
        eng.sync()
        outs.append((eng.stats(steps).copy(), eng.v["params"].cpu().numpy().copy()))
        eng.close()
    ref = np.array([[o["q1_loss"], o["q2_loss"], o["p_loss"]] for o in (oracle_step(st, ocfg, nrm, buf, R, expert)
                                                                        for R in Rs)])
    dev = outs[0][0]
    assert np.max(np.abs(dev[:, :2] - ref[:, :2]) / np.abs(ref[:, :2])) < 1e-4
    assert np.max(np.abs(dev[:, 2] - ref[:, 2])) / np.max(np.abs(ref[:, 2])) < 1e-4
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
