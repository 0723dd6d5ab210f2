"""Variants of the update orchestration (A13) against the fp64 oracle.

* ``target_update_int`` 2 and 3: the Polyak sync runs only when ``num_timesteps %
  target_update_int == 0`` (sac_eo/algs/SAC_expert.py:475-477, SAC.py:248-250); the
  device gate is the dW + Adam epilogue's (csrc/k_sac.hip, ``polyak = nts % tui == 0``).
* ``SAC.train``'s G updates at ONE ``num_timesteps`` (SAC.py:345-348: ``ts_increment`` 0):
  every one of the G updates sees the same gate.
Targets and losses are compared after every call; the target nets are the quantity the
gate changes, so a wrong gate shows as an O(tau) difference at once.
"""
import numpy as np
import pytest

import sac_oracle as O
from helpers import make_pair, oracle_step, relerr

pytestmark = pytest.mark.gpu


def _targets_err(eng, st):
    return max(relerr(a, b) for k in range(2) for a, b in zip(eng.get_net(f"t{k}"), st.q_targ[k]))


def _run(eng, ocfg, st, nrm, buf, calls, B, use_expert=False, expert=None):
    """calls: [(num_timesteps, n_updates, ts_increment)]; compares after every call."""
    N = buf["r"].shape[0]
    rs = np.random.RandomState(44)
    gen = np.random.default_rng(8)
    eng.rng_set_state(rs.get_state())
    ref, worst_t = [], 0.0
    tui = eng.cfg.target_update_int
    for (t0, n, inc) in calls:
        Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen) for _ in range(n)]
        if use_expert:
            eng.push_perms(np.stack([R["perm"] for R in Rs]))
        eng.step(n, num_timesteps=t0, ts_increment=inc)
        for i, R in enumerate(Rs):
            ts = t0 + i * inc
            n_ = [O.f32_noise(R[k]) for k in ("noise_t", "noise_pi", "noise_alpha")]
            ex = None
            if use_expert:
                sec = R["sections"]
                ex = O.Expert(expert["s"][sec[0]], expert["sp"][sec[0]], expert["s"][sec[1]], expert["sp"][sec[1]],
                              O.f32_noise(R["noise_e1"]), O.f32_noise(R["noise_e2"]), ocfg.epsilon)
            o = O.sac_update(st, ocfg, nrm, O.gather(buf, R["idx"]), *n_, expert=ex, do_polyak=(ts % tui == 0))
            ref.append([o["q1_loss"], o["q2_loss"], o["p_loss"]])
        eng.sync()
        worst_t = max(worst_t, _targets_err(eng, st))
    dev = eng.stats(len(ref))[:, :3]
    ref = np.array(ref)
    return relerr(dev, ref), worst_t, eng.ctl()["num_timesteps"]


@pytest.mark.parametrize("tui", [2, 3])
def test_target_update_int(gpu_available, tui):
    B = 128
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=B, seed=31, target_update_int=tui, graph_steps=8)
    # num_timesteps 5.. advancing by one per update: the gate opens on every tui-th update
    calls = [(5, 7, 1), (12, 6, 1), (18, 1, 1), (19, 9, 1)]
    loss_err, targ_err, nts = _run(eng, ocfg, st, nrm, buf, calls, B)
    print(f"target_update_int {tui}: losses {loss_err:.2e}, targets {targ_err:.2e}")
    assert loss_err < 1e-4 and targ_err < 1e-4, (loss_err, targ_err)
    assert nts == 28
    eng.close()


@pytest.mark.parametrize("tui,use_expert", [(1, False), (2, False), (3, True)])
def test_G_updates_at_one_timestep(gpu_available, tui, use_expert):
    """SAC.train: G = 3 updates with num_timesteps fixed (ts_increment = 0) every
    real_step_mod = 3 environment steps; the gate is the same for all three."""
    B = 128
    eng, ocfg, st, buf, nrm, expert = make_pair(act="tanh", B=B, seed=32, target_update_int=tui,
                                                use_expert=use_expert, graph_steps=8)
    calls = [(t, 3, 0) for t in range(0, 24, 3)]          # episode steps 0, 3, 6, ... (SAC.py:345)
    loss_err, targ_err, nts = _run(eng, ocfg, st, nrm, buf, calls, B, use_expert, expert)
    print(f"G=3 at one timestep, target_update_int {tui}: losses {loss_err:.2e}, targets {targ_err:.2e}")
    assert loss_err < 1e-4 and targ_err < 1e-4, (loss_err, targ_err)
    assert nts == 21                                       # ts_increment 0: num_timesteps stays at the call's
    eng.close()
