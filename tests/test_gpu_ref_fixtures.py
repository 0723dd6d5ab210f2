"""The device ring, sampler gather and world-model rollout against vectors the REFERENCE's own
code produced (tests/golden/make_ref_fixtures.py): TrajectoryBuffer.add / get_offmodel_info
(buffers.py:41-71, :126-144) and batch_simtrajectory_sampler (samplers.py:73-122).
Bit for bit for the ring, the sampled rows and the RNG stream; the rollout's float trajectories
within 1e-4 relative (fp32 device vs the fp64 oracle objects that drove the reference sampler)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def F():
    with np.load(os.path.join(GOLD, "ref_fixtures.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def M():
    with open(os.path.join(GOLD, "ref_fixtures.json")) as fh:
        return json.load(fh)


def _filled_engine(F, M):
    from sac_eo.engine import Engine, EngineConfig
    B = M["buf"]
    eng = Engine(EngineConfig(s_dim=B["S"], a_dim=B["A"], hidden=(64, 64), activation="tanh", batch=B["B"],
                              buffer_capacity=B["cap"], graph_steps=1))
    for i, _n in enumerate(B["lens"]):
        eng.append(*(F[f"buf.add{i}.{k}"] for k in ("s", "a", "r", "sp", "d")))     # host rows, as the loops add
        assert eng.ctl()["cur_size"] == F["buf.sizes"][i][0]
    return eng


def test_device_ring_equals_trajectory_buffer(gpu_available, F, M):
    """After the same adds (crossing buffer_size): the ring's logical rows == s_all / a_all /
    sp_all and f32(r_all) / f32(d_all) (the reference keeps r and d as float64)."""
    B = M["buf"]
    S, A, cap = B["S"], B["A"], B["cap"]
    eng = _filled_engine(F, M)
    c = eng.ctl()
    rep = eng.v["replay"].cpu().numpy()
    phys = (c["start"] + np.arange(c["cur_size"])) % cap
    assert np.array_equal(rep[phys, 0:S], F["buf.s_all"])
    assert np.array_equal(rep[phys, S:S + A], F["buf.a_all"])
    assert np.array_equal(rep[phys, S + A:2 * S + A], F["buf.sp_all"])
    assert np.array_equal(rep[phys, 2 * S + A], F["buf.r_all"].astype(np.float32))
    assert np.array_equal(rep[phys, 2 * S + A + 1], F["buf.d_all"].astype(np.float32))
    eng.close()


@pytest.mark.parametrize("normalizers", ["identity", "updated"])
def test_sampler_gather_equals_get_offmodel_info(gpu_available, F, M, normalizers):
    """np.random.seed(k); get_offmodel_info(256) on the reference buffer == the device sampler's
    first draw of an update from the same stream state, gathered into the update's input slabs
    (normalised with RunningNormalizer.normalize when the normalisers are not the identity)."""
    from sac_eo.common.normalizer import RunningNormalizers
    B = M["buf"]
    S, A, Bn = B["S"], B["A"], B["B"]
    eng = _filled_engine(F, M)
    nr = RunningNormalizers(S, A, 0.99)
    if normalizers == "updated":
        nr.update_rms(*(F[f"buf.add3.{k}"] for k in ("s", "a", "r", "sp")))
        nr.push_to(eng, which="main")
    for seed in B["seeds"]:
        eng.rng_set_state(np.random.RandomState(seed).get_state())
        eng.step(1, eager=True)
        eng.sync()
        s, a, sp = (F[f"buf.sample{seed}.{k}"] for k in ("s", "a", "sp"))
        xq = eng.v["slot0.Xq"].cpu().numpy()
        xa = eng.v["slot0.Xa"].cpu().numpy()
        assert np.array_equal(xq[:Bn, :S], nr.s_rms.normalize(s)), seed
        assert np.array_equal(xq[:Bn, S:S + A], nr.a_rms.normalize(a)), seed
        assert np.array_equal(xa[:Bn, :S], nr.s_rms.normalize(sp)), seed            # target rows: sp
        assert np.array_equal(xa[Bn:2 * Bn, :S], nr.s_rms.normalize(s)), seed       # policy rows: s
        assert np.array_equal(eng.v["slot0.r"].cpu().numpy()[0, :Bn], F[f"buf.sample{seed}.r"].astype(np.float32))
        assert np.array_equal(eng.v["slot0.d"].cpu().numpy()[0, :Bn], F[f"buf.sample{seed}.d"].astype(np.float32))
    eng.close()


@pytest.mark.parametrize("j", range(3))
def test_rollout_equals_batch_simtrajectory_sampler(gpu_available, F, M, j):
    """sacx_rollout on the weights that drove the reference's batch_simtrajectory_sampler: the
    trajectories within 1e-4 relative, the global stream after the rollout bit-exact."""
    import sac_oracle as O
    from sac_eo.engine import Engine, EngineConfig
    c = M["samplers"]["roll_cases"][j]
    cfg = O.Config(S=17, A=6, hidden=(32, 32), act="tanh", B=8, model_hidden=(64, 64))
    st = O.init_state(cfg, seed=c["seed"], with_models=True, bias_scale=0.05, actor_gain=0.5, model_gain=0.3)
    eng = Engine(EngineConfig(s_dim=17, a_dim=6, hidden=(32, 32), activation="tanh", batch=8, buffer_capacity=16,
                              use_expert=True, model_hidden=(64, 64), graph_steps=1))
    eng.set_net("actor", st.actor)
    eng.set_logstd(st.logstd)
    for k in range(2):
        eng.set_net(f"m{k}", st.models[k])
    eng.rng_set_state(np.random.RandomState(600 + j).get_state())
    got = [t.cpu().numpy() for t in eng.rollout(1, F[f"roll{j}.s_init"], c["H"], c["det"])]
    for g, k in zip(got, ("s", "a", "r", "sp", "d")):
        ref = F[f"roll{j}.{k}"]
        assert g.shape == ref.shape, (k, g.shape, ref.shape)
        if k == "d":
            assert np.array_equal(g.astype(bool), ref)
        else:
            err = np.max(np.abs(g - ref)) / max(np.max(np.abs(ref)), 1e-30)
            assert err < 1e-4, (k, err)
    rs = np.random.RandomState()
    rs.set_state(eng.rng_get_state())
    assert np.array_equal(rs.randint(2 ** 31, size=4), F[f"roll{j}.after"])
    eng.close()
