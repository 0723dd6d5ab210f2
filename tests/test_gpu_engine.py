"""Device parity tests: the HIP engine (through the C ABI) against the CPU
oracle on identical seeded inputs.  Run on the MI355X box (-m gpu).

Tolerances (fp32 device vs fp64 oracle):
  * sampler indices: bit-exact; noise: bit-exact after the f64->f32 cast
  * per-stage activations / losses: 2e-5 relative to the tensor's max
  * gradients (read back through Adam's first moment): 2e-4 relative to max
  * Q-loss trajectory over 100 updates: 1e-4 relative (BASELINE.json north_star)
"""
import numpy as np
import pytest

import sac_oracle as O
from helpers import B1, load_learner, make_learner, make_pair, oracle_step, relerr

pytestmark = pytest.mark.gpu


def _draw(seed, N, B, A, ne=0):
    rs = np.random.RandomState(seed)
    gen = np.random.default_rng(seed + 7) if ne else None
    return rs, gen


def test_rng_matches_numpy(gpu_available):
    eng, ocfg, st, buf, nrm, _ = make_pair(S=5, A=3, hidden=(32, 32), B=37, N=777)
    for seed in (0, 2590541744, 12345):
        rs = np.random.RandomState(seed)
        rs.normal(size=1)                                    # leave a cached gaussian (has_gauss)
        eng.rng_set_state(rs.get_state())
        for _ in range(3):
            eng.step(1, eager=True)
            eng.sync()
            idx = rs.randint(777, size=37)
            noise = rs.normal(size=(3 * 37 * 3,))
            assert np.array_equal(eng.v["slot0.idx"][0].cpu().numpy(), idx)
            assert np.array_equal(eng.v["slot0.noise"][0].cpu().numpy(), noise.astype(np.float32))
        got = eng.rng_get_state()
        ref = rs.get_state()
        assert np.array_equal(got[1], ref[1]) and got[2] == ref[2] and got[3] == ref[3] and got[4] == ref[4]
    eng.close()


def test_rng_big_draws(gpu_available):
    """Many twists per update (B*A large) and a near-power-of-two bound."""
    eng, *_ = make_pair(S=4, A=17, hidden=(16, 16), B=1024, N=(1 << 20) + 3)
    rs = np.random.RandomState(99)
    eng.rng_set_state(rs.get_state())
    eng.step(2, eager=True)
    eng.sync()
    for _ in range(2):
        idx = rs.randint((1 << 20) + 3, size=1024)
        nz = rs.normal(size=3 * 1024 * 17).astype(np.float32)
    assert np.array_equal(eng.v["slot0.idx"][0].cpu().numpy(), idx)
    assert np.array_equal(eng.v["slot0.noise"][0].cpu().numpy(), nz)
    eng.close()


@pytest.mark.parametrize("mode", ["segmented", "fallback", "k_rng"])
def test_rng_segmented_batches(gpu_available, monkeypatch, mode):
    """Humanoid-sized draws (~135k MT words per update) take the segmented sampler (k_mtj_*:
    jumped-ahead segments, flag / prefix / resolve / emit over the GPU).  Over a captured graph
    (two batches of 4 updates after a cached gaussian) and then eager updates, the draws and the
    final state equal NumPy's stream -- on the segmented path, on its fallback (forced: one
    segment, too few words, rng_body redraws the batch) and on the one-workgroup k_rng."""
    if mode == "fallback":
        monkeypatch.setenv("SACX_MTJ_UNDER", "1")
    if mode == "k_rng":
        monkeypatch.setenv("SACX_RNG_JUMP", "0")
    S, A, B, N = 4, 17, 1024, (1 << 20) + 3
    eng, *_ = make_pair(S=S, A=A, hidden=(16, 16), B=B, N=N, graph_steps=8)
    rs = np.random.RandomState(2024)
    rs.normal(size=1)                                    # a cached gaussian (has_gauss)
    eng.rng_set_state(rs.get_state())
    eng.step(8)
    eng.sync()
    ctl = eng.v["ctl"][0].cpu().numpy()
    seq0 = int(ctl[6]) - 8                               # step_seq before the call
    for u in range(8):
        idx = rs.randint(N, size=B)
        nz = rs.normal(size=3 * B * A).astype(np.float32)
        slots = [k for k in range(8) if int(ctl[16 + k]) == seq0 + u]
        assert len(slots) == 1, (u, ctl[16:24])
        k = slots[0]
        assert np.array_equal(eng.v[f"slot{k}.idx"][0].cpu().numpy(), idx), (mode, u)
        assert np.array_equal(eng.v[f"slot{k}.noise"][0].cpu().numpy(), nz), (mode, u)
    rs.normal(size=3)                                    # an odd draw: the next update starts cached
    eng.rng_set_state(rs.get_state())
    for _ in range(2):
        eng.step(1, eager=True)
        eng.sync()
        idx = rs.randint(N, size=B)
        nz = rs.normal(size=3 * B * A).astype(np.float32)
        assert np.array_equal(eng.v["slot0.idx"][0].cpu().numpy(), idx), mode
        assert np.array_equal(eng.v["slot0.noise"][0].cpu().numpy(), nz), mode
    got, ref = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(got[1], ref[1]) and got[2] == ref[2] and got[3] == ref[3] and got[4] == ref[4]
    eng.close()


@pytest.mark.parametrize("host", [True, False])
def test_replay_ring_fifo(gpu_available, host):
    """TrajectoryBuffer.add truncation (buffers.py:60-66) on the device ring, from host rows
    (sacx_buffer_append_host: pinned staging, chunked at 64 Ki floats -- the 7000-row add
    spans two chunks) and from device rows (sacx_buffer_append)."""
    import torch
    from sac_eo.engine import Engine, EngineConfig
    eng = Engine(EngineConfig(s_dim=3, a_dim=2, hidden=(16, 16), batch=4, buffer_capacity=10))
    rs = np.random.RandomState(0)
    ref = {k: np.zeros((0,) + sh, np.float32) for k, sh in (("s", (3,)), ("a", (2,)), ("r", ()), ("sp", (3,)), ("d", ()))}
    for n in (4, 5, 3, 12, 1, 7000, 2):
        rows = dict(s=rs.normal(size=(n, 3)), a=rs.normal(size=(n, 2)), r=rs.normal(size=n),
                    sp=rs.normal(size=(n, 3)), d=(rs.uniform(size=n) < .5).astype(np.float64))
        args = [rows[k] for k in ("s", "a", "r", "sp", "d")]
        if not host:
            args = [torch.as_tensor(x, dtype=torch.float32, device=eng.device) for x in args]
        eng.append(*args)
        for k in ref:
            ref[k] = np.concatenate([ref[k], rows[k].astype(np.float32)])[-10:]
    c = eng.ctl()
    assert c["cur_size"] == 10
    rep = eng.v["replay"].cpu().numpy()
    phys = (c["start"] + np.arange(10)) % 10
    assert np.array_equal(rep[phys, 0:3], ref["s"])
    assert np.array_equal(rep[phys, 3:5], ref["a"])
    assert np.array_equal(rep[phys, 5:8], ref["sp"])
    assert np.array_equal(rep[phys, 8], ref["r"])
    assert np.array_equal(rep[phys, 9], ref["d"])
    eng.close()


def _one_step_compare(act, normalizers="identity", per_state_std=False, use_expert=False, B=256, seed=0,
                      done_p=0.05, S=17, A=6, hidden=(256, 256)):
    eng, ocfg, st, buf, nrm, expert = make_pair(act=act, normalizers=normalizers, per_state_std=per_state_std,
                                               use_expert=use_expert, B=B, seed=seed, done_p=done_p, S=S, A=A,
                                               hidden=hidden)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(seed + 5)
    gen = np.random.default_rng(seed + 6)
    eng.rng_set_state(rs.get_state())
    R = O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen)
    if use_expert:
        eng.push_perms(R["perm"][None, :])
    keep = {}
    st0 = st.copy()
    stats = oracle_step(st, ocfg, nrm, buf, R, expert, keep)
    eng.step(1, eager=True)
    eng.sync()
    v = {k: t.cpu().numpy() for k, t in eng.v.items()}
    S, A = ocfg.S, ocfg.A
    # sampler: bit-exact
    assert np.array_equal(v["slot0.idx"][0], R["idx"])
    # forward stages
    assert relerr(v["slot0.Xa"][:B, :S], keep["sp_n"]) < 1e-6
    assert relerr(v["ws.Ha1"][:B], keep["actor_h_t"][0]) < 2e-5
    assert relerr(v["ws.Ha2"][B:2 * B], keep["actor_h_p"][1]) < 2e-5
    assert relerr(v["ws.nlp_t"][0], keep["nlp_t"]) < 2e-5
    assert relerr(v["ws.nlp_p"][0], keep["nlp_p"]) < 2e-5
    assert relerr(v["ws.Hq2"][2 * B:3 * B], keep["q0_h"][1]) < 2e-5
    # losses (stats ring)
    row = eng.stats(1)[0]
    for i, k in enumerate(("q1_loss", "q2_loss", "p_loss", "alpha_loss")):
        assert abs(row[i] - stats[k]) <= 2e-5 * abs(stats[k]) + 1e-7, (k, row[i], stats[k])
    assert abs(row[4] - stats["alpha"]) <= 1e-6 * abs(stats["alpha"])
    # gradients through Adam's first moment (m_1 = g * (1 - beta1))
    def grads_of(net):
        m = eng.v["adam_m"][0]
        out = []
        for i in range(3):
            seg = eng.segments[f"{net}.l{i}"]
            off = seg["offset"] // 4
            n = seg["rows"] * seg["cols"]
            w = m[off: off + n].cpu().numpy().reshape(seg["rows"], seg["cols"]) / B1
            out += [w[:-1], w[-1]]
        return out
    for k in range(2):
        for gd, go in zip(grads_of(f"q{k}"), keep[f"q{k}_grads"]):
            assert relerr(gd, go) < 2e-4
    for gd, go in zip(grads_of("actor"), keep["actor_grads"]):
        assert relerr(gd, go) < 2e-4, (relerr(gd, go))
    if not per_state_std:
        seg = eng.segments["actor.logstd"]
        gl = eng.v["adam_m"][0][seg["offset"] // 4: seg["offset"] // 4 + A].cpu().numpy() / B1
        assert relerr(gl, keep["g_logstd"][0]) < 2e-4
    # Polyak: targets = keep*f32(1-tau) + updated q * f32(tau)
    for k in range(2):
        tgt = eng.get_net(f"t{k}")
        for a_, b_ in zip(tgt, st.q_targ[k]):
            assert np.max(np.abs(a_ - b_)) < 1e-5
    eng.close()
    return True


@pytest.mark.parametrize("act", ["relu", "tanh", "elu"])
def test_one_update_matches_oracle(gpu_available, act):
    _one_step_compare(act)


def test_one_update_nontrivial_normalizers(gpu_available):
    _one_step_compare("tanh", normalizers="random", seed=3)


def test_one_update_per_state_std(gpu_available):
    _one_step_compare("relu", per_state_std=True, seed=4)


def test_one_update_sac_eo(gpu_available):
    _one_step_compare("relu", use_expert=True, seed=5)


def test_one_update_odd_draws(gpu_available):
    """A = 1, B = 37: every normal(size=(B, A)) draw is odd, so the legacy gauss cache carries
    a value from one draw into the next (target -> policy -> alpha noise)."""
    _one_step_compare("tanh", B=37, S=3, A=1, seed=7)


def test_one_update_wide_hidden(gpu_available):
    """Hidden 320 / 384: row kernels on 8 registers per lane, the folded head with K = 384."""
    _one_step_compare("relu", hidden=(320, 384), seed=8)


def test_one_update_narrow_hidden(gpu_available):
    """Hidden 100 / 60 (not multiples of 16 or 4): scalar operand loads and the separate
    actor.head launch (the fold needs H1 % 16 == 0)."""
    _one_step_compare("elu", hidden=(100, 60), seed=9)


def test_one_update_unfused_head(gpu_available, monkeypatch):
    """SACX_FUSE_HEAD=0: the standalone actor.head launch path of plain SAC."""
    monkeypatch.setenv("SACX_FUSE_HEAD", "0")
    _one_step_compare("relu", seed=10)


def test_one_update_small_batch(gpu_available):
    _one_step_compare("relu", B=37, seed=6)


def test_one_update_humanoid_shapes(gpu_available):
    """Config C3 shapes (S=376, A=17, B=1024, SAC-EO): wide layer-0 K (unfused forward),
    multi-chunk gather rows and the 47-chunk world-model head."""
    _one_step_compare("relu", use_expert=True, B=1024, seed=7, S=376, A=17, normalizers="random")


@pytest.mark.parametrize("use_expert", [False, True])
def test_qloss_trajectory_100(gpu_available, use_expert):
    """Q-loss trajectory over 100 updates within 1e-4 relative (north_star)."""
    B = 256
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=11, use_expert=use_expert, done_p=0.01)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(123)
    gen = np.random.default_rng(77)
    eng.rng_set_state(rs.get_state())
    steps = 100
    Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen) for _ in range(steps)]
    if use_expert:
        eng.push_perms(np.stack([R["perm"] for R in Rs]))
    eng.step(steps, num_timesteps=0, ts_increment=1)     # graph replay path
    eng.sync()
    dev = eng.stats(steps)
    ref = []
    for R in Rs:
        o = oracle_step(st, ocfg, nrm, buf, R, expert)      # one oracle update per step
        ref.append([o["q1_loss"], o["q2_loss"], o["alpha_loss"]])
    ref = np.array(ref)
    rel = np.abs(dev[:, :2] - ref[:, :2]) / np.abs(ref[:, :2])
    assert rel.max() < 1e-4, rel.max()
    # the alpha loss (-alpha * mean(-nlp + H) over the alpha rows) catches a wrong alpha
    # branch that the Q losses barely see once alpha is clamped at 1e-5
    rel_a = np.abs(dev[:, 3] - ref[:, 2]) / np.abs(ref[:, 2])
    assert rel_a.max() < 1e-3, rel_a.max()
    got = eng.rng_get_state()
    exp = rs.get_state()
    assert np.array_equal(got[1], exp[1]) and got[2] == exp[2]
    eng.close()


@pytest.mark.parametrize("use_expert", [False, True])
def test_graph_equals_eager(gpu_available, use_expert):
    """hipGraph replay (sampler + gather forked ahead on a side stream, alpha.final on a
    third) is bit-identical to eager launches; 19 = two 8-update graphs + 3 single ones."""
    outs = []
    n = 19
    for eager in (True, False):
        eng, ocfg, st, buf, nrm, _ = make_pair(act="tanh", B=128, seed=21, use_expert=use_expert)
        eng.rng_set_state(np.random.RandomState(5).get_state())
        if use_expert:
            rs = np.random.RandomState(8)
            eng.push_perms(np.stack([rs.permutation(eng.cfg.expert_batch) for _ in range(n)]))
        eng.step(n, eager=eager)
        eng.sync()
        outs.append((eng.stats(n).copy(), eng.v["params"].cpu().numpy().copy()))
        eng.close()
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("eager", [True, False])
def test_model_fit_matches_oracle(gpu_available, eager):
    """World-model fitting steps (mbrl_onpolicy_alg.py:301-319) vs oracle.model_fit_step."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=31, use_expert=True, normalizers="random")
    N = buf["r"].shape[0]
    mb = eng.cfg.model_batch
    rs = np.random.RandomState(9)
    steps = 5
    idx = rs.randint(N, size=(steps, 2, mb))
    eng.model_fit(idx, eager=eager)
    eng.sync()
    dev = eng.model_stats(steps)
    ref = []
    for j in range(steps):
        batches = [(buf["s"][idx[j, k]], buf["a"][idx[j, k]], buf["sp"][idx[j, k]], buf["r"][idx[j, k]])
                   for k in range(2)]
        ref.append(O.model_fit_step(st, ocfg, nrm, batches))
    ref = np.array(ref)
    assert np.max(np.abs(dev - ref) / np.abs(ref)) < 1e-4, (dev, ref)
    for k in range(2):
        for a_, b_ in zip(eng.get_net(f"m{k}"), st.models[k]):
            assert np.max(np.abs(a_ - b_)) < 5e-5
    assert eng.ctl()["t_model"] == steps
    eng.close()


@pytest.mark.parametrize("act,B,eager", [("relu", 256, False), ("tanh", 256, True), ("elu", 100, False)])
def test_fused_forward_pair_bit_identical(gpu_available, monkeypatch, act, B, eager):
    """The two-layer forward pairs as ONE k_fwd2 launch each (both layers per workgroup, layer 0 in
    LDS, SACX_FWD2=1, the default): the policy-loss critics' pair, the actor pair (with the head's
    partial dots), the alpha branch's pair folded into the next update's actor launch, and the
    target / critic pair with the actor-head prologue, the previous update's alpha rows and their
    finalisation by the last alpha block -- the updates equal the k_gemm chain's bit for bit, eager
    and graph."""
    outs = []
    for fused, afin in (("0", "1"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("SACX_FWD2", fused)
        monkeypatch.setenv("SACX_AFIN", afin)     # the folded alpha finalisation: ticket (0) or split (1)
        eng, ocfg, st, buf, nrm, _ = make_pair(act=act, B=B, seed=41, normalizers="random", graph_steps=8)
        names = [L["name"] for L in eng.plan_info()]
        for pair in ("pi.q.fwd01", "actor.fwd01", "alpha.fwd01", "q.fwd01+actor.head"):
            assert (pair in names) == (fused == "1"), names
        eng.rng_set_state(np.random.RandomState(6).get_state())
        eng.step(19, eager=eager)
        # a host write of the weights between calls
        for net in ("actor", "q1", "t0"):
            w = eng.get_net(net)
            w[1] = w[1] * np.float32(0.75)
            eng.set_net(net, w)
        eng.step(6, eager=eager)
        eng.sync()
        outs.append((eng.stats(25).copy(), eng.v["params"].cpu().numpy().copy(), eng.v["adam_v"].cpu().numpy().copy()))
        eng.close()
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("S,A,B,clip", [(17, 6, 256, 0.0), (376, 17, 1024, 0.0), (17, 6, 64, 5.0)])
def test_model_fit_folds_bit_identical(gpu_available, monkeypatch, S, A, B, clip):
    """The folded world-model fit chain (the loss and its gradient in model.fwd2's epilogue,
    k_mfinal as an extra workgroup of model.bwd2: SACX_MFUSE=1; the rows gathered on model.fwd0's
    operand loads: 2; model.bwd2 generated on model.bwd1's operand loads for heads of <= 32
    outputs: 3, the default; the gathered layer 0 and layer 1 as one k_fwd2 launch: SACX_MFWD2=1,
    the default, when S + A <= 32; the fit's own tile shapes: SACX_MTILE=1, the default, or 16x16
    everywhere: 0) leaves the weights and Adam state of the unfolded chain
    (SACX_MFUSE=0, SACX_MTILE=2) bit for bit, eager and graph; the loss statistic sums the
    same squares in another order (<= 1e-6 relative)."""
    outs = []
    steps = 12      # (> 8: a graph block of 8 steps reads pre-gather slots 0 .. 7, then 1-step blocks slot 0)
    for fuse, tile, f2, mt32, pre in (("0", "2", "0", "5", "0"), ("1", "1", "0", "5", "0"), ("2", "1", "0", "5", "0"),
                                      ("2", "1", "1", "5", "0"), ("2", "1", "1", "0", "0"), ("2", "1", "0", "3", "0"),
                                      ("2", "1", "1", "15", "0"), ("2", "1", "0", "15", "0"), ("3", "1", "0", "5", "0"),
                                      ("3", "1", "1", "5", "0"), ("3", "0", "1", "5", "0"),
                                      # SACX_MPRE=1 (default): the rows of a block of steps pre-gathered
                                      ("0", "2", "0", "5", "1"), ("2", "1", "1", "5", "1"), ("2", "1", "0", "5", "1"),
                                      ("2", "1", "1", "15", "1"), ("3", "1", "0", "5", "1")):
        monkeypatch.setenv("SACX_MFUSE", fuse)
        monkeypatch.setenv("SACX_MTILE", tile)
        monkeypatch.setenv("SACX_MFWD2", f2)
        monkeypatch.setenv("SACX_MT32", mt32)
        monkeypatch.setenv("SACX_MPRE", pre)
        eng, ocfg, st, buf, nrm, _ = make_pair(S=S, A=A, B=B, act="tanh", N=3000, seed=33, use_expert=True,
                                               normalizers="random", model_max_grad_norm=clip)
        names = [L["name"] for L in eng.model_plan_info()]
        pair = f2 == "1" and S + A <= 32 and (fuse != "1" if pre == "0" else tile != "2")
        assert (("model.gather+fwd01" if pre == "0" else "model.fwd01") in names) == pair, names
        mb = eng.cfg.model_batch
        idx = np.random.RandomState(4).randint(buf["r"].shape[0], size=(steps, 2, mb))
        eng.model_fit(idx[:3], eager=True)
        eng.model_fit(idx[3:])
        eng.sync()
        P = np.concatenate([eng.v[k].cpu().numpy().ravel() for k in ("params", "adam_m", "adam_v")])
        outs.append((eng.model_stats(steps).copy(), P, eng.ctl()["t_model"]))
        eng.close()
    for o in outs[1:]:
        assert o[2] == outs[0][2] == steps
        assert np.array_equal(o[1], outs[0][1])
        assert np.max(np.abs(o[0] - outs[0][0]) / np.abs(outs[0][0])) < 1e-6, (o[0], outs[0][0])


@pytest.mark.parametrize("deterministic,per_state_std,n,host", [(True, False, 37, False), (False, False, 37, False),
                                                                (False, True, 5, False), (False, False, 1, False),
                                                                (False, False, 1, True), (True, False, 37, True),
                                                                (False, True, 3000, True), (True, True, 16, False),
                                                                (False, False, 16, True), (False, True, 2, True)])
def test_actor_act_matches_oracle(gpu_available, deterministic, per_state_std, n, host):
    """Behaviour-policy inference (sample(), continuous_actors.py:270-306) vs the oracle;
    the stochastic draw advances the device stream exactly as np.random.normal(size=(n, A))."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="tanh", B=64, seed=41, normalizers="random",
                                           per_state_std=per_state_std)
    S, A = ocfg.S, ocfg.A
    obs = np.random.RandomState(3).normal(size=(n, S)) * 2.0
    eng.rng_set_state(np.random.RandomState(17).get_state())
    ref_rs = np.random.RandomState(17)
    if host:    # sacx_actor_act_host: host rows in and out (3000 rows span 3 ACT_CAP chunks)
        got = np.asarray(eng.act_host(obs[0] if n == 1 else obs, deterministic)).reshape(n, A)
    else:
        got = eng.act(obs[0] if n == 1 else obs, deterministic).cpu().numpy().reshape(n, A)
    x = (obs.astype(np.float32) - nrm.s_mean) / nrm.s_den
    out, _ = O.mlp_forward(st.actor, x.astype(np.float64), ocfg.act)
    mu, lraw = O.split_head(out, st.logstd, ocfg)
    u = np.zeros((n, A)) if deterministic else O.f32_noise(ref_rs.normal(size=(n, A))).astype(np.float64)
    pi, _ = O.head_sample(mu, lraw, u, ocfg.act_limit, np.float64)
    assert relerr(got, pi) < 2e-5, relerr(got, pi)
    dev, ref = eng.rng_get_state(), ref_rs.get_state()
    assert np.array_equal(dev[1], ref[1]) and dev[2] == ref[2] and dev[3] == ref[3] and dev[4] == ref[4]
    eng.close()


@pytest.mark.parametrize("S,A,act,per_state_std,n", [(376, 17, "tanh", False, 3), (376, 17, "relu", True, 1),
                                                      (17, 6, "elu", True, 16), (17, 6, "relu", False, 1),
                                                      (17, 6, "tanh", True, 1)])
def test_actor_act_rows_shapes(gpu_available, S, A, act, per_state_std, n):
    """k_act_rows on both of its paths (the prefetching one, S <= 128 and H <= 256; the generic
    one, Humanoid S = 376), stochastic, vs the oracle; the device stream advances as NumPy's;
    repeats from the same stream state give the same action."""
    eng, ocfg, st, buf, nrm, _ = make_pair(S=S, A=A, act=act, B=64, N=500, seed=43, normalizers="random",
                                           per_state_std=per_state_std)
    obs = np.random.RandomState(5).normal(size=(n, S)) * 2.0
    eng.rng_set_state(np.random.RandomState(19).get_state())
    ref_rs = np.random.RandomState(19)
    got = np.asarray(eng.act_host(obs[0] if n == 1 else obs, False)).reshape(n, A)
    x = (obs.astype(np.float32) - nrm.s_mean) / nrm.s_den
    out, _ = O.mlp_forward(st.actor, x.astype(np.float64), ocfg.act)
    mu, lraw = O.split_head(out, st.logstd, ocfg)
    u = O.f32_noise(ref_rs.normal(size=(n, A))).astype(np.float64)
    pi, _ = O.head_sample(mu, lraw, u, ocfg.act_limit, np.float64)
    assert relerr(got, pi) < 2e-5, relerr(got, pi)
    dev, ref = eng.rng_get_state(), ref_rs.get_state()
    assert np.array_equal(dev[1], ref[1]) and dev[2] == ref[2] and dev[3] == ref[3] and dev[4] == ref[4]
    for _ in range(3):
        eng.rng_set_state(np.random.RandomState(19).get_state())
        again = np.asarray(eng.act_host(obs[0] if n == 1 else obs, False)).reshape(n, A)
        assert np.array_equal(again, got)
    eng.close()


@pytest.mark.parametrize("deterministic,n,horizon,clip", [(False, 37, 5, 0.0), (True, 8, 3, 0.0),
                                                         (False, 4100, 2, 0.05)])
def test_rollout_matches_oracle(gpu_available, deterministic, n, horizon, clip):
    """World-model rollout (samplers.py:73-122 over MSEModel.step) vs oracle.rollout: the
    noise stream bit-exact (one normal(size=(n, A)) per step, chunked at 4096 rows), the
    trajectories within 1e-4 relative (fp32 device vs fp64 oracle over the horizon)."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="tanh", B=64, seed=51, use_expert=True, normalizers="random")
    S = ocfg.S
    s0 = (np.random.RandomState(5).normal(size=(n, S)) * 1.5).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(23).get_state())
    ref_rs = np.random.RandomState(23)
    got = [t.cpu().numpy() for t in eng.rollout(1, s0, horizon, deterministic, delta_clip=clip)]
    ref = O.rollout(st, ocfg, nrm, s0, horizon, 1, ref_rs, deterministic, delta_clip=clip)
    for g, r, name in zip(got, ref, ("s", "a", "r", "sp", "d")):
        assert g.shape == r.shape, (name, g.shape, r.shape)
        if name == "d":
            assert not g.any()
        else:
            assert relerr(g, r) < 1e-4, (name, relerr(g, r))
    assert np.array_equal(got[0][:, 0], s0)
    assert np.array_equal(got[0][:, 1:], got[3][:, :-1])
    dev, rr = eng.rng_get_state(), ref_rs.get_state()
    assert np.array_equal(dev[1], rr[1]) and dev[2] == rr[2] and dev[3] == rr[3] and dev[4] == rr[4]
    eng.close()


@pytest.mark.parametrize("eager", [True, False])
def test_dp_single_rank_equals_fused(gpu_available, eager):
    """Data-parallel mode (sacx_dp_init) with one RCCL rank: local gradients stored, summed
    by ncclAllReduce inside the update graph, then k_adam_apply / k_alpha_apply -- the same
    arithmetic as the fused dW+Adam epilogue, so parameters, Adam state, targets and
    statistics are bit-identical to the fused path over 19 updates (2 graphs + 3 singles)."""
    from sac_eo.engine import Engine
    outs = []
    n = 19
    for dp in (None, (Engine.dp_unique_id(), 1, 0)):
        eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=128, seed=61, dp=dp)
        eng.rng_set_state(np.random.RandomState(6).get_state())
        eng.step(n, eager=eager)
        eng.sync()
        plan = [p["name"] for p in eng.plan_info()]
        outs.append((eng.stats(n).copy(), eng.arena[:eng.segments["grad"]["offset"]].cpu().numpy().copy(), plan))
        eng.close()
    assert "critic.allreduce" in outs[1][2] and "alpha.allreduce" in outs[1][2]
    assert "critic.allreduce" not in outs[0][2]
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])       # params, adam_m, adam_v (targets included)


@pytest.mark.parametrize("use_expert_actions,n", [(False, 20), (True, 7), (False, 1000)])
def test_expert_diag_matches_oracle(gpu_available, use_expert_actions, n):
    """Expert diagnostics (SAC_expert.py:579-608, _calc_disc :427-460) vs the oracle; the
    counterfactual draws advance the device stream exactly like the reference's."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=71, use_expert=True, normalizers="random")
    S, A = ocfg.S, ocfg.A
    r = np.random.RandomState(9)
    s_e = (r.normal(size=(n, S)) * 2).astype(np.float32)
    a_e = r.uniform(-1, 1, (n, A)).astype(np.float32)
    sp_e = (s_e + r.normal(size=(n, S)) * 0.1).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(29).get_state())
    rs = np.random.RandomState(29)
    got = eng.expert_diag(s_e, a_e, sp_e, use_expert_actions=use_expert_actions)
    m_data, m_cf, per_data, per_cf = O.expert_mse_diag(st, ocfg, nrm, s_e, a_e, sp_e, rs, use_expert_actions)
    assert abs(got["mse_expert_data"] - m_data) <= 1e-4 * abs(m_data)
    assert abs(got["mse_counterfactual"] - m_cf) <= 1e-4 * abs(m_cf)
    assert np.max(np.abs(got["mse_counterfactual_per_model"] - per_cf) / np.abs(per_cf)) < 1e-4
    got_d = eng.expert_diag(s_e, a_e, sp_e, disc=True, use_expert_actions=use_expert_actions)
    ratio, mx, med, tot = O.calc_disc(st, ocfg, nrm, s_e, a_e, rs, use_expert_actions)
    assert abs(got_d["s_disc_total"] - tot) <= 1e-4 * tot
    assert abs(got_d["max_disc"] - mx) <= 1e-4 * mx
    assert abs(got_d["median_disc"] - med) <= 1e-4 * med
    assert relerr(got_d["disc_ratio"], ratio) < 1e-4
    dev, ref = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(dev[1], ref[1]) and dev[2] == ref[2] and dev[3] == ref[3] and dev[4] == ref[4]
    eng.close()


@pytest.mark.parametrize("use_expert", [False, True])
def test_snapshot_resume_bit_identical(gpu_available, tmp_path, use_expert):
    """Full-state snapshot (F4): 11 updates, save, 13 more; a fresh engine loading the
    snapshot runs the same 13 updates bit-identically (weights, Adam, RNG stream, counters,
    replay ring, permutation ring, stats)."""
    def fresh():
        eng, *_ = make_pair(act="tanh", B=64, seed=81, use_expert=use_expert)
        return eng
    eng = fresh()
    eng.rng_set_state(np.random.RandomState(4).get_state())
    if use_expert:
        rs = np.random.RandomState(2)
        eng.push_perms(np.stack([rs.permutation(eng.cfg.expert_batch) for _ in range(24)]))
    eng.step(11)
    eng.save_state(str(tmp_path / "snap"))
    eng.step(13)
    eng.sync()
    ref = (eng.stats(13).copy(), eng.v["params"].cpu().numpy().copy(), eng.rng_get_state())
    eng.close()
    eng2 = fresh()
    eng2.load_state(str(tmp_path / "snap"))
    eng2.step(13)
    eng2.sync()
    got = (eng2.stats(13).copy(), eng2.v["params"].cpu().numpy().copy(), eng2.rng_get_state())
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])
    assert np.array_equal(ref[2][1], got[2][1]) and ref[2][2] == got[2][2]
    assert eng2.ctl()["step_seq"] == 24
    eng2.close()


BF16_QLOSS_TOL = 5e-3     # config C5: bf16 operands (8-bit mantissa), fp32 accumulate; measured 1.3e-3


@pytest.mark.parametrize("use_expert", [False, True])
def test_bf16_qloss_trajectory(gpu_available, use_expert):
    """Config C5 (bf16 MFMA MLP path, fp32 accumulate and master weights): the Q-loss
    trajectory over 100 updates against the fp64 oracle within BF16_QLOSS_TOL relative
    (the fp32 path's bar is 1e-4; bf16 rounds every GEMM operand to 8 mantissa bits), and
    the sampler stream still bit-exact."""
    B = 256
    eng, ocfg, st, buf, nrm, expert = make_pair(act="relu", B=B, seed=11, use_expert=use_expert, done_p=0.01,
                                                gemm_bf16=True)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(123)
    gen = np.random.default_rng(77)
    eng.rng_set_state(rs.get_state())
    steps = 100
    Rs = [O.draw_step_randoms(rs, N, B, ocfg.A, n_expert=20 if use_expert else 0, gen=gen) for _ in range(steps)]
    if use_expert:
        eng.push_perms(np.stack([R["perm"] for R in Rs]))
    eng.step(steps)
    eng.sync()
    dev = eng.stats(steps)
    ref = np.array([[o["q1_loss"], o["q2_loss"]] for o in (oracle_step(st, ocfg, nrm, buf, R, expert) for R in Rs)])
    rel = np.abs(dev[:, :2] - ref) / np.abs(ref)
    print("bf16 q-loss max rel err", rel.max(), "median", np.median(rel))
    assert rel.max() < BF16_QLOSS_TOL, rel.max()
    assert np.all(np.isfinite(dev))
    got, exp = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(got[1], exp[1]) and got[2] == exp[2]
    eng.close()


def test_bf16_graph_equals_eager(gpu_available):
    outs = []
    for eager in (True, False):
        eng, *_ = make_pair(act="tanh", B=128, seed=21, gemm_bf16=True)
        eng.rng_set_state(np.random.RandomState(5).get_state())
        eng.step(19, eager=eager)
        eng.sync()
        outs.append((eng.stats(19).copy(), eng.v["params"].cpu().numpy().copy()))
        eng.close()
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


def test_rollout_graph_replay_equals_eager(gpu_available, monkeypatch):
    """The captured rollout graph (replayed on the second call with the same shapes) gives
    the eager launches' results bit for bit, and advances the stream identically."""
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=53, use_expert=True, normalizers="random")
    s0 = (np.random.RandomState(6).normal(size=(50, ocfg.S))).astype(np.float32)
    outs = []
    for mode in ("1", "1", "0"):          # capture, replay, eager
        monkeypatch.setenv("SACX_ROLL_GRAPH", mode)
        eng.rng_set_state(np.random.RandomState(31).get_state())
        res = [t.cpu().numpy() for t in eng.rollout(0, s0, 4)]
        outs.append((res, eng.rng_get_state()))
    for res, stt in outs[1:]:
        for x, y in zip(outs[0][0], res):
            assert np.array_equal(x, y)
        assert np.array_equal(outs[0][1][1], stt[1]) and outs[0][1][2] == stt[2]
    eng.close()


@pytest.mark.parametrize("K,use_expert,eager,t32,bf16,folds",
                         [(3, False, False, None, False, None), (3, True, False, None, False, None),
                          (3, False, True, None, False, None), (4, False, False, None, False, "0"),
                          (4, True, False, None, False, "0"), (4, False, False, "1", False, "0"),
                          (4, False, False, "1", True, "0"), (4, False, False, "2", True, "0"),
                          (4, False, False, "2", False, "1"), (4, False, True, "1", True, "1")])
def test_packed_seeds_equal_single(gpu_available, monkeypatch, K, use_expert, eager, t32, bf16, folds):
    """cfg.seeds = K (the reference's --runs packed into one handle, grid z = seed): every
    seed ends bit-identical to a one-seed engine fed the same state, buffer, RNG stream and
    permutations -- stats, every parameter / Adam / target value, and the RNG key.  19
    updates = two 8-update graphs + remainder graphs.  At K = 4 the packed plan takes 32x32
    tiles for its forward / dX launches and the one-seed engines 16x16 (both with the
    separate actor.head launch): the two tilings must agree bit for bit -- in fp32 and with
    bf16 MFMA operands (config C5: the 32x32 tiles split the k slabs over acc0 / acc1 exactly
    as the 16x16 path does)."""
    from sac_eo.engine import Engine, EngineConfig
    n, B, N, eps = 19, 128, 3000, 0.1
    if K >= 4:                                  # the packed plan: 32x32 tiles ("1": dW + Adam too)
        monkeypatch.setenv("SACX_FUSE_HEAD", "0")
        monkeypatch.setenv("SACX_T32", t32 or "2")
        # the partial-dot folds (off by default on 32x32 plans) set alike in both plans; "1": the
        # partial epilogues on 32x32 tiles against the one-seed 16x16 ones
        monkeypatch.setenv("SACX_FOLD_HBW", folds)
        monkeypatch.setenv("SACX_HEAD_PART", folds)
    learners = [make_learner(act="tanh", B=B, N=N, seed=40 + 7 * k, use_expert=use_expert, epsilon=eps)
                for k in range(K)]

    def cfg(seeds):
        return EngineConfig(s_dim=17, a_dim=6, activation="tanh", batch=B, buffer_capacity=N, use_expert=use_expert,
                            expert_capacity=20, expert_batch=20, graph_steps=8, epsilon=eps, seeds=seeds,
                            gemm_bf16=bf16)

    def drive(eng, k):
        _, st, buf, nrm, ex = learners[k]
        load_learner(eng, st, buf, nrm, ex, eps)
        eng.rng_set_state(np.random.RandomState(500 + k).get_state())
        if use_expert:
            rs = np.random.RandomState(900 + k)
            eng.push_perms(np.stack([rs.permutation(20) for _ in range(n)]))

    packed = Engine(cfg(K))
    if K >= 4:
        monkeypatch.setenv("SACX_T32", "0")     # the one-seed references: 16x16 tiles
    for k in range(K):
        packed.select_seed(k)
        drive(packed, k)
    packed.select_seed(0)
    packed.step(n, eager=eager)
    packed.sync()
    got = []
    for k in range(K):
        packed.select_seed(k)
        got.append((packed.stats(n).copy(), packed.v["params"].cpu().numpy().copy(),
                    packed.v["adam_v"].cpu().numpy().copy(), packed.rng_get_state()[1].copy()))
    packed.close()
    for k in range(K):
        e = Engine(cfg(1))
        drive(e, k)
        e.step(n, eager=eager)
        e.sync()
        ref = (e.stats(n), e.v["params"].cpu().numpy(), e.v["adam_v"].cpu().numpy(), e.rng_get_state()[1])
        e.close()
        for i, (a, b) in enumerate(zip(got[k], ref)):
            assert np.array_equal(a, b), (k, i)
    assert np.all(np.isfinite(got[0][0]))
    assert not np.array_equal(got[0][1], got[1][1])     # the seeds are different learners



@pytest.mark.parametrize("act,S,A,B,graph,bf16", [("relu", 17, 6, 256, True, False), ("tanh", 17, 6, 100, False, False),
                                                  ("relu", 376, 17, 1024, True, False),
                                                  ("relu", 376, 17, 1024, True, True)])
def test_launch_header_fallback_bit_identical(gpu_available, monkeypatch, act, S, A, B, graph, bf16):
    """k_gemm / k_dwl take the scalars that pick a workgroup's role from a launch header preloaded
    into SGPRs (sacx_internal.h KHdr); SACX_KHDR=0 marks every header invalid, so the kernels read
    the same values from GemmArgs.  Both paths give the same updates bit for bit."""
    outs = []
    for kh in ("1", "0"):
        monkeypatch.setenv("SACX_KHDR", kh)
        eng, ocfg, st, buf, nrm, _ = make_pair(S=S, A=A, act=act, B=B, N=4000, seed=17, normalizers="random",
                                               graph_steps=8, gemm_bf16=bf16)
        eng.rng_set_state(np.random.RandomState(3).get_state())
        eng.step(19, eager=not graph)
        eng.sync()
        outs.append((eng.stats(19).copy(), eng.v["params"].cpu().numpy().copy(), eng.v["adam_v"].cpu().numpy().copy()))
        eng.close()
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)
