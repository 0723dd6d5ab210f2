"""BASELINE.json configs exercised at their own shapes on the device.

* C3 (Humanoid-v3, S=376, A=17): the world-model fit (2 models x minibatch 200,
  mbrl_onpolicy_alg.py:301-319) and the rollout (samplers.py:73-122) vs the oracle.
* C5 (Humanoid-v3, B=1024, bf16 MFMA operands / fp32 accumulate, 4e6-row buffer in HBM):
  the Q-loss trajectory of 100 updates vs the fp64 oracle within BF16_QLOSS_TOL (the graph
  schedule at its production graph_steps = 128), and on a full 4e6-row ring (12.3 GB, byte
  offsets past 2^32) the device sampler's indices and noise bit-exact against NumPy and the
  gathered rows equal to the ring rows they name.
"""
import numpy as np
import pytest

import sac_oracle as O
from helpers import make_pair, oracle_step, relerr

pytestmark = pytest.mark.gpu

HUM = dict(S=376, A=17)
BF16_QLOSS_TOL = 5e-3       # as tests/test_gpu_engine.py: 8-bit-mantissa operands, fp32 accumulate


@pytest.mark.parametrize("eager", [True, False])
def test_humanoid_model_fit(gpu_available, eager):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=33, use_expert=True, normalizers="random", **HUM)
    N = buf["r"].shape[0]
    mb = eng.cfg.model_batch
    idx = np.random.RandomState(10).randint(N, size=(4, 2, mb))
    eng.model_fit(idx, eager=eager)
    eng.sync()
    dev = eng.model_stats(4)
    ref = np.array([O.model_fit_step(st, ocfg, nrm, [(buf["s"][idx[j, k]], buf["a"][idx[j, k]], buf["sp"][idx[j, k]],
                                                      buf["r"][idx[j, k]]) for k in range(2)]) for j in range(4)])
    assert np.max(np.abs(dev - ref) / np.abs(ref)) < 1e-4, (dev, ref)
    for k in range(2):
        for a_, b_ in zip(eng.get_net(f"m{k}"), st.models[k]):
            assert np.max(np.abs(a_ - b_)) < 5e-5
    eng.close()


def test_humanoid_rollout(gpu_available):
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=64, seed=35, use_expert=True, normalizers="random", **HUM)
    s0 = (np.random.RandomState(7).normal(size=(1000, ocfg.S)) * 0.5).astype(np.float32)
    eng.rng_set_state(np.random.RandomState(24).get_state())
    rs = np.random.RandomState(24)
    got = [t.cpu().numpy() for t in eng.rollout(0, s0, 5)]
    ref = O.rollout(st, ocfg, nrm, s0, 5, 0, rs)
    for g, r, name in zip(got, ref, ("s", "a", "r", "sp", "d")):
        assert g.shape == r.shape
        if name != "d":
            assert relerr(g, r) < 1e-4, (name, relerr(g, r))
    dev, rr = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(dev[1], rr[1]) and dev[2] == rr[2]
    eng.close()


def test_humanoid_bf16_trajectory(gpu_available):
    B, steps = 1024, 100
    eng, ocfg, st, buf, nrm, _ = make_pair(act="relu", B=B, N=20000, seed=37, done_p=0.01, gemm_bf16=True,
                                           graph_steps=128, **HUM)
    N = buf["r"].shape[0]
    rs = np.random.RandomState(77)
    eng.rng_set_state(rs.get_state())
    Rs = [O.draw_step_randoms(rs, N, B, ocfg.A) for _ in range(steps)]
    eng.prepare(steps)
    eng.step(steps)
    eng.sync()
    dev = eng.stats(steps)
    ref = np.array([[o["q1_loss"], o["q2_loss"]] for o in (oracle_step(st, ocfg, nrm, buf, R) for R in Rs)])
    rel = np.abs(dev[:, :2] - ref) / np.abs(ref)
    print("humanoid bf16 q-loss max rel err", rel.max(), "median", np.median(rel))
    assert rel.max() < BF16_QLOSS_TOL, rel.max()
    got, exp = eng.rng_get_state(), rs.get_state()
    assert np.array_equal(got[1], exp[1]) and got[2] == exp[2]
    eng.close()


def test_sampler_on_4e6_ring(gpu_available):
    """Config C5's replay ring: 4e6 Humanoid rows resident in HBM (12.3 GB)."""
    import torch
    from sac_eo.engine import Engine, EngineConfig
    S, A, B, N = 376, 17, 1024, 4_000_000
    eng = Engine(EngineConfig(s_dim=S, a_dim=A, batch=B, buffer_capacity=N, gemm_bf16=True, graph_steps=1))
    g = torch.Generator(device=eng.device)
    g.manual_seed(5)
    for c0 in range(0, N, 500_000):                   # fill on the device in chunks
        n = min(500_000, N - c0)
        s = torch.randn(n, S, device=eng.device, generator=g)
        eng.append(s, torch.rand(n, A, device=eng.device, generator=g) * 2 - 1,
                   torch.randn(n, device=eng.device, generator=g), s * 0.5, torch.zeros(n, device=eng.device))
        eng.sync()
        del s
    assert eng.ctl()["cur_size"] == N and eng.ctl()["start"] == 0
    for seed in (2590541744, 11):
        rs = np.random.RandomState(seed)
        eng.rng_set_state(rs.get_state())
        eng.step(1, external=False, eager=True)
        eng.sync()
        idx = rs.randint(N, size=B)
        noise = rs.normal(size=3 * B * A)
        assert np.array_equal(eng.v["slot0.idx"][0].cpu().numpy(), idx)
        assert np.array_equal(eng.v["slot0.noise"][0].cpu().numpy(), noise.astype(np.float32))
        assert idx.max() > 3_500_000                      # rows past 2^32 bytes into the ring
        rows = eng.v["replay"][torch.as_tensor(idx, device=eng.device)]
        xq = eng.v["slot0.Xq"][:B]
        assert torch.equal(xq[:, :S], rows[:, :S]) and torch.equal(xq[:, S:S + A], rows[:, S:S + A])
        assert torch.equal(eng.v["slot0.r"][0], rows[:, 2 * S + A])
    eng.close()


def _wbf_expected(W):
    """The bf16 shadow of W [K x N] in the kernels' pair layout (sacx_internal.h wbf_pos), as uint16."""
    import torch
    K, N = W.shape
    per = (((K + 15) >> 4) + 3) >> 2
    ld = 4 * ((per + 1) >> 1) * 32
    bits = torch.from_numpy(np.ascontiguousarray(W, np.float32)).to(torch.bfloat16).view(torch.int16).numpy()
    out = np.zeros((N, ld), np.uint16)
    k = np.arange(K)
    s = k >> 4
    w = s // per
    i = s - w * per
    pos = (w * ((per + 1) >> 1) + (i >> 1)) * 32 + ((k >> 2) & 3) * 8 + (i & 1) * 4 + (k & 3)
    out[:, pos] = bits.view(np.uint16).T
    return out


@pytest.mark.parametrize("eager", [False, True])
def test_bf16_weight_shadows_bit_identical(gpu_available, monkeypatch, eager):
    """C5's forward tiles reading layer 1's A from the layer-0 outputs' bf16 shadows (SACX_WBF=3,
    the default), B from the weights' shadows (2), or both (1) equal the converting loads
    (SACX_WBF=0) bit for bit over 2 x 24 Humanoid updates at B = 1,024, with a host write of the
    parameters in between (the weight shadows are rebuilt at the next step call); after each run
    every weight shadow equals the bf16 image of its fp32 weights in the wbf_pos layout, and the
    critics' layer-0 output shadow that of the last update's activations.  critic.adam reading X^T
    from transposed images (opt-in SACX_XBF=1: critic rows and layer-0 outputs, 2: the rows only)
    equals it too, and the images equal the bf16 transposes of every slot's critic rows and of the
    last update's q0 / q1 layer-0 outputs."""
    B, n = 1024, 24
    S, A = HUM["S"], HUM["A"]
    outs = []
    for wbf, xbf in (("0", "1"), ("3", "0"), ("3", "1"), ("3", "2"), ("2", "1"), ("1", "1")):
        monkeypatch.setenv("SACX_WBF", wbf)
        monkeypatch.setenv("SACX_XBF", xbf)
        eng, *_ = make_pair(act="relu", B=B, N=6000, seed=41, done_p=0.01, gemm_bf16=True, graph_steps=8, **HUM)
        eng.rng_set_state(np.random.RandomState(8).get_state())
        eng.step(n, eager=eager)
        eng.sync()
        p = eng.v["params"]
        p.mul_(0.999)                      # a host-side write between step calls
        eng.step(n, eager=eager)
        eng.sync()
        outs.append((eng.stats(2 * n).copy(), eng.v["params"].cpu().numpy().copy(),
                     eng.v["adam_v"].cpu().numpy().copy()))
        if wbf in ("1", "2"):
            names = [f"{net}.l{l}" for net in ("actor", "q0", "q1", "t0", "t1") for l in (0, 1)]
            for nm in names:
                assert "wbf." + nm in eng.v, nm
                Wx = eng.v[nm].cpu().numpy()
                exp = _wbf_expected(Wx[:-1])             # W_ext without the bias row
                got = eng.v["wbf." + nm].cpu().numpy().view(np.uint16).reshape(exp.shape[0], -1)
                assert np.array_equal(got, exp), nm
        if wbf in ("1", "3"):
            hq = eng.v["ws.Hq1"].cpu().numpy()
            exp = _wbf_expected(hq.T)
            got = eng.v["abf.ws.Hq1"].cpu().numpy().view(np.uint16).reshape(exp.shape[0], -1)
            assert np.array_equal(got, exp)
        assert ("xbf.ws.Hq1" in eng.v) == (xbf == "1")
        if wbf != "0" and xbf != "0":
            names = [nm for nm in eng.v if nm.startswith("slot") and nm.endswith(".xbfq")]
            assert len(names) == 8                   # Humanoid: an 8-slot ring
            for nm in names:
                xq = eng.v[nm.replace(".xbfq", ".Xq")].cpu().numpy()[:B, :S + A]
                exp = _wbf_expected(xq)
                got = eng.v[nm].cpu().numpy().view(np.uint16).reshape(exp.shape[0], -1)
                assert np.array_equal(got, exp), nm
        if wbf != "0" and xbf == "1":
            hq = eng.v["ws.Hq1"].cpu().numpy()
            img = eng.v["xbf.ws.Hq1"].cpu().numpy().view(np.uint16)
            img = img.reshape(4, hq.shape[1], -1)
            for k in (2, 3):                         # q0, q1 (critic.adam's consumers; t0 / t1 unwritten)
                assert np.array_equal(img[k], _wbf_expected(hq[k * B:(k + 1) * B])), k
        eng.close()
    for o in outs[1:]:
        for i, (a, b) in enumerate(zip(outs[0], o)):
            assert np.array_equal(a, b), i


def test_bf16_shadows_packed_seeds(gpu_available, monkeypatch):
    """The shadows of packed seeds (one arena block per seed, relocated by grid z): 4 HC-shaped
    bf16 seeds (4 x 256 rows: 32x32 forward tiles) over a 16-update graph, a host write, and 16
    more, SACX_WBF=1 equal to SACX_WBF=0 bit for bit for every seed."""
    from helpers import load_learner, make_learner
    from sac_eo.engine import Engine, EngineConfig
    K, n, B, N = 4, 16, 256, 3000
    learners = [make_learner(act="relu", B=B, N=N, seed=90 + 3 * k) for k in range(K)]
    outs = []
    for wbf in ("0", "1"):
        monkeypatch.setenv("SACX_WBF", wbf)
        eng = Engine(EngineConfig(s_dim=17, a_dim=6, activation="relu", batch=B, buffer_capacity=N, graph_steps=16,
                                  seeds=K, gemm_bf16=True))
        for k in range(K):
            eng.select_seed(k)
            _, st, buf, nrm, ex = learners[k]
            load_learner(eng, st, buf, nrm, ex, 0.1)
            eng.rng_set_state(np.random.RandomState(300 + k).get_state())
        eng.select_seed(0)
        eng.step(n)
        eng.sync()
        eng.select_seed(2)
        eng.v["params"].mul_(0.999)
        eng.select_seed(0)
        eng.step(n)
        eng.sync()
        got = []
        for k in range(K):
            eng.select_seed(k)
            got.append((eng.stats(2 * n).copy(), eng.v["params"].cpu().numpy().copy(),
                        eng.v["adam_v"].cpu().numpy().copy()))
        outs.append(got)
        eng.close()
    for k in range(K):
        for i, (a, b) in enumerate(zip(outs[0][k], outs[1][k])):
            assert np.array_equal(a, b), (k, i)
