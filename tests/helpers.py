"""Shared setup for the parity tests: one oracle state (tests' checker) and
the same state loaded into the device engine (the product)."""
from __future__ import annotations

import numpy as np

import sac_oracle as O

B1 = np.float32(1.0) - np.float32(0.9)   # Keras (1 - beta_1) in fp32: m_1 = g * B1


def synthetic_buffer(rs: np.random.RandomState, N: int, S: int, A: int, done_p: float = 0.0):
    """SURVEY.md §8(d) synthetic data: per-dim scales U(0.1, 5), a ~ U(-1, 1)."""
    sig = rs.uniform(0.1, 5.0, size=S)
    buf = dict(s=(rs.normal(size=(N, S)) * sig).astype(np.float32),
               a=rs.uniform(-1, 1, size=(N, A)).astype(np.float32),
               sp=(rs.normal(size=(N, S)) * sig).astype(np.float32),
               r=rs.normal(size=N).astype(np.float32),
               d=(rs.uniform(size=N) < done_p).astype(np.float64))
    return buf


def nontrivial_normalizers(rs, S, A):
    return O.Normalizers(
        (rs.normal(size=S) * 0.2).astype(np.float32), rs.uniform(0.5, 3.0, S).astype(np.float32),
        (rs.normal(size=A) * 0.05).astype(np.float32), rs.uniform(0.8, 1.2, A).astype(np.float32),
        (rs.normal(size=S) * 0.1).astype(np.float32), rs.uniform(0.5, 2.0, S).astype(np.float32),
        0.0, 1.0, 1.0)


def make_learner(S=17, A=6, hidden=(256, 256), B=256, act="relu", N=5000, seed=0, per_state_std=False,
                 use_expert=False, ne=20, model_hidden=(512, 512), normalizers="identity", done_p=0.0,
                 bias_scale=0.05, actor_gain=0.5, epsilon=0.1, layer_norm=False, actor_acts=None, critic_acts=None,
                 wm=None, num_models=2):
    """The seeded inputs of one learner: (oracle_cfg, oracle_state_f32, buffer, normalizers, expert).
    ``wm``: world-model variant flags (gaussian_model, scale_model_loss, separate_reward_nn,
    reward_hidden, reward_act) of O.Config."""
    wm = dict(wm or {})
    ocfg = O.Config(S=S, A=A, hidden=hidden, act=act, B=B, per_state_std=per_state_std,
                    critic_hidden=wm.pop("critic_hidden", None),
                    model_hidden=model_hidden, epsilon=epsilon, layer_norm=layer_norm, actor_acts=actor_acts,
                    critic_acts=critic_acts, num_models=num_models, **wm)
    st = O.init_state(ocfg, seed=seed + 1, with_models=use_expert, bias_scale=bias_scale,
                      actor_gain=actor_gain, model_gain=0.3, model_std_mult=0.7, reward_gain=0.3)
    rs = np.random.RandomState(seed + 100)
    buf = synthetic_buffer(rs, N, S, A, done_p)
    nrm = O.Normalizers.identity(S, A) if normalizers == "identity" else nontrivial_normalizers(rs, S, A)
    expert = None
    if use_expert:
        ers = np.random.RandomState(seed + 200)
        sig = ers.uniform(0.1, 5.0, size=S)
        expert = dict(s=(ers.normal(size=(ne, S)) * sig).astype(np.float32),
                      sp=(ers.normal(size=(ne, S)) * sig).astype(np.float32))
    return ocfg, st, buf, nrm, expert


def load_learner(eng, st, buf, nrm, expert, epsilon):
    """Writes one learner's state into the engine's selected seed."""
    eng.set_net("actor", st.actor)
    eng.set_logstd(st.logstd)
    for k in range(2):
        eng.set_net(f"q{k}", st.q[k])
        eng.set_net(f"t{k}", st.q_targ[k])
    if expert is not None:
        for k in range(len(st.models)):
            if f"m{k}.l0" in eng.segments:      # --num_models 1: model 0 only
                eng.set_net(f"m{k}", st.models[k])
                if st.model_logstd is not None:
                    eng.set_model_logstd(k, st.model_logstd[k])
                if st.reward_nets is not None:
                    eng.set_net(f"r{k}", st.reward_nets[k])
    eng.set_alpha(float(st.alpha))
    eng.set_normalizers(nrm.s_mean, nrm.s_den, nrm.a_mean, nrm.a_den, nrm.d_mean, nrm.d_den,
                        nrm.r_mean, nrm.r_den, nrm.ret_den)
    eng.append(buf["s"], buf["a"], buf["r"], buf["sp"], buf["d"].astype(np.float32))
    if expert is not None:
        eng.set_expert(expert["s"], expert["sp"], epsilon)


def make_pair(S=17, A=6, hidden=(256, 256), B=256, act="relu", N=5000, seed=0, per_state_std=False,
              use_expert=False, ne=20, model_hidden=(512, 512), normalizers="identity", done_p=0.0,
              graph_steps=8, bias_scale=0.05, actor_gain=0.5, epsilon=0.1, dp=None, gemm_bf16=False, layer_norm=False,
              actor_acts=None, critic_acts=None, wm=None, **ekw):
    """Returns (engine, oracle_cfg, oracle_state_fp64, buffer, normalizers, expert)."""
    from sac_eo.engine import Engine, EngineConfig
    ocfg, st, buf, nrm, expert = make_learner(S, A, hidden, B, act, N, seed, per_state_std, use_expert, ne,
                                              model_hidden, normalizers, done_p, bias_scale, actor_gain, epsilon,
                                              layer_norm, actor_acts, critic_acts, wm, ekw.get("num_models", 2))
    if wm:                                 # the oracle's world-model flags -> the engine's
        ekw = dict(ekw, gaussian_model=ocfg.gaussian_model, scale_model_loss=ocfg.scale_model_loss,
                   separate_reward_nn=ocfg.separate_reward_nn, reward_hidden=tuple(ocfg.reward_hidden),
                   reward_activations=(ocfg.reward_act,))
    if ocfg.critic_hidden is not None:
        ekw = dict(ekw, critic_hidden=tuple(ocfg.critic_hidden))
    ecfg = EngineConfig(s_dim=S, a_dim=A, hidden=hidden, activation=act, batch=B, buffer_capacity=N,
                        per_state_std=per_state_std, use_expert=use_expert, expert_capacity=max(ne, 2),
                        expert_batch=ne, model_hidden=model_hidden, graph_steps=graph_steps, epsilon=epsilon,
                        gemm_bf16=gemm_bf16, actor_layer_norm=layer_norm, actor_activations=actor_acts,
                        critic_activations=critic_acts, **ekw)
    eng = Engine(ecfg, dp=dp)
    load_learner(eng, st, buf, nrm, expert, epsilon)
    return eng, ocfg, st.astype(np.float64), buf, nrm, expert


def oracle_step(st, ocfg, nrm, buf, R, expert=None, keep=None):
    """One oracle update with the randoms R drawn in the reference order."""
    n = [O.f32_noise(R[k]) for k in ("noise_t", "noise_pi", "noise_alpha")]
    ex = None
    if expert is not None:
        sec = R["sections"]
        if len(sec) == 1:                      # one world model: every expert row, in order
            ex = O.Expert(expert["s"][sec[0]], expert["sp"][sec[0]], None, None,
                          O.f32_noise(R["noise_e1"]), None, ocfg.epsilon)
        else:
            ex = O.Expert(expert["s"][sec[0]], expert["sp"][sec[0]], expert["s"][sec[1]], expert["sp"][sec[1]],
                          O.f32_noise(R["noise_e1"]), O.f32_noise(R["noise_e2"]), ocfg.epsilon)
    return O.sac_update(st, ocfg, nrm, O.gather(buf, R["idx"]), *n, expert=ex, keep=keep)


def relerr(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))
