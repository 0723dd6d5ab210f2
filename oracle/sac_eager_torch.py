"""Eager, op-by-op PyTorch-CPU restatement of the reference's gradient step: the CPU BASELINE.

TEST / MEASUREMENT INFRASTRUCTURE ONLY (like ``sac_oracle.py``): only ``bench.py``'s
``cpu_baseline`` leg and ``tests/`` use it.  It is the "reference-equivalent CPU path"
SURVEY.md §8(d) asks for, because the reference itself (TensorFlow 2 eager) cannot be installed:
the same op sequence with the same per-op dispatch structure as the reference's eager code,
autodiff tapes instead of closed-form backward passes, Keras Adam per variable.

  sampler + gather      np.random.randint + fancy indexing       buffers.py:126-144
  target (no tape)      evaluate(sp), two target critics, min    SAC_expert.py:211-229
  critics               one tape + Adam per critic, in turn      SAC_expert.py:232-259
  actor (+ expert term) tape over evaluate(s) -> min Q (-> models) SAC_expert.py:262-338
  alpha                 evaluate(s) again, tape over alpha       SAC_expert.py:340-348
  Polyak                per tensor, two products and an add      SAC_expert.py:362-373
  world-model fit step  2 models x minibatch, one tape + Adam    mbrl_onpolicy_alg.py:301-319
Keras Adam (legacy OptimizerV2): m, v updates, lr_t = lr sqrt(1-b2^t)/(1-b1^t), eps outside sqrt.

``tests/test_eager_torch.py`` checks one update of this restatement against ``sac_oracle`` (fp32),
so the timed baseline computes what the product computes."""
from __future__ import annotations

import math
import time

import numpy as np
import torch
import torch.nn.functional as Fn

LN2 = math.log(2.0)
LN2PI = math.log(2.0 * math.pi)


class KerasAdam:
    def __init__(self, params, lr, b1=0.9, b2=0.999, eps=1e-7):
        self.p, self.lr, self.b1, self.b2, self.eps = list(params), lr, b1, b2, eps
        self.m = [torch.zeros_like(x) for x in self.p]
        self.v = [torch.zeros_like(x) for x in self.p]
        self.t = 0

    @torch.no_grad()
    def apply(self, grads):
        self.t += 1
        lr_t = self.lr * math.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        for p, g, m, v in zip(self.p, grads, self.m, self.v):
            m.add_((g - m) * (1 - self.b1))
            v.add_((g * g - v) * (1 - self.b2))
            p.sub_(m * lr_t / (v.sqrt() + self.eps))


def _act(x, kind):
    return torch.relu(x) if kind == "relu" else torch.tanh(x) if kind == "tanh" else Fn.elu(x)


class EagerSAC:
    """One learner: actor, two critics + targets, alpha (+ two world models for SAC-EO)."""

    def __init__(self, st, cfg, use_expert=False, threads=1):
        """st: a ``sac_oracle.SACState`` (weights, Keras layout), cfg: its ``sac_oracle.Config``."""
        t = lambda x: torch.tensor(np.asarray(x, np.float32), requires_grad=True)
        self.cfg = cfg
        self.act = cfg.act
        self.actor = [t(w) for w in st.actor]
        self.logstd = t(np.asarray(st.logstd, np.float32).reshape(1, -1))
        self.q = [[t(w) for w in net] for net in st.q]
        self.qt = [[t(w).detach() for w in net] for net in st.q_targ]
        self.alpha = t(np.float32(st.alpha))
        self.opt_q = [KerasAdam(n, cfg.lr_q) for n in self.q]
        self.opt_pi = KerasAdam(self.actor + [self.logstd], cfg.lr_pi)
        self.opt_alpha = KerasAdam([self.alpha], cfg.lr_alpha)
        self.use_expert = use_expert
        if use_expert:
            self.models = [[t(w) for w in m] for m in st.models]
            self.opt_model = KerasAdam([w for m in self.models for w in m], cfg.lr_model)
        self.H = -float(cfg.A)
        # the default (identity) running normalisers: the reference still runs their ops
        z = lambda n: torch.zeros(n)
        self.s_mu, self.s_sd, self.a_mu, self.a_sd = z(cfg.S), z(cfg.S) + 1, z(cfg.A), z(cfg.A) + 1
        self.ret_sd, self.r_mu, self.r_sd = torch.tensor(1.0), torch.tensor(0.0), torch.tensor(1.0)

    # -------------------------------------------------------------- nets (Keras Dense per layer)
    def _mlp(self, params, x, act):
        n = len(params) // 2
        for i in range(n):
            x = x @ params[2 * i] + params[2 * i + 1]
            if i < n - 1:
                x = _act(x, act)
        return x

    def evaluate(self, s, u):
        """SquashedGaussianActor.evaluate (continuous_actors.py:327-379): (a, neglogp)."""
        mu = self._mlp(self.actor, (s - self.s_mu) / self.s_sd, self.act)
        logstd = torch.clamp(self.logstd, -5.0, 2.0)
        std = torch.exp(logstd)
        x = mu + std * u
        nlp = 0.5 * torch.sum(((x - mu) / std) ** 2 + 2.0 * logstd + LN2PI, dim=-1)
        nlp = nlp + torch.sum(2.0 * (LN2 - x - Fn.softplus(-2.0 * x)), dim=-1)
        return torch.tanh(x), nlp

    def qval(self, net, s, a, value=False):
        """QCritic._forward (value=True: .value, x ret sigma) on normalised inputs."""
        x = torch.cat([(s - self.s_mu) / self.s_sd, (a - self.a_mu) / self.a_sd], -1)
        q = self._mlp(net, x, self.act)[:, 0]
        return q * self.ret_sd if value else q

    def model_sample(self, k, s, a):
        x = torch.cat([(s - self.s_mu) / self.s_sd, (a - self.a_mu) / self.a_sd], -1)
        out = self._mlp(self.models[k], x, "relu")
        return s + (out[:, : s.shape[1]] * self.s_sd + self.s_mu)

    # -------------------------------------------------------------- one _update
    def update(self, s, a, sp, r, d, u_t, u_pi, u_al, expert=None):
        cfg = self.cfg
        with torch.no_grad():                                     # _get_Q_target
            a2, nlp2 = self.evaluate(sp, u_t)
            q_next = torch.min(self.qval(self.qt[0], sp, a2, True), self.qval(self.qt[1], sp, a2, True))
            y = r + cfg.gamma * ((1 - d) * (q_next + self.alpha * nlp2))
        losses = []
        for k in range(2):                                        # _update_critic: one tape per critic
            q = self.qval(self.q[k], s, a)
            L = 0.5 * torch.mean((q - y) ** 2)
            self.opt_q[k].apply(torch.autograd.grad(L, self.q[k]))
            losses.append(L)
        a_pi, nlp = self.evaluate(s, u_pi)                        # _update_actor_and_alpha
        qm = torch.min(self.qval(self.q[0], s, a_pi), self.qval(self.q[1], s, a_pi))
        p = torch.mean(-self.alpha.detach() * nlp - qm)
        if expert is not None:                                    # SAC-EO expert term, 2 models
            (se1, spe1, ue1), (se2, spe2, ue2), eps = expert
            ae1, _ = self.evaluate(se1, ue1)
            ae2, _ = self.evaluate(se2, ue2)
            e1 = self.model_sample(0, se1, ae1) - spe1
            e2 = self.model_sample(1, se2, ae2) - spe2
            mse = torch.mean(0.5 * (torch.sum(e1 * e1, -1) + torch.sum(e2 * e2, -1)))
            p = (1 - eps) * p + eps * mse
        self.opt_pi.apply(torch.autograd.grad(p, self.actor + [self.logstd]))
        with torch.no_grad():
            _, nlp3 = self.evaluate(s, u_al)
        La = -self.alpha * torch.mean(-nlp3 + self.H)
        self.opt_alpha.apply(torch.autograd.grad(La, [self.alpha]))
        with torch.no_grad():
            self.alpha.clamp_(min=1e-5)
            for k in range(2):                                    # _update_q_target
                for tw, w in zip(self.qt[k], self.q[k]):
                    tw.copy_(tw * (1 - cfg.tau) + w * cfg.tau)
        return [float(x.detach()) for x in losses] + [float(p.detach()), float(La.detach())]

    def model_fit_step(self, batches):
        """_apply_model_grads: the summed MSE losses of the two models on their own minibatches."""
        S = self.cfg.S
        total = 0.0
        for k, (s, a, sp, r) in enumerate(batches):
            x = torch.cat([(s - self.s_mu) / self.s_sd, (a - self.a_mu) / self.a_sd], -1)
            out = self._mlp(self.models[k], x, "relu")
            ed = ((sp - s) - self.s_mu) / self.s_sd - out[:, :S]          # delta_rms (identity)
            er = (r - self.r_mu) / self.r_sd - out[:, S]
            total = total + torch.mean(0.5 * torch.sum(ed * ed, -1) + 0.5 * er * er)
        params = [w for m in self.models for w in m]
        self.opt_model.apply(torch.autograd.grad(total, params))
        return float(total.detach())


def time_updates(st, cfg, seconds, threads, use_expert=False, n_rows=100_000, seed=0):
    """Gradient steps per second of EagerSAC on a synthetic buffer (NumPy sampler as the
    reference's: randint + normal from the legacy global-style stream)."""
    torch.set_num_threads(int(threads))
    S, A, B = cfg.S, cfg.A, cfg.B
    rs = np.random.RandomState(seed)
    buf = dict(s=rs.normal(size=(n_rows, S)).astype(np.float32), a=rs.uniform(-1, 1, (n_rows, A)).astype(np.float32),
               sp=rs.normal(size=(n_rows, S)).astype(np.float32), r=rs.normal(size=n_rows).astype(np.float32),
               d=np.zeros(n_rows, np.float32))
    eng = EagerSAC(st, cfg, use_expert=use_expert)
    g = np.random.RandomState(1)
    ex_s = torch.tensor(rs.normal(size=(20, S)).astype(np.float32))
    ex_sp = torch.tensor(rs.normal(size=(20, S)).astype(np.float32))
    gen = np.random.default_rng(2)
    tn = lambda x: torch.from_numpy(np.ascontiguousarray(x))
    n, t0 = 0, None
    while True:
        idx = g.randint(n_rows, size=B)
        u = [tn(g.normal(size=(B, A)).astype(np.float32)) for _ in range(2)]
        expert = None
        if use_expert:
            perm = np.arange(20)
            gen.shuffle(perm)
            h1, h2 = np.array_split(perm, 2)
            ue = [tn(g.normal(size=(len(h), A)).astype(np.float32)) for h in (h1, h2)]
            expert = ((ex_s[h1], ex_sp[h1], ue[0]), (ex_s[h2], ex_sp[h2], ue[1]), cfg.epsilon)
        u.append(tn(g.normal(size=(B, A)).astype(np.float32)))
        eng.update(tn(buf["s"][idx]), tn(buf["a"][idx]), tn(buf["sp"][idx]), tn(buf["r"][idx]), tn(buf["d"][idx]),
                   u[0], u[1], u[2], expert)
        n += 1
        if n == 2:
            t0 = time.perf_counter()          # after the first two (allocator warm-up)
        if t0 is not None and n > 4 and time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    return (n - 2) / el, n - 2, el, eng, buf


def time_model_fit(eng, buf, cfg, seconds, mb=200):
    S = cfg.S
    rs = np.random.RandomState(5)
    tn = lambda x: torch.from_numpy(np.ascontiguousarray(x))
    n_rows = buf["r"].shape[0]
    n, t0 = 0, None
    while True:
        bs = []
        for _ in range(2):
            i = rs.randint(n_rows, size=mb)
            bs.append((tn(buf["s"][i]), tn(buf["a"][i]), tn(buf["sp"][i][:, :S]), tn(buf["r"][i])))
        eng.model_fit_step(bs)
        n += 1
        if n == 2:
            t0 = time.perf_counter()
        if t0 is not None and n > 4 and time.perf_counter() - t0 >= seconds:
            break
    el = time.perf_counter() - t0
    return (n - 2) / el, n - 2, el

