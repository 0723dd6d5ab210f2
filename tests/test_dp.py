"""Data-parallel mode (config C4, include/sacx.h sacx_dp_init) on CPU: world_size 2 over
gloo.  Each rank runs the oracle update on its half of a global batch and sums every
optimiser's gradients over the ranks (scale 1/2) before Adam -- the protocol libsacx runs
with RCCL inside the update graph.  Both ranks must end bit-identical to each other and
equal (fp64 rounding) to the single-learner update on the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import sac_oracle as O

S, A, B, STEPS = 5, 2, 16, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup():
    cfg = O.Config(S=S, A=A, hidden=(16, 16), act="tanh", B=B)
    st = O.init_state(cfg, seed=4, bias_scale=0.05).astype(np.float64)
    rs = np.random.RandomState(11)
    steps = []
    for _ in range(STEPS):
        batch = (rs.normal(size=(B, S)), rs.uniform(-1, 1, (B, A)), rs.normal(size=(B, S)),
                 rs.normal(size=B), (rs.uniform(size=B) < 0.2).astype(np.float64))
        noise = [O.f32_noise(rs.normal(size=(B, A))).astype(np.float64) for _ in range(3)]
        steps.append((batch, noise))
    return cfg, st, O.Normalizers.identity(S, A), steps


def _flat(st):
    return np.concatenate([x.ravel() for x in st.actor + [st.logstd] + st.q[0] + st.q[1] + st.q_targ[0]
                           + st.q_targ[1] + [np.atleast_1d(st.alpha)]])


def _worker(rank, ws, port, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    cfg, st, nrm, steps = _setup()
    lo, hi = rank * B // ws, (rank + 1) * B // ws
    cfg.B = hi - lo

    def allreduce_mean(name, grads):
        out = []
        for g in grads:
            t = torch.from_numpy(np.array(g, np.float64, copy=True))
            dist.all_reduce(t)
            out.append((t.numpy() * (1.0 / ws)).astype(np.float64))
        return out

    for batch, noise in steps:
        local = tuple(x[lo:hi] for x in batch)
        O.sac_update(st, cfg, nrm, local, *(n[lo:hi] for n in noise), grad_hook=allreduce_mean)
    dist.destroy_process_group()
    q.put((rank, _flat(st)))


def test_dp_two_ranks_equal_global_batch():
    ws = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, qu)) for r in range(ws)]
    for p in procs:
        p.start()
    out = sorted(qu.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(out[0][1], out[1][1])          # replicas stay identical
    cfg, st, nrm, steps = _setup()
    for batch, noise in steps:
        O.sac_update(st, cfg, nrm, batch, *noise)
    ref = _flat(st)
    assert np.max(np.abs(out[0][1] - ref)) <= 1e-10 * np.max(np.abs(ref))
