"""Multi-replica plumbing on CPU: world_size 2 over gloo (the GPU path uses RCCL for the
same barrier / max-time calls and nothing else).  Seeds follow the reference's
derivation (sac_eo/train.py:108-118)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sac_eo.common.seeding import derive_seeds


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, ws, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(ws), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from sac_eo.common.replicas import init_replica
    rep = init_replica(backend="gloo", use_cuda=False)
    seeds = rep.seeds(0)
    rep.barrier()
    t = rep.max_over_ranks(1.0 + rank)          # each rank's "elapsed"
    total = rep.sum_over_ranks(100.0)           # each rank did 100 updates
    uid = rep.broadcast_bytes(bytes(range(128)) if rank == 0 else None)   # dp-mode RCCL id hand-off
    rep.close()
    q.put((rank, seeds, t, total, uid))


@pytest.mark.parametrize("ws", [2])
def test_two_replicas_gloo(ws):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    ref = derive_seeds(0, runs=ws)
    for rank, seeds, t, total, uid in out:
        assert uid == bytes(range(128))
        assert t == float(ws)                   # max over ranks of (1 + rank)
        assert total == 100.0 * ws              # aggregate = sum of per-replica work
        for k, v in seeds.items():
            assert v == int(ref[k][rank])
    # independent learners: every stream differs between the replicas
    assert all(out[0][1][k] != out[1][1][k] for k in out[0][1])


def test_seed_derivation_known_answers():
    """--seed 0, run 0 -> the seeds logged in the reference's sac_eo/logs/TEMPLOG_0."""
    s = derive_seeds(0, runs=1)
    assert int(s["setup"][0]) == 2773201285
    assert int(s["sim"][0]) == 397334063
    assert int(s["eval"][0]) == 3968933684
    assert int(s["expert"][0]) == 2590541744
    # runs_start slices the same streams
    s2 = derive_seeds(0, runs=3)
    s3 = derive_seeds(0, runs=2, runs_start=1)
    assert np.array_equal(s2["setup"][1:], s3["setup"])
