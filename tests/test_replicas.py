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


def test_bench_gpus_flag_spawns_ranks():
    """bench.py --gpus 2 (no launcher environment) relaunches itself as two ranks through
    torch.distributed.run; each rank's learner seeds are run index = rank of the reference's
    derivation (sac_eo/train.py:108-128).  --plan-only keeps it on the CPU (gloo)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plan-only"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == [0, 1] and all(r["world_size"] == 2 for r in ranks)
    ref = derive_seeds(0, runs=2)
    for r in ranks:
        for k, v in r["seeds"].items():
            assert v == int(ref[k][r["rank"]])
        assert r["group_world_size"] == 2                 # the process group the ranks joined
    # the N > 1 line carries every rank's time, the group size and the C4 RCCL leg
    assert {"rank_times_s", "group_world_size", "dp_c4"} <= set(line["line_fields_n_gt_1"])
    leg = line["dp_c4_leg"]
    assert leg["ranks"] == 2 and leg["mode"] == "dpcheck" and "dp_ranks_identical" in leg["fields"]


def test_bench_gpus_mismatch_fails_loudly():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--plan-only"],
                         capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr
