"""The host side of the drop-in training loop on CPU, over a stand-in engine (tests/fake_engine.py):
``sac_eo.train``'s construction sequence, both algorithms' loops (request generators), the
per-episode normaliser hooks, checkpoints and gathered logs, and --runs in lock-step (one batched
act / update / append per round) against the same runs one after another.  The arithmetic is the
GPU tests' (test_gpu_loop.py, test_gpu_train.py)."""
import numpy as np
import pytest

import fake_engine


def _argv(alg, tmp, extra=()):
    return ["--alg_type", alg, "--env_name", "HalfCheetah-v3", "--actor_layers", "16", "16", "--critic_layers", "16",
            "16", "--model_layers", "16", "16", "--total_timesteps", "2600", "--env_batch_size_init", "300",
            "--env_horizon", "200", "--sac_batch_size", "32", "--model_batch_size", "50", "--model_num_epochs", "1",
            "--seed", "3", "--save_path", str(tmp)] + list(extra)


@pytest.mark.parametrize("alg", ["sac", "sac_imit"])
@pytest.mark.parametrize("extra", [(), ("--update_normalizers",), ("--update_normalizers", "--only_model_normalizer"),
                                   ("--eval_freq", "1000", "--eval_num_traj", "1")])
def test_train_loop_host(monkeypatch, tmp_path, alg, extra):
    fake_engine.install(monkeypatch)
    from sac_eo.train import main
    from sac_eo.common.logger import load_log
    log = load_log(main(_argv(alg, tmp_path, extra)))[0]
    tr = log["train"]
    assert len(tr["J_tot"]) >= 3                           # the collection + two finished 1000-step episodes
    if alg == "sac_imit":
        assert len(tr["p_loss"]) == 2600 - 300             # one update per env step
        assert len(tr["model_MSE_on_expert_data"]) == 3    # one model fit per episode start
    if "--eval_freq" in extra:
        assert len(tr["J_tot_eval"]) == 4 and list(tr["steps_eval"]) == [0, 1000, 1000, 600]
    if "--update_normalizers" in extra:
        rms = log["final"]["rms_stats"]
        assert rms["s_rms"]["t"] == (0 if "--only_model_normalizer" in extra else 300 + 2000)


@pytest.mark.parametrize("alg", ["sac", "sac_imit"])
def test_packed_runs_host(monkeypatch, tmp_path, alg):
    """--runs 3 in lock-step: one batched act / append and ONE packed step per env step; the
    logs equal the serial runs' (the stand-in engine is deterministic per seed)."""
    fake_engine.install(monkeypatch)
    from sac_eo.train import main
    from sac_eo.common.logger import load_log
    engines = []
    orig = fake_engine.FakeEngine.__init__

    def track(self, cfg, *a, **k):
        orig(self, cfg, *a, **k)
        engines.append(self)
    monkeypatch.setattr(fake_engine.FakeEngine, "__init__", track)
    packed = load_log(main(_argv(alg, tmp_path / "p", ["--runs", "3", "--cores", "1"])))
    big = [e for e in engines if e.seeds == 3]
    assert len(big) == 1 and big[0].cfg.single_seed_plan
    steps = [c for c in big[0].calls if isinstance(c, tuple)]
    assert big[0].calls.count("act_seeds") == 300 + 2300 and big[0].calls.count("append_seeds") == 2300
    assert len(steps) == (2300 if alg == "sac_imit" else 2 * 334 + 1 * 100)
    serial = load_log(main(_argv(alg, tmp_path / "s", ["--runs", "3", "--serial_runs", "--cores", "1"])))
    for a, b in zip(packed, serial):
        for k in a["train"]:
            if "time" not in k:
                assert np.array_equal(np.asarray(a["train"][k]), np.asarray(b["train"][k]), equal_nan=True), k


def test_pool_size_and_split():
    """--cores as the reference's Pool size (train.py:148-152), capped by the usable cores and
    MAX_PROCS_PER_GPU; without it one packed process per GPU (processes sharing a GPU time-slice
    it); runs dealt round-robin over the processes."""
    import argparse
    from sac_eo import train as T
    ns = lambda cores: argparse.Namespace(cores=cores)
    usable = len(__import__("os").sched_getaffinity(0))
    assert T.pool_size(ns(None), 1) == 1
    assert T.pool_size(ns(1), 8) == 1
    assert T.pool_size(ns(None), 8) == 1
    assert T.pool_size(ns(8), 8) == min(8, usable, T.MAX_PROCS_PER_GPU)
    assert T.pool_size(ns(3), 2) == min(2, usable)
