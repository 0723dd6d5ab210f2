"""End-to-end ``sac_eo.train`` on the GPU at tiny sizes: the reference's construction
sequence, env loop, model fitting and checkpoint, through the device engine."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("alg", ["sac", "sac_imit"])
def test_train_entry_point(gpu_available, tmp_path, alg):
    from sac_eo.train import main
    argv = ["--alg_type", alg, "--env_name", "HalfCheetah-v3", "--actor_layers", "64", "64",
            "--critic_layers", "64", "64", "--actor_activations", "relu", "--critic_activations", "relu",
            "--model_layers", "64", "64", "--total_timesteps", "2600", "--env_batch_size_init", "300",
            "--env_horizon", "200", "--sac_batch_size", "64", "--model_batch_size", "50",
            "--model_num_epochs", "1", "--seed", "3", "--save_path", str(tmp_path)]
    path = main(argv)
    # the reference's gathered log: a list of runs, each {param, train, final} (train.py:159-191)
    from sac_eo.common.logger import load_log
    logs = load_log(path)
    assert isinstance(logs, list) and len(logs) == 1
    log = logs[0]
    assert set(log) == {"param", "train", "final"}
    assert os.listdir(tmp_path) == [os.path.basename(path)]        # per-run checkpoints gathered and removed
    w = log["final"]["actor_weights"]
    assert len(w) == 7 and all(np.all(np.isfinite(x)) for x in w)    # [W0, b0, W1, b1, W2, b2, logstd]
    assert np.isfinite(log["final"]["alpha"])
    assert len(log["train"]["J_tot"]) >= 3          # the collection batch + 2 finished 1000-step episodes
    if alg == "sac_imit":
        assert log["train"]["model_updates"][-1] > 0
        assert np.isfinite(log["train"]["model_loss_last"][-1])
        # expert diagnostics on the device (SAC_expert.py:579-608)
        assert np.isfinite(log["train"]["model_MSE_on_expert_data"][-1])
        assert np.isfinite(log["train"]["model_MSE_on_expert_counterfactual_action"][-1])
        # one alpha_loss / p_loss / epsilon entry per gradient step (SAC_expert.py:351-356)
        n_upd = 2600 - 300
        for k in ("alpha_loss", "p_loss", "epsilon"):
            assert len(log["train"][k]) == n_upd, (k, len(log["train"][k]))
        assert np.all(np.isfinite(log["train"]["p_loss"]))
        assert len(log["final"]["model_weights"]) == 2


def test_train_one_model_and_imported_expert(gpu_available, tmp_path):
    """--num_models 1 with --model_max_grad_norm, and --expert_file pointing at a log this
    build wrote (its actor, built as the reference's plain GaussianActor, collects the expert
    data)."""
    from sac_eo.train import main
    from sac_eo.common.logger import load_log
    base = ["--env_name", "HalfCheetah-v3", "--actor_layers", "64", "64", "--critic_layers", "64", "64",
            "--actor_activations", "relu", "--critic_activations", "relu", "--model_layers", "64", "64",
            "--env_batch_size_init", "300", "--env_horizon", "200", "--sac_batch_size", "64",
            "--model_batch_size", "50", "--model_num_epochs", "1", "--seed", "5"]
    exp_dir = tmp_path / "experts"
    expert_log = main(base + ["--alg_type", "sac", "--total_timesteps", "600", "--save_path", str(exp_dir)])
    path = main(base + ["--alg_type", "sac_imit", "--num_models", "1", "--model_max_grad_norm", "0.5",
                        "--total_timesteps", "1600", "--expert_path", str(exp_dir),
                        "--expert_file", os.path.basename(expert_log), "--save_path", str(tmp_path / "run")])
    log = load_log(path)[0]
    assert len(log["final"]["model_weights"]) == 1
    assert np.all(np.isfinite(log["train"]["p_loss"])) and len(log["train"]["p_loss"]) == 1600 - 300
    assert log["train"]["expert_steps"][-1] == 20           # the imported expert collected the expert rows


def _same(x, y, what):
    """Nested lists / dicts of arrays and scalars, bit for bit."""
    if isinstance(x, dict):
        assert set(x) == set(y), what
        for k in x:
            _same(x[k], y[k], f"{what}.{k}")
    elif isinstance(x, (list, tuple)):
        assert len(x) == len(y), what
        for i, (u, v) in enumerate(zip(x, y)):
            _same(u, v, f"{what}[{i}]")
    elif x is None:
        assert y is None, what
    else:
        assert np.array_equal(np.asarray(x), np.asarray(y), equal_nan=True), what


def _logs_equal(a, b):
    """Two runs' checkpoint logs, bit for bit except wall-clock fields."""
    assert set(a["train"]) == set(b["train"])
    for k in a["train"]:
        if "time" not in k:
            _same(a["train"][k], b["train"][k], k)
    _same(a["final"], b["final"], "final")


@pytest.mark.parametrize("alg,extra", [("sac_imit", ["--cores", "1"]), ("sac", ["--cores", "1"]),
                                       ("sac_imit", ["--cores", "1", "--update_normalizers", "--only_model_normalizer"]),
                                       ("sac_imit", ["--cores", "2"])])
def test_packed_runs_equal_serial_runs(gpu_available, tmp_path, alg, extra):
    """--runs 3 as three lock-step seeds of one packed handle (sac_eo.algs.lockstep) -- or, with
    --cores 2, as two spawned processes on the GPU with runs {0, 2} packed and {1} alone (the
    reference's process pool) -- vs the same three runs one after another: every run's log
    identical, bit for bit."""
    from sac_eo.train import main
    from sac_eo.common.logger import load_log
    argv = ["--alg_type", alg, "--env_name", "HalfCheetah-v3", "--actor_layers", "64", "64",
            "--critic_layers", "64", "64", "--actor_activations", "relu", "--critic_activations", "relu",
            "--model_layers", "64", "64", "--total_timesteps", "1400", "--env_batch_size_init", "300",
            "--env_horizon", "200", "--sac_batch_size", "64", "--model_batch_size", "50",
            "--model_num_epochs", "1", "--seed", "11", "--runs", "3"] + extra
    packed = load_log(main(argv + ["--save_path", str(tmp_path / "packed")]))
    serial = load_log(main(argv + ["--serial_runs", "--cores", "1", "--save_path", str(tmp_path / "serial")]))
    assert len(packed) == len(serial) == 3
    for a, b in zip(packed, serial):
        _logs_equal(a, b)
    # the runs are different learners (different seeds)
    assert not np.array_equal(packed[0]["final"]["actor_weights"][0], packed[1]["final"]["actor_weights"][0])
