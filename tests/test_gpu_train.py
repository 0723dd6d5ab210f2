"""End-to-end ``sac_eo.train`` on the GPU at tiny sizes: the reference's construction
sequence, env loop, model fitting and checkpoint, through the device engine."""
import json
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
    names = main(argv)
    assert len(names) == 1
    with open(os.path.join(tmp_path, names[0] + ".json")) as fh:
        log = json.load(fh)
    assert "actor_weights" in log["final"]
    arrs = np.load(os.path.join(tmp_path, names[0] + ".npz"))
    w = [arrs[k] for k in arrs.files if k.startswith("log.final.actor_weights")]
    assert w and all(np.all(np.isfinite(x)) for x in w)
    assert np.isfinite(log["final"]["alpha"])
    assert len(log["train"]["J_tot"]) >= 3          # the collection batch + 2 finished 1000-step episodes
    if alg == "sac_imit":
        assert log["train"]["model_updates"][-1] == 2 * 2600 // 50 // 2 or log["train"]["model_updates"][-1] > 0
        assert np.isfinite(log["train"]["model_loss_last"][-1])
        # expert diagnostics on the device (SAC_expert.py:579-608), no longer NaN placeholders
        assert np.isfinite(log["train"]["model_MSE_on_expert_data"][-1])
        assert np.isfinite(log["train"]["model_MSE_on_expert_counterfactual_action"][-1])
