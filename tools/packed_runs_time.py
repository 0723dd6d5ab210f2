"""Wall time of ``python -m sac_eo.train --runs K`` as K lock-step packed seeds vs the same K runs
one after another (--serial_runs), on one GPU.  Usage: packed_runs_time.py [K] [alg] [steps]."""
import os
import sys
import tempfile
import time

sys.path[:0] = ["sac-expert_amd"]

from sac_eo.train import main   # noqa: E402
from sac_eo.common.logger import load_log   # noqa: E402
import numpy as np   # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
alg = sys.argv[2] if len(sys.argv) > 2 else "sac_imit"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
argv = ["--alg_type", alg, "--env_name", "HalfCheetah-v3", "--actor_layers", "256", "256",
        "--critic_layers", "256", "256", "--actor_activations", "relu", "--critic_activations", "relu",
        "--total_timesteps", str(steps), "--env_batch_size_init", "1000", "--model_num_epochs", "1",
        "--seed", "0", "--runs", str(K)]
out = {}
for mode in ("packed", "serial"):
    d = tempfile.mkdtemp()
    t0 = time.perf_counter()
    path = main(argv + ["--save_path", d] + (["--serial_runs"] if mode == "serial" else []))
    out[mode] = time.perf_counter() - t0
    logs = load_log(path)
    parts = {k: sum(float(np.sum(lg["train"].get(k, 0.0))) for lg in logs)
             for k in ("time_env_data", "time_model_fit", "expert_time")}
    print(f"  {mode} parts summed over runs (s): " + ", ".join(f"{k} {v:.2f}" for k, v in parts.items()))
    print(f"{mode}: {K} runs of {alg} (256x2, {steps} steps: 1000 collected, {steps - 1000} loop steps with updates) "
          f"in {out[mode]:.1f} s", flush=True)
print(f"packed / serial speed-up: {out['serial'] / out['packed']:.2f}x")
