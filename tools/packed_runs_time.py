"""Wall time of ``python -m sac_eo.train --runs K`` on one GPU: the K runs one after another
(--serial_runs --cores 1), as K lock-step packed seeds of one handle (--cores 1), and as P spawned
processes (--cores P) each packing K/P seeds -- the reference's process pool.
Usage: packed_runs_time.py [K] [alg] [steps] [P,P,...]."""
import os
import sys
import tempfile
import time

sys.path[:0] = ["sac-expert_amd"]

from sac_eo.train import main   # noqa: E402
from sac_eo.common.logger import load_log   # noqa: E402
import numpy as np   # noqa: E402


def run():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    alg = sys.argv[2] if len(sys.argv) > 2 else "sac_imit"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    pools = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else [2, 4]
    argv = ["--alg_type", alg, "--env_name", "HalfCheetah-v3", "--actor_layers", "256", "256",
            "--critic_layers", "256", "256", "--actor_activations", "relu", "--critic_activations", "relu",
            "--total_timesteps", str(steps), "--env_batch_size_init", "1000", "--model_num_epochs", "1",
            "--seed", "0", "--runs", str(K)]
    modes = [("serial", ["--serial_runs", "--cores", "1"]), ("packed", ["--cores", "1"])] + \
            [(f"pool{p}", ["--cores", str(p)]) for p in pools]
    out, ref = {}, None
    for mode, extra in modes:
        d = tempfile.mkdtemp()
        t0 = time.perf_counter()
        path = main(argv + ["--save_path", d] + extra)
        out[mode] = time.perf_counter() - t0
        logs = load_log(path)
        if ref is None:
            ref = logs
        same = all(np.array_equal(np.asarray(a["train"][k]), np.asarray(b["train"][k]), equal_nan=True)
                   for a, b in zip(logs, ref) for k in a["train"] if "time" not in k)
        print(f"{mode}: {K} runs of {alg} (256x2, {steps} steps: 1000 collected, {steps - 1000} loop steps with "
              f"updates) in {out[mode]:.1f} s = {out['serial'] / out[mode]:.2f}x serial; logs equal serial: {same}",
              flush=True)


if __name__ == "__main__":     # spawned pool workers import this module: no work at import
    run()
