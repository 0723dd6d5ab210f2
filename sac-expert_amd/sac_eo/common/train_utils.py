"""Log-driven inputs (reference ``sac_eo/common/train_utils.py:20-131`` and the expert
import of ``sac_eo/train.py:65-91``).

* ``import_inputs``: ``--import_file`` / ``--import_idx`` / ``--import_all`` re-initialise
  the actor, the (V) critics, the world models and the normalisers from a log's ``final``
  entry, and take the env / net kwargs from its ``param`` entry.
* ``load_expert``: ``--expert_file`` -> (expert actor kwargs with the log's actor weights,
  the expert's normaliser stats).
* ``organize_rms_inputs``: a log's normaliser stats in the ``rms_stats`` schema
  ``{s_rms, a_rms, r_rms, delta_rms, ret_rms}: {t, mean, var}``, also from the flat
  ``s_t`` / ``s_mean`` / ... keys of older logs.
Logs are read with ``logger.load_log`` (allow-list unpickler: nothing in the file runs)."""
import copy
import os

from .logger import load_log

RMS_KEYS = ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms")


def organize_rms_inputs(final: dict) -> dict:
    if "rms_stats" in final:
        return final["rms_stats"]
    return {k: {"t": final[f"{k[:-4]}_t"], "mean": final[f"{k[:-4]}_mean"], "var": final[f"{k[:-4]}_var"]}
            for k in RMS_KEYS}


def import_inputs(inputs_dict: dict) -> dict:
    """train_utils.py:20-92: fills actor / critic / model weights and init_rms_stats (None
    without --import_file)."""
    sk = inputs_dict["setup_kwargs"]
    path, name = sk.get("import_path"), sk.get("import_file")
    actor_w = critic_w = model_w = reward_w = rms = None
    if path and name:
        logs = load_log(os.path.join(path, name))
        logs = logs if isinstance(logs, list) else [logs]
        run = sk["idx"] - sk.get("runs_start", 0)
        idx = sk.get("import_idx")
        if idx is None:
            idx = run if len(logs) > run else 0
        elif idx >= len(logs):
            raise AssertionError("import_idx too large")            # train_utils.py:43
        param, final = logs[idx]["param"], logs[idx]["final"]
        if sk.get("import_all"):
            setup = sk
            inputs_dict = copy.deepcopy(param)
            inputs_dict["setup_kwargs"] = setup
        else:
            for k in ("env_kwargs", "actor_kwargs", "critic_kwargs"):
                inputs_dict[k] = copy.deepcopy(param[k])
        actor_w, critic_w, rms = final["actor_weights"], final["critic_weights"], final["rms_stats"]
        if "model_weights" in final and "reward_weights" in final:
            model_w, reward_w = final["model_weights"], final["reward_weights"]
            inputs_dict["model_kwargs"] = copy.deepcopy(param["model_kwargs"])
            inputs_dict["model_setup_kwargs"] = copy.deepcopy(param["model_setup_kwargs"])
    inputs_dict["actor_kwargs"]["actor_weights"] = actor_w
    inputs_dict["critic_kwargs"]["critic_weights"] = critic_w
    inputs_dict["model_kwargs"]["model_weights"] = model_w
    inputs_dict["model_kwargs"]["reward_weights"] = reward_w
    inputs_dict["alg_kwargs"]["init_rms_stats"] = rms
    return inputs_dict


def load_expert(expert_path: str, expert_file: str):
    """train.py:65-86: the first run of an expert log -> (actor kwargs carrying its weights,
    its normaliser stats).  The reference drops ``actor_squash`` / ``actor_adversary_prob``
    from the kwargs (so the expert is built by init_actor's defaults)."""
    logs = load_log(os.path.join(expert_path, expert_file))
    log = logs[0] if isinstance(logs, list) else logs
    kw = copy.deepcopy(log["param"]["actor_kwargs"])
    kw["actor_weights"] = log["final"]["actor_weights"]
    for k in ("actor_squash", "actor_adversary_prob"):
        if kw.get(k) is not None:
            kw.pop(k)
    return kw, organize_rms_inputs(log["final"])
