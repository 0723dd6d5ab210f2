"""Log / import compatibility on CPU: the reference's pickled
{param, train, final} layout (sac_eo/common/logger.py:43-86), the run-list file train.py
gathers (:159-191), --import_file (train_utils.py:20-92) and --expert_file (train.py:65-86).

The reference's own log pickles under sac_eo/logs are not loaded here: the environment
forbids unpickling files shipped with the reference, even with an allow-list.  The layouts
below are the ones its writer code produces (weight lists [W0, b0, W1, b1, W2, b2] (+ logstd
(1, A)), a per_state_std expert head of 2A outputs, rms stats {t, mean, var} with the extra
'ignore' key of the MPO expert log), built by our own Logger."""
import os
import pickle

import numpy as np
import pytest

from sac_eo.common.logger import Logger, load_log
from sac_eo.common.normalizer import RunningNormalizers
from sac_eo.common.train_parser import create_train_parser, gather_inputs
from sac_eo.common.train_utils import import_inputs, load_expert, organize_rms_inputs


def _weights(rs, sizes):
    out = []
    for i, o in zip(sizes[:-1], sizes[1:]):
        out += [rs.normal(size=(i, o)).astype(np.float32), rs.normal(size=o).astype(np.float32)]
    return out


def _rms(rs, S, A, ignore=False):
    d = {}
    for k, n in (("s_rms", S), ("a_rms", A), ("r_rms", 1), ("delta_rms", S), ("ret_rms", 1)):
        d[k] = {"t": 50, "mean": rs.normal(size=n).astype(np.float32), "var": rs.uniform(.5, 2, n).astype(np.float32)}
        if ignore:
            d[k]["ignore"] = None
    return d


def _run_log(tmp_path, name, per_state_std=False, ignore=False, with_models=True):
    rs = np.random.RandomState(0)
    S, A = 3, 1
    inputs = gather_inputs(create_train_parser().parse_args(
        ["--env_name", "Pendulum-v1", "--actor_layers", "8", "8", "--critic_layers", "8", "8"]
        + (["--actor_per_state_std"] if per_state_std else [])))
    lg = Logger()
    for t in range(3):
        lg.log_train({"J_tot": float(t), "alpha_loss": np.float32(t * .1)})
    lg.log_params(inputs)
    aw = _weights(rs, [S, 8, 8, 2 * A if per_state_std else A]) + ([] if per_state_std else [np.zeros((1, A), np.float32)])
    final = {"actor_weights": aw, "critic_weights": [_weights(rs, [S, 8, 8, 1])], "rms_stats": _rms(rs, S, A, ignore)}
    if with_models:
        final["model_weights"] = [_weights(rs, [S + A, 512, 512, S + 1]) for _ in range(2)]
        final["reward_weights"] = [None, None]
    lg.log_final(final)
    lg.dump_and_save(str(tmp_path), name)
    return inputs, final


def test_logger_reference_layout_and_append(tmp_path):
    inputs, final = _run_log(tmp_path, "TEMPLOG_0")
    lg = Logger()
    lg.log_train({"J_tot": 9.0, "alpha_loss": np.float32(1.0), "new_key": 1})
    lg.log_params(inputs)
    lg.log_final(final)
    lg.dump_and_save(str(tmp_path), "TEMPLOG_0")           # appends the train arrays
    log = load_log(os.path.join(tmp_path, "TEMPLOG_0"))
    assert set(log) == {"param", "train", "final"}
    assert list(log["train"]["J_tot"]) == [0.0, 1.0, 2.0, 9.0]
    assert log["train"]["alpha_loss"].dtype == np.float32 and len(log["train"]["alpha_loss"]) == 4
    assert [w.shape for w in log["final"]["actor_weights"]] == [(3, 8), (8,), (8, 8), (8,), (8, 1), (1,), (1, 1)]
    assert log["param"]["actor_kwargs"]["actor_layers"] == [8, 8]


def test_load_log_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    p = os.path.join(tmp_path, "bad")
    with open(p, "wb") as fh:
        pickle.dump({"param": {}, "train": {}, "final": {"x": Evil()}}, fh)
    with pytest.raises(pickle.UnpicklingError):
        load_log(p)


def test_import_inputs_from_log(tmp_path):
    _, final = _run_log(tmp_path, "run0")
    with open(os.path.join(tmp_path, "runs"), "wb") as fh:         # the gathered run list
        pickle.dump([load_log(os.path.join(tmp_path, "run0"))], fh)
    d = gather_inputs(create_train_parser().parse_args(["--import_path", str(tmp_path), "--import_file", "runs"]))
    d["setup_kwargs"].update(idx=0)
    d = import_inputs(d)
    assert d["actor_kwargs"]["actor_layers"] == [8, 8]           # taken from the log's param
    for a, b in zip(d["actor_kwargs"]["actor_weights"], final["actor_weights"]):
        assert np.array_equal(a, b)
    assert len(d["model_kwargs"]["model_weights"]) == 2
    rms = RunningNormalizers(3, 1, 0.99, d["alg_kwargs"]["init_rms_stats"])
    assert np.array_equal(rms.s_rms.mean, final["rms_stats"]["s_rms"]["mean"])
    d2 = gather_inputs(create_train_parser().parse_args([]))
    d2["setup_kwargs"].update(idx=0)
    assert import_inputs(d2)["actor_kwargs"]["actor_weights"] is None


def test_expert_import_per_state_std_and_ignore_key(tmp_path):
    """An MPO-style expert log: per_state_std head (2A outputs) and rms stats with 'ignore'."""
    _, final = _run_log(tmp_path, "expert", per_state_std=True, ignore=True, with_models=False)
    with open(os.path.join(tmp_path, "expert_runs"), "wb") as fh:
        pickle.dump([load_log(os.path.join(tmp_path, "expert"))], fh)
    kw, rms_stats = load_expert(str(tmp_path), "expert_runs")
    assert "actor_squash" not in kw and kw["actor_per_state_std"] is True
    assert kw["actor_weights"][4].shape == (8, 2)
    rms = RunningNormalizers(3, 1, 0.99, rms_stats)               # instantiate(..., ignore=None)
    assert np.array_equal(rms.a_rms.mean, final["rms_stats"]["a_rms"]["mean"])
    flat = {"s_t": 1, "s_mean": np.zeros(3), "s_var": np.ones(3)}
    for k in ("a", "r", "delta", "ret"):
        flat.update({f"{k}_t": 1, f"{k}_mean": np.zeros(1), f"{k}_var": np.ones(1)})
    assert set(organize_rms_inputs(flat)) == {"s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms"}


def test_protocol5_log_round_trip_and_unreadable_file(tmp_path):
    """A log pickled with protocol 5 (numpy arrays through numeric._frombuffer) loads through
    the allow-list; our own writer uses protocol 4; an unreadable existing file is overwritten
    (the reference's ``except: pass``, logger.py:71-83)."""
    p = os.path.join(tmp_path, "p5")
    arr = np.arange(12, dtype=np.float32).reshape(3, 4)
    with open(p, "wb") as fh:
        pickle.dump({"param": {}, "train": {"x": arr}, "final": {"w": [arr.T.copy()]}}, fh, protocol=5)
    log = load_log(p)
    assert np.array_equal(log["train"]["x"], arr) and np.array_equal(log["final"]["w"][0], arr.T)
    lg = Logger()
    lg.log_train({"x": np.ones(4, np.float32)})
    lg.dump_and_save(str(tmp_path), "p5")                 # appends to the protocol-5 file
    assert load_log(p)["train"]["x"].shape == (4, 4)
    with open(p, "rb") as fh:
        assert fh.read(2) == b"\x80\x04"                  # protocol 4 header
    bad = os.path.join(tmp_path, "bad")
    with open(bad, "wb") as fh:
        fh.write(b"not a pickle")
    lg = Logger()
    lg.log_train({"y": 1.0})
    lg.dump_and_save(str(tmp_path), "bad")
    assert list(load_log(bad)["train"]["y"]) == [1.0]
