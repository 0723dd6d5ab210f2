"""The build's host mirrors (and the oracle's restatements) against vectors the REFERENCE's own
NumPy-only modules produced (tests/golden/make_ref_fixtures.py, run in the build container
with /root/reference on sys.path): bit for bit.

  buffers.py:41-71, :107-144          TrajectoryBuffer.add FIFO / get_offmodel_info  (oracle ring)
  normalizer.py:26-190                RunningNormalizers: update_rms, normalize, instantiate
  buffer_utils.py:8-9                 discounted_sum (scipy lfilter)
  logger.py:5-91                      Logger.dump_and_save over two checkpoints
  train_parser.py                     every default, all_kwargs groups, parsed command lines
  train_utils.py:20-131               import_inputs / organize_rms_inputs
  samplers.py:3-122, corruptor.py     trajectory_sampler (+ corruptor), batch_simtrajectory_sampler
The device-side counterparts (ring, sampler gather, rollout) are in test_gpu_ref_fixtures.py."""
import json
import os

import numpy as np
import pytest

import ref_ducks as D

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def F():
    with np.load(os.path.join(GOLD, "ref_fixtures.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def M():
    with open(os.path.join(GOLD, "ref_fixtures.json")) as fh:
        return json.load(fh)


def same(a, b):
    """Bit-identical values and identical dtype."""
    a, b = np.asarray(a), np.asarray(b)
    return a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


def from_json(x):
    if isinstance(x, dict):
        if "__nd__" in x:
            return np.array(x["__nd__"], dtype=x["dtype"]).reshape(x["shape"])
        if "__np__" in x:
            return np.dtype(x["dtype"]).type(x["__np__"])
        return {k: from_json(v) for k, v in x.items()}
    if isinstance(x, list):
        return [from_json(v) for v in x]
    return x


def deep_equal(a, b, path="$"):
    if isinstance(b, dict):
        assert isinstance(a, dict) and set(a) == set(b), (path, sorted(a) if isinstance(a, dict) else a, sorted(b))
        for k in b:
            deep_equal(a[k], b[k], f"{path}.{k}")
    elif isinstance(b, (list, tuple)):
        assert isinstance(a, (list, tuple)) and len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            deep_equal(x, y, f"{path}[{i}]")
    elif isinstance(b, (np.ndarray, np.generic)):
        assert same(a, b), (path, a, b)
    else:
        assert type(a) is type(b) and a == b, (path, a, b)


# ------------------------------------------------------------------ parser
def test_parser_defaults_and_groups(M):
    from sac_eo.common.train_parser import all_kwargs, create_train_parser, gather_inputs
    ref = M["parser"]
    assert all_kwargs == ref["all_kwargs"]                 # the logged param layout, group order included
    for cli, parsed in zip(ref["cli"], ref["parsed"]):
        ns = create_train_parser().parse_args(cli)
        got = vars(ns)
        extra = {k: got.pop(k) for k in ("gpus", "serial_runs")}   # the build's own two flags
        assert extra == {"gpus": None, "serial_runs": False}
        assert got == parsed
        assert {k: type(v) for k, v in got.items()} == {k: type(v) for k, v in parsed.items()}
        grouped = gather_inputs(ns)
        assert {g: list(d) for g, d in grouped.items()} == ref["all_kwargs"]


# ------------------------------------------------------------------ normalisers
def _norm_classes():
    from sac_eo.common.normalizer import RunningNormalizers
    import sac_loop
    return [RunningNormalizers, sac_loop.RunningNorms]


@pytest.mark.parametrize("which", [0, 1], ids=["product", "oracle"])
def test_running_normalizers_update_rms(F, which):
    cls = _norm_classes()[which]
    nr = cls(5, 2, 0.995)
    for i in range(6):
        nr.update_rms(*(F[f"norm.upd{i}.{k}"] for k in ("s", "a", "r", "sp")))
        for k in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms"):
            n = getattr(nr, k)
            p = f"norm.upd{i}.{k}"
            assert n.t_last == int(F[p + ".t"])
            # dim-1 normalisers hold NumPy scalars / 0-d arrays after an update: compare values and dtype
            for f in ("mean", "var", "std"):
                assert same(np.asarray(getattr(n, f)), F[f"{p}.{f}"]), (i, k, f, getattr(n, f), F[f"{p}.{f}"])


def test_normalize_denormalize_instantiate(F):
    from sac_eo.common.normalizer import RunningNormalizers
    nr = RunningNormalizers(5, 2, 0.995)
    for i in range(6):
        nr.update_rms(*(F[f"norm.upd{i}.{k}"] for k in ("s", "a", "r", "sp")))
    x = F["norm.nd.x"]
    assert same(nr.s_rms.normalize(x), F["norm.nd.n"])
    assert same(nr.s_rms.normalize(x, center=False), F["norm.nd.nc"])
    assert same(nr.s_rms.denormalize(x), F["norm.nd.dn"])
    assert same(nr.s_rms.denormalize(x, center=False), F["norm.nd.dnc"])
    for t in (0, 1, 5):
        m = RunningNormalizers(5, 2, 0.995)
        ks = ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms")
        m.set_rms_stats({k: {"t": t, "mean": F[f"norm.inst{t}.{k}.mean"], "var": F[f"norm.inst{t}.{k}.var"]}
                         for k in ks})
        for k in ks:
            assert same(np.asarray(getattr(m, k).std), F[f"norm.inst{t}.{k}.std"]), (t, k)
            assert same(np.asarray(getattr(m, k).mean), F[f"norm.inst{t}.{k}.mean_out"]), (t, k)


@pytest.mark.parametrize("which", [0, 1], ids=["product", "oracle"])
def test_discounted_sum(F, which):
    from sac_eo.common.normalizer import discounted_sum as P
    import sac_loop
    f = (P, sac_loop.discounted_sum)[which]
    for i in range(4):
        y = f(F[f"dsum{i}.x"], float(F[f"dsum{i}.rate"]))
        assert same(y, F[f"dsum{i}.y"]), i


# ------------------------------------------------------------------ replay buffer (oracle ring)
def test_oracle_buffer_fifo_and_sample(F, M):
    import sac_loop
    B = M["buf"]
    buf = sac_loop.Buffer(B["S"], B["A"], B["cap"])
    for i, _n in enumerate(B["lens"]):
        buf.add(*(F[f"buf.add{i}.{k}"] for k in ("s", "a", "r", "sp", "d")))
        assert buf.current_size == F["buf.sizes"][i][0]
    for k in ("s", "a", "sp"):
        assert np.array_equal(getattr(buf, k), F[f"buf.{k}_all"]), k
    assert same(buf.r, F["buf.r_all"]) and same(buf.d, F["buf.d_all"])      # float64 r and d, as the reference's
    for seed in B["seeds"]:
        rs = np.random.RandomState(seed)
        idx = rs.randint(buf.current_size, size=B["B"])          # buffers.py:136
        for k in ("s", "a", "sp"):
            assert np.array_equal(getattr(buf, k)[idx], F[f"buf.sample{seed}.{k}"])
        assert np.array_equal(rs.randint(2 ** 31, size=4), F[f"buf.sample{seed}.after"])


# ------------------------------------------------------------------ logger + train_utils
def test_logger_two_checkpoints(F, tmp_path):
    from sac_eo.common.logger import Logger, load_log
    rs = np.random.RandomState(31)
    lg = D.fill_run_log(Logger, rs, 0, 5)
    lg.dump_and_save(str(tmp_path), "LOG_0")
    lg.reset()
    lg2 = D.fill_run_log(Logger, rs, 0, 3)
    lg2.log_train({"new_key": 7.0})
    lg2.dump_and_save(str(tmp_path), "LOG_0")
    ref = load_log(os.path.join(GOLD, "ref_logger.pkl"))          # the allow-list loader reads the reference's file
    got = load_log(str(tmp_path / "LOG_0"))
    deep_equal(got, ref)
    assert list(got["train"]) == list(ref["train"])                # key order (the merged dict's)
    with open(os.path.join(GOLD, "ref_logger.pkl"), "rb") as fh, open(tmp_path / "LOG_0", "rb") as gh:
        assert fh.read() == gh.read()                              # the same bytes on disk


def test_import_inputs_and_rms_organisation(M):
    from sac_eo.common.train_utils import import_inputs, organize_rms_inputs
    from sac_eo.common.train_parser import all_kwargs
    for case in M["import_cases"]:
        c = case["case"]
        inp = {g: {} for g in all_kwargs}
        inp["setup_kwargs"] = {"import_path": GOLD, "import_file": "ref_runs.pkl", "import_idx": c["import_idx"],
                               "import_all": c["import_all"], "idx": c["idx"], "runs_start": 0}
        inp["env_kwargs"] = {"env_name": "mine"}
        deep_equal(import_inputs(inp), from_json(case["out"]))
    deep_equal(organize_rms_inputs(from_json(M["rms_flat"])), from_json(M["rms_organized"]))


def test_import_idx_too_large():
    from sac_eo.common.train_utils import import_inputs
    from sac_eo.common.train_parser import all_kwargs
    inp = {g: {} for g in all_kwargs}
    inp["setup_kwargs"] = {"import_path": GOLD, "import_file": "ref_runs.pkl", "import_idx": 2, "import_all": False,
                           "idx": 0, "runs_start": 0}
    with pytest.raises(AssertionError):
        import_inputs(inp)


# ------------------------------------------------------------------ samplers + corruptor
def _corruptor_norm(F):
    from sac_eo.common.normalizer import RunningNormalizers
    nr = RunningNormalizers(4, 2, 0.99)
    rs = np.random.RandomState(41)
    s0 = rs.normal(size=(40, 4)).astype(np.float32)
    assert np.array_equal(s0, F["samp.norm_upd.s"])
    nr.update_rms(s0, rs.normal(size=(40, 2)).astype(np.float32), rs.normal(size=40).astype(np.float32),
                  (s0 + rs.normal(size=(40, 4))).astype(np.float32))
    return nr, rs


def _sampler_case(F, M, i, runner):
    from sac_eo.common.corruptor import TrajectoryCorruptor
    c = M["samplers"]["traj_cases"][i]
    nr, _ = _corruptor_norm(F)
    env = D.DuckEnv(4, 2, seed=100 + i, term_at=c["term_at"])
    actor = D.DuckActor(4, 2, seed=200 + i)
    corr = None
    if c["noise"] > 0 or i == 0:
        corr = TrajectoryCorruptor(c["noise"], c["ntype"])
        corr.set_rms(nr)
    np.random.seed(300 + i)
    res = runner(env, actor, c, corr)
    names = ("s", "a", "r", "sp", "d") + (("J",) if c["eval"] else ())
    assert len(res) == len(names)
    for k, v in zip(names, res):
        assert same(v, F[f"samp{i}.{k}"]), (i, k)
    assert np.array_equal(np.random.randint(2 ** 31, size=4), F[f"samp{i}.after"])
    if corr is not None:
        assert np.array_equal(corr.s_noise_rng.integers(2 ** 31, size=4), F[f"samp{i}.cafter"])


@pytest.mark.parametrize("i", range(5))
def test_trajectory_sampler(F, M, i):
    from sac_eo.common.samplers import trajectory_sampler
    _sampler_case(F, M, i, lambda env, actor, c, corr: trajectory_sampler(
        env, actor, c["h"], eval=c["eval"], deterministic=c["det"], corruptor=corr))


@pytest.mark.parametrize("i", [0, 1, 2, 3, 4])
def test_train_loop_trajectory_steps(F, M, i):
    """The training loops' own collection (SACBase._trajectory_steps: the act requests of
    trajectory_sampler(eval=True) as a generator) against the same reference vectors."""
    from sac_eo.algs.base import SACBase
    c = M["samplers"]["traj_cases"][i]
    if not c["eval"]:
        pytest.skip("the loops always collect with eval=True")

    class Host:
        pass

    def run(env, actor, c, corr):
        from sac_eo.common.corruptor import TrajectoryCorruptor
        h = Host()
        h.actor = actor
        h.corruptor = corr if corr is not None else TrajectoryCorruptor(0.0)
        gen = SACBase._trajectory_steps(h, env, c["h"], c["det"])
        try:
            req = next(gen)
            while True:
                assert req[0] == "act"
                req = gen.send(actor.sample(req[1], deterministic=req[2]).numpy())
        except StopIteration as stop:
            return stop.value
    _sampler_case(F, M, i, run)


def test_corruptor_stream(F):
    from sac_eo.common.corruptor import TrajectoryCorruptor
    nr, rs = _corruptor_norm(F)
    corr = TrajectoryCorruptor(0.7, "all")
    corr.set_rms(nr)
    for i in range(3):
        assert same(corr.corrupt_samples(F[f"corr{i}.x"]), F[f"corr{i}.y"]), i


@pytest.mark.parametrize("j", range(3))
def test_oracle_rollout_vs_batch_simtrajectory_sampler(F, M, j):
    """oracle.rollout (the checker of the device rollout) against the reference's
    batch_simtrajectory_sampler driven by the oracle's actor.sample and MSEModel.step."""
    import sac_oracle as O
    c = M["samplers"]["roll_cases"][j]
    cfg = O.Config(S=17, A=6, hidden=(32, 32), act="tanh", B=8, model_hidden=(64, 64))
    st = O.init_state(cfg, seed=c["seed"], with_models=True, bias_scale=0.05, actor_gain=0.5,
                      model_gain=0.3).astype(np.float64)
    rs = np.random.RandomState(600 + j)
    got = O.rollout(st, cfg, O.Normalizers.identity(17, 6), F[f"roll{j}.s_init"], c["H"], 1, rs, c["det"])
    for k, v in zip(("s", "a", "r", "sp", "d"), got):
        assert np.array_equal(v, F[f"roll{j}.{k}"]), (j, k)
    assert np.array_equal(rs.randint(2 ** 31, size=4), F[f"roll{j}.after"])
