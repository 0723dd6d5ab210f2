"""Generates tests/golden/ref_*.{npz,json,pkl}: input / output vectors of the REFERENCE's own
NumPy-only modules, run here in the build container (they need no TensorFlow).

Build-container only: it puts /root/reference on sys.path and imports
  sac_eo.common.buffers.TrajectoryBuffer            (buffers.py:5-186)
  sac_eo.common.normalizer.RunningNormalizers       (normalizer.py:5-190)
  sac_eo.common.buffer_utils.discounted_sum         (buffer_utils.py:8-9)
  sac_eo.common.logger.Logger                       (logger.py:5-91)
  sac_eo.common.train_parser.create_train_parser / all_kwargs  (train_parser.py)
  sac_eo.common.train_utils.import_inputs / organize_rms_inputs (train_utils.py:20-131)
  sac_eo.common.samplers.trajectory_sampler / batch_simtrajectory_sampler (samplers.py:3-122)
  sac_eo.common.corruptor.TrajectoryCorruptor       (corruptor.py:3-30)
and records what they return on seeded inputs.  The fixtures are data only (arrays, JSON,
and pickles the reference's Logger wrote, read back in the tests through the build's
allow-list loader); no reference source text is stored.  The GPU box never runs this.

Run:  python tests/golden/make_ref_fixtures.py
"""
import json
import os
import pickle
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, REF)
from sac_eo.common.buffers import TrajectoryBuffer                       # noqa: E402
from sac_eo.common.normalizer import RunningNormalizers                  # noqa: E402
from sac_eo.common.buffer_utils import discounted_sum                    # noqa: E402
from sac_eo.common.logger import Logger                                  # noqa: E402
from sac_eo.common.train_parser import create_train_parser, all_kwargs   # noqa: E402
from sac_eo.common.train_utils import import_inputs, organize_rms_inputs  # noqa: E402
from sac_eo.common.samplers import trajectory_sampler, batch_simtrajectory_sampler  # noqa: E402
from sac_eo.common.corruptor import TrajectoryCorruptor                  # noqa: E402
import sac_eo                                                            # noqa: E402
assert sac_eo.__file__.startswith(REF), sac_eo.__file__
sys.path.pop(0)
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import ref_ducks as D                                                    # noqa: E402
import sac_oracle as O                                                   # noqa: E402

OUT = {}


def put(prefix, **kv):
    for k, v in kv.items():
        OUT[f"{prefix}.{k}"] = np.asarray(v)


# ----------------------------------------------------------------- A. the replay buffer
# ADD_LENS[i] rows per add; buffer_size crossed at the 4th add; sampled twice afterwards
BUF = dict(S=17, A=6, cap=600, lens=[250, 1, 1, 400, 3, 1, 120, 1], B=256, seeds=[7, 2590541744])


def make_buffer():
    S, A, cap = BUF["S"], BUF["A"], BUF["cap"]
    rs = np.random.RandomState(11)
    buf = TrajectoryBuffer(S, A, 0.99, 0.97, cap)
    unb = TrajectoryBuffer(S, A, 0.99, 0.97, None)
    sizes = []
    for i, n in enumerate(BUF["lens"]):
        s = (rs.normal(size=(n, S)) * 2).astype(np.float32)
        a = rs.uniform(-1, 1, size=(n, A)).astype(np.float32)
        r = rs.normal(size=n) if i % 2 else rs.normal(size=n).astype(np.float32)   # float64 / float32 r
        sp = (rs.normal(size=(n, S)) * 2).astype(np.float32)
        d = rs.uniform(size=n) < 0.1
        put(f"buf.add{i}", s=s, a=a, r=r, sp=sp, d=d)
        buf.add(s, a, r, sp, d)
        unb.add(s, a, r, sp, d)
        sizes.append((buf.current_size, buf.traj_total, buf.steps_total, unb.current_size))
    put("buf", sizes=np.array(sizes), s_all=buf.s_all, a_all=buf.a_all, r_all=buf.r_all, sp_all=buf.sp_all,
        d_all=buf.d_all, idx_all=buf.idx_all, unb_idx_all=unb.idx_all, r_dtype=str(buf.r_all.dtype),
        d_dtype=str(buf.d_all.dtype))
    for seed in BUF["seeds"]:
        np.random.seed(seed)
        s, a, sp, r, d = buf.get_offmodel_info(BUF["B"])
        after = np.random.randint(2 ** 31, size=4)
        put(f"buf.sample{seed}", s=s, a=a, sp=sp, r=r, d=d, after=after)
        np.random.seed(seed)
        s2, a2, sp2, r2 = buf.get_model_info(33)
        put(f"buf.model{seed}", s=s2, a=a2, sp=sp2, r=r2)


# ----------------------------------------------------------------- B. normalisers
def make_normalizers():
    S, A = 5, 2
    rs = np.random.RandomState(21)
    nr = RunningNormalizers(S, A, 0.995)
    lens = [1, 7, 30, 1, 13, 200]
    for i, n in enumerate(lens):
        s = (rs.normal(size=(n, S)) * rs.uniform(0.1, 5, S) + 1).astype(np.float32)
        a = rs.uniform(-1, 1, size=(n, A)).astype(np.float32)
        r = rs.normal(size=n) * 3 + 1 if i % 2 else (rs.normal(size=n) * 3 + 1).astype(np.float32)
        sp = (s + rs.normal(size=(n, S)) * 0.1).astype(np.float32)
        nr.update_rms(s, a, r, sp)
        put(f"norm.upd{i}", s=s, a=a, r=r, sp=sp)
        st = nr.get_rms_stats()
        for k, v in st.items():
            put(f"norm.upd{i}.{k}", t=v["t"], mean=v["mean"], var=v["var"],
                std=getattr(nr, k).std)
    x = (rs.normal(size=(9, S)) * 3).astype(np.float32)
    put("norm.nd", x=x, n=nr.s_rms.normalize(x), nc=nr.s_rms.normalize(x, center=False),
        dn=nr.s_rms.denormalize(x), dnc=nr.s_rms.denormalize(x, center=False))
    # instantiate from stats: t = 0, 1 and > 1 (normalizer.py:104-114)
    for t in (0, 1, 5):
        m = RunningNormalizers(S, A, 0.995)
        stats = {k: {"t": t, "mean": (rs.normal(size=S if k in ("s_rms", "delta_rms") else A if k == "a_rms" else 1)
                                      ).astype(np.float32),
                     "var": rs.uniform(0.5, 2, size=S if k in ("s_rms", "delta_rms") else A if k == "a_rms" else 1
                                       ).astype(np.float32)} for k in ("s_rms", "a_rms", "r_rms", "delta_rms", "ret_rms")}
        m.set_rms_stats(stats)
        for k in stats:
            put(f"norm.inst{t}.{k}", mean=stats[k]["mean"], var=stats[k]["var"], std=getattr(m, k).std,
                mean_out=getattr(m, k).mean)
    # discounted_sum (scipy lfilter): float32 / float64 inputs, several rates and lengths
    for i, (n, rate, dt) in enumerate([(1, 0.99, np.float32), (7, 0.995, np.float64), (1000, 0.995, np.float32),
                                       (333, 0.9, np.float64)]):
        x = (rs.normal(size=n) * 2).astype(dt)
        put(f"dsum{i}", x=x, rate=rate, y=discounted_sum(x, rate))


# ----------------------------------------------------------------- C. logger (+ train_utils)
def make_logger(tmp):
    rs = np.random.RandomState(31)
    lg = D.fill_run_log(Logger, rs, 0, 5)
    lg.dump_and_save(tmp, "LOG_0")                 # checkpoint 1: a new file
    lg.reset()
    lg2 = D.fill_run_log(Logger, rs, 0, 3)
    lg2.log_train({"new_key": 7.0})
    lg2.dump_and_save(tmp, "LOG_0")                # checkpoint 2: train arrays appended
    with open(os.path.join(tmp, "LOG_0"), "rb") as fh:
        data = fh.read()
    with open(os.path.join(HERE, "ref_logger.pkl"), "wb") as fh:
        fh.write(data)
    # the aggregated multi-run file of train.py:159-187 (a list of run dicts)
    runs = [D.fill_run_log(Logger, rs, i, 2).dump() for i in range(2)]
    runs[1]["final"].pop("model_weights")          # a run without world models (train_utils.py:68-77)
    runs[1]["final"].pop("reward_weights")
    path = os.path.join(HERE, "ref_runs.pkl")
    with open(path, "wb") as fh:
        pickle.dump(runs, fh, protocol=4)
    cases = []
    for c in [dict(idx=0, import_idx=None, import_all=False), dict(idx=1, import_idx=None, import_all=False),
              dict(idx=5, import_idx=None, import_all=True), dict(idx=0, import_idx=1, import_all=True)]:
        inp = {g: {} for g in all_kwargs}
        inp["setup_kwargs"] = {"import_path": HERE, "import_file": "ref_runs.pkl", "import_idx": c["import_idx"],
                               "import_all": c["import_all"], "idx": c["idx"], "runs_start": 0}
        inp["env_kwargs"] = {"env_name": "mine"}
        out = import_inputs(inp)
        cases.append(dict(case=c, out=_jsonable(out)))
    # organize_rms_inputs on the flat keys of older logs (train_utils.py:94-129)
    flat = {f"{k}_{f}": (rs.normal(size=3).astype(np.float32) if f != "t" else 4)
            for k in ("s", "a", "r", "delta", "ret") for f in ("t", "mean", "var")}
    org = organize_rms_inputs(flat)
    return cases, _jsonable(flat), _jsonable(org)


def _jsonable(x):
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, np.ndarray):
        return {"__nd__": x.tolist(), "dtype": str(x.dtype), "shape": list(x.shape)}
    if isinstance(x, np.generic):
        return {"__np__": x.item(), "dtype": str(x.dtype)}
    return x


# ----------------------------------------------------------------- D. parser
CLIS = [
    [],
    "--env_name HalfCheetah-v3 --alg_type sac_imit --actor_layers 256 256 --critic_layers 256 256 "
    "--actor_squash --total_timesteps 1e6 --env_buffer_size 1e6 --runs 4".split(),
    "--env_name Humanoid-v3 --sac_batch_size 1024 --env_buffer_size 4e6 --runs 8 --no_model_batch_shuffle "
    "--no_adv_center --delta_clip_pred 5 --model_holdout_ratio 0.2 --s_noise_std 0.1 --s_noise_type next".split(),
]


def make_parser():
    p = create_train_parser()
    return {"all_kwargs": all_kwargs, "cli": [c for c in CLIS],
            "parsed": [vars(p.parse_args(c)) for c in CLIS]}


# ----------------------------------------------------------------- E. samplers + corruptor
def make_samplers():
    S, A = 4, 2
    out = {}
    nr = RunningNormalizers(S, A, 0.99)
    rs = np.random.RandomState(41)
    s0 = rs.normal(size=(40, S)).astype(np.float32)
    nr.update_rms(s0, rs.normal(size=(40, A)).astype(np.float32), rs.normal(size=40).astype(np.float32),
                  (s0 + rs.normal(size=(40, S))).astype(np.float32))
    put("samp.norm_upd", s=s0)
    cases = [dict(h=50, eval=True, det=False, noise=0.0, ntype="all", term_at=None),
             dict(h=50, eval=False, det=False, noise=0.3, ntype="all", term_at=None),
             dict(h=25, eval=True, det=True, noise=0.5, ntype="next", term_at=None),
             dict(h=12, eval=True, det=False, noise=0.0, ntype="all", term_at=12),
             dict(h=1, eval=True, det=False, noise=0.2, ntype="all", term_at=None)]
    for i, c in enumerate(cases):
        env = D.DuckEnv(S, A, seed=100 + i, term_at=c["term_at"])
        actor = D.DuckActor(S, A, seed=200 + i)
        corr = None
        if c["noise"] > 0 or i == 0:
            corr = TrajectoryCorruptor(c["noise"], c["ntype"])
            corr.set_rms(nr)
        np.random.seed(300 + i)
        res = trajectory_sampler(env, actor, c["h"], eval=c["eval"], deterministic=c["det"], corruptor=corr)
        after = np.random.randint(2 ** 31, size=4)
        cafter = corr.s_noise_rng.integers(2 ** 31, size=4) if corr is not None else np.zeros(4, np.int64)
        names = ("s", "a", "r", "sp", "d") + (("J",) if c["eval"] else ())
        put(f"samp{i}", after=after, cafter=cafter, **dict(zip(names, res)))
        for k, v in zip(names, res):
            put(f"samp{i}.dtype", **{k: str(np.asarray(v).dtype)})
    out["traj_cases"] = cases
    # batch_simtrajectory_sampler over an oracle actor and an oracle world model
    roll = []
    for j, (n, H, det) in enumerate([(37, 5, False), (8, 3, True), (1, 4, False)]):
        cfg = O.Config(S=17, A=6, hidden=(32, 32), act="tanh", B=8, model_hidden=(64, 64))
        st = O.init_state(cfg, seed=400 + j, with_models=True, bias_scale=0.05, actor_gain=0.5,
                          model_gain=0.3).astype(np.float64)
        nrm = O.Normalizers.identity(17, 6)
        s_init = (np.random.RandomState(500 + j).normal(size=(n, 17)) * 1.5).astype(np.float32)
        np.random.seed(600 + j)
        res = batch_simtrajectory_sampler(D.OracleModelEnv(O, st, cfg, nrm, 1), D.OracleActor(O, st, cfg, nrm), H,
                                          s_init, deterministic=det)
        after = np.random.randint(2 ** 31, size=4)
        put(f"roll{j}", s_init=s_init, after=after, **dict(zip(("s", "a", "r", "sp", "d"), res)))
        roll.append(dict(n=n, H=H, det=det, seed=400 + j))
    out["roll_cases"] = roll
    # the corruptor on its own (its default_rng(0) stream across calls)
    corr = TrajectoryCorruptor(0.7, "all")
    corr.set_rms(nr)
    xs = [rs.normal(size=(S,)), rs.normal(size=(3, S)).astype(np.float32), rs.normal(size=(S,))]
    for i, x in enumerate(xs):
        put(f"corr{i}", x=x, y=corr.corrupt_samples(x))
    return out


def main():
    make_buffer()
    make_normalizers()
    with tempfile.TemporaryDirectory() as tmp:
        imp_cases, flat, org = make_logger(tmp)
    meta = {"parser": make_parser(), "samplers": make_samplers(), "buf": BUF,
            "import_cases": imp_cases, "rms_flat": flat, "rms_organized": org}
    np.savez_compressed(os.path.join(HERE, "ref_fixtures.npz"), **OUT)
    with open(os.path.join(HERE, "ref_fixtures.json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
    print(f"wrote {len(OUT)} arrays; logger pickle {os.path.getsize(os.path.join(HERE, 'ref_logger.pkl'))} B")


if __name__ == "__main__":
    main()
