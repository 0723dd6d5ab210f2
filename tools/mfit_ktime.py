"""Per-launch workgroup timing of the world-model fit (diagnostic): eager fit steps with libsacx's
SACX_MFIT_KTIME stamps; per launch the mean over steps of its span, mean / max workgroup duration,
last-start offset and gap to the previous launch (us).  usage: python tools/mfit_ktime.py [config] [steps]"""
import collections
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sac-expert_amd"))
path = os.path.join(tempfile.mkdtemp(), "mk.csv")
os.environ["SACX_MFIT_KTIME"] = path
import bench  # noqa: E402
import torch  # noqa: E402
from sac_eo.common.seeding import derive_seeds  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "hc_eo"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 48
cfgd = dict(bench.CONFIGS[cfg], buffer=200_000)
sd = {k: int(v[0]) for k, v in derive_seeds(0, 1).items()}
eng = bench.build_engine(cfgd, sd, device=torch.device("cuda", 0))
mb = eng.cfg.model_batch
idx = np.random.RandomState(3).randint(cfgd["buffer"], size=(n, 2, mb)).astype(np.int32)
eng.model_fit(idx, eager=True)
eng.sync()
eng.close()
rows = collections.OrderedDict()
with open(path) as f:
    for line in f:
        name, *v = line.strip().split(",")
        rows.setdefault(name, []).append([float(x) for x in v])
print(f"{cfg}: {n} eager fit steps; per launch (mean over steps after the first 8): wgs span wg_mean wg_max last_start gap")
tot = 0.0
for name, v in rows.items():
    a = np.array(v[8:] if len(v) > 8 else v)
    m = a.mean(0)
    tot += m[1] + m[5]
    print(f"  {name:28s} {int(m[0]):5d} {m[1]:7.2f} {m[2]:7.2f} {m[3]:7.2f} {m[4]:7.2f} {m[5]:7.2f}")
print(f"  sum of spans + gaps {tot:.2f} us")
