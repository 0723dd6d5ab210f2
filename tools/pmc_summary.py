"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) into profiles/pmc_<config>.json.

Per kernel family: mean over dispatches of FETCH_SIZE and WRITE_SIZE (KB), and
traffic_bytes_per_launch = (f * FETCH_SIZE + WRITE_SIZE) * 1024.  The factor f depends on the
access shape (tools/fetch_calib.hip, profiles/r03_fetch_calib_v1.txt: each shape reading a fresh
64 MiB once): FETCH_SIZE reports 0.50x the bytes of coalesced streaming reads (16 B or 4 B per
lane, 1 KiB / 256 B per wave-instruction; MI355X_MICROARCH.md, section HBM) but 1.00x for
k_gemm's MFMA-fragment loads (16 lanes x 4 B = one 64-B piece of a row, 4 rows per
instruction).  So f = 1 for k_gemm (its operand and epilogue loads are all 64-B row pieces),
f = 2 for the row-streaming kernels.
Families follow sacx kernel names (template arguments folded: k_gemm<1, 1> -> k_gemm;
k_gemm_head, k_fwd2 -> k_gemm).
usage: python tools/pmc_summary.py gpurun_out/pmc hc [source-tag] [extra-copy-path]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def family(name):
    n = name.replace("void ", "")
    m = re.search(r"sacx::(k_[a-z_0-9]+)", n)      # (digits: k_fwd2 is not k_fwd)
    if not m:
        return None
    # k_gemm_head is k_gemm with the actor-head prologue, k_fwd2 two forward layers in one launch:
    # launches of the k_gemm family (the plan's GEMM launches)
    return "k_gemm" if m.group(1).startswith("k_gemm") or m.group(1) == "k_fwd2" else m.group(1)


def subfamily(name):
    """k_gemm launches split by operand mode (template argument 0): fwd / dx / dw (+ Adam) / fwd2."""
    if "k_gemm_head" in name:              # the forward launch with the actor-head prologue
        return "k_gemm.fwd_head"
    if "k_fwd2" in name:                   # two forward layers in one launch
        return "k_gemm.fwd2"
    m = re.search(r"sacx::k_gemm<(\d+)", name)
    if not m:
        return None
    return "k_gemm." + {"0": "fwd", "1": "dx", "2": "dw_adam", "3": "fwd2"}.get(m.group(1), m.group(1))


def main():
    d, config = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(os.path.normpath(d))
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            if fam is None or fam == "k_append":
                continue
            vals[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
            sub = subfamily(r["Kernel_Name"])
            if sub is not None:
                vals[sub][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"config": config, "source": tag, "kernels": {}}
    for fam, cs in sorted(vals.items()):
        k = {c: sum(v) / len(v) for c, v in cs.items()}
        k["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
            f = 1.0 if fam.startswith("k_gemm") else 2.0
            k["fetch_factor"] = f
            k["traffic_bytes_per_launch"] = (f * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024.0
        out["kernels"][fam] = k
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "profiles", f"pmc_{config}.json")
    paths = [path] + sys.argv[4:5]
    for pth in paths:
        with open(pth, "w") as fh:
            json.dump(out, fh, indent=1, sort_keys=True)
    print(paths)
    for fam, k in out["kernels"].items():
        print(fam, {c: round(v, 1) for c, v in k.items() if isinstance(v, float)})


if __name__ == "__main__":
    main()
