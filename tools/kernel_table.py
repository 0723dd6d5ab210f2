"""Per-kernel roofline table from one profiling call (tools/gpu_profile.sh): rocprofv3
kernel-trace stats (average duration per kernel) joined with the PMC summary
(profiles/pmc_<config>.json: HBM traffic per launch from FETCH_SIZE / WRITE_SIZE with the
gfx950 correction, SQ_VALU_MFMA_BUSY_CYCLES).

  HBM GB/s        = traffic bytes per launch / average duration
  MFMA busy frac  = MFMA busy cycles per launch / (average duration x 2.4 GHz x 1024 SIMDs)

usage: python tools/kernel_table.py <kernel_stats.csv> <pmc json> [out.md]
"""
import csv
import json
import re
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import family, subfamily  # noqa: E402

CLK_HZ = 2.4e9
SIMDS = 1024
HBM_PEAK = 8000.0


def main():
    stats, pmcp = sys.argv[1], sys.argv[2]
    pmc = json.load(open(pmcp))["kernels"]
    dur = defaultdict(lambda: [0.0, 0])          # family / subfamily -> [total ns, calls]
    for r in csv.DictReader(open(stats)):
        name = r["Name"]
        for key in (family(name), subfamily(name)):
            if key:
                dur[key][0] += float(r["TotalDurationNs"])
                dur[key][1] += int(r["Calls"])
    lines = ["| kernel | calls | avg us | HBM traffic / launch (MB) | HBM GB/s | % of 8 TB/s | MFMA busy |",
             "|---|---|---|---|---|---|---|"]
    for key in sorted(pmc, key=lambda k: -dur[k][0]):
        if dur[key][1] == 0:
            continue
        avg = dur[key][0] / dur[key][1]
        k = pmc[key]
        tr = k.get("traffic_bytes_per_launch")
        gbs = tr / avg if tr else None                      # bytes / ns = GB/s
        mf = k.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mfrac = mf / (avg * 1e-9 * CLK_HZ * SIMDS) if mf else 0.0
        lines.append(f"| {key} | {dur[key][1]} | {avg / 1e3:.2f} | {tr / 1e6:.3f} | {gbs:.0f} | "
                     f"{100 * gbs / HBM_PEAK:.1f} % | {100 * mfrac:.2f} % |" if tr else
                     f"| {key} | {dur[key][1]} | {avg / 1e3:.2f} | - | - | - | {100 * mfrac:.2f} % |")
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(out + "\n")


if __name__ == "__main__":
    main()
