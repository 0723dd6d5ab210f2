"""Print one update's worth of the kernel trace: queue, start, duration, gap to the previous
kernel on the same queue.  usage: python tools/trace_view.py <kernel_trace.csv> [n] [first-kernel]
(first-kernel: start the window at a dispatch of that kernel, e.g. k_mgather for a model-fit step;
 comma-separated: the first marker the trace holds)"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "sacx" in r["Kernel_Name"]]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
mid = len(rows) * 2 // 3
if len(sys.argv) > 3:       # comma-separated markers: the first one present in the trace
    for mark in sys.argv[3].split(","):
        hits = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
        if hits:
            mid = hits[len(hits) * 5 // 6]
            break
w = rows[mid: mid + n]
t0 = w[0]["s"]
last = {}
busy = 0
for r in w:
    q = r["Queue_Id"]
    gap = (r["s"] - last[q]) / 1e3 if q in last else float("nan")
    last[q] = r["e"]
    name = r["Kernel_Name"].replace("sacx::", "").replace("void ", "").split("(")[0]
    print(f"q{q:>3s} {name:22s} start={(r['s'] - t0) / 1e3:8.2f} dur={(r['e'] - r['s']) / 1e3:6.2f} "
          f"gap={gap:6.2f} grid={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}")
