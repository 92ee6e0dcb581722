"""Split a rocprofv3 kernel trace of tools/single_trace.py into per-call kernel duration and the
boundary to the next call (start of call i+1 - end of call i), per kernel name, over the replayed
calls (the last REPLAYS x CALLS dispatches of each kernel name run back to back inside a graph).
usage: python3 tools/trace_gaps.py OUT_DIR [--min-us 3]"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 3.0
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # consecutive dispatches of the same quantize kernel with < 50 us between them = one replay run
    runs = []
    cur = []
    for s, e, n in rows:
        if "k_group" not in n and "k_row" not in n:
            continue
        if cur and (n != cur[-1][2] or s - cur[-1][1] > 50_000):
            runs.append(cur)
            cur = []
        cur.append((s, e, n))
    if cur:
        runs.append(cur)
    by = defaultdict(lambda: {"dur": [], "gap": []})
    for run in runs:
        if len(run) < 8:
            continue
        n = run[0][2]
        for i, (s, e, _) in enumerate(run):
            by[n]["dur"].append((e - s) / 1e3)
            if i + 1 < len(run):
                by[n]["gap"].append((run[i + 1][0] - e) / 1e3)
    for n, v in by.items():
        ds, gs = v["dur"], v["gap"]
        if statistics.median(ds) < min_us:
            continue
        print(f"{n[:120]}\n  calls {len(ds)}  kernel_us median {statistics.median(ds):.2f}  "
              f"min {min(ds):.2f}  boundary_us median {statistics.median(gs):.2f}  "
              f"per_call_us {statistics.median(ds) + statistics.median(gs):.2f}")


if __name__ == "__main__":
    main()
