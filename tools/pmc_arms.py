"""Cut a rocprofv3 --pmc run of `tools/ab_outplace.py --pmc` into its arms: the tool launches
iwq_fill_synthetic on 16 elements (k_synth, grid 16) before the fresh-buffer ceiling and before every
arm x variant; the dispatches between two separators belong to the arm printed in that order in the
tool's log.  Prints per arm the median of each counter over the arm's measured dispatches and the
per-dispatch duration.

usage: python tools/pmc_arms.py gpurun_out/<pmc dir> gpurun_out/<tool log> [-o out.jsonl]
"""
import argparse
import collections
import csv
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("log")
    ap.add_argument("-o", "--out", default=None)
    a = ap.parse_args()
    arms = []
    for ln in open(a.log):
        if ln.startswith("{"):
            r = json.loads(ln)
            if "arm" in r:
                arms.append(f"{r['arm']}/v{r['variant']}")
    rows = collections.defaultdict(dict)  # dispatch -> {counter: value, name, dur}
    for r in csv.DictReader(open(os.path.join(a.pmc_dir, "run_counter_collection.csv"))):
        d = int(r["Dispatch_Id"])
        rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
        rows[d]["_name"] = r["Kernel_Name"]
        rows[d]["_grid"] = int(r["Grid_Size"])
        rows[d]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    seq = [rows[d] for d in sorted(rows)]
    groups, cur = [], None
    for x in seq:
        if "k_synth" in x["_name"] and x["_grid"] <= 256:
            cur = []
            groups.append(cur)
        elif cur is not None:
            cur.append(x)
    out = open(a.out, "w") if a.out else None
    for arm, g in zip(arms, groups):
        if not g:
            continue
        ctr = sorted(k for k in g[0] if not k.startswith("_"))
        rec = {"arm": arm, "dispatches": len(g), "kernel": g[0]["_name"][:60],
               "us_median": round(statistics.median(x["_ns"] for x in g) / 1e3, 2)}
        for c in ctr:
            rec[c] = statistics.median(x.get(c, 0.0) for x in g)
        line = json.dumps(rec)
        print(line)
        if out:
            out.write(line + "\n")
    if len(arms) != len(groups):
        print(f"# note: {len(arms)} arms in the log, {len(groups)} separated groups in the trace")


if __name__ == "__main__":
    main()
