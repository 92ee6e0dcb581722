"""Cut a rocprofv3 kernel trace of `bench.py --mark-file MARKS` into bench.py's timed regions.

Every number bench.py reports comes from HIP events around one timed region (the headline's K
launches, each cold `shapes` replay, each fused-forward arm, each formats path, the 70B steps).  With
--mark-file bench.py also writes the host-clock interval of each region (synchronized on both sides),
so every kernel a region ran lies inside its interval.  This tool assigns the traced dispatches to
the regions and prints, per region and kernel name: dispatches, average / median / min / max kernel
duration and (graph replays) the median boundary to the next dispatch, beside bench.py's own
figure for that region -- the per-workload rocprof summary each BENCH number is read against.

    cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d OUT -o run -- \\
        python3 $ROOT/bench.py --mark-file $ROOT/gpurun_out/marks.jsonl
    python3 tools/trace_sections.py OUT gpurun_out/marks.jsonl -o profiles/rNN_sections.json

Which host clock the trace's timestamps share is found from the data (the clock under which the
most regions contain a dispatch): rocprofv3 stamps kernels on the system clock of the host.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def load_trace(d):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def load_marks(path):
    return [json.loads(line) for line in open(path) if line.strip()]


def assign(rows, marks, clock):
    """{region index: [(start, end, name)]} of the dispatches inside each region's interval."""
    import bisect
    starts = [r[0] for r in rows]
    out = {}
    for i, m in enumerate(marks):
        t0, t1 = m["t0"][clock], m["t1"][clock]
        lo = bisect.bisect_left(starts, t0)
        hi = bisect.bisect_right(starts, t1)
        out[i] = [r for r in rows[lo:hi] if r[1] <= t1]
    return out


def short(name, n=110):
    return name if len(name) <= n else name[:n] + "..."


def summarize(rows, marks):
    best = None
    for clock in ("boot", "mono", "real"):
        got = assign(rows, marks, clock)
        hit = sum(1 for v in got.values() if v)
        if best is None or hit > best[0]:
            best = (hit, clock, got)
    hit, clock, got = best
    # regions of the same name (e.g. the rounds of one interleaved arm) are merged
    merged = defaultdict(lambda: {"dispatches": defaultdict(list), "gaps": defaultdict(list), "bench": []})
    order = []
    for i, m in enumerate(marks):
        name = m["region"]
        if name not in merged:
            order.append(name)
        g = merged[name]
        for k in ("bench_kernel_ms", "bench_us_per_call", "bench_ms_per_call", "bench_ms_per_call_this_round"):
            if k in m:
                g["bench"].append((k, m[k]))
        ds = got[i]
        for j, (s, e, n) in enumerate(ds):
            g["dispatches"][n].append((e - s) / 1e3)
            if j + 1 < len(ds) and ds[j + 1][2] == n:
                g["gaps"][n].append((ds[j + 1][0] - e) / 1e3)
    res = {"clock": clock, "regions_with_dispatches": hit, "regions": len(marks), "rows": []}
    for name in order:
        g = merged[name]
        bench = {}
        for k, v in g["bench"]:
            bench.setdefault(k, []).append(v)
        bench = {k: (statistics.median(v) if len(v) > 1 else v[0]) for k, v in bench.items()}
        kernels = []
        for n, ds in sorted(g["dispatches"].items(), key=lambda kv: -sum(kv[1])):
            gs = g["gaps"].get(n, [])
            kernels.append({"kernel": n, "dispatches": len(ds), "avg_us": round(statistics.fmean(ds), 3),
                            "median_us": round(statistics.median(ds), 3), "min_us": round(min(ds), 3),
                            "max_us": round(max(ds), 3),
                            "median_gap_us": round(statistics.median(gs), 3) if gs else None})
        row = {"region": name, "bench": bench, "kernels": kernels}
        # the dominant kernel's average against bench.py's own per-call figure
        if kernels:
            top = kernels[0]["avg_us"]
            ref = None
            if "bench_kernel_ms" in bench:
                ref = bench["bench_kernel_ms"] * 1e3
            elif "bench_us_per_call" in bench:
                ref = bench["bench_us_per_call"]
            elif "bench_ms_per_call" in bench:
                ref = bench["bench_ms_per_call"] * 1e3
            elif "bench_ms_per_call_this_round" in bench:  # interleaved arm: median over its rounds
                ref = bench["bench_ms_per_call_this_round"] * 1e3
            if ref:
                row["dominant_avg_over_bench"] = round(top / ref, 4)
        res["rows"].append(row)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("marks")
    ap.add_argument("-o", "--out", default="")
    ap.add_argument("--min-us", type=float, default=0.0, help="hide kernels whose average is below this")
    a = ap.parse_args()
    rows = load_trace(a.trace_dir)
    if not rows:
        raise SystemExit(f"no *kernel_trace.csv under {a.trace_dir}")
    res = summarize(rows, load_marks(a.marks))
    print(f"clock {res['clock']}: {res['regions_with_dispatches']} of {res['regions']} regions hold dispatches")
    for row in res["rows"]:
        print(f"{row['region']}  bench {row['bench']}  avg/bench {row.get('dominant_avg_over_bench')}")
        for k in row["kernels"]:
            if k["avg_us"] < a.min_us:
                continue
            print(f"    {k['dispatches']:5d} x avg {k['avg_us']:10.3f} us  median {k['median_us']:10.3f}  "
                  f"min {k['min_us']:10.3f}  max {k['max_us']:10.3f}  gap {k['median_gap_us']}  {short(k['kernel'])}")
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
