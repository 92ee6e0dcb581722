"""Per-kernel median PMC values from a rocprofv3 output dir (counter_collection.csv, and
kernel_trace.csv when present for durations): one block per distinct kernel name, with the implied
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and MFMA busy fraction of 1024 SIMDs when available."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    dur = {}
    for path in kt:
        for r in csv.DictReader(open(path)):
            dur[(r["Kernel_Name"], r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for path in cc:
        for r in csv.DictReader(open(path)):
            per[r["Kernel_Name"]][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for name, ctrs in per.items():
        if "k_synth" in name or "elementwise" in name or "k_rowwave" in name:
            continue
        print(name[:140])
        med = {}
        for c in sorted(ctrs):
            vals = list(ctrs[c].values())
            med[c] = statistics.median(vals)
            print(f"  {c} = {med[c]:.0f}  (dispatches {len(vals)})")
        ds = [v for (n, _), v in dur.items() if n == name]
        if ds:
            t = statistics.median(ds)
            print(f"  duration_us = {t * 1e6:.1f}")
            if "GRBM_GUI_ACTIVE" in med:
                clk = med["GRBM_GUI_ACTIVE"] / 8 / t
                print(f"  implied_clock_GHz = {clk / 1e9:.3f}")
                if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
                    print(f"  mfma_busy_frac = {med['SQ_VALU_MFMA_BUSY_CYCLES'] / (clk * t * 1024):.3f}")


if __name__ == "__main__":
    main()
