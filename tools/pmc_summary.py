"""Median per-dispatch value of each PMC counter for one kernel (rocprofv3 counter_collection.csv)."""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path, needle = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "k_group")
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        if needle in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for name in sorted(per):
        vals = list(per[name].values())
        print(f"{name} median_per_dispatch={statistics.median(vals):.0f} dispatches={len(vals)}")


if __name__ == "__main__":
    main()
