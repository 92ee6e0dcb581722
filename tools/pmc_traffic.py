"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes for bench.py.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide (16 B/lane) coalesced streaming
read, so it is doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.

usage: python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --numel N --bits 4 --group 128 \
           --kernel k_group -o profiles/traffic.json
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def counter(dirname, name, kernel):
    path = os.path.join(dirname, "run_counter_collection.csv")
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == name and kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit(f"no {name} rows for kernel '{kernel}' in {path}")
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--numel", type=int, required=True)
    ap.add_argument("--bits", type=int, default=4)
    ap.add_argument("--group", type=int, default=128)
    ap.add_argument("--kernel", default="k_group")
    ap.add_argument("--placement", default="out-of-place", choices=["out-of-place", "in-place"])
    ap.add_argument("-o", "--out", default="profiles/traffic.json")
    a = ap.parse_args()
    fetch_kib, nf = counter(a.fetch_dir, "FETCH_SIZE", a.kernel)
    write_kib, nw = counter(a.write_dir, "WRITE_SIZE", a.kernel)
    read_bytes = fetch_kib * 1024 * 2
    write_bytes = write_kib * 1024
    rec = {"workload_numel": a.numel, "bits": a.bits, "group": a.group, "kernel": a.kernel, "placement": a.placement,
           "fetch_size_kib": fetch_kib, "write_size_kib": write_kib, "dispatches": [nf, nw],
           "read_bytes_per_launch": read_bytes, "write_bytes_per_launch": write_bytes,
           "hbm_bytes_per_launch": read_bytes + write_bytes,
           # bench.py trusts this record only while the headline kernel's sources are unchanged
           "kernel_sources_sha": __import__("bench").kernel_sources_sha(),
           "correction": "FETCH_SIZE x 1024 x 2 (gfx950 half-count of 16B/lane streaming reads), WRITE_SIZE x 1024"}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(rec, open(a.out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
