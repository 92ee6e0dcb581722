"""A/B of two library builds on bench.py's formats section (FP8 / FP4 pack and unpack on [11008, 4096],
cold over 16 copies): one process per (library, round), alternate and compare medians.
    python tools/ab_formats_lib.py --lib iron_weight_only_quant_amd/_lib/libiwq_base.so --tag base"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--tag", required=True)
    a = ap.parse_args()
    from iron_weight_only_quant_amd import _lib
    _lib.LIB_PATH = os.path.abspath(a.lib)
    import bench
    for r in bench.formats_section()["rows"]:
        print(json.dumps({"tag": a.tag, **r}), flush=True)


if __name__ == "__main__":
    main()
