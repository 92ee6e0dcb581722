"""Tabulate bench_gemm.py JSON lines: per (shape, M) the time / weight GB/s of every variant."""
import json
import sys
from collections import defaultdict

t = defaultdict(dict)
hb = {}
for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    r = json.loads(line)
    t[(r["shape"], r["M"])][r.get("variant", 0)] = (r["fused_ms"] * 1000, r.get("fused_weight_GBps", 0))
    hb[(r["shape"], r["M"])] = r["hipblaslt_fp16_ms"] * 1000
for k, v in t.items():
    best = min(v, key=lambda x: v[x][0])
    print(f"{k[0]:>10} M={k[1]:<5} hipblaslt {hb[k]:7.1f}us  best v{best}  " +
          " ".join(f"v{vv}:{a:.1f}/{b:.0f}" for vv, (a, b) in sorted(v.items())))
