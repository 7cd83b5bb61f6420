"""Summarise tools/ab_latency.sh output: per case and variant, the kernel / first-ball /
walk times of each run.   python3 tools/ab_latency_summary.py gpurun_out/x.log"""
import collections
import json
import sys

rows = collections.defaultdict(list)
order = []
for line in open(sys.argv[1]):
    v, _, j = line.partition(" ")
    try:
        d = json.loads(j)
    except ValueError:
        continue
    if v not in order:
        order.append(v)
    rows[(d["case"], v)].append(d)
cases = []
for (c, _) in rows:
    if c not in cases:
        cases.append(c)
for c in cases:
    for v in order:
        ds = rows.get((c, v), [])
        if ds:
            k = min(d["kernel_ms"] for d in ds)
            print(f"{c:12s} {v:8s} kernel {k:7.3f}  " +
                  " ".join(f"[fb {d['first_ball_ms']:.3f} walk {d['walk_ms']:.3f}]" for d in ds))
