"""Median kernel / first-ball / walk ms per (variant, config) of a tools/ab.sh log.
    python3 tools/ab_summary.py gpurun_out/x_ab.log"""
import collections
import json
import statistics
import sys

r = collections.defaultdict(list)
for line in open(sys.argv[1]):
    v, _, js = line.partition(" ")
    try:
        d = json.loads(js)
    except ValueError:
        continue
    r[(d["config"], v)].append((d["kernel_ms"], d["first_ball_ms"], d["walk_ms"]))
for (cfg, v), vals in sorted(r.items()):
    med = [statistics.median(x[i] for x in vals) for i in range(3)]
    print(f"{cfg:16s} {v:10s} kernel {med[0]:8.3f}  first_ball {med[1]:7.3f}  walk {med[2]:8.3f}  (n={len(vals)})")
