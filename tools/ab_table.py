"""Table of an A/B run (tools/ab_generic.sh TAG ...): kernel / first-ball / walk ms per
(case, variant), every round side by side.   python3 tools/ab_table.py TAG"""
import collections
import json
import sys

tag = sys.argv[1]
for f in (f"gpurun_out/{tag}_ab.log", f"gpurun_out/{tag}_ab_cfg.log"):
    d = collections.defaultdict(list)
    try:
        rows = open(f).read().splitlines()
    except OSError:
        continue
    for line in rows:
        if not line.strip():
            continue
        v, js = line.split(" ", 1)
        r = json.loads(js)
        d[(r.get("case", r.get("config")), v)].append((r["kernel_ms"], r["first_ball_ms"], r["walk_ms"]))
    for (k, v), xs in sorted(d.items()):
        mean = sum(x[0] for x in xs) / len(xs)
        print(f"{k:15s} {v:7s} mean {mean:7.3f}  " + "  ".join(f"{a:.3f}[fb {b:.3f} w {c:.3f}]" for a, b, c in xs))
