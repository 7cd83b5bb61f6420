"""HBM traffic of the walk kernel from rocprofv3 PMC counters (run on the GPU box).

Two separate --pmc passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one pass
on gfx950) over `bench.py --steps 2 --warmup 1 --no-cpu-baseline`; the per-dispatch
values of wos_walk_kernel are averaged and written to profiles/<tag>_walk_traffic.json,
which bench.py reports as roofline.traffic for the same configuration.

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB (TCC_EA0_RDREQ /
_WRREQ based).  MI355X_MICROARCH.md: FETCH_SIZE counts exactly half the bytes of a
wide (16 B/lane) coalesced streaming read; this kernel's reads are 4-byte gathers
(walk-task fields and source texels), an uncalibrated width, so the raw value is
reported together with the 2x-corrected upper estimate.
    python3 tools/collect_traffic.py [tag] [config]
This script itself never touches the GPU: rocprofv3 runs as a child process.
"""
import csv
import glob
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import lib_sha16  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = sys.argv[1] if len(sys.argv) > 1 else "r1"
CONFIG = sys.argv[2] if len(sys.argv) > 2 else "B"
OUT = os.path.join(REPO, "gpurun_out", f"traffic_{TAG}")  # per tag: the csv glob below must see only this run


def run_pass(counter):
    d = os.path.join(OUT, counter.lower())
    os.makedirs(d, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", counter, "-d", d, "-o", counter.lower(), "--output-format", "csv", "--",
           sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1", "--config", CONFIG, "--no-cpu-baseline", "--no-projection-wall", "--no-strong"]
    subprocess.run(cmd, check=True, cwd=REPO, env=dict(os.environ, TMPDIR="/tmp"),
                   stdout=open(os.path.join(d, "log.txt"), "w"), stderr=subprocess.STDOUT, timeout=600)
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = {}
        for r in csv.DictReader(open(f)):
            if "wos_walk_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        vals += list(per.values())
    if not vals:
        raise SystemExit(f"no wos_walk_kernel {counter} records found under {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_kib, nf = run_pass("FETCH_SIZE")
    write_kib, nw = run_pass("WRITE_SIZE")
    raw = (fetch_kib + write_kib) * 1024.0
    res = {
        "config": CONFIG, "lib_sha16": lib_sha16(), "kernel": "wos_walk_kernel",
        "fetch_bytes": fetch_kib * 1024.0, "write_bytes": write_kib * 1024.0, "dispatches": [nf, nw],
        "bytes_per_launch": raw,
        "bytes_per_launch_fetch_x2": 2.0 * fetch_kib * 1024.0 + write_kib * 1024.0,
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), mean over {nf}/{nw} dispatches; "
                  "raw KiB x 1024 (4-byte gathers: FETCH_SIZE width correction uncalibrated, x2 bound alongside)",
    }
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    path = os.path.join(REPO, "gpurun_out", f"{TAG}_walk_traffic.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
