"""Instruction issue of the walk kernel from rocprofv3 SQ counters (GPU box): one
--pmc pass (8 SQ counters) over `bench.py --steps 2 --warmup 1`, averaged over the
wos_walk_kernel dispatches and written to gpurun_out/<tag>_walk_sq.json (copy it to
profiles/ to have bench.py report it as roofline.valu).

The path is bound by neither HBM nor MFMA: the meaningful ceiling
is the vector-instruction issue rate.  valu_issue_frac = SQ_INSTS_VALU x 4 cycles
(a wave64 VALU instruction occupies a 16-lane SIMD for 4 cycles) / (kernel time x
2.4 GHz x 256 CUs x 4 SIMDs), the kernel time from the same pass's dispatch
timestamps; the SQ_WAIT_* split says how much of a wave's life is spent parked on
memory / LDS waits (s_waitcnt) versus stalled at issue.
    python3 tools/collect_sq.py [tag] [config] [set]

set "issue" (default) is the pass above; "mix" and "mix2" are the instruction-mix passes
(VALU by type: F64 add/mul/fma/transcendental, F32, INT32/64, conversions; SALU and
scalar-pipe active cycles, branches, scalar loads); "icache" the instruction cache (requests,
hits, misses) with LDS bank conflicts and LDS issue waits; "dcache" the scalar data cache and
the LDS load / store / atomic split.  Written to <tag>_<set>_walk_sq.json.
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
SET = sys.argv[3] if len(sys.argv) > 3 else "issue"
SETS = {
    "issue": ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
              "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"],
    "mix": ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64",
            "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT"],
    "mix2": ["SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_ACTIVE_INST_VALU",
             "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM"],
    "icache": ["SQC_ICACHE_REQ", "SQC_ICACHE_HITS", "SQC_ICACHE_MISSES", "SQC_ICACHE_MISSES_DUPLICATE", "SQ_IFETCH",
               "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS", "SQ_LDS_IDX_ACTIVE"],
    "dcache": ["SQC_DCACHE_REQ", "SQC_DCACHE_HITS", "SQC_DCACHE_MISSES", "SQC_DCACHE_MISSES_DUPLICATE",
               "SQ_INSTS_LDS_LOAD", "SQ_INSTS_LDS_STORE", "SQ_INSTS_LDS_ATOMIC", "SQ_INSTS_SMEM"],
}
COUNTERS = SETS[SET]
PFX = TAG if SET == "issue" else f"{TAG}_{SET}"
OUT = os.path.join(REPO, "gpurun_out", f"{PFX}_sq")
CLOCK_HZ, SIMDS = 2.4e9, 256 * 4


def main():
    os.makedirs(OUT, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", *COUNTERS, "-d", OUT, "-o", "sq", "--output-format", "csv", "--",
           sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1", "--config", CONFIG, "--no-cpu-baseline",
           "--no-projection-wall", "--no-strong"]
    subprocess.run(cmd, check=True, cwd=REPO, env=dict(os.environ, TMPDIR="/tmp"),
                   stdout=open(os.path.join(OUT, "log.txt"), "w"), stderr=subprocess.STDOUT, timeout=280)
    per, dur, kname = {}, {}, {}
    for f in glob.glob(os.path.join(OUT, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = r["Dispatch_Id"]
            kname[d] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("wos::", "")
            per.setdefault(d, {}).setdefault(r["Counter_Name"], 0.0)
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9

    def summary(name):
        ds = [d for d in per if kname[d] == name]
        n = len(ds)
        mean = {c: sum(per[d].get(c, 0.0) for d in ds) / n for c in COUNTERS}
        t = sum(dur[d] for d in ds) / n
        res = {"kernel": name, "config": CONFIG, "lib_sha16": lib_sha16(), "dispatches": n, "kernel_s": t,
               "counters": mean,
               "source": "rocprofv3 --pmc " + " ".join(COUNTERS) + " (one pass), bench.py --steps 2 --warmup 1"}
        if SET != "issue":
            return res
        return {**res,
                "valu_issue_frac": mean["SQ_INSTS_VALU"] * 4 / (t * CLOCK_HZ * SIMDS),
                "wait_any_frac": mean["SQ_WAIT_ANY"] / max(mean["SQ_WAVE_CYCLES"], 1.0),
                "wait_inst_frac": mean["SQ_WAIT_INST_ANY"] / max(mean["SQ_WAVE_CYCLES"], 1.0),
                "active_frac": mean["SQ_ACTIVE_INST_ANY"] / max(mean["SQ_WAVE_CYCLES"], 1.0),
                "source": "rocprofv3 --pmc " + " ".join(COUNTERS) + " (one pass), bench.py --steps 2 --warmup 1; "
                          "VALU issue = INSTS_VALU x 4 cycles / (kernel time x 2.4 GHz x 1024 SIMDs)"}

    if "wos_walk_kernel" not in kname.values():
        raise SystemExit(f"no wos_walk_kernel records under {OUT}")
    # every kernel of the projection (the first-ball and setup kernels too)
    allk = {k: summary(k) for k in sorted(set(kname.values()))}
    json.dump(allk, open(os.path.join(REPO, "gpurun_out", f"{PFX}_all_sq.json"), "w"), indent=1)
    for k, v in allk.items():
        print(k, json.dumps({x: v[x] for x in ("kernel_s", "valu_issue_frac", "wait_any_frac", "active_frac") if x in v}))
    res = allk["wos_walk_kernel"]
    path = os.path.join(REPO, "gpurun_out", f"{PFX}_walk_sq.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
