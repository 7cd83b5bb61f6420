"""Instruction issue of the walk kernel from rocprofv3 SQ counters (GPU box): one
--pmc pass (8 SQ counters) over `bench.py --steps 2 --warmup 1`, averaged over the
wos_walk_kernel dispatches and written to gpurun_out/<tag>_walk_sq.json (copy it to
profiles/ to have bench.py report it as roofline.valu).

The path is bound by neither HBM nor MFMA: the meaningful ceiling
is the vector-instruction issue rate.  The issue pass's valu_issue_frac_4cyc =
SQ_INSTS_VALU x 4 cycles / (kernel time x 2.4 GHz x 256 CUs x 4 SIMDs) is the CDNA3
rule of thumb (16-lane SIMDs); gfx950's are 32 lanes wide, so a wave64 f32 / int
instruction costs about 2 SIMD-cycles.  The calibrated figure (`combine`, below)
weights each instruction type by its measured SIMD-cycles per wave64 instruction
(tools/mb_latency.hip `issue`: 16 independent chains of one type, 4 waves per SIMD,
one workgroup per CU) over the instruction mix of the same launches (mix / mix2
passes): valu_issue_frac = sum_t n_t c_t / (kernel time x 2.4 GHz x 1024 SIMDs).
The SQ_WAIT_* split says how much of a wave's life is spent parked on memory / LDS
waits (s_waitcnt) versus stalled at issue.
    python3 tools/collect_sq.py [tag] [config] [set]
    python3 tools/collect_sq.py combine TAG CONFIG MB_ISSUE_JSON   (after issue, mix, mix2)

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
TAG = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "combine" else "r1"
CONFIG = sys.argv[2] if len(sys.argv) > 2 else "B"
SET = sys.argv[3] if len(sys.argv) > 3 and sys.argv[1] != "combine" else "issue"
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
                "valu_issue_frac_4cyc": mean["SQ_INSTS_VALU"] * 4 / (t * CLOCK_HZ * SIMDS),
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
        print(k, json.dumps({x: v[x] for x in ("kernel_s", "valu_issue_frac_4cyc", "wait_any_frac", "active_frac")
                             if x in v}))
    res = allk["wos_walk_kernel"]
    path = os.path.join(REPO, "gpurun_out", f"{PFX}_walk_sq.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res))


# instruction type (mix counter) -> the microbenchmark instruction whose issue cost stands for it
TYPE_OPS = {
    "SQ_INSTS_VALU_ADD_F64": "v_add_f64", "SQ_INSTS_VALU_MUL_F64": "v_mul_f64",
    "SQ_INSTS_VALU_FMA_F64": "v_fma_f64", "SQ_INSTS_VALU_TRANS_F64": "v_rcp_f64",
    "SQ_INSTS_VALU_TRANS_F32": "v_exp_f32", "SQ_INSTS_VALU_ADD_F32": "v_add_f32",
    "SQ_INSTS_VALU_MUL_F32": "v_fma_f32", "SQ_INSTS_VALU_FMA_F32": "v_fma_f32",
    "SQ_INSTS_VALU_INT32": "v_add_u32", "SQ_INSTS_VALU_INT64": "v_lshlrev_b64",
    "SQ_INSTS_VALU_CVT": "v_cvt_f64_f32",
}
OTHER_OPS = ("v_mov_b32", "v_cndmask_b32")  # untyped VALU (moves, selects, compares, lane ops): at the
# move's cost (the calibrated figure) and at the SGPR-mask select's (the upper bound, `_hi`)


def issue_cycles(mb, waves=4):
    """op -> SIMD-cycles per wave64 instruction at `waves` waves per SIMD (mb_latency issue)."""
    return {r["op"]: r["simd_cycles_per_wave_instr"] for r in mb["results"] if r["waves_per_simd"] == waves}


def weighted_issue(issue, mix, mix2, cyc, other_op="v_mov_b32"):
    """Calibrated VALU issue fraction of one kernel: sum over types of count x cycles / SIMD-cycles."""
    n = dict(mix["counters"], **mix2["counters"])
    parts, typed = {}, 0.0
    for ctr, op in TYPE_OPS.items():
        parts[ctr] = n.get(ctr, 0.0) * cyc[op]
        typed += n.get(ctr, 0.0)
    other = max(0.0, issue["counters"]["SQ_INSTS_VALU"] - typed)
    c_other = cyc[other_op]
    parts["untyped"] = other * c_other
    busy = sum(parts.values())
    denom = issue["kernel_s"] * CLOCK_HZ * SIMDS
    return busy / denom, {k: v / denom for k, v in parts.items()}, other


def combine(tag, config, mb_path):
    """<tag>[_<config>]_walk_sq.json gains valu_issue_frac (calibrated) from its mix / mix2 passes."""
    mb = json.load(open(mb_path))
    cyc = issue_cycles(mb)
    pfx = tag if config == "B" else f"{tag}_{config}"
    out = os.path.join(REPO, "gpurun_out")
    issue = json.load(open(os.path.join(out, f"{pfx}_walk_sq.json")))
    mix = json.load(open(os.path.join(out, f"{pfx}_mix_walk_sq.json")))
    mix2 = json.load(open(os.path.join(out, f"{pfx}_mix2_walk_sq.json")))
    frac, parts, other = weighted_issue(issue, mix, mix2, cyc)
    frac_hi, _, _ = weighted_issue(issue, mix, mix2, cyc, other_op="v_cndmask_b32")
    issue.update({
        "valu_issue_frac": frac, "valu_issue_frac_hi": frac_hi, "valu_issue_parts": parts,
        "valu_untyped_instr": other,
        "issue_cycles": {op: cyc[op] for op in sorted(set(TYPE_OPS.values()) | set(OTHER_OPS))},
        "issue_calibration": f"{os.path.basename(mb_path)}: tools/mb_latency.hip issue, SIMD-cycles per wave64 "
                             "instruction at 4 waves/SIMD; counts from the mix / mix2 passes of the same launches "
                             "(untyped VALU at the move's cost; valu_issue_frac_hi: at the SGPR-mask select's)",
    })
    issue["source"] = issue["source"].replace(
        "VALU issue = INSTS_VALU x 4 cycles / (kernel time x 2.4 GHz x 1024 SIMDs)",
        "VALU issue = sum over instruction types of count x measured SIMD-cycles / (kernel time x 2.4 GHz x 1024 "
        "SIMDs); valu_issue_frac_4cyc = INSTS_VALU x 4 cycles / the same")
    path = os.path.join(out, f"{pfx}_walk_sq.json")
    json.dump(issue, open(path, "w"), indent=1)
    print(json.dumps({"config": config, "valu_issue_frac": frac, "valu_issue_frac_hi": frac_hi,
                      "valu_issue_frac_4cyc": issue["valu_issue_frac_4cyc"],
                      "parts": parts}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "combine":
        combine(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        main()
