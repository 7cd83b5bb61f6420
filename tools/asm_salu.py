"""Static instruction census of one kernel in an amdgcn .s file built with -gline-tables-only:
SALU by kind (exec-mask moves, constants / selects, s_nop hazards, branches, arithmetic,
s_waitcnt, compares, scalar loads) and VALU by kind, each attributed to the device function
whose body holds the instruction's source line (wos_device.h / wos_detmath.h function spans).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w \\
          -gline-tables-only --cuda-device-only -S csrc/wos_kernel.hip -o /tmp/wk.s
    python3 tools/asm_salu.py /tmp/wk.s wos_walk_kernelILi2ELb0ELb0ELb0ELb0E
"""
import collections
import os
import re
import sys

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "neural-monte-carlo-fluid-simulation_amd", "csrc")
FN = re.compile(r"^(?:template\s*<[^>]*>\s*)?(?:__device__|__global__|WOS_HD|static __device__)")
NOT_NAMES = {"__launch_bounds__", "__attribute__", "amdgpu_waves_per_eu", "amdgpu_flat_work_group_size"}


def fn_name(line):
    """the declared function's name: the first `name(` that is not an attribute"""
    for m in re.finditer(r"\b(\w+)\s*\(", line):
        if m.group(1) not in NOT_NAMES:
            return m.group(1)
    return None


def spans(path):
    """[(first line, last line, name)] of the functions and named lambdas of a header: from the
    declaration to the brace that closes its body (comments and strings are not parsed; the
    headers keep braces out of them)."""
    text = open(path).read().split("\n")
    out = []
    for i, line in enumerate(text):
        lam = re.match(r"\s+auto (\w+) = \[", line)
        name = lam.group(1) if lam else (fn_name(line) if FN.match(line) else None)
        if not name:
            continue
        depth, opened, j = 0, False, i
        while j < len(text):
            code = text[j].split("//")[0]
            if not opened and ";" in code and "{" not in code and j > i + 6:
                break  # a declaration without a body
            for ch in code:
                if ch == "{":
                    depth += 1
                    opened = True
                elif ch == "}":
                    depth -= 1
            if opened and depth <= 0:
                break
            j += 1
        if opened:
            out.append((i + 1, j + 1, name))
    return out


def owner(tab, line):
    """the innermost function / lambda whose span holds the line"""
    best, width = "?", None
    for first, last, nm in tab:
        if first <= line <= last and (width is None or last - first < width):
            best, width = nm, last - first
    return best


def salu_kind(op, line):
    if "exec" in line and op.startswith(("s_and", "s_or", "s_xor", "s_andn2", "s_orn2", "s_mov", "s_cselect")):
        return "exec mask"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc", "s_getpc")):
        return "branch"
    if op == "s_nop":
        return "s_nop (hazard)"
    if op == "s_waitcnt":
        return "s_waitcnt"
    if op.startswith(("s_load", "s_buffer_load")):
        return "scalar load"
    if op.startswith("s_cmp") or op.startswith("s_bitcmp"):
        return "compare"
    if op.startswith(("s_mov", "s_cselect", "s_movk")):
        return "move / select"
    if op in ("s_barrier", "s_sleep", "s_setprio", "s_endpgm", "s_memtime", "s_sethalt", "s_trap", "s_icache_inv"):
        return "other"
    return "arithmetic / bit"


def valu_kind(op):
    if op.startswith(("v_readlane", "v_writelane")):
        return "readlane / writelane"
    if op.startswith("v_readfirstlane"):
        return "readfirstlane"
    if "f64" in op:
        return "f64"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "compare"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith(("v_mov", "v_accvgpr")):
        return "move"
    if "f32" in op or "f16" in op:
        return "f32"
    return "int / bit"


def main():
    asm, sym = sys.argv[1], sys.argv[2]
    lines = open(asm).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = os.path.basename(m.group(3) or m.group(2))
    tabs = {f: spans(os.path.join(PKG, f)) for f in ("wos_device.h", "wos_detmath.h")}
    s = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0])
    e = next(i for i in range(s, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cur = "?"
    salu, valu = collections.Counter(), collections.Counter()
    by_fn = collections.defaultdict(collections.Counter)
    for l in lines[s:e]:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            f, ln = files.get(m.group(1), "?"), int(m.group(2))
            cur = f"{f.split('.')[0]}:{owner(tabs[f], ln)}" if f in tabs and ln > 0 else f
            continue
        t = l.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        if op.startswith("s_"):
            k = salu_kind(op, l)
            salu[k] += 1
            by_fn[cur]["salu"] += 1
            by_fn[cur]["salu:" + k] += 1
        elif op.startswith("v_"):
            valu[valu_kind(op)] += 1
            by_fn[cur]["valu"] += 1
    ts, tv = sum(salu.values()), sum(valu.values())
    print(f"{sym}: {ts} SALU, {tv} VALU static instructions")
    print("SALU by kind:")
    for k, n in salu.most_common():
        print(f"  {k:22s} {n:6d} {100.0 * n / ts:5.1f} %")
    print("VALU by kind:")
    for k, n in valu.most_common():
        print(f"  {k:22s} {n:6d} {100.0 * n / tv:5.1f} %")
    print("by source function (SALU, VALU; SALU kinds > 10 %):")
    for fn, c in sorted(by_fn.items(), key=lambda kv: -kv[1]["salu"])[:24]:
        kinds = ", ".join(f"{k[5:]} {v}" for k, v in c.most_common() if k.startswith("salu:") and v > 0.1 * c["salu"])
        print(f"  {fn:40s} {c['salu']:5d} {c['valu']:6d}   {kinds}")


if __name__ == "__main__":
    main()
