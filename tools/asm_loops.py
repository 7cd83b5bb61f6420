"""Lists the loops of one kernel in an amdgcn .s file: for every backward branch,
the label range, its instruction count and the mix (VALU / SALU / LDS / VMEM / branch).
    python3 tools/asm_loops.py file.s kernel_symbol_substring
"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
sub = sys.argv[2]
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sub in l and l.rstrip().endswith(":") or
             (l.startswith("_Z") and sub in l.split(":")[0]))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i


def kind(ins):
    op = ins.split()[0]
    if op.startswith("v_"): return "valu"
    if op.startswith("s_cbranch") or op.startswith("s_branch"): return "br"
    if op.startswith("s_"): return "salu"
    if op.startswith("ds_"): return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")): return "vmem"
    return "other"


loops = []
for i, l in enumerate(body):
    m = re.match(r"\s+(s_cbranch_\w+|s_branch)\s+(\.LBB\d+_\d+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        a = labels[m.group(2)]
        mix = {}
        n = 0
        for x in body[a:i + 1]:
            x = x.strip()
            if not x or x.startswith((";", ".")) or x.endswith(":"): continue
            k = kind(x)
            mix[k] = mix.get(k, 0) + 1
            n += 1
        loops.append((a + start + 1, i + start + 1, n, mix))
for a, b, n, mix in loops:
    print(f"lines {a}-{b}: {n} instrs {mix}")
total = sum(1 for x in body if x.strip() and not x.strip().startswith((";", ".")) and not x.strip().endswith(":"))
print("kernel instructions:", total)
