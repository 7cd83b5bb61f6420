"""Summarises a rocprofv3 --pmc counter_collection.csv: per kernel name, the
counters of its LAST dispatch (one value per counter, summed over dimensions).
    python3 tools/pmc_summary.py gpurun_out/pmc1/pmc1_counter_collection.csv [kernel-substring]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else "wos_solve"
last = {}
for r in rows:
    if sub in r["Kernel_Name"]:
        last[r["Kernel_Name"]] = max(last.get(r["Kernel_Name"], 0), int(r["Dispatch_Id"]))
for name, d in last.items():
    agg = collections.OrderedDict()
    dur = None
    for r in rows:
        if r["Kernel_Name"] == name and int(r["Dispatch_Id"]) == d:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"{name[:60]}  dispatch {d}  {dur:.3f} ms")
    for k, v in agg.items():
        print(f"  {k:28s} {v:16.0f}")
