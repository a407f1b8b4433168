"""Average each PMC counter per kernel over the runs of tools/pmc_groups.sh (tooling).
  python tools/pmc_sum.py gpurun_out/<tag> [kernel-substring] [per-unit divisor]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
div = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/p*/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"] and "rocclr" not in r["Kernel_Name"]:
            agg[(r["Kernel_Name"].split("(")[0][-60:], int(r["Grid_Size"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    m = sum(v) / len(v)
    print(f"{k[0]} | {k[1]} | {k[2]} | {m:.4g} | per-unit {m / div:.4g}")
