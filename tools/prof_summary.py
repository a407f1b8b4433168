"""Summarize rocprofv3 outputs (kernel_stats.csv / counter_collection.csv) into a text table."""
import collections
import csv
import sys


def kernel_stats(path, top=8):
    rows = list(csv.DictReader(open(path)))
    out = ["kernel | calls | avg_us | total_ms | pct"]
    for r in rows[:top]:
        out.append(f"{r['Name'][:110]} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f}")
    return "\n".join(out)


def counters(path, name_filter, min_grid=0):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(list)
    for r in rows:
        if name_filter in r["Kernel_Name"] and int(r["Grid_Size"]) >= min_grid:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


if __name__ == "__main__":
    kind = sys.argv[1]
    if kind == "stats":
        print(kernel_stats(sys.argv[2]))
    else:
        flt = sys.argv[3] if len(sys.argv) > 3 else "check_kernel"
        for k, v in sorted(counters(sys.argv[2], flt, int(sys.argv[4]) if len(sys.argv) > 4 else 0).items()):
            print(f"{k} = {v:.6g}")
