"""Turn one gpu_round.sh run into the committed profile summary that bench.py's `roofline.traffic`
reads (tooling).

  python tools/traffic.py gpurun_out/<tag> profiles/<round>_<tag>

writes <out>_kernel_stats.txt (rocprofv3 --kernel-trace --stats summary of the bench command) and
<out>_traffic.json (per-launch HBM bytes of the dominant kernel from the FETCH_SIZE / WRITE_SIZE
PMC passes).  Correction (calibrated with tools/calib.hip on an MI355X, profiles/r01_calib.txt):
FETCH_SIZE tallies 64 B per L2 miss while every miss is a 128-B DRAM read (TCC_EA0_RDREQ_128B =
TCC_EA0_RDREQ), for streaming reads and for random 4-16 B gathers alike, so read bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE x 1024 is taken as is.
The json carries the sha256 of engine.hip and its compile flags, so bench.py only uses it for the kernel it was measured on.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def engine_sha():
    import importlib.util
    spec = importlib.util.spec_from_file_location("_keto_build", os.path.join(ROOT, "keto_amd", "build.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.engine_build_id()   # engine.hip and its compile flags


def pmc(path, counter, kernel):
    vals = []
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals), len(vals)


def stats(path, kernel):
    out, avg = ["kernel | calls | avg_us | total_ms | pct"], None
    for r in csv.DictReader(open(path)):
        out.append(f"{r['Name'][:110]} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                   f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f}")
        if kernel in r["Name"] and avg is None:
            avg = float(r["AverageNs"]) / 1e6
    return "\n".join(out), avg


def main(src, dst):
    line = [l for l in open(os.path.join(src, "bench.log")) if l.startswith("{")][-1]
    bench = json.loads(line)
    cfg = bench["config"]
    kernel = bench["roofline"]["kernel"]
    txt, avg_ms = stats(os.path.join(src, "kt", "kt_kernel_stats.csv"), kernel)
    fetch, nf = pmc(os.path.join(src, "pmc_FETCH_SIZE", "pmc_counter_collection.csv"), "FETCH_SIZE", kernel)
    write, nw = pmc(os.path.join(src, "pmc_WRITE_SIZE", "pmc_counter_collection.csv"), "WRITE_SIZE", kernel)
    with open(dst + "_kernel_stats.txt", "w") as f:
        f.write(f"# rocprofv3 --kernel-trace --stats -- python bench.py --no-work  ({src})\n")
        f.write(txt + "\n")
    rd = 2.0 * fetch * 1024
    wr = write * 1024
    j = {"kernel": kernel, "engine_sha256": engine_sha(), "launches": [nf, nw],
         "workload": {k: cfg[k] for k in ("tuples", "checks_per_gpu_per_step", "max_depth", "scale")},
         "FETCH_SIZE_kb": fetch, "WRITE_SIZE_kb": write, "read_bytes": rd, "write_bytes": wr,
         "traffic_bytes": rd + wr, "kernel_trace_avg_ms": avg_ms,
         "traffic_GBps_at_trace_ms": (rd + wr) / (avg_ms * 1e-3) / 1e9 if avg_ms else None,
         "correction": "read = 2 x FETCH_SIZE KB (tools/calib.hip: 64 B tallied per 128-B line miss); write = WRITE_SIZE KB"}
    with open(dst + "_traffic.json", "w") as f:
        json.dump(j, f, indent=1)
    print(json.dumps(j, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
