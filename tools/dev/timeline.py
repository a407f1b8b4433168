"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace run (CSV): every kernel and copy with
its start / end relative to the first event, in time order, optionally only a window of them.

  python tools/dev/timeline.py <dir with *_kernel_trace.csv / *_memory_copy_trace.csv> [--last N]
"""
import argparse
import csv
import glob
import os


def rows(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        s = int(r.get("Start_Timestamp") or r.get("start_timestamp"))
        e = int(r.get("End_Timestamp") or r.get("end_timestamp"))
        if kind == "K":
            name = r.get("Kernel_Name") or r.get("kernel_name") or "?"
        else:
            name = (r.get("Direction") or r.get("Operation") or r.get("Kind") or "copy") + \
                   f" {int(r.get('Size', 0) or 0) / 1e6:.1f} MB"
        out.append((s, e, kind, name[:90]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=60)
    a = ap.parse_args()
    ev = []
    for p in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        ev += rows(p, "K")
    for p in glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True):
        ev += rows(p, "C")
    ev.sort()
    ev = ev[-a.last:]
    t0 = ev[0][0]
    for s, e, k, n in ev:
        print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} us  {k} {n}")


if __name__ == "__main__":
    main()
