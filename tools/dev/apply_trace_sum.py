"""Summarize KETO_APPLY_TRACE lines (stderr of tools/apply_concurrent.py): per write, the staged part
(shared lock), the wait for the exclusive lock, the exclusive part (host commit + device), and the
device phases inside it (images, copies, closures, maps).  Prints one JSON line of p50 / p99 / max
per field and the closures' share of the exclusive part.  Dev tooling.

  python tools/dev/apply_trace_sum.py <log>
"""
import json
import re
import sys

import numpy as np


def main():
    fields = {}
    excl, clos = [], []
    for ln in open(sys.argv[1], errors="replace"):
        m = re.match(r"\[apply\] staged ([\d.]+) ms, lock wait ([\d.]+) ms, host commit \+ device ([\d.]+) ms", ln)
        if m:
            for k, v in zip(("staged", "lock_wait", "exclusive"), m.groups()):
                fields.setdefault(k, []).append(float(v))
            excl.append(float(m.group(3)))
            continue
        m = re.match(r"\[apply\] device phases \(ms\):(.*)", ln)
        if m:
            toks = m.group(1).split()
            for k, v in zip(toks[::2], toks[1::2]):
                fields.setdefault("device_" + k, []).append(float(v))
            c = dict(zip(toks[::2], map(float, toks[1::2]))).get("closures")
            if c is not None:
                clos.append(c)
    out = {k: {"p50": round(float(np.percentile(v, 50)), 3), "p99": round(float(np.percentile(v, 99)), 3),
               "max": round(max(v), 3), "n": len(v)} for k, v in fields.items()}
    if excl and clos and len(excl) == len(clos):
        out["closures_share_of_exclusive"] = round(sum(clos) / max(1e-9, sum(excl)), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
