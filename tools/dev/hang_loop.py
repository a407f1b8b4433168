"""Run one GPU test function repeatedly in this process with KETO_TRACE_LOCKS on; if an iteration
takes more than --limit seconds, print every thread's Python stack and exit (the lock trace on
stderr shows where each thread waits).  Dev tooling.
  python tools/dev/hang_loop.py tests.test_gpu_resolve_device:test_packed_batches_concurrent_with_writes --n 30"""
import argparse
import faulthandler
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("target")
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--limit", type=int, default=60)
    a = ap.parse_args()
    os.environ["KETO_TRACE_LOCKS"] = "1"
    mod, fn = a.target.split(":")
    f = getattr(importlib.import_module(mod), fn)
    for i in range(a.n):
        faulthandler.dump_traceback_later(a.limit, exit=True)
        t = time.time()
        f()
        faulthandler.cancel_dump_traceback_later()
        print(f"iteration {i}: {time.time() - t:.2f} s", flush=True)


if __name__ == "__main__":
    main()
