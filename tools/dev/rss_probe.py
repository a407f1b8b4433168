"""Host memory of the plain CSR snapshot path at a given scale (dev tooling): generate the power-law
graph, build + upload its snapshot, print the process's peak RSS after each step."""
import resource
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rss_gb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    from tools import synth
    t = time.time()
    g = synth.SynthGraph(synth.scaled(synth.POWERLAW_1B, scale), threads=16)
    print(f"gen {time.time() - t:.1f} s peak {rss_gb():.1f} GB ({g.n_edges} tuples)", flush=True)
    t = time.time()
    s = g.snapshot(device=0)
    print(f"snapshot {time.time() - t:.1f} s peak {rss_gb():.1f} GB arena {s.part_stats(0, 1)['arena_bytes'] / 2**30 if False else 0}", flush=True)
    st = s.stats()
    print(f"device bytes {st['device_bytes'] / 2**30:.2f} GiB", flush=True)


if __name__ == "__main__":
    main()
