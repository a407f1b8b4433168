"""Host-to-device copy bandwidth from pinned memory (the end-to-end leg's link ceiling): one 134 MB
copy, 8 MB chunks on one stream, and 8 MB chunks alternating over two streams.  Dev tooling."""
import time

import torch


def main():
    n = 16 * 1024 * 1024 * 8
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ch = 8 << 20

    def one():
        d.copy_(h, non_blocking=True)

    def chunks(two):
        for i, lo in enumerate(range(0, n, ch)):
            with torch.cuda.stream(s2 if two and i & 1 else s1):
                d[lo:lo + ch].copy_(h[lo:lo + ch], non_blocking=True)

    for name, f in [("one copy", one), ("8 MB chunks, one stream", lambda: chunks(False)),
                    ("8 MB chunks, two streams", lambda: chunks(True))]:
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 10
        print(f"{name}: {n / dt / 1e9:.1f} GB/s ({dt * 1e3:.2f} ms for {n / 1e6:.0f} MB)", flush=True)
    hd = torch.empty(n, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        hd.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
    print(f"device to host, one copy: {n / dt / 1e9:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
