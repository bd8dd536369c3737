"""Device -> pinned host copy of one step's SB3 outputs at 65,536 envs (obs + reward + done, 3.7 MB):
one hipMemcpyAsync on the current stream against the same bytes split over 2 / 4 streams (whether
the copies then run on several DMA engines at once), host-timed to the event wait.

    python tools/d2h_split.py [bytes]
"""
import sys
import time

import numpy as np
import torch


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 65536 * 57
    dev = torch.device("cuda", 0)
    src = torch.randint(0, 255, (nb,), dtype=torch.uint8, device=dev)
    dst = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
    cur = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(4)]
    ev = torch.cuda.Event()

    def one():
        dst.copy_(src, non_blocking=True)
        ev.record(cur)
        ev.synchronize()

    def split(k):
        evs = []
        fork = torch.cuda.Event()
        fork.record(cur)
        step = -(-nb // k)
        for j in range(k):
            s = side[j]
            s.wait_event(fork)
            with torch.cuda.stream(s):
                dst[j * step:(j + 1) * step].copy_(src[j * step:(j + 1) * step], non_blocking=True)
                e = torch.cuda.Event()
                e.record(s)
                evs.append(e)
        for e in evs:
            e.synchronize()

    for name, fn in (("1 copy", one), ("2 streams", lambda: split(2)), ("4 streams", lambda: split(4)),
                     ("1 copy again", one)):
        for _ in range(50):
            fn()
        ts = np.empty(500)
        for i in range(500):
            t0 = time.perf_counter()
            fn()
            ts[i] = time.perf_counter() - t0
        print(f"{name:14s} {nb / 1e6:.2f} MB  median {np.median(ts) * 1e6:8.1f} us  "
              f"({nb / np.median(ts) / 1e9:.1f} GB/s)", flush=True)
    assert torch.equal(dst.to(dev), src)


if __name__ == "__main__":
    main()
