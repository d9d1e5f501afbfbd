#!/usr/bin/env python3
"""PCIe host->device copy rates from pinned memory (the ceiling of the from-host legs of
bench.py): one copy of the whole buffer, and the buffer in chunks spread over
1..4 streams (each stream copies its chunks back to back), timed on the host around a sync.
Prints one JSON line.  Usage: python tools/h2d_probe.py [MB] [reps]"""
import json
import sys
import time

import torch


def main():
    mb = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n = mb << 20
    dev = torch.device("cuda", 0)
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    host.fill_(1)
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    out = {"MB": mb, "reps": reps}
    for nst in (1, 2, 3, 4):
        for chunk_mb in (8, 32, 128, mb):
            if chunk_mb > mb or (nst > 1 and chunk_mb == mb):
                continue
            sts = [torch.cuda.Stream(dev) for _ in range(nst)]
            c = chunk_mb << 20
            chunks = [(o, min(c, n - o)) for o in range(0, n, c)]

            def once():
                for k, (o, ln) in enumerate(chunks):
                    with torch.cuda.stream(sts[k % nst]):
                        d[o:o + ln].copy_(host[o:o + ln], non_blocking=True)
                torch.cuda.synchronize(dev)
            once()
            t = time.perf_counter()
            for _ in range(reps):
                once()
            dt = (time.perf_counter() - t) / reps
            out[f"streams{nst}_chunk{chunk_mb}MB_GBps"] = round(n / dt / 1e9, 2)
    # device -> host of the same buffer (the results direction, for reference)
    t = time.perf_counter()
    for _ in range(reps):
        host.copy_(d, non_blocking=True)
        torch.cuda.synchronize(dev)
    out["d2h_GBps"] = round(n * reps / (time.perf_counter() - t) / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
