#!/usr/bin/env python3
"""Proofs in host memory -> statuses (GPU box): p2v_verify_batch_devices on device 0 with
pageable and pinned input (pinned up to 65 536 proofs), per chunk size.  usage: host_batch_probe.py [n_proofs]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "plonky2-verifier_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import p2v  # noqa: E402
from support import gen_circuit  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
gc = gen_circuit(12, 4, 0)
proofs = [gc.proof(1 + i % 4, 300 + i) for i in range(16)]
vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
packed = vk.pack_many(proofs)
host = np.ascontiguousarray(packed[np.arange(N) % len(proofs)])
pinned = torch.from_numpy(host.view(np.int64)).pin_memory().numpy().view(np.uint64) if N <= 65536 else None
print(f"N={N}, {host.nbytes / 1e9:.2f} GB of packed proofs", flush=True)


def rate(fn, k=2):
    fn()
    t = time.perf_counter()
    for _ in range(k):
        r = fn()
    dt = (time.perf_counter() - t) / k
    assert (r == 1).all()
    return N / dt


CHUNKS = tuple(int(c) for c in os.environ.get("P2V_PROBE_CHUNKS", "4096,16384").split(","))   # 0: auto (about n/8)
for chunk in CHUNKS:
    for name, arr in (("pageable", host), ("pinned", pinned)):
        if arr is None:
            continue
        print(f"verify_batch_devices chunk {chunk} {name}: {rate(lambda: p2v.verify_batch_devices(vk, arr, [0], chunk)):.0f} proofs/s", flush=True)
bv = p2v.BatchVerifier(vk, 0, 4096)
