#!/usr/bin/env python3
"""Where the time of p2v_verifier_run_json goes (GPU box): raw pinned H2D of the JSON blob,
the k_json_pack kernel (rocprofv3 shows it; here: run_json minus the other legs), and the
device-resident verification of the same batch."""
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
gc = gen_circuit(12, 4, 0)
proofs = [gc.proof(1 + i % 4, 100 + i) for i in range(16)]
vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
texts = [proofs[i % len(proofs)] for i in range(B)]
offs = np.zeros(B + 1, dtype=np.uint64)
offs[1:] = np.cumsum([len(t) for t in texts])
blob = torch.from_numpy(np.frombuffer(b"".join(texts), dtype=np.uint8).copy()).pin_memory()
bv = p2v.BatchVerifier(vk, 0, B)
res, codes = bv.run_json((blob.numpy(), offs))
assert os.environ.get("P2V_PROBE_NOCHECK") or ((codes == 0).all() and (res == 1).all())


def timeit(fn, k=3):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e3


dev = torch.empty(blob.numel(), dtype=torch.uint8, device="cuda")
t_h2d = timeit(lambda: dev.copy_(blob, non_blocking=True))
t_json = timeit(lambda: bv.run_json((blob.numpy(), offs)))
packed = vk.pack_many(proofs)
d = torch.from_numpy(np.ascontiguousarray(packed[np.arange(B) % len(proofs)]).view(np.int64)).cuda()
r = torch.empty(B, dtype=torch.int8, device="cuda")
t_ver = timeit(lambda: bv.run_device(d.data_ptr(), B, r.data_ptr()))
t_pack = timeit(lambda: vk.pack_many(texts[:512], threads=16), k=1) * B / 512
print(f"B={B} blob {blob.numel() / 1e6:.0f} MB: H2D {t_h2d:.2f} ms ({blob.numel() / t_h2d / 1e6:.1f} GB/s), run_json {t_json:.2f} ms, "
      f"verify {t_ver:.2f} ms, remainder (k_json_pack + host work) {t_json - t_h2d - t_ver:.2f} ms; host packer (16 threads) {t_pack:.1f} ms")
