import os, sys, time
import numpy as np, torch
sys.path.insert(0, "plonky2-verifier_amd"); sys.path.insert(0, "tests")
import p2v
from support import gen_circuit
gc = gen_circuit(12, 4, 0)
proofs = [gc.proof(1 + i % 4, 300 + i) for i in range(16)]
vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
packed = vk.pack_many(proofs)
B = 4096
host = torch.from_numpy(np.ascontiguousarray(packed[np.arange(B) % 16]).view(np.int64)).pin_memory()
d1 = torch.empty_like(host, device="cuda"); d2 = torch.empty_like(host, device="cuda")
r = torch.empty(B, dtype=torch.int8, device="cuda")
bv = p2v.BatchVerifier(vk, 0, B)
s1 = torch.cuda.Stream(); s2 = torch.cuda.Stream()
def t(fn, k=5):
    fn(); torch.cuda.synchronize(); a = time.perf_counter()
    for _ in range(k): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - a) / k * 1e3
with torch.cuda.stream(s1):
    d1.copy_(host, non_blocking=True)
torch.cuda.synchronize()
h2d = t(lambda: d1.copy_(host, non_blocking=True))
ver = t(lambda: bv.run_device(d2.data_ptr(), B, r.data_ptr(), stream=s2.cuda_stream, sync=False))
def both():
    with torch.cuda.stream(s1):
        d1.copy_(host, non_blocking=True)
    bv.run_device(d2.data_ptr(), B, r.data_ptr(), stream=s2.cuda_stream, sync=False)
bo = t(both)
print(f"H2D {h2d:.2f} ms ({host.numel()*8/h2d/1e6:.1f} GB/s), verify {ver:.2f} ms, both concurrently {bo:.2f} ms")
