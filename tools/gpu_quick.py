#!/usr/bin/env python3
"""Quick GPU-vs-oracle parity sweep (developer tool; the pytest suite is the gate)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from support import gen_circuit, oracle, mutate, p2v_module  # noqa: E402


def case_set(gc):
    out = []
    for w in (1, 2):
        for s in (1, 2):
            out.append((f"valid w{w} s{s}", gc.proof(w, s)))
    base = gc.proof(1, 3)
    out.append(("flag1 step-eval", gc.proof(1, 4, flags=1)))
    out.append(("flag2 final", gc.proof(1, 5, flags=2)))
    out.append(("flag4 quotient", gc.proof(1, 6, flags=4)))

    def leaf(d):
        d["proof"]["opening_proof"]["query_round_proofs"][3]["initial_trees_proof"]["evals_proofs"][1][0][5] += 1
    out.append(("leaf q3", mutate(base, leaf)))

    def sib(d):
        d["proof"]["opening_proof"]["query_round_proofs"][0]["steps"][0]["merkle_proof"]["siblings"][0]["elements"][0] += 1
    out.append(("step sib q0", mutate(base, sib)))

    def powm(d):
        d["proof"]["opening_proof"]["pow_witness"] += 1
    out.append(("pow witness", mutate(base, powm)))

    def wire(d):
        d["proof"]["openings"]["wires"][7][0] += 1
    out.append(("wire opening", mutate(base, wire)))
    return out


def main():
    p2v = p2v_module()
    O = oracle()
    bad = 0
    for (nb, lk) in ((6, 0), (6, 1), (12, 0)):
        t = time.time()
        gc = gen_circuit(nb, 4, lk)
        cases = case_set(gc) if nb < 12 else [("valid", gc.proof(1, 1))]
        vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
        packed = vk.pack_many([c[1] for c in cases])
        bv = p2v.BatchVerifier(vk, 0, len(cases))
        res, tr = bv.run(packed, trace=True)
        print(f"n={nb} lookups={lk}: gen+run {time.time() - t:.1f}s timings {bv.last_timings()}")
        for i, (name, pj) in enumerate(cases):
            st, otr = O.verify_json(gc.common, gc.vkey, pj, trace=True)
            diff = np.nonzero(otr != tr[i])[0]
            ok = st == res[i] and len(diff) == 0
            bad += not ok
            print(f"  {name:18s} oracle={st:3d} gpu={res[i]:3d} trace_mismatch_words={len(diff)} {'' if ok else 'FAIL ' + str(diff[:12])}")
    print("ALL OK" if bad == 0 else f"{bad} FAILURES")
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
