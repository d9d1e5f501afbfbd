"""Real circuits (generator modes 1 and 2, csrc/gen/gen.cpp + gates.hpp), checked by the ORACLE on
the CPU.

The degenerate generator circuit makes every gate filter and every permutation-argument term
identically 0, so a verifier could mis-evaluate them and still accept.  A real circuit places
every gate of the recursion set on rows, selects each row's gate with selector polynomials
(Gate/Selector.hs:83-95), carries copy constraints through a real sigma permutation with Z and
the partial products (Plonk/Vanishing.hs:97-111), and commits a genuine quotient C/Z_H.  Its
witness rows follow plonky2's gate semantics, derived independently of the constraint programs
where the gate has a meaning of its own (the Poseidon output from the KAT-pinned permutation,
the CosetInterpolation result by Lagrange interpolation, base^e, Horner sums, list[index]).
A valid proof therefore accepts only if the verifier's every vanishing term agrees with the
prover's at zeta, and each of them is a non-zero field element there."""
import json

import numpy as np
import pytest

from support import P, circuit_shape, gen_circuit, mutate, oracle, trace_offsets


def _flags(gc, tr):
    r, S, Q = circuit_shape(gc.common)
    return int(tr[trace_offsets(r, S, Q)["flags"]])


@pytest.mark.parametrize("mode,nb", [(1, 6), (2, 6), (1, 8)])
def test_real_proofs_accept_with_nonzero_terms(mode, nb):
    O = oracle()
    gc = gen_circuit(nb, 4, 0, 1, 28, 16, 0, mode)
    c = json.loads(gc.common)
    if mode == 1:
        assert len(c["selectors_info"]["groups"]) > 1 and c["num_gate_constraints"] == 123
    else:
        assert len(c["selectors_info"]["groups"]) == 1
    for w in (1, 2):
        p = gc.proof(w, 1)
        st, tr = O.verify_json(gc.common, gc.vkey, p, trace=True)
        assert st == 1
        r, S, Q = circuit_shape(gc.common)
        off = trace_offsets(r, S, Q)
        comb = tr[off["combined"]: off["combined"] + 2 * r]
        assert (comb != 0).all()                       # C_i(zeta) = Q_i(zeta)(zeta^n - 1) != 0
        o = json.loads(p)["proof"]["openings"]
        for k in ("plonk_zs", "plonk_zs_next", "partial_products", "quotient_polys", "constants"):
            assert all(v != [1, 0] and v != [0, 0] for v in o[k]), k


def _real_reject_cases(gc):
    base = gc.proof(1, 3)

    def perturb(key, i):
        def f(d):
            d["proof"]["openings"][key][i][0] = (d["proof"]["openings"][key][i][0] + 1) % P
        return f
    return [
        (base, 1, 3),
        (gc.proof(1, 4, flags=1), -3, 3),    # step-0 evaluation mismatch
        (gc.proof(1, 5, flags=2), 0, 1),     # final polynomial (PoW still ok, identity ok)
        (gc.proof(1, 6, flags=4), 0, None),  # quotient opening: identity fails
        (mutate(base, perturb("wires", 3)), 0, None),
        (mutate(base, perturb("plonk_sigmas", 7)), 0, None),
        (mutate(base, perturb("plonk_zs", 1)), 0, None),
        (mutate(base, perturb("plonk_zs_next", 0)), 0, None),
        (mutate(base, perturb("partial_products", 11)), 0, None),
        (mutate(base, perturb("constants", 0)), 0, None),   # a gate-selector column S_0(zeta)
    ]


@pytest.mark.parametrize("mode", [1, 2])
def test_real_reject_paths(mode):
    """On a real circuit every opening feeds a non-zero term: perturbing a wire, sigma, Z,
    Z(omega zeta), partial product or selector opening breaks the Plonk identity (flags bit 0
    clear), where on the degenerate circuit it would only move the transcript."""
    O = oracle()
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, mode)
    for i, (proof, expect, flags) in enumerate(_real_reject_cases(gc)):
        st, tr = O.verify_json(gc.common, gc.vkey, proof, trace=True)
        assert st == expect, i
        fl = _flags(gc, tr)
        if flags is None:
            assert fl & 1 == 0, i           # eqs_ok = False
        else:
            assert fl & 1 == 1, i


def _eval_gate(gate: str, wires, consts, pih):
    """The oracle's constraint program of one gate string (or_eval_gate, F^2 inputs)."""
    O = oracle().L
    w2 = np.zeros(2 * len(wires), np.uint64)
    w2[0::2] = wires
    k2 = np.zeros(2 * len(consts), np.uint64)
    k2[0::2] = consts
    out = np.zeros(2 * 512, np.uint64)
    n = O.or_eval_gate(gate.encode(), w2.ctypes.data, len(wires), k2.ctypes.data, len(consts), pih.ctypes.data,
                       out.ctypes.data, 512)
    assert n >= 0
    return out[: 2 * n]


def test_gate_rows_satisfy_oracle_constraint_programs():
    """each gate kind's plonky2-semantics witness row makes every one of the
    ORACLE's constraints zero (Gate/Constraints.hs:40-128, Gate/Custom/*.hs), and corrupting any
    single wire that a constraint reads makes some constraint non-zero."""
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, 1)
    gates = json.loads(gc.common)["gates"]
    rng = np.random.default_rng(5)
    for g, s in enumerate(gates):
        for seed in (1, 2, 3):
            w, k, h, n = gc.gate_row(g, seed)
            out = _eval_gate(s, w, k, h)
            assert len(out) == 2 * n, s
            assert not out.any(), (s, seed, np.nonzero(out)[0][:5])
        if n == 0:
            continue   # NoopGate
        read = 0
        for wi in range(len(w)):
            w2 = w.copy()
            w2[wi] = (int(w2[wi]) + 1 + int(rng.integers(1 << 40))) % P
            read += bool(_eval_gate(s, w2, k, h).any())
        assert read > 0, s


def test_coset_interpolation_row_is_lagrange():
    """The CosetInterpolationGate row's result is the Lagrange interpolant of the 16 values at
    the shifted subgroup, evaluated at eval_loc: recomputed here in Python with big integers
    (F^2 = F[X]/(X^2 - 7), GoldilocksExt.hs:54-61), independently of both C restatements."""
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, 1)
    gates = json.loads(gc.common)["gates"]
    g = next(i for i, s in enumerate(gates) if s.startswith("CosetInterpolationGate"))
    w, _, _, _ = gc.gate_row(g, 9)
    w = [int(x) for x in w]

    def emul(a, b):
        return ((a[0] * b[0] + 7 * a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)
    h = 0x64fdd1a46201e246
    gen = pow(h, 2 ** 28, P)
    shift = w[0]
    vals = [(w[1 + 2 * k], w[2 + 2 * k]) for k in range(16)]
    z = (w[33], w[34])
    xs = [shift * pow(gen, k, P) % P for k in range(16)]
    acc = (0, 0)
    for k in range(16):
        num, den = (1, 0), 1
        for j in range(16):
            if j != k:
                num = emul(num, ((z[0] - xs[j]) % P, z[1]))
                den = den * (xs[k] - xs[j]) % P
        t = emul(vals[k], num)
        inv = pow(den, P - 2, P)
        acc = ((acc[0] + t[0] * inv) % P, (acc[1] + t[1] * inv) % P)
    assert (w[35], w[36]) == acc


def _lookup_reject_cases(gc):
    """(proof, expected status, eqs bit or None) on a real lookup circuit: valid proofs, an FRI
    reject, and openings that only lookup terms read (RE / SLDC at zeta and omega zeta, a
    lookup selector, the output wire of the first lookup slot) perturbed."""
    c = json.loads(gc.common)
    ng, nlp = len(c["selectors_info"]["groups"]), c["num_lookup_polys"]
    base = gc.proof(1, 3)

    def perturb(key, i, part=0):
        def f(d):
            d["proof"]["openings"][key][i][part] = (d["proof"]["openings"][key][i][part] + 1) % P
        return f
    return [
        (base, 1, 3),
        (gc.proof(2, 4), 1, 3),
        (gc.proof(1, 4, flags=1), -3, 3),
        (mutate(base, perturb("lookup_zs", 0)), 0, None),                 # RE, round 0
        (mutate(base, perturb("lookup_zs", nlp + 3, 1)), 0, None),        # an SLDC column, round 1
        (mutate(base, perturb("lookup_zs_next", nlp - 1)), 0, None),      # the last SLDC at omega zeta
        (mutate(base, perturb("constants", ng + 1)), 0, None),            # TransLdc selector
        (mutate(base, perturb("constants", ng + 4)), 0, None),            # StartEnd_0 selector
        (mutate(base, perturb("wires", 1)), 0, None),                     # a looked-up output
    ]


@pytest.mark.parametrize("nb,lk,mode", [(6, 5, 1), (6, 4, 2)])
def test_real_lookup_proofs_accept_and_reject(nb, lk, mode):
    """Real lookup circuits (LookupGate / LookupTableGate blocks, lookup selectors, RE and
    SLDC polynomials built by the prover, Plonk/Lookups.hs:45-132): valid proofs accept with
    C_i != 0, and each perturbed lookup opening breaks the identity."""
    O = oracle()
    gc = gen_circuit(nb, 4, lk, 1, 28, 16, 0, mode)
    c = json.loads(gc.common)
    assert c["num_lookup_polys"] == 7 and c["num_lookup_selectors"] == 4 + len(c["luts"])
    assert any(g.startswith("LookupGate") for g in c["gates"]) and any(g.startswith("LookupTableGate") for g in c["gates"])
    for i, (proof, expect, flags) in enumerate(_lookup_reject_cases(gc)):
        st, tr = O.verify_json(gc.common, gc.vkey, proof, trace=True)
        assert st == expect, i
        fl = _flags(gc, tr)
        assert (fl & 1 == 0) if flags is None else (fl & 1 == 1), i


def test_real_lookup_generator_refuses_a_table_too_large():
    """A 2^16-entry table needs 2 521 LookupTableGate rows: it does not fit 2^8 rows."""
    with pytest.raises(RuntimeError, match="do not fit"):
        gen_circuit(8, 4, 6, 1, 28, 16, 0, 1)
