"""Pins the ORACLE (oracle/oracle.c, the CPU restatement of the reference) against the
reference's own known answers, and checks generator self-consistency (CPU only)."""
import gzip
import json
import os

import numpy as np
import pytest

from support import GOLDEN, KAT_IN, KAT_OUT, P, gen_circuit, mutate, oracle


def test_poseidon_kat():
    # the reference's only result-pinning vector: Hash/Poseidon.hs:27-35
    assert oracle().permute(KAT_IN) == KAT_OUT


def test_roots_of_unity_sage_identities():
    # Algebra/Goldilocks.hs:58-67: h = g^((p-1)/2^32) == twoAdicGen; rootsOfUnity!k = h^(2^(32-k))
    O = oracle().L
    g, h = 0xc65c18b67785d900, 0x64fdd1a46201e246
    assert pow(g, (P - 1) // 2**32, P) == h
    for q in (2, 3, 5, 17, 257, 65537):   # p - 1 = 2^32 * 3 * 5 * 17 * 257 * 65537
        assert pow(g, (P - 1) // q, P) != 1
    assert O.or_subgroup_gen(32) == h
    for k in range(0, 33):
        w = O.or_subgroup_gen(k)
        assert w == pow(h, 2 ** (32 - k), P)
        assert pow(w, 2**k, P) == 1
        if k > 0:
            assert pow(w, 2 ** (k - 1), P) != 1


def test_field_inverse_semantics():
    O = oracle().L
    assert O.or_finv(0) == 0          # inv = pow x (p-2): inv 0 = 0 (Goldilocks.hs:155-156)
    rng = np.random.default_rng(1)
    for x in [1, 2, P - 1, P - 2, 2**32 - 1, 2**32] + [int(v) for v in rng.integers(1, 2**63, 50)]:
        assert O.or_fmul(x % P, O.or_finv(x % P)) == 1


@pytest.mark.parametrize("gate,kind", [
    ("ArithmeticGate { num_ops: 20 }", 0),
    ("ArithmeticGate { num_ops: 20 } trailing", 16),          # withEOF -> UnknownGate
    ("ArithmeticExtensionGate { num_ops: 10 }", 1),
    ("BaseSumGate { num_limbs: 63 } + Base: 2", 2),
    ("ConstantGate { num_consts: 2 }<anything>", 4),           # no EOF check
    ("ExponentiationGate { num_power_bits: 66 }", 5),
    ("ExponentiationGate { num_power_bits: 66, _phantom: PhantomData<x> }<D=2>", 16),
    ("LookupGate { num_slots: 40, lut_hash: [1, 2, 3] }", 6),
    ("LookupTableGate { num_slots: 26, lut_hash: [], last_lut_row: 7 }", 7),
    ("MulExtensionGate { num_ops: 13 }", 8),
    ("NoopGate", 9),
    ("PublicInputGate", 10),
    ("PoseidonGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=12>", 11),
    ("PoseidonMdsGate(PhantomData<plonky2_field::goldilocks_field::GoldilocksField>)<WIDTH=12>", 12),
    ("RandomAccessGate { bits: 4, num_copies: 4, num_extra_constants: 2, _phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField> }<D=2>", 13),
    ("ReducingGate { num_coeffs: 43 }", 14),
    ("ReducingExtensionGate { num_coeffs: 32 }", 15),
    ("SomethingElse", 16),
])
def test_gate_parser_grammar(gate, kind):
    # Gate/Parser.hs:112-240
    assert oracle().L.or_gate_kind(gate.encode()) == kind


def test_generated_proofs_accept_and_perm_count():
    O = oracle()
    for lk in (0, 1):
        for ng in (0, 1):   # 3 selector groups / one group (the column is NoopGate's index)
            gc = gen_circuit(6, 4, lk, 1, 28, 16, ng)
            for w, s in ((1, 1), (2, 3)):
                assert O.verify_json(gc.common, gc.vkey, gc.proof(w, s)) == 1
    # permutation-count model of SURVEY.md §8d at n = 6 (1727) + ceil(#PI/8) for the PI hash
    gc = gen_circuit(6, 4, 0)
    pr = gc.proof(1, 1)
    c, p = O.circuit(gc.common, gc.vkey), O.proof(pr)
    O.L.or_perm_count_reset()
    assert O.verify(c, p) == 1
    assert O.L.or_perm_count() == 1727 + 1


@pytest.mark.slow
def test_perm_count_matches_commentary_at_n12():
    # commentary/FRI.md:263-265: 114 + 28 x (77 + 11 + 7) = 2774 permutations (+1: PI hash)
    O = oracle()
    gc = gen_circuit(12, 4, 0)
    c, p = O.circuit(gc.common, gc.vkey), O.proof(gc.proof(1, 1))
    O.L.or_perm_count_reset()
    assert O.verify(c, p) == 1
    assert O.L.or_perm_count() == 2774 + 1


def _reject_cases(gc):
    base = gc.proof(1, 3)

    def leaf(d):
        d["proof"]["opening_proof"]["query_round_proofs"][3]["initial_trees_proof"]["evals_proofs"][0][0][1] += 1

    def sib(d):
        d["proof"]["opening_proof"]["query_round_proofs"][2]["steps"][0]["merkle_proof"]["siblings"][0]["elements"][1] += 1

    def powm(d):
        d["proof"]["opening_proof"]["pow_witness"] += 1

    def wire(d):
        d["proof"]["openings"]["wires"][3][0] += 1

    def later_leaf_after_final_fail(d):   # round 0 is decided first
        d["proof"]["opening_proof"]["query_round_proofs"][9]["initial_trees_proof"]["evals_proofs"][1][0][0] += 1
    return [
        (gc.proof(1, 4, flags=1), -3),   # step-0 evaluation mismatch  (Plonk/FRI.hs:311)
        (gc.proof(1, 5, flags=2), 0),    # final polynomial mismatch -> False
        (gc.proof(1, 6, flags=4), 0),    # Plonk identity fails: FRI never evaluated
        (mutate(base, leaf), -1),        # initial-tree Merkle failure (Plonk/FRI.hs:108)
        (mutate(base, sib), -2),         # step Merkle failure (Plonk/FRI.hs:310)
        (mutate(base, powm), 0),         # proof-of-work (Plonk/FRI.hs:212-216)
        (mutate(base, wire), 0),         # opening changed: on this degenerate circuit C_i stays 0,
                                         # the transcript moves and the proof fails by its PoW
        (mutate(gc.proof(1, 5, flags=2), later_leaf_after_final_fail), 0),
    ]


@pytest.mark.parametrize("lk", [0, 1])
def test_reject_paths_follow_reference_order(lk):
    O = oracle()
    gc = gen_circuit(6, 4, lk)
    for proof, expect in _reject_cases(gc):
        assert O.verify_json(gc.common, gc.vkey, proof) == expect


def test_degenerate_wire_mutation_fails_by_pow_not_identity():
    """on the degenerate circuit a changed wire opening leaves C_i = 0 (gate filters
    0, sigma = k X); the proof is rejected by its proof of work.  The real circuits of
    test_real_circuits.py are the ones where the same mutation breaks the Plonk identity."""
    from support import circuit_shape, trace_offsets
    O = oracle()
    gc = gen_circuit(6, 4, 0)
    proof = _reject_cases(gc)[6][0]
    st, tr = O.verify_json(gc.common, gc.vkey, proof, trace=True)
    fl = int(tr[trace_offsets(*circuit_shape(gc.common))["flags"]])
    assert st == 0 and fl == 1   # eqs_ok, not pow_ok


def test_value_canonicalisation_in_json():
    # aeson Integer then mod p (Goldilocks.hs:98-102): x + p and x - p decode to x
    O = oracle()
    gc = gen_circuit(6, 4, 0)
    pr = gc.proof(2, 3)

    def plus_p(d):
        d["public_inputs"][0] += P
        d["proof"]["openings"]["wires"][5][1] -= P
    assert O.verify_json(gc.common, gc.vkey, mutate(pr, plus_p)) == 1


def _golden():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        exp = json.load(f)["cases"]

    def rd(name):
        with gzip.open(os.path.join(GOLDEN, name), "rb") as f:
            return f.read()
    return exp, rd


def test_golden_fixtures_oracle():
    exp, rd = _golden()
    O = oracle()
    for case in exp:
        common, vkey = rd(case["circuit"] + "_common.json.gz"), rd(case["circuit"] + "_vkey.json.gz")
        st, tr = O.verify_json(common, vkey, rd(case["name"] + "_proof.json.gz"), trace=True)
        assert st == case["status"], case["name"]
        assert [int(x) for x in tr] == [int(x) for x in case["trace"]], case["name"]


def test_coset_gate_matches_reference_example():
    """Gate/Parser.hs:150 quotes a CosetInterpolationGate string from a real Plonky2 circuit:
    `subgroup_bits: 4, degree: 6, barycentric_weights: [17293822565076172801, ...`.  The
    generator derives degree and weights itself (CosetInterp.hs:36-49: w_i = 1/prod_{j!=i}
    (x_i - x_j) over the size-16 subgroup, so w_0 = 1/16); the reference's example pins both,
    and with them the field inverse and the 2-adic subgroup generator."""
    gc = gen_circuit(6, 4, 0)
    gates = [g for g in json.loads(gc.common)["gates"] if g.startswith("CosetInterpolationGate")]
    assert gates
    assert gates[0].startswith("CosetInterpolationGate { subgroup_bits: 4, degree: 6, "
                               "barycentric_weights: [17293822565076172801, ")
    assert oracle().L.or_gate_kind(gates[0].encode()) == oracle().L.or_gate_kind(
        b"CosetInterpolationGate { subgroup_bits: 4, degree: 6, barycentric_weights: [17293822565076172801], "
        b"_phantom: PhantomData<plonky2_field::goldilocks_field::GoldilocksField> }<D=2>")


def test_first_round_wrap_states_hit_their_targets():
    """The crafted permutation states of the GPU S-box tests: round 0's constant addition (as
    p2::add_nc computes it) lands exactly on the S-box edge value, except where no 64-bit word
    can (then on the congruent y + p)."""
    from support import EPS, add_nc, first_round_wrap_states, preimage_round0, round0_constants, sbox_edge_values
    rc0 = round0_constants()
    exact = 0
    for y in sbox_edge_values():
        for i in range(12):
            w = preimage_round0(y, i, rc0)
            assert 0 <= w < 1 << 64
            got = add_nc(w, rc0[i])
            assert got % P == y % P
            exact += got == y
            if y >= rc0[i] or y >= EPS:
                assert got == y
    assert exact > 0.6 * 12 * len(sbox_edge_values())   # y < min(rc0[i], 2^32 - 1): no 64-bit word reaches y itself
    st = first_round_wrap_states()
    assert any(add_nc(w, rc0[i]) == 1 << 48 for s in st for i, w in enumerate(s))


def test_chunked_reduce_powers_algebra():
    """k_fri's combineInitial (round 5, kernels.hip reduce_powers): Horner in chunks of 8,
    g <- g a^8 + sum_{k<8} y_{j+k} a^k, whose inner sums of base-field products are kept as
    lo + hi 2^64 + top 2^128 and reduced with 2^128 == -2^32 (mod p), equals the reference's
    reduceWithPowers sum_i a^i y_i (Goldilocks.hs:180-183) in F^2 = F[X]/(X^2 - 7), for list
    lengths that are and are not multiples of 8."""
    import random
    rng = random.Random(9)
    assert pow(2, 128, P) == (P - (1 << 32)) % P

    def emul(x, y):
        return ((x[0] * y[0] + 7 * x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)

    def acc_sum(ys, cs):   # the device accumulator: 64-bit words with explicit carries
        lo = hi = top = 0
        for y, c in zip(ys, cs):
            prod = y * c
            l, h = prod & ((1 << 64) - 1), prod >> 64
            lo2 = (lo + l) & ((1 << 64) - 1)
            c0 = 1 if lo2 < l else 0
            hi2 = (hi + h) & ((1 << 64) - 1)
            c1 = 1 if hi2 < h else 0
            hi3 = (hi2 + c0) & ((1 << 64) - 1)
            c2 = 1 if hi3 < c0 else 0
            lo, hi, top = lo2, hi3, top + c1 + c2
        assert top <= 8
        r = (lo + hi * (1 << 64)) % P
        return (r - (top << 32)) % P
    for n in (1, 7, 8, 9, 16, 85, 135, 256, 258):
        a = (rng.randrange(P), rng.randrange(P))
        ys = [rng.randrange(P) for _ in range(n)]
        ref = (0, 0)
        pw = (1, 0)
        for y in ys:
            ref = ((ref[0] + pw[0] * y) % P, (ref[1] + pw[1] * y) % P)
            pw = emul(pw, a)
        ap = [(1, 0)]
        for _ in range(8):
            ap.append(emul(ap[-1], a))
        g = (0, 0)
        rem = n & 7
        for v in range(n - 1, n - rem - 1, -1):
            g = emul(g, a)
            g = ((g[0] + ys[v]) % P, g[1])
        for j in range(n - rem - 8, -1, -8):
            ch = ys[j:j + 8]
            sa = (ch[0] + acc_sum(ch[1:], [ap[k][0] for k in range(1, 8)])) % P
            sb = acc_sum(ch[1:], [ap[k][1] for k in range(1, 8)])
            g = emul(g, ap[8])
            g = ((g[0] + sa) % P, (g[1] + sb) % P)
        assert g == ref, n
