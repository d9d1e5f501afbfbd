"""Opt-in plonky2 conventions the reference does not implement (SURVEY.md §8f row 4;
include/p2v.h P2V_EXT_*): FRI steps from fri_params.reduction_arity_bits (MinSize), salted
leaves under `hiding`, hash_or_noop leaves.  Parity unpinned: the reference rejects all of these
(MinSize is an `error` at Plonk/FRI.hs:342, salted leaves fail buildListOracle at :74, leaves are
always sponged at Hash/Merkle.hs:27-28), so the checks are (a) the generator's valid proofs accept
and its malicious modes reject under the flags, in the oracle; (b) with the flags off every path
keeps the reference's behaviour; (c) the words path packs exactly as the JSON path."""
import numpy as np
import pytest

from support import gen_circuit, oracle, p2v_module

CONFIGS = [  # (degree_bits, generator mode, ext, arities)
    (6, 1, 7, (3, 2)), (8, 1, 5, (1, 1, 1, 1)), (6, 2, 6, (3, 1)), (8, 1, 7, (3, 2, 1, 1)),
    (6, 0, 7, (2, 2, 1)), (6, 1, 4, (1, 1, 1)), (6, 1, 1, (2, 2)),
]


@pytest.mark.parametrize("nb,mode,ext,arities", CONFIGS)
def test_oracle_accepts_and_rejects_under_ext(nb, mode, ext, arities):
    gc = gen_circuit(nb, 4, 0, 1, 28, 8, 0, mode, ext, arities)
    O = oracle()
    assert O.verify_json(gc.common, gc.vkey, gc.proof(1, 1), ext=ext) == 1
    assert O.verify_json(gc.common, gc.vkey, gc.proof(2, 2), ext=ext) == 1
    # malicious modes: corrupted first layer (step eval), final polynomial, quotient opening
    assert [O.verify_json(gc.common, gc.vkey, gc.proof(1, 3, flags=f), ext=ext) for f in (1, 2, 4)] == [-3, 0, 0]


def test_reference_semantics_without_ext():
    """ext = 0 is the reference: MinSize is a circuit error, salted leaves a shape error, and a
    hash_or_noop tree fails the step Merkle check (the reference sponges every leaf)."""
    p2v = p2v_module()
    O = oracle()
    gc = gen_circuit(6, 4, 0, 1, 28, 8, 0, 1, 1, (2, 2))     # MinSize
    with pytest.raises(p2v.P2VError) as e:
        p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    assert e.value.code == p2v.E_CIRCUIT
    assert O.verify_json(gc.common, gc.vkey, gc.proof(1, 1)) == -6
    gc = gen_circuit(6, 4, 0, 1, 28, 8, 0, 2, 2, (3, 1))     # hiding, Fixed strategy
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    assert vk.info.leaf_widths == vk.info.oracle_widths
    with pytest.raises(p2v.P2VError) as e:
        vk.pack(gc.proof(1, 1))
    assert e.value.code == p2v.E_SHAPE
    assert O.verify_json(gc.common, gc.vkey, gc.proof(1, 1)) == -5
    gc = gen_circuit(6, 4, 0, 1, 28, 8, 0, 1, 4, (1, 1, 1))  # hash_or_noop, arity-2 steps, Fixed
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    vk.pack(gc.proof(1, 1))                                    # same shapes
    assert O.verify_json(gc.common, gc.vkey, gc.proof(1, 1)) == -2   # step leaves of 4 elements differ
    assert O.verify_json(gc.common, gc.vkey, gc.proof(1, 1), ext=4) == 1


@pytest.mark.parametrize("nb,mode,ext,arities", CONFIGS[:4])
def test_ext_layout_and_words_path(nb, mode, ext, arities):
    p2v = p2v_module()
    gc = gen_circuit(nb, 4, 0, 1, 28, 8, 0, mode, ext, arities)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, ext)
    inf = vk.info
    assert inf.ext == ext and inf.step_arity_bits == tuple(arities)
    salt = 4 if ext & p2v.EXT_HIDING else 0
    assert inf.leaf_widths == (inf.oracle_widths[0],) + tuple(w + salt for w in inf.oracle_widths[1:])
    assert inf.final_poly_len == 1 << (nb - sum(arities))
    vw = p2v.VerifierCircuitData.from_words(p2v.circuit_words(gc.common, gc.vkey), ext)
    assert vw.info == inf
    pr = gc.proof(1, 1)
    assert np.array_equal(vk.pack(pr), vw.pack_words(p2v.proof_words(pr)))


def test_ext_flag_validation():
    p2v = p2v_module()
    gc = gen_circuit(6, 4, 0, 1, 28, 8)
    with pytest.raises(p2v.P2VError) as e:
        p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, 8)
    assert e.value.code == p2v.E_ARG
    # plain circuits are unchanged by the flags (ConstantArityBits expands to the params' list,
    # no hiding, no leaf of <= 4 elements)
    a = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    b = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, p2v.EXT_PLONKY2)
    assert a.info.proof_words == b.info.proof_words and a.info.step_arity_bits == b.info.step_arity_bits
    pr = gc.proof(1, 1)
    assert np.array_equal(a.pack(pr), b.pack(pr))
    assert oracle().verify_json(gc.common, gc.vkey, pr, ext=p2v.EXT_PLONKY2) == 1
