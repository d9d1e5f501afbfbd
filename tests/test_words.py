"""The typed-host boundary (include/p2v.h "word-encoded Types.hs values"): VerifierCircuitData
and ProofWithPublicInputs marshalled field by field into u64 words, as the Haskell shim
(bindings/haskell/Plonk/VerifierGPU.hs) writes them from decoded values, must give exactly what
the JSON entry points give: the same circuit shape and the same packed words, bit for bit, and
the same error classes (host only, no GPU)."""
import gzip
import json
import os

import numpy as np
import pytest

from support import GOLDEN, P, gen_circuit, mutate, p2v_module

CIRCUITS = [dict(degree_bits=6), dict(degree_bits=6, lookups=1), dict(degree_bits=8, lookups=2),
            dict(degree_bits=7, num_pis=17, queries=12, pow_bits=0), dict(degree_bits=6, mode=1),
            dict(degree_bits=6, mode=2), dict(degree_bits=6, ngroups=1)]


def _gc(kw):
    a = dict(degree_bits=6, num_pis=4, lookups=0, seed=1, queries=28, pow_bits=16, ngroups=0, mode=0)
    a.update(kw)
    return gen_circuit(**a)


@pytest.mark.parametrize("kw", CIRCUITS, ids=[str(k) for k in CIRCUITS])
def test_circuit_and_proof_words_equal_json_path(kw):
    p2v = p2v_module()
    gc = _gc(kw)
    vj = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    vw = p2v.VerifierCircuitData.from_words(p2v.circuit_words(gc.common, gc.vkey))
    assert vw.info == vj.info
    proofs = [gc.proof(1, 1), gc.proof(2, 3), gc.proof(1, 4, flags=1), gc.proof(1, 6, flags=4)]
    for pr in proofs:
        a = vj.pack(pr)
        assert np.array_equal(vw.pack_words(p2v.proof_words(pr)), a)   # words circuit, words proof
        assert np.array_equal(vj.pack_words(p2v.proof_words(pr)), a)   # JSON circuit, words proof
        assert np.array_equal(vw.pack(pr), a)                         # words circuit, JSON proof


def test_words_path_on_golden_fixtures():
    p2v = p2v_module()
    exp = json.load(open(os.path.join(GOLDEN, "expected.json")))["cases"]

    def rd(n):
        with gzip.open(os.path.join(GOLDEN, n), "rb") as f:
            return f.read()
    for c in exp:
        common, vkey = rd(c["circuit"] + "_common.json.gz"), rd(c["circuit"] + "_vkey.json.gz")
        vw = p2v.VerifierCircuitData.from_words(p2v.circuit_words(common, vkey))
        pr = rd(c["name"] + "_proof.json.gz")
        assert np.array_equal(vw.pack_words(p2v.proof_words(pr)), p2v.VerifierCircuitData.from_json(common, vkey).pack(pr))


def test_words_values_reduced_mod_p_and_errors():
    """F values >= p reduce like aeson's Integer (Goldilocks.hs:98-102); a wrong list length is
    a shape error, a truncated / bad-magic / trailing encoding a parse error, and circuit-level
    errors (unknown gate, MinSize, selector tally) surface at creation as from JSON."""
    p2v = p2v_module()
    gc = _gc({})
    cw = p2v.circuit_words(gc.common, gc.vkey)
    vw = p2v.VerifierCircuitData.from_words(cw)
    pr = mutate(gc.proof(1, 1), lambda d: d["public_inputs"].__setitem__(-1, 12345))
    pw = p2v.proof_words(pr)
    base = vw.pack_words(pw)
    big = pw.copy()
    big[-1] = np.uint64(12345 + P)                                 # last public input + p
    assert np.array_equal(vw.pack_words(big), base)
    for bad, code in ((pw[:-1], p2v.E_PARSE), (np.concatenate([pw, [np.uint64(0)]]), p2v.E_PARSE)):
        with pytest.raises(p2v.P2VError) as e:
            vw.pack_words(bad)
        assert e.value.code == code
    wrong = p2v.proof_words(mutate(pr, lambda d: d["public_inputs"].append(5)))
    with pytest.raises(p2v.P2VError) as e:
        vw.pack_words(wrong)
    assert e.value.code == p2v.E_SHAPE
    bad_magic = cw.copy()
    bad_magic[0] ^= np.uint64(1)
    with pytest.raises(p2v.P2VError) as e:
        p2v.VerifierCircuitData.from_words(bad_magic)
    assert e.value.code == p2v.E_PARSE
    c = json.loads(gc.common)
    for edit, code in ((lambda c: c["gates"].__setitem__(3, "FancyGate { x: 1 }"), p2v.E_CIRCUIT),
                       (lambda c: c["config"]["fri_config"].__setitem__("reduction_strategy", {"MinSize": None}), p2v.E_CIRCUIT),
                       (lambda c: c.__setitem__("num_constants", c["num_constants"] + 1), p2v.E_CIRCUIT)):
        cc = json.loads(gc.common)
        edit(cc)
        cj = json.dumps(cc).encode()
        with pytest.raises(p2v.P2VError) as ej:
            p2v.VerifierCircuitData.from_json(cj, gc.vkey)
        with pytest.raises(p2v.P2VError) as ew:
            p2v.VerifierCircuitData.from_words(p2v.circuit_words(cj, gc.vkey))
        assert ej.value.code == ew.value.code == code


def test_c_host_words_mode_equals_json_mode(tmp_path):
    """examples/p2v_verify.c (plain C over include/p2v.h): --words reads the word-encoded values
    (p2v_circuit_from_words + p2v_pack_proof_words), and its packed words (--dump) equal the
    JSON mode's for the same proofs; a malformed words file is a decode failure (exit 4)."""
    import subprocess
    p2v = p2v_module()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "plonky2-verifier_amd", "p2v_verify")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.join(root, "plonky2-verifier_amd"), "p2v_verify"])
    gc = _gc(dict(mode=1))
    (tmp_path / "c.json").write_bytes(gc.common)
    (tmp_path / "v.json").write_bytes(gc.vkey)
    p2v.circuit_words(gc.common, gc.vkey).tofile(tmp_path / "c.words")
    js, ws = [], []
    for i, pr in enumerate([gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 4, flags=1)]):
        (tmp_path / f"p{i}.json").write_bytes(pr)
        p2v.proof_words(pr).tofile(tmp_path / f"p{i}.words")
        js.append(str(tmp_path / f"p{i}.json"))
        ws.append(str(tmp_path / f"p{i}.words"))
    a = subprocess.run([exe, "--pack-only", "--dump", str(tmp_path / "a.bin"), str(tmp_path / "c.json"), str(tmp_path / "v.json")] + js,
                       capture_output=True, text=True)
    b = subprocess.run([exe, "--words", "--pack-only", "--dump", str(tmp_path / "b.bin"), str(tmp_path / "c.words")] + ws,
                       capture_output=True, text=True)
    assert a.returncode == 0 and b.returncode == 0, (a.stderr, b.stderr)
    da, db = np.fromfile(tmp_path / "a.bin", np.uint64), np.fromfile(tmp_path / "b.bin", np.uint64)
    assert da.size == 3 * p2v.VerifierCircuitData.from_json(gc.common, gc.vkey).info.proof_words
    assert np.array_equal(da, db)
    p2v.proof_words(gc.proof(1, 1))[:-3].tofile(tmp_path / "bad.words")
    assert subprocess.run([exe, "--words", "--pack-only", str(tmp_path / "c.words"), str(tmp_path / "bad.words")],
                          capture_output=True).returncode == 4
