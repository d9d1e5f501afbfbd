"""verifyProof restated literally in Python (tests/verifier_literal.py: transcript, Plonk
identity with every gate and the lookup argument, PoW, initial Merkle proofs, combineInitial,
folding steps with their Merkle / evaluation / arity checks, final polynomial, in the
reference's evaluation order) must give the oracle's status on every committed fixture and on a
random mutation campaign over real circuits: a second, independent verifier pinning the
oracle's statuses (and through test_gpu, libp2v's)."""
import gzip
import json
import os
import random

import pytest

import verifier_literal as VLIT
from support import GOLDEN, P, gen_circuit, mutate, oracle


def _cases():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        return json.load(f)["cases"]


def _rd(name):
    with gzip.open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("idx", range(len(_cases())))
def test_literal_verify_proof_matches_golden_status(idx):
    case = _cases()[idx]
    if case["circuit"].startswith("circuit_n16"):
        pytest.skip("degree_bits 16: too slow for the pure-Python verifier")
    common = json.loads(_rd(case["circuit"] + "_common.json.gz"))
    vkey = json.loads(_rd(case["circuit"] + "_vkey.json.gz"))
    pwpi = json.loads(_rd(case["name"] + "_proof.json.gz"))
    assert VLIT.verify_proof(common, vkey, pwpi) == case["status"], case["name"]


def _number_paths(d, path=()):
    if isinstance(d, dict):
        for k, v in d.items():
            yield from _number_paths(v, path + (k,))
    elif isinstance(d, list):
        for i, v in enumerate(d):
            yield from _number_paths(v, path + (i,))
    elif isinstance(d, int) and not isinstance(d, bool):
        yield path


@pytest.mark.parametrize("lk,mode", [(0, 1), (5, 1), (4, 2)])
def test_literal_verify_proof_mutation_campaign(lk, mode):
    """Each of 24 mutants changes one number anywhere in a valid real-circuit proof (openings,
    caps, leaves, siblings, step evaluations, final polynomial, PoW witness, public inputs):
    the literal verifier's status equals the oracle's, and the campaign reaches several outcome
    classes."""
    gc = gen_circuit(6, 4, lk, 1, 28, 16, 0, mode)
    base = gc.proof(1, 1)
    common, vkey = json.loads(gc.common), json.loads(gc.vkey)
    paths = list(_number_paths(json.loads(base)))
    rnd = random.Random(1000 + 10 * lk + mode)
    seen = set()
    O = oracle()
    for _ in range(24):
        path = rnd.choice(paths)

        def f(d, path=path):
            x = d
            for k in path[:-1]:
                x = x[k]
            x[path[-1]] = (x[path[-1]] + 1 + rnd.randrange(1 << 20)) % P
        pj = mutate(base, f)
        want = O.verify_json(gc.common, gc.vkey, pj)
        assert VLIT.verify_proof(common, vkey, json.loads(pj)) == want, path
        seen.add(want)
    assert VLIT.verify_proof(common, vkey, json.loads(base)) == 1
    assert len(seen) >= 3, seen
