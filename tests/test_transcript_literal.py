"""A second, independent restatement of the Fiat-Shamir transcript, checked against the oracle.

The oracle (oracle/oracle.c) and the GPU kernels share one author's reading of the reference.
This file is a literal Python transliteration of the transcript, written clause by clause
from the Haskell and sharing no code with either. The only shared piece is the Poseidon
permutation, taken from the oracle and pinned by the reference's KAT (Hash/Poseidon.hs:27-35).
It re-derives every challenge of the golden fixtures straight from their JSON and requires the
oracle's trace words to match:

- public-input hash
- betas, gammas, alphas
- lookup deltas
- zeta
- FRI alpha and betas
- PoW response
- query indices

test_gpu pins the GPU trace to the oracle word for word, so this check covers the device
transcript as well. Pure Python loops, small cases only; CPU suite."""
import gzip
import json
import os

import pytest

from support import GOLDEN, P, oracle

RATE = 8


def F(x):
    """JSON numbers are Integers reduced mod p (Algebra/Goldilocks.hs:101-102)."""
    return int(x) % P


def permutation(state):
    return oracle().permute(list(state))


# ---- Hash/Sponge.hs:26-31: overwrite mode, no padding, [] -> zero digest
def sponge(xs):
    state = [0] * 12
    while xs:
        this, xs = xs[:8], xs[8:]
        state = permutation(this + state[len(this):])
    return state[:4]


# ---- Challenge/Pure.hs:27-107.  A mode is ("A", old, inp) or ("S", old, out).
def overwrite(new, old):
    return new + old[len(new):]


def duplex(inp, old):
    return permutation(overwrite(inp, old))


def extract(state):
    return list(reversed(state[:RATE]))


def fresh_squeezing(new):
    return ("S", new, extract(new))


def absorb_felt(x, mode):
    if mode[0] == "S":
        return absorb_felt(x, ("A", mode[1], []))
    _, old, inp = mode
    if len(inp) < RATE:
        return ("A", old, inp + [x])
    return absorb_felt(x, ("A", duplex(inp, old), []))


def squeeze_felt(mode):
    kind, old, lst = mode
    if kind == "S":
        if not lst:
            return squeeze_felt(fresh_squeezing(permutation(old)))
        return lst[0], ("S", old, lst[1:])
    if not lst:
        return squeeze_felt(fresh_squeezing(permutation(old)))
    return squeeze_felt(fresh_squeezing(duplex(lst, old)))


class Duplex:
    def __init__(self):
        self.mode = ("A", [0] * 12, [])           # zeroState, no domain separator

    def absorb(self, xs):                         # instance Absorb [a]: left to right
        for x in xs:
            self.mode = absorb_felt(x, self.mode)

    def squeeze(self):
        x, self.mode = squeeze_felt(self.mode)
        return x

    def squeeze_n(self, n):
        return [self.squeeze() for _ in range(n)]

    def squeeze_ext(self):                        # instance Squeeze GoldilocksExt: (re, im)
        return [self.squeeze(), self.squeeze()]


def cap(c):
    """instance Absorb MerkleCap / Digest: the digests' elements in order."""
    return [F(x) for d in c for x in d["elements"]]


def ext_list(xs):
    """instance Absorb FExt: [re, im]."""
    return [F(v) for e in xs for v in e]


def proof_challenges(common, vkey, pwpi):
    """Challenge/Verifier.hs:58-103 followed by Challenge/FRI.hs:65-104."""
    cfg = common["config"]
    r = cfg["num_challenges"]
    has_lookup = common["num_lookup_polys"] > 0
    proof = pwpi["proof"]
    pi_hash = sponge([F(x) for x in pwpi["public_inputs"]])
    d = Duplex()
    d.absorb([F(x) for x in vkey["circuit_digest"]["elements"]])
    d.absorb(pi_hash)
    d.absorb(cap(proof["wires_cap"]))
    betas = d.squeeze_n(r)
    gammas = d.squeeze_n(r)
    deltas = []
    if has_lookup:
        deltas = betas + gammas + d.squeeze_n(2 * r)   # mkLookupDeltaList: chunks of 4
    d.absorb(cap(proof["plonk_zs_partial_products_cap"]))
    alphas = d.squeeze_n(r)
    d.absorb(cap(proof["quotient_polys_cap"]))
    zeta = d.squeeze_ext()
    # friChallenges, Challenge/FRI.hs:65-104; toFriOpenings order :46-61
    o = proof["openings"]
    batch_this = sum((o[k] for k in ("constants", "plonk_sigmas", "wires", "plonk_zs", "partial_products",
                                      "quotient_polys", "lookup_zs")), [])
    batch_next = o["plonk_zs_next"] + o["lookup_zs_next"]
    d.absorb(ext_list(batch_this))
    d.absorb(ext_list(batch_next))
    fri_alpha = d.squeeze_ext()
    fp = proof["opening_proof"]
    fri_betas = []
    for c in fp["commit_phase_merkle_caps"]:
        d.absorb(cap(c))
        fri_betas += d.squeeze_ext()
    d.absorb(ext_list(fp["final_poly"]["coeffs"]))
    d.absorb([F(fp["pow_witness"])])
    pow_response = d.squeeze()
    lde_size = 1 << (common["fri_params"]["degree_bits"] + cfg["fri_config"]["rate_bits"])
    qidx = [x % lde_size for x in d.squeeze_n(cfg["fri_config"]["num_query_rounds"])]
    return {"pi_hash": pi_hash, "betas": betas, "gammas": gammas, "alphas": alphas, "deltas": deltas,
            "zeta": zeta, "fri_alpha": fri_alpha, "fri_betas": fri_betas, "pow_response": [pow_response],
            "qidx": qidx}


def _fixtures():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        cases = json.load(f)["cases"]

    def rd(name):
        with gzip.open(os.path.join(GOLDEN, name), "rb") as f:
            return f.read()
    return cases, rd


def test_sponge_of_nothing_is_zero_digest():
    assert sponge([]) == [0, 0, 0, 0]            # Hash/Sponge.hs:28, #PI = 0 -> pi_hash = 0^4


@pytest.mark.parametrize("idx", range(len(_fixtures()[0])))
def test_literal_transcript_matches_oracle_trace(idx):
    cases, rd = _fixtures()
    case = cases[idx]
    common_b, vkey_b = rd(case["circuit"] + "_common.json.gz"), rd(case["circuit"] + "_vkey.json.gz")
    proof_b = rd(case["name"] + "_proof.json.gz")
    common, vkey, pwpi = json.loads(common_b), json.loads(vkey_b), json.loads(proof_b)
    ch = proof_challenges(common, vkey, pwpi)
    _, tr = oracle().verify_json(common_b, vkey_b, proof_b, trace=True)
    tr = [int(x) for x in tr]
    r = common["config"]["num_challenges"]
    S = len(pwpi["proof"]["opening_proof"]["commit_phase_merkle_caps"])
    Q = common["config"]["fri_config"]["num_query_rounds"]
    # trace layout: include/p2v.h (off_pi_hash .. off_query_idx)
    k = 0
    got = {}
    for name, n in (("pi_hash", 4), ("betas", r), ("gammas", r), ("alphas", r), ("deltas", 4 * r), ("zeta", 2),
                    ("fri_alpha", 2), ("fri_betas", 2 * S), ("pow_response", 1), ("qidx", Q)):
        got[name] = tr[k:k + n]
        k += n
    if not ch["deltas"]:
        ch["deltas"] = [0] * (4 * r)                # zero when the circuit has no lookups
    for name in got:
        assert got[name] == ch[name], (case["name"], name)
