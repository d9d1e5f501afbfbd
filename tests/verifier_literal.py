"""A literal Python restatement of the whole of verifyProof (src/Plonk/Verifier.hs:56-65):
the transcript (test_transcript_literal.py), the Plonk identity (vanishing_literal.py) and,
here, checkFRIProof (src/Plonk/FRI.hs:358-407) with the Merkle checks (src/Hash/Merkle.hs)
and the reference's evaluation order, so that it returns the same status code libp2v and the
oracle report: 1 True, 0 False, -1..-4 the `error` the reference raises first.

Independent of the oracle (oracle/oracle.c), the kernels and the generator: it shares only the
KAT-pinned Poseidon permutation (through the oracle's or_poseidon) and the constant tables.
Test infrastructure only; pure Python, small circuits.

Evaluation order (laziness, StrictData in Plonk/FRI.hs):
- verifyProof = eqs_ok && fri_ok: the identity first, FRI only if it holds (:62);
- checkFRIProof = pow_ok && and oks: PoW first, then the query rounds in order (:370);
- in a round, forcing round_ok forces the final state of foldl' foldingStep, whose first step
  pattern-matches the initial state: its strict upstream value forces combineInitial, whose
  MkOracles pattern forces checkInitialTreeProofs (initial Merkle proofs, -1) before anything
  else; then each step's guards in order: Merkle (-2), evaluation (-3), arity (-4); finally the
  final polynomial comparison (False)."""
from __future__ import annotations

import vanishing_literal as VL
from test_transcript_literal import (F, MUL_GEN, P, ROOTS, eadd, emul, epow, esub, escale, fold_coset, fpow,
                                     proof_challenges, reduce_with_powers, rev_bits, sponge, permutation, einv)


# ---- Hash/Merkle.hs
def compress(x, y):                                        # :21-23
    return permutation(list(x) + list(y) + [0, 0, 0, 0])[:4]


def check_merkle_proof(cap, idx, leaf, siblings):          # :27-42
    cur = sponge(list(leaf))                               # reconstructMerkleRoot: sponge of the leaf
    for sib in siblings:
        cur = compress(cur, sib) if idx % 2 == 0 else compress(sib, cur)
        idx >>= 1
    return cap[idx] == cur                                 # cap_roots !! rootidx


class Raise(Exception):
    """the reference's `error` (the status libp2v reports for it)"""

    def __init__(self, status):
        self.status = status


def digests(c):
    return [[F(x) for x in d["elements"]] for d in c]


def expand_reduction_strategy(degree_logn, strategy):      # Plonk/FRI.hs:337-354
    if "ConstantArityBits" in strategy:
        a, fbits = strategy["ConstantArityBits"]
        out, logn = [], degree_logn
        while logn > fbits:
            out.append(a)
            logn -= a
        return out
    if "Fixed" in strategy:
        return list(strategy["Fixed"])
    raise Raise(-6)                                         # "reduction strategy not implemented"


def check_fri_proof(common, vkey, pwpi, ch):
    """checkFRIProof, Plonk/FRI.hs:358-407: True / False, or Raise(status)."""
    cfg = common["config"]
    fc = cfg["fri_config"]
    r = cfg["num_challenges"]
    proof = pwpi["proof"]
    fp = proof["opening_proof"]
    # pow_ok (:212-216): the top pow_bits bits of the canonical response are zero
    bits = fc["proof_of_work_bits"]
    mask = ((1 << bits) - 1) << (64 - bits) if bits else 0
    if ch["pow_response"][0] & mask:
        return False
    # toMerkleOracles (:87-97) with validateMerkleCapLength
    caps = [digests(vkey["constants_sigmas_cap"]), digests(proof["wires_cap"]),
            digests(proof["plonk_zs_partial_products_cap"]), digests(proof["quotient_polys_cap"])]
    for c in caps:
        if len(c) != 1 << fc["cap_height"]:
            raise Raise(-5)
    widths = [common["num_constants"] + cfg["num_routed_wires"], cfg["num_wires"],
              r * (1 + common["num_partial_products"] + common["num_lookup_polys"]), r * common["quotient_degree_factor"]]
    o = proof["openings"]
    ext = lambda xs: [(F(a), F(b)) for a, b in xs]   # noqa: E731
    alpha = tuple(ch["fri_alpha"])
    zeta = tuple(ch["zeta"])
    y0 = reduce_with_powers(alpha, ext(sum((o[k] for k in ("constants", "plonk_sigmas", "wires", "plonk_zs",
                                                          "partial_products", "quotient_polys", "lookup_zs")), [])))
    y1 = reduce_with_powers(alpha, ext(o["plonk_zs_next"] + o["lookup_zs_next"]))
    logn = common["fri_params"]["degree_bits"]
    logn_lde = logn + fc["rate_bits"]
    arities = expand_reduction_strategy(logn, fc["reduction_strategy"])
    betas = [tuple(ch["fri_betas"][2 * i:2 * i + 2]) for i in range(len(ch["fri_betas"]) // 2)]
    step_caps = [digests(c) for c in fp["commit_phase_merkle_caps"]]
    final_coeffs = ext(fp["final_poly"]["coeffs"])
    qdf = common["quotient_degree_factor"]
    npp = -(-cfg["num_routed_wires"] // qdf)
    rounds = fp["query_round_proofs"]
    if len(rounds) != len(ch["qidx"]):
        raise Raise(-5)                                   # safeZipWith
    for idx, rnd in zip(ch["qidx"], rounds):
        # checkInitialTreeProofs (:105-117)
        ep = rnd["initial_trees_proof"]["evals_proofs"]
        if len(ep) != 4:
            raise Raise(-5)
        for cap, (leaf, mp) in zip(caps, ep):
            if not check_merkle_proof(cap, idx, [F(x) for x in leaf], digests(mp["siblings"])):
                raise Raise(-1)
        leaves = [[F(x) for x in lp[0]] for lp in ep]
        if [len(x) for x in leaves] != widths:            # buildListOracle
            raise Raise(-5)
        consts, wires, pp_lookup, quot = leaves
        if r * (npp + common["num_lookup_polys"]) != len(pp_lookup):   # combineInitial sanityCheck
            raise Raise(-6)
        pp, lookup = pp_lookup[:r * npp], pp_lookup[r * npp:]
        first = consts + wires + pp + quot + lookup        # :177-185
        second = pp[:r] + lookup
        g0 = reduce_with_powers(alpha, [(x, 0) for x in first])
        g1 = reduce_with_powers(alpha, [(x, 0) for x in second])
        omega, eta = ROOTS[logn], ROOTS[logn_lde]
        point_x = (MUL_GEN * pow(eta, rev_bits(logn_lde, idx), P) % P, 0)
        one = emul(esub(g0, y0), einv(esub(point_x, zeta)))
        two = emul(esub(g1, y1), einv(esub(point_x, escale(omega, zeta))))
        cur = eadd(emul(epow(alpha, len(second)), one), two)
        # foldl' foldingStep (:306-323) over safeZipWith4 steps betas caps query steps
        steps = rnd["steps"]
        if not (len(arities) == len(betas) == len(step_caps) == len(steps)):
            raise Raise(-5)
        shift, size, qi = MUL_GEN, logn_lde, idx
        for a, beta, cap, st in zip(arities, betas, step_caps, steps):
            evals = ext(st["evals"])
            new_qi = qi >> a
            flat = [v for e in evals for v in e]            # flattenExt
            if not check_merkle_proof(cap, new_qi, flat, digests(st["merkle_proof"]["siblings"])):
                raise Raise(-2)
            arity = 1 << a
            if qi % arity >= len(evals):
                raise Raise(-5)                              # (!!): index too large
            if evals[qi % arity] != cur:
                raise Raise(-3)
            if len(evals) == 0 or (len(evals) & (len(evals) - 1)) or len(evals).bit_length() - 1 != a:
                raise Raise(-4)                              # arityCheckOK (safeLog2)
            start = rev_bits(size, (qi >> a) << a)          # prepareCoset (:248-259)
            offset = shift * fpow(ROOTS[size], start) % P
            xs = [evals[rev_bits(a, i)] for i in range(arity)]
            cur = fold_coset(beta, a, offset, xs)
            shift = fpow(shift, arity)
            size, qi = size - a, new_qi
        x_final = shift * fpow(ROOTS[size], rev_bits(size, qi)) % P   # folding_query_loc
        val, xp = (0, 0), 1
        for c in final_coeffs:                              # evalPolynomialAt
            val = eadd(val, escale(xp, c))
            xp = xp * x_final % P
        if val != cur:
            return False
    return True


def verify_proof(common, vkey, pwpi):
    """verifyProof (Plonk/Verifier.hs:56-65) as a status code: 1 / 0 / the reference's error."""
    try:
        ch = proof_challenges(common, vkey, pwpi)
        comb, _ = VL.eval_combined_plonk_constraints(common, pwpi, ch, sponge)
        nn = 1 << common["fri_params"]["degree_bits"]
        zn1 = esub(epow(tuple(ch["zeta"]), nn), (1, 0))
        qdf = common["quotient_degree_factor"]
        qpolys = [(F(a), F(b)) for a, b in pwpi["proof"]["openings"]["quotient_polys"]]
        qs = [qpolys[i:i + qdf] for i in range(0, len(qpolys), qdf)]   # partition maxdeg
        zeta_n = epow(tuple(ch["zeta"]), nn)
        quot = []
        for chunk in qs:                                    # Verifier.hs:43-49
            acc = (0, 0)
            for x in reversed(chunk):
                acc = eadd(x, emul(zeta_n, acc))
            quot.append(acc)
        if len(quot) != len(comb):
            raise Raise(-5)                                 # safeZip
        if not all(emul(q, zn1) == c for q, c in zip(quot, comb)):
            return 0
        return 1 if check_fri_proof(common, vkey, pwpi, ch) else 0
    except Raise as e:
        return e.status
