"""A literal Python restatement of the Plonk identity's full combined value C_i(zeta):
the gate constraint programs of all 16 gate kinds, the gate selector polynomials, the
vertical gate sum, the lookup argument, the permutation argument and the alpha-combination.

Written clause by clause from the reference (file:line below), independently of the
oracle (oracle/oracle.c), the GPU kernels (csrc/vanish.hip) and the proof generator
(csrc/gen/gates.hpp, gen.cpp).  Shared with them: only the Poseidon constant tables, read
as data from oracle/poseidon_constants.h (generated from Hash/Constants.hs; the round
constants are pinned by the KAT), and the transcript restatement of
test_transcript_literal.py.  Test infrastructure only; pure Python, small cases.

The reference builds each gate's constraints as a symbolic straight-line program over
`Expr` (Gate/Computation.hs:117-129) and evaluates it over F^2 (:157-211).  Here each
gate is evaluated directly over F^2 values with the same operations in the same order;
`wireExt i` is the "doubly extended" element Ext (w_i, w_{i+1}) whose arithmetic is
GoldilocksExt.hs:54-61 instantiated at F^2 (so the 7 in the product is the literal 7).
"""
from __future__ import annotations

import os
import re

from test_transcript_literal import (F, P, chunks, eadd, einv, emul, epow, escale, esub, eval_lagrange0,
                                     eprod, ROOTS)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ZERO, ONE = (0, 0), (1, 0)


def fb(x):                                   # fromBase
    return (x % P, 0)


def eneg(x):
    return esub(ZERO, x)


def esum(xs):
    acc = ZERO
    for x in xs:
        acc = eadd(acc, x)
    return acc


# ---- Ext (FExt): GoldilocksExt.hs:54-71 over the F^2 "Expr" values of Gate/Vars.hs:56-57
def xadd(u, v):
    return (eadd(u[0], v[0]), eadd(u[1], v[1]))


def xsub(u, v):
    return (esub(u[0], v[0]), esub(u[1], v[1]))


def xmul(u, v):                              # (r1 r2 + 7 i1 i2, r1 i2 + r2 i1)
    (r1, i1), (r2, i2) = u, v
    return (eadd(emul(r1, r2), emul(fb(7), emul(i1, i2))), eadd(emul(r1, i2), emul(r2, i1)))


def xscale(s, u):                            # scaleExt
    return (emul(s, u[0]), emul(s, u[1]))


def xbase(x):                                # fromBase
    return (x, ZERO)


# ---- Poseidon constants (Hash/Constants.hs:19-208), as data
def _poseidon_tables():
    text = open(os.path.join(ROOT, "oracle", "poseidon_constants.h")).read()
    out = {}
    for name, body in re.findall(r"static const uint64_t OR_(\w+)\[\d+\] = \{(.*?)\};", text, re.S):
        out[name] = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", body)]
    return out


_PT = _poseidon_tables()


def mds_coeff(i, j):                         # Constants.hs:24-25
    return _PT["MDS_CIRC"][(j - i) % 12] + (_PT["MDS_DIAG"][i] if i == j else 0)


def partial_mds_coeff(i, j):                 # Constants.hs:112-113: INITIAL_MATRIX ! (j, i)
    return _PT["FAST_PARTIAL_ROUND_INITIAL_MATRIX"][11 * j + i]


def round_constants(r):
    return _PT["ALL_ROUND_CONSTANTS"][12 * r:12 * r + 12]


# ---- Gate/Parser.hs:107-242: the Rust Debug strings
def parse_gate(s):
    name = re.match(r"\s*(\w+)", s).group(1)
    ints = {k: int(v) for k, v in re.findall(r"(\w+): (-?\d+)(?=[,} ])", s)}
    g = {"name": name, "s": s}
    if name == "BaseSumGate":                       # "BaseSumGate { num_limbs: 63 } + Base: 2"
        g["num_limbs"] = ints["num_limbs"]
        g["base"] = int(re.search(r"Base: (\d+)", s).group(1))
    elif name == "CosetInterpolationGate":
        g.update(subgroup_bits=ints["subgroup_bits"], degree=ints["degree"])
        g["weights"] = [int(x) % P for x in re.search(r"barycentric_weights: \[([^\]]*)\]", s).group(1).split(",")]
    elif name in ("PoseidonGate", "PoseidonMdsGate"):
        g["width"] = int(re.search(r"<WIDTH=(\d+)>", s).group(1))
    else:
        g.update(ints)
    return g


# ---- Gate/Constraints.hs:40-128 and Gate/Custom/*.hs, evaluated at one opening set
class Vars:
    """EvaluationVars (Gate/Computation.hs:177-184): F^2 values of the row."""

    def __init__(self, constants, wires, pi_hash):
        self.c, self.w, self.h = constants, wires, pi_hash

    def wire(self, i):
        return self.w[i]

    def cnst(self, i):
        return self.c[i]

    def hash(self, i):
        return fb(self.h[i])

    def wire_ext(self, i):
        return (self.w[i], self.w[i + 1])


def sbox(x):                                  # Custom/Poseidon.hs:29-36
    x2 = emul(x, x)
    x3 = emul(x, x2)
    x4 = emul(x2, x2)
    return emul(x3, x4)


def poseidon_gate(v):                          # Custom/Poseidon.hs:63-150
    out = []
    inp = v.wire
    swap = v.wire(24)
    delta = lambda i: v.wire(25 + i)
    out.append(emul(swap, esub(swap, ONE)))
    out += [esub(emul(swap, esub(inp(i + 4), inp(i))), delta(i)) for i in range(4)]
    state = [eadd(inp(i), delta(i)) for i in range(4)] + [esub(inp(i), delta(i - 4)) for i in range(4, 8)] + \
            [inp(i) for i in range(8, 12)]

    def mds(st):
        return [esum(emul(fb(mds_coeff(i, j)), x) for j, x in enumerate(st)) for i in range(12)]

    def plus_rc(r, st):
        return [eadd(x, fb(c)) for x, c in zip(st, round_constants(r))]
    for r in range(4):
        s2 = plus_rc(r, state)
        if r == 0:
            s3 = s2
        else:
            sin = [v.wire(29 + 12 * (r - 1) + i) for i in range(12)]
            out += [esub(s2[i], sin[i]) for i in range(12)]
            s3 = sin
        state = mds([sbox(x) for x in s3])
    state = [eadd(x, fb(c)) for x, c in zip(state, _PT["FAST_PARTIAL_FIRST_ROUND_CONSTANT"])]
    first, rest = state[0], state[1:]
    state = [first] + [esum(emul(fb(partial_mds_coeff(i, j)), x) for j, x in enumerate(rest)) for i in range(11)]
    for r in range(22):
        sin = v.wire(29 + 36 + r)
        out.append(esub(state[0], sin))
        y = sbox(sin)
        z = eadd(y, fb(_PT["FAST_PARTIAL_ROUND_CONSTANTS"][r])) if r < 21 else y
        s2 = [z] + state[1:]
        cs = [mds_coeff(0, 0)] + _PT["FAST_PARTIAL_ROUND_W_HATS"][11 * r:11 * r + 11]   # mdsFastPartial
        d = esum(emul(e, fb(c)) for e, c in zip(s2, cs))
        vs = _PT["FAST_PARTIAL_ROUND_VS"][11 * r:11 * r + 11]
        state = [d] + [eadd(x, emul(s2[0], fb(t))) for x, t in zip(s2[1:], vs)]
    for r in range(4):
        s2 = plus_rc(r + 26, state)
        sin = [v.wire(29 + 36 + 22 + 12 * r + i) for i in range(12)]
        out += [esub(s2[i], sin[i]) for i in range(12)]
        state = mds([sbox(x) for x in sin])
    out += [esub(state[i], v.wire(i + 12)) for i in range(12)]
    return out


def coset_interpolation_gate(g, v):            # Custom/CosetInterp.hs:51-121
    n_points = 1 << g["subgroup_bits"]
    degree = g["degree"]
    n_int = (n_points - 2) // (degree - 1)
    gen = ROOTS[g["subgroup_bits"]]
    domain = [pow(gen, k, P) for k in range(n_points)]        # enumerateSubgroup
    values = [v.wire_ext(1 + 2 * k) for k in range(n_points)]
    coset_shift = v.wire(0)
    eval_loc = v.wire_ext(1 + 2 * n_points)
    eval_result = v.wire_ext(1 + 2 * n_points + 2)
    tmp_eval = lambda i: v.wire_ext(1 + 2 * (n_points + 2) + 2 * i)
    tmp_prod = lambda i: v.wire_ext(1 + 2 * (n_points + 2) + 2 * (n_int + i))
    shifted_loc = v.wire_ext(1 + 2 * (n_points + 2) + 4 * n_int)

    def chunk(xs):
        return [xs[:degree]] + chunks(degree - 1, xs[degree:])
    out = []
    d = xsub(eval_loc, xscale(coset_shift, shifted_loc))
    out += [d[0], d[1]]
    initials = [(xbase(ZERO), xbase(ONE))] + [(tmp_eval(i), tmp_prod(i)) for i in range(n_int)]
    stuff = []
    for ini, (dom, vals, ws) in zip(initials, zip(chunk(domain), chunk(values), chunk(g["weights"]))):
        ev, pr = ini
        for val, xi in zip([xscale(fb(w), x) for w, x in zip(ws, vals)], dom):
            term = xsub(shifted_loc, xbase(fb(xi)))
            ev, pr = xadd(xmul(term, ev), xmul(val, pr)), xmul(term, pr)
        stuff.append((ev, pr))
    for i, (ev, pr) in enumerate(stuff[:-1]):
        a, b = xsub(tmp_eval(i), ev), xsub(tmp_prod(i), pr)
        out += [a[0], a[1], b[0], b[1]]
    a = xsub(eval_result, stuff[-1][0])
    return out + [a[0], a[1]]


def random_access_gate(g, v):                   # Custom/RandomAccess.hs:47-88
    nb, copies, extra = g["bits"], g["num_copies"], g["num_extra_constants"]
    veclen = 1 << nb
    width = 2 + veclen
    bstart = width * copies + extra
    bits = lambda k, j: v.wire(bstart + k * nb + j)
    out = []
    for k in range(copies):
        out += [emul(bits(k, j), esub(bits(k, j), ONE)) for j in range(nb)]
        reconstr = ZERO
        for b in reversed([bits(k, j) for j in range(nb)]):   # foldr (\b acc -> 2 acc + b) 0
            reconstr = eadd(emul(fb(2), reconstr), b)
        out.append(esub(reconstr, v.wire(k * width)))
        vals = [v.wire(k * width + 2 + i) for i in range(veclen)]
        for j in range(nb):
            b = bits(k, j)
            vals = [eadd(x, emul(b, esub(y, x))) for x, y in zip(vals[0::2], vals[1::2])]
        out.append(esub(vals[0], v.wire(k * width + 1)))
    out += [esub(v.cnst(j), v.wire(copies * width + j)) for j in range(extra)]
    return out


def reducing_gate(n, v, ext):                   # Custom/Reducing.hs:28-60
    output, alpha, initial = v.wire_ext(0), v.wire_ext(2), v.wire_ext(4)
    coeff = (lambda i: v.wire_ext(6 + 2 * i)) if ext else (lambda i: xbase(v.wire(6 + i)))
    acc0 = 6 + 2 * n if ext else 6 + n
    accum = lambda i: v.wire_ext(acc0 + 2 * i) if i < n - 1 else output
    prev = lambda i: initial if i == 0 else accum(i - 1)
    out = []
    for i in range(n):
        d = xsub(xadd(xmul(prev(i), alpha), coeff(i)), accum(i))
        out += [d[0], d[1]]
    return out


def gate_constraints(g, v):
    """gateComputation (Gate/Constraints.hs:40-108), evaluated (runStraightLine)."""
    name, out = g["name"], []
    if name == "ArithmeticGate":                                   # :45-46
        for i in range(g["num_ops"]):
            j = 4 * i
            out.append(esub(esub(v.wire(j + 3), emul(emul(v.cnst(0), v.wire(j)), v.wire(j + 1))),
                            emul(v.cnst(1), v.wire(j + 2))))
    elif name == "ArithmeticExtensionGate":                        # :49-54
        c0, c1 = xbase(v.cnst(0)), xbase(v.cnst(1))
        for i in range(g["num_ops"]):
            j = 8 * i
            d = xsub(xsub(v.wire_ext(j + 6), xmul(xmul(c0, v.wire_ext(j)), v.wire_ext(j + 2))), xmul(c1, v.wire_ext(j + 4)))
            out += [d[0], d[1]]
    elif name == "BaseSumGate":                                    # :57-62
        nl, base = g["num_limbs"], g["base"]
        limb = lambda i: v.wire(i + 1)

        def go(k):
            return eadd(limb(k), emul(fb(base), go(k + 1))) if k < nl - 1 else limb(k)
        out.append(esub(go(0), v.wire(0)))
        out += [eprod([esub(limb(i), fb(k)) for k in range(base)]) for i in range(nl)]
    elif name == "CosetInterpolationGate":
        out = coset_interpolation_gate(g, v)
    elif name == "ConstantGate":                                   # :68-69
        out = [esub(v.cnst(i), v.wire(i)) for i in range(g["num_consts"])]
    elif name == "ExponentiationGate":                             # :114-128
        n = g["num_power_bits"]
        base, out_w = v.wire(0), v.wire(n + 1)
        tmp = lambda i: v.wire(n + 2 + i)
        cur_bit = lambda i: v.wire((n - 1 - i) + 1)
        for i in range(n):
            prev = ONE if i == 0 else emul(tmp(i - 1), tmp(i - 1))
            comp = emul(prev, eadd(emul(cur_bit(i), base), esub(ONE, cur_bit(i))))
            out.append(esub(comp, tmp(i)))
        out.append(esub(out_w, tmp(n - 1)))
    elif name in ("LookupGate", "LookupTableGate", "NoopGate"):   # :76-77, :85
        out = []
    elif name == "MulExtensionGate":                               # :80-83
        for i in range(g["num_ops"]):
            j = 6 * i
            d = xsub(v.wire_ext(j + 4), xmul(xmul(xbase(v.cnst(0)), v.wire_ext(j)), v.wire_ext(j + 2)))
            out += [d[0], d[1]]
    elif name == "PublicInputGate":                                # :88-89
        out = [esub(v.wire(i), v.hash(i)) for i in range(4)]
    elif name == "PoseidonGate":
        assert g["width"] == 12
        out = poseidon_gate(v)
    elif name == "PoseidonMdsGate":                                # Custom/Poseidon.hs:49-59
        assert g["width"] == 12
        for i in range(12):
            res = (ZERO, ZERO)
            for j in range(12):
                res = xadd(res, xscale(fb(mds_coeff(i, j)), v.wire_ext(2 * j)))
            d = xsub(v.wire_ext(2 * (i + 12)), res)
            out += [d[0], d[1]]
    elif name == "RandomAccessGate":
        out = random_access_gate(g, v)
    elif name == "ReducingGate":
        out = reducing_gate(g["num_coeffs"], v, False)
    elif name == "ReducingExtensionGate":
        out = reducing_gate(g["num_coeffs"], v, True)
    else:
        raise ValueError("gateConstraints: unknown gate " + name)   # :108
    return out


# ---- Gate/Selector.hs
def split_constant_columns(common, xs):                            # :31-72
    ngroups = len(common["selectors_info"]["groups"])
    nls = common["num_lookup_selectors"]
    nk = common["config"]["num_constants"]
    nluts = len(common["luts"])
    assert nls == (4 + nluts if nluts else 0)
    assert common["num_constants"] == ngroups + nls + nk
    assert len(xs) == ngroups + nls + nk
    return xs[:ngroups], xs[ngroups:ngroups + nls], xs[ngroups + nls:]


def eval_gate_selector_poly(sel_info, x, k):                       # :83-89
    grp = sel_info["groups"][sel_info["selector_indices"][k]]
    initial = esub(fb(2 ** 32 - 1), x) if len(sel_info["groups"]) > 1 else ONE
    return emul(initial, eprod([esub(fb(j), x) for j in range(grp["start"], grp["end"]) if j != k]))


def eval_gate_selectors(sel_info, xs):                             # :93-95
    return [eval_gate_selector_poly(sel_info, xs[grp], i) for i, grp in enumerate(sel_info["selector_indices"])]


# ---- Plonk/Lookups.hs:45-132
def remove1(xs):                                                   # Misc/Aux.hs:116-123
    return [xs[:i] + xs[i + 1:] for i in range(len(xs))]


def pairs(xs):                                                     # Misc/Aux.hs:76-79
    return list(zip(xs, xs[1:]))


def div_ceil(a, b):
    return -(-a // b)


def eval_lookup_equations(common, lkp_sels, o, deltas):
    cfg = common["config"]
    nlp = common["num_lookup_polys"]
    ext = lambda xs: [(F(a), F(b)) for a, b in xs]
    wires = ext(o["wires"])
    selector = lambda idx: lkp_sels[idx]       # TransSre 0, TransLdc 1, InitSre 2, LastLdc 3, StartEnd k: 4+k
    round_chunks = chunks(nlp, list(zip(ext(o["lookup_zs"]), ext(o["lookup_zs_next"]))))
    num_lu_slots = cfg["num_routed_wires"] // 2
    num_lut_slots = cfg["num_routed_wires"] // 3
    num_sldc_polys = nlp - 1
    lu_degree = common["quotient_degree_factor"] - 1
    lut_degree = div_ceil(num_lut_slots, num_sldc_polys)
    final = []
    assert len(deltas) == len(round_chunks)                       # safeZipWith
    for (A, B, lk_alpha, lk_delta), columns in zip(deltas, round_chunks):
        re_pair, sldc_pairs = columns[0], columns[1:]
        re, re_next = re_pair
        sldc = [p[0] for p in sldc_pairs]
        sldc_next = [p[1] for p in sldc_pairs]
        lu_combos = [eadd(inp, escale(A, out)) for inp, out in chunks(2, wires)[:num_lu_slots]]
        lut3 = [c for c in chunks(3, wires)[:num_lut_slots] if len(c) == 3]   # the [inp,out,mult] pattern
        lut_combos_A = [eadd(inp, escale(A, out)) for inp, out, _ in lut3]
        lut_combos_B = [eadd(inp, escale(B, out)) for inp, out, _ in lut3]
        mults = [wires[3 * i + 2] for i in range(num_lut_slots)]
        chunks_lu_combo = chunks(lu_degree, lu_combos)
        chunks_lut_combo = chunks(lut_degree, lut_combos_A)
        chunks_mults = chunks(lut_degree, mults)
        eq_last_sldc = emul(selector(3), sldc[-1])
        eq_ini_sum = emul(selector(2), sldc[0])
        eq_ini_re = emul(selector(2), re)
        eq_finals_re = []
        for k, table in enumerate(common["luts"]):
            lut = [(F(a), F(b)) for a, b in table]
            lut_nrows = div_ceil(len(lut), num_lut_slots)
            padded = (lut + [lut[0]] * (lut_nrows * num_lut_slots))[:lut_nrows * num_lut_slots]
            cur = 0
            for inp, out in padded:
                cur = (lk_delta * cur + (inp + B * out)) % P
            eq_finals_re.append(emul(selector(4 + k), esub(re, fb(cur))))
        cur_sum = re_next
        for elt in lut_combos_B:
            cur_sum = eadd(escale(lk_delta, cur_sum), elt)
        eq_re_trans = emul(selector(0), esub(re, cur_sum))
        prev_this = pairs([sldc_next[-1]] + sldc)
        eqs_sldc = []
        alpha = fb(lk_alpha)
        for (prev, this), (lu_c, lut_c, mu) in zip(prev_this, zip(chunks_lu_combo, chunks_lut_combo, chunks_mults)):
            lu_prod = eprod([esub(alpha, c) for c in lu_c])
            lut_prod = eprod([esub(alpha, c) for c in lut_c])
            lu_prods_i = [eprod([esub(alpha, c) for c in one_less]) for one_less in remove1(lu_c)]
            lut_prods_i = [emul(m, eprod([esub(alpha, c) for c in one_less])) for m, one_less in zip(mu, remove1(lut_c))]
            eq_ldc = emul(selector(1), eadd(emul(lu_prod, esub(this, prev)), esum(lu_prods_i)))
            eq_sum = emul(selector(0), esub(emul(lut_prod, esub(this, prev)), esum(lut_prods_i)))
            eqs_sldc += [eq_sum, eq_ldc]
        final += [eq_last_sldc, eq_ini_sum, eq_ini_re] + eq_finals_re + [eq_re_trans] + eqs_sldc
    return final


# ---- Plonk/Vanishing.hs:48-137
def long_zip_add(xs, ys):                                          # longZipWith 0 0 (+)
    n = max(len(xs), len(ys))
    xs = xs + [ZERO] * (n - len(xs))
    ys = ys + [ZERO] * (n - len(ys))
    return [eadd(a, b) for a, b in zip(xs, ys)]


def all_plonk_constraints(common, pwpi, ch, sponge):
    """evalAllPlonkConstraints: (terms, {"zs1", "pp", "lookup", "gates"} -> the sublists)."""
    cfg = common["config"]
    r, qdf = cfg["num_challenges"], common["quotient_degree_factor"]
    nn = 1 << common["fri_params"]["degree_bits"]
    o = pwpi["proof"]["openings"]
    ext = lambda xs: [(F(a), F(b)) for a, b in xs]
    zeta = tuple(ch["zeta"])
    gate_sels, lkp_sels, konst = split_constant_columns(common, ext(o["constants"]))
    pi_hash = sponge([F(x) for x in pwpi["public_inputs"]])
    v = Vars(konst, ext(o["wires"]), pi_hash)
    gates = [parse_gate(s) for s in common["gates"]]
    sel_values = eval_gate_selectors(common["selectors_info"], gate_sels)
    unfiltered = [gate_constraints(g, v) for g in gates]
    filtered = [[emul(s, c) for c in cons] for s, cons in zip(sel_values, unfiltered)]
    gate_terms = filtered[0]
    for f in filtered[1:]:                                         # foldl1 (longZipWith 0 0 (+))
        gate_terms = long_zip_add(gate_terms, f)
    zs, zs_next = ext(o["plonk_zs"]), ext(o["plonk_zs_next"])
    zs1 = [emul(eval_lagrange0(nn, zeta), esub(z, ONE)) for z in zs]
    wires, sigmas = ext(o["wires"]), ext(o["plonk_sigmas"])
    k_is = [F(k) for k in common["k_is"]]
    pp_checks = []
    for z, znext, beta, gamma, pp_chunk in zip(zs, zs_next, ch["betas"], ch["gammas"],
                                               chunks(common["num_partial_products"], ext(o["partial_products"]))):
        numers = chunks(qdf, [eadd(eadd(w, escale(beta * k % P, zeta)), fb(gamma)) for k, w in zip(k_is, wires)])
        denoms = chunks(qdf, [eadd(eadd(w, escale(beta, s)), fb(gamma)) for s, w in zip(sigmas, wires)])
        current = [z] + pp_chunk + [znext]
        for (prev, nxt), nu, de in zip(pairs(current), numers, denoms):
            pp_checks.append(esub(emul(prev, eprod(nu)), emul(nxt, eprod(de))))
    lookup_checks = []
    if common["luts"]:
        d = ch["deltas"]
        deltas = [tuple(d[i:i + 4]) for i in range(0, len(d), 4)]   # mkLookupDeltaList
        lookup_checks = eval_lookup_equations(common, lkp_sels, o, deltas)
    parts = {"zs1": zs1, "pp": pp_checks, "lookup": lookup_checks, "gates": gate_terms, "sel_values": sel_values,
             "unfiltered": unfiltered}
    return zs1 + pp_checks + lookup_checks + gate_terms, parts


def combine_with_powers_of_alpha(alpha, xs):                      # Vanishing.hs:54-56
    acc = ZERO
    for x in reversed(xs):
        acc = eadd(x, escale(alpha, acc))
    return acc


def eval_combined_plonk_constraints(common, pwpi, ch, sponge):   # Vanishing.hs:48-51
    terms, parts = all_plonk_constraints(common, pwpi, ch, sponge)
    return [combine_with_powers_of_alpha(a, terms) for a in ch["alphas"]], parts
