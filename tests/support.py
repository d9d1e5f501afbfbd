"""Shared test helpers: ctypes wrappers for the ORACLE (CPU restatement, tests only) and
the synthetic proof generator, plus the product module (p2v) import."""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys
from functools import lru_cache

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "plonky2-verifier_amd")
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
GEN_SO = os.path.join(PKG, "libp2v_gen.so")
P2V_SO = os.path.join(PKG, "libp2v.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

if PKG not in sys.path:
    sys.path.insert(0, PKG)

P = 0xFFFFFFFF00000001
KAT_IN = list(range(12))
KAT_OUT = [0xd64e1e3efc5b8e9e, 0x53666633020aaa47, 0xd40285597c6a8825, 0x613a4f81e81231d2,
           0x414754bfebd051f0, 0xcb1f8980294a023f, 0x6eb2a9e4d54a9d0f, 0x1902bc3af467e056,
           0xf045d5eafdc6021f, 0xe4150f77caaa3be5, 0xc9bfd01d39b50cce, 0x5c0a27fcb0e1459b]   # Hash/Poseidon.hs:27-32


def ensure_built():
    """Build the oracle / generator / libp2v in-tree if missing (make; no network)."""
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if not os.path.exists(GEN_SO) or not os.path.exists(P2V_SO):
        subprocess.check_call(["make", "-s", "-j4", "-C", PKG])


# ----------------------------------------------------------------------------- oracle
class Oracle:
    """ORACLE — test infrastructure only (oracle/oracle.c)."""

    def __init__(self):
        ensure_built()
        L = ctypes.CDLL(ORACLE_SO)
        vp = ctypes.c_void_p
        L.or_circuit_load.restype = vp
        L.or_circuit_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.or_proof_load.restype = vp
        L.or_proof_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.or_circuit_free.argtypes = [vp]
        L.or_proof_free.argtypes = [vp]
        L.or_verify.argtypes = [vp, vp, vp, ctypes.c_int]
        L.or_trace_words.argtypes = [vp]
        L.or_last_error.restype = ctypes.c_char_p
        L.or_perm_count.restype = ctypes.c_longlong
        L.or_subgroup_gen.restype = ctypes.c_uint64
        L.or_fmul.restype = ctypes.c_uint64
        L.or_fmul.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_finv.restype = ctypes.c_uint64
        L.or_finv.argtypes = [ctypes.c_uint64]
        L.or_eval_gate.argtypes = [ctypes.c_char_p, vp, ctypes.c_int, vp, ctypes.c_int, vp, vp, ctypes.c_int]
        L.or_gate_kind.argtypes = [ctypes.c_char_p]
        L.or_verify_many.argtypes = [vp, ctypes.POINTER(vp), ctypes.c_long, vp, ctypes.c_int]
        L.or_verify_many.restype = ctypes.c_long
        L.or_circuit_set_ext.argtypes = [vp, ctypes.c_uint]
        self.L = L

    def circuit(self, common: bytes, vkey: bytes, ext: int = 0):
        """ext: the P2V_EXT_* conventions (include/p2v.h), 0 = the reference's."""
        h = self.L.or_circuit_load(common, len(common), vkey, len(vkey))
        if not h:
            raise ValueError(self.L.or_last_error().decode())
        self.L.or_circuit_set_ext(h, ext)
        return h

    def proof(self, text: bytes):
        h = self.L.or_proof_load(text, len(text))
        if not h:
            raise ValueError(self.L.or_last_error().decode())
        return h

    def verify(self, circ, proof, trace=False, full=True, unit_filters=False):
        if trace:
            tw = self.L.or_trace_words(circ)
            tr = np.zeros(tw, dtype=np.uint64)
            st = self.L.or_verify(circ, proof, tr.ctypes.data, (1 if full else 0) | (2 if unit_filters else 0))
            return st, tr
        return self.L.or_verify(circ, proof, None, 0)

    def verify_json(self, common: bytes, vkey: bytes, proof: bytes, trace=False, unit_filters=False, ext=0):
        c = self.circuit(common, vkey, ext)
        p = self.proof(proof)
        try:
            return self.verify(c, p, trace=trace, unit_filters=unit_filters)
        finally:
            self.L.or_proof_free(p)
            self.L.or_circuit_free(c)

    def permute(self, st):
        a = (ctypes.c_uint64 * 12)(*st)
        self.L.or_poseidon(a)
        return list(a)


@lru_cache(maxsize=1)
def oracle() -> Oracle:
    return Oracle()


# ----------------------------------------------------------------------------- generator
class Generator:
    """Synthetic valid-proof generator (csrc/gen/gen.cpp): degenerate circuit, real FRI prover."""

    def __init__(self):
        ensure_built()
        L = ctypes.CDLL(GEN_SO)
        vp = ctypes.c_void_p
        L.p2v_gen_circuit_new.restype = vp
        L.p2v_gen_circuit_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.p2v_gen_circuit_new2.restype = vp
        L.p2v_gen_circuit_new2.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int]
        L.p2v_gen_circuit_new3.restype = vp
        L.p2v_gen_circuit_new3.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_uint, vp, ctypes.c_int]
        L.p2v_gen_common_json.restype = ctypes.c_char_p
        L.p2v_gen_common_json.argtypes = [vp]
        L.p2v_gen_vkey_json.restype = ctypes.c_char_p
        L.p2v_gen_vkey_json.argtypes = [vp]
        L.p2v_gen_witness_new.restype = vp
        L.p2v_gen_witness_new.argtypes = [vp, ctypes.c_uint64]
        L.p2v_gen_witness_free.argtypes = [vp]
        L.p2v_gen_circuit_free.argtypes = [vp]
        L.p2v_gen_proof_json.restype = vp
        L.p2v_gen_proof_json.argtypes = [vp, vp, ctypes.c_uint64]
        L.p2v_gen_proof_json_flags.restype = vp
        L.p2v_gen_proof_json_flags.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint]
        L.p2v_gen_free_str.argtypes = [vp]
        L.p2v_gen_gate_row.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, vp, vp, vp]
        L.p2v_gen_num_gates.argtypes = [vp]
        L.p2v_gen_last_error.restype = ctypes.c_char_p
        self.L = L

    def circuit(self, degree_bits=12, num_pis=4, lookups=0, seed=1, queries=28, pow_bits=16, ngroups=0, mode=0, ext=0, arities=()):
        """mode 0: degenerate circuit (every gate filter 0), `ngroups` selector groups (0: 3);
        mode 1: real circuit over the recursion gate set; mode 2: real circuit, small gate set
        in one selector group.  ext / arities: the opt-in plonky2 conventions (P2V_EXT_*: 1 the
        `arities` as fri_params.reduction_arity_bits under MinSize, 2 hiding salts, 4
        hash_or_noop leaves; `arities` without 1: a Fixed strategy)."""
        arr = (ctypes.c_int * max(1, len(arities)))(*arities)
        h = self.L.p2v_gen_circuit_new3(degree_bits, num_pis, lookups, seed, queries, pow_bits, ngroups, mode, ext, arr, len(arities))
        if not h:
            raise RuntimeError(self.L.p2v_gen_last_error().decode())
        return GenCircuit(self, h)


class GenCircuit:
    def __init__(self, g: Generator, h):
        self.g, self.h = g, h
        self.common = g.L.p2v_gen_common_json(h)
        self.vkey = g.L.p2v_gen_vkey_json(h)
        self._wit = {}

    def witness(self, seed):
        if seed not in self._wit:
            w = self.g.L.p2v_gen_witness_new(self.h, seed)
            if not w:
                raise RuntimeError(self.g.L.p2v_gen_last_error().decode())
            self._wit[seed] = w
        return self._wit[seed]

    def gate_row(self, gate: int, seed: int, num_wires=135, num_consts=2):
        """(wires, consts, pih) of a witness row that satisfies gate `gate` (real modes)."""
        w = np.zeros(num_wires, np.uint64)
        k = np.zeros(num_consts, np.uint64)
        h = np.zeros(4, np.uint64)
        n = self.g.L.p2v_gen_gate_row(self.h, gate, seed, w.ctypes.data, k.ctypes.data, h.ctypes.data)
        if n < 0:
            raise RuntimeError(self.g.L.p2v_gen_last_error().decode())
        return w, k, h, n

    def proof(self, wseed=1, pseed=1, flags=0) -> bytes:
        w = self.witness(wseed)
        ptr = self.g.L.p2v_gen_proof_json_flags(self.h, w, pseed, flags)
        if not ptr:
            raise RuntimeError(self.g.L.p2v_gen_last_error().decode())
        s = ctypes.string_at(ptr)
        self.g.L.p2v_gen_free_str(ptr)
        return s


@lru_cache(maxsize=1)
def generator() -> Generator:
    return Generator()


@lru_cache(maxsize=16)
def gen_circuit(degree_bits=6, num_pis=4, lookups=0, seed=1, queries=28, pow_bits=16, ngroups=0, mode=0, ext=0, arities=()) -> GenCircuit:
    return generator().circuit(degree_bits, num_pis, lookups, seed, queries, pow_bits, ngroups, mode, ext, tuple(arities))


# ----------------------------------------------------------------------------- plonky2 bytes
def proof_bytes(proof_json: bytes, pi_prefix: bool = False) -> bytes:
    """plonky2's binary serialization of a ProofWithPublicInputs (Write::
    write_proof_with_public_inputs, restated here independently of the C++ reader in
    csrc/circuit.cpp): u64 LE words, caps without length, Merkle proofs as a u8 count then the
    hashes, circuit-sized vectors without length; public inputs raw, or after a u64 count."""
    import struct
    d = json.loads(proof_json)
    pr, out = d["proof"], bytearray()

    def f(x):
        out.extend(struct.pack("<Q", int(x) % 0xFFFFFFFF00000001))

    def cap(c):
        for h in c:
            for x in h["elements"]:
                f(x)

    def exts(v):
        for a, b in v:
            f(a)
            f(b)

    def mproof(sib):
        out.append(len(sib["siblings"]))
        cap(sib["siblings"])
    cap(pr["wires_cap"])
    cap(pr["plonk_zs_partial_products_cap"])
    cap(pr["quotient_polys_cap"])
    o = pr["openings"]
    for k in ("constants", "plonk_sigmas", "wires", "plonk_zs", "plonk_zs_next", "lookup_zs", "lookup_zs_next",
              "partial_products", "quotient_polys"):
        exts(o[k])
    fp = pr["opening_proof"]
    for c in fp["commit_phase_merkle_caps"]:
        cap(c)
    for qr in fp["query_round_proofs"]:
        for leaf, mp in qr["initial_trees_proof"]["evals_proofs"]:
            for x in leaf:
                f(x)
            mproof(mp)
        for st in qr["steps"]:
            exts(st["evals"])
            mproof(st["merkle_proof"])
    exts(fp["final_poly"]["coeffs"])
    f(fp["pow_witness"])
    if pi_prefix:
        out.extend(struct.pack("<Q", len(d["public_inputs"])))
    for x in d["public_inputs"]:
        f(x)
    return bytes(out)


# ----------------------------------------------------------------------------- mutations
def mutate(proof: bytes, fn) -> bytes:
    d = json.loads(proof)
    fn(d)
    return json.dumps(d, separators=(",", ":")).encode()


OPENING_KEYS = ("constants", "plonk_sigmas", "plonk_zs", "plonk_zs_next", "partial_products", "lookup_zs", "lookup_zs_next")


def randomize_openings(proof: bytes, seed: int, keys=OPENING_KEYS) -> bytes:
    """Replace the opened values under `keys` (OpeningSet, Types.hs:265-279) by uniform F^2
    elements: gate selectors S_g(zeta), lookup selectors, sigmas, Z, partial products and the
    lookup polynomials then take arbitrary values, so every vanishing term is non-trivial."""
    import random
    rnd = random.Random(seed)

    def f(d):
        o = d["proof"]["openings"]
        for k in keys:
            o[k] = [[rnd.randrange(P), rnd.randrange(P)] for _ in o[k]]
    return mutate(proof, f)


def trace_offsets(r: int, S: int, Q: int) -> dict:
    """Word offsets of the debug trace (include/p2v.h)."""
    o = {"pi_hash": 0, "betas": 4}
    o["gammas"] = o["betas"] + r
    o["alphas"] = o["gammas"] + r
    o["deltas"] = o["alphas"] + r
    o["zeta"] = o["deltas"] + 4 * r
    o["fri_alpha"] = o["zeta"] + 2
    o["fri_betas"] = o["fri_alpha"] + 2
    o["pow"] = o["fri_betas"] + 2 * S
    o["query_idx"] = o["pow"] + 1
    o["combined"] = o["query_idx"] + Q
    o["quotient"] = o["combined"] + 2 * r
    o["q_initial"] = o["quotient"] + 2 * r
    o["q_folded"] = o["q_initial"] + 2 * Q
    o["q_final"] = o["q_folded"] + 2 * Q
    o["flags"] = o["q_final"] + 2 * Q
    o["lut_re"] = o["flags"] + 1
    return o


def circuit_shape(common: bytes):
    """(r, S, Q) of a generated circuit's common data (ConstantArityBits strategy)."""
    c = json.loads(common)
    fc = c["config"]["fri_config"]
    a, fb = fc["reduction_strategy"]["ConstantArityBits"]
    logn, S = c["fri_params"]["degree_bits"], 0
    while logn > fb:
        logn -= a
        S += 1
    return c["config"]["num_challenges"], S, fc["num_query_rounds"]


def p2v_module():
    ensure_built()
    import p2v  # noqa: E402  (plonky2-verifier_amd/p2v.py)
    return p2v


# ----------------------------------------------------------------------------- S-box edge inputs
EPS = (1 << 32) - 1   # 2^64 mod p


def round0_constants():
    """Round 0's constants (Hash/Constants.hs all_ROUND_CONSTANTS row 0), from the generated header."""
    import re
    hdr = os.path.join(PKG, "csrc", "poseidon_constants.h")
    body = re.search(r"P2V_ALL_ROUND_CONSTANTS_INIT\s*\{([^}]*)\}", open(hdr).read()).group(1)
    return [int(v, 16) for v in re.findall(r"0x([0-9a-fA-F]+)", body)][:12]


def sbox_edge_values():
    """S-box inputs whose products take the rare -2^64 wrap of the device multiply (product bits
    64..95 zero, bits 0..63 below 2^32, e.g. 2^48 -> 2^96): 2^k and 2^k +- 1 for every k, p - 1,
    p - 2^k, and 2^k (2^32 - 1)."""
    vals = {P - 1, P - 2, 0, 1}
    for k in range(64):
        for v in ((1 << k), (1 << k) - 1, (1 << k) + 1, P - (1 << k), ((1 << k) * EPS) % P):
            if 0 <= v < (1 << 64):
                vals.add(v)
    return sorted(vals)


def add_nc(a, b):
    """p2::add_nc (csrc/poseidon.h): a < 2^64, b < p; a wrap adds 2^64 mod p."""
    s = a + b
    return s - (1 << 64) + EPS if s >= 1 << 64 else s


def preimage_round0(y, i, rc0):
    """A u64 state word w with add_nc(w, rc0[i]) == y exactly (so the first round's S-box sees
    the 64-bit value y itself), or y + p when no such word exists (y < rc0[i] and y < 2^32 - 1)."""
    c = rc0[i]
    if y >= c:
        return y - c
    if y >= EPS:                           # through the wrap: w + c - 2^64 + EPS == y
        return y - EPS - c + (1 << 64)
    return y + P - c                       # the congruent representative y + p (< 2^64)


def first_round_wrap_states(n_extra=0, seed=5):
    """Permutation states whose round-0 S-box inputs (state + rc0, Hash/Poseidon.hs:50-56) are the
    S-box edge values, 12 per state (the device S-box's rare fix-up on the first round
    of every permutation form)."""
    import random
    rc0 = round0_constants()
    ev = sbox_edge_values()
    rng = random.Random(seed)
    targets = ev + [1 << 48] * 12
    states = []
    for k in range(0, len(targets), 12):
        chunk = (targets[k:k + 12] + ev)[:12]
        states.append([preimage_round0(y, i, rc0) for i, y in enumerate(chunk)])
    for _ in range(n_extra):
        chunk = [rng.choice(ev) for _ in range(12)]
        states.append([preimage_round0(y, i, rc0) for i, y in enumerate(chunk)])
    return states
