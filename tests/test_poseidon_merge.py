"""The merged partial rounds of the device permutation (csrc/poseidon.h `PBlock`, `dv::pblock`).

D consecutive partial rounds (Hash/Poseidon.hs:48-60) are computed as D S-boxes, D-1 chain
rows and one 12-row output layer whose coefficients are products of the MDS matrix
(Hash/Constants.hs:19-25).  This checks, in exact integer arithmetic:
  * the algebra: every merge schedule the build can select reproduces the plain permutation
    (KAT of Hash/Poseidon.hs:27-35 and random states), with the device's lazy
    representatives in [0, 2^64) and its two row reductions modelled bit for bit;
  * the bounds the device code relies on: every row's 32-bit-half accumulators stay below
    2^64 for any input representatives, and the reductions never wrap twice.
"""
import os
import random
import re

import pytest

P = 2**64 - 2**32 + 1
CIRC = [17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20]
M = [[CIRC[(j - i) % 12] + (8 if i == j == 0 else 0) for j in range(12)] for i in range(12)]
KAT = [0xd64e1e3efc5b8e9e, 0x53666633020aaa47, 0xd40285597c6a8825, 0x613a4f81e81231d2,
       0x414754bfebd051f0, 0xcb1f8980294a023f, 0x6eb2a9e4d54a9d0f, 0x1902bc3af467e056,
       0xf045d5eafdc6021f, 0xe4150f77caaa3be5, 0xc9bfd01d39b50cce, 0x5c0a27fcb0e1459b]
SCHEDULES = {4: [4, 4, 4, 4, 4, 2], 3: [3] * 7 + [1], 2: [2] * 11}   # P2V_PMERGE -> PM_SCHED


def _round_constants():
    hdr = os.path.join(os.path.dirname(__file__), "..", "plonky2-verifier_amd", "csrc", "poseidon_constants.h")
    src = open(hdr).read()
    body = re.search(r"P2V_ALL_ROUND_CONSTANTS_INIT\s*\{([^}]*)\}", src).group(1)
    rc = [int(v, 16) for v in re.findall(r"0x([0-9a-fA-F]+)", body)]
    assert len(rc) == 360
    return rc


RC = _round_constants()


def sbox(x):
    return pow(x, 7, P)


def perm_plain(s):
    s = list(s)
    for r in range(30):
        s = [(s[i] + RC[12 * r + i]) % P for i in range(12)]
        if r < 4 or r >= 26:
            s = [sbox(x) for x in s]
        else:
            s[0] = sbox(s[0])
        s = [sum(M[i][j] * s[j] for j in range(12)) % P for i in range(12)]
    return s


def levels(D):
    """G[k], H[k][m] of PBlock: level-k output = G[k] s' + sum_m H[k][m] y_m + d_k."""
    G, H = {1: M}, {1: {}}
    for k in range(2, D + 1):
        G[k] = [[sum(M[i][l] * G[k - 1][l][j] for l in range(1, 12)) for j in range(12)] for i in range(12)]
        H[k] = {m: [sum(M[i][l] * H[k - 1][m][l] for l in range(1, 12)) for i in range(12)] for m in range(2, k)}
        H[k][k] = [M[i][0] for i in range(12)]
    return G, H


def dconsts(r, D):
    c = lambda k: [RC[12 * (r + k) + i] for i in range(12)]   # noqa: E731
    d = {1: c(1)}
    for k in range(2, D + 1):
        d[k] = [(sum(M[i][l] * d[k - 1][l] for l in range(1, 12)) + c(k)[i]) % P for i in range(12)]
    return d


def row(coefs, vals, dconst, wide):
    """One device row: accumulate over 32-bit halves from the constant's halves, then
    dv::reduce_t (wide=False) or dv::reduce_w (wide=True); returns a value in [0, 2^64)."""
    al, ah = dconst & 0xFFFFFFFF, dconst >> 32
    for c, v in zip(coefs, vals):
        assert 0 <= c < 2**32
        al += c * (v & 0xFFFFFFFF)
        ah += c * (v >> 32)
    assert al < 2**64 and ah < 2**64
    if not wide:
        t = al + (ah >> 32) * (2**32 - 1)
        assert t < 2**64
        r = t + ((ah & 0xFFFFFFFF) << 32)
    else:
        lo = al + ((ah & 0xFFFFFFFF) << 32)
        hi = (ah >> 32) + (lo >> 64)
        assert hi < 2**32
        r = (lo % 2**64) + hi * (2**32 - 1)
    if r >= 2**64:
        r = r - 2**64 + 2**32 - 1
    assert r < 2**64
    return r


def lift(x, rng):
    """a random 64-bit representative of x mod p (the device keeps lazy values)"""
    return x + P if x < 2**64 - P and rng.random() < 0.5 else x


def block(s, r, D, rng):
    G, H = levels(D)
    d = dconsts(r, D)
    sp = list(s)
    sp[0] = lift(sbox(s[0]), rng)
    ys = {}
    for k in range(1, D):   # chain row k -> y_{k+1}
        z = row(G[k][0] + [H[k][m][0] for m in range(2, k + 1)], sp + [ys[m] for m in range(2, k + 1)],
                d[k][0], wide=(D == 4 and k == 4))
        ys[k + 1] = lift(sbox(z), rng)
    return [row(G[D][i] + [H[D][m][i] for m in range(2, D + 1)], sp + [ys[m] for m in range(2, D + 1)],
                d[D][i], wide=(D == 4)) for i in range(12)]


def perm_merged(s, sched, rng):
    s = [(s[i] + RC[i]) % P for i in range(12)]
    for r in range(4):
        s = [sbox(x) for x in s]
        s = [(sum(M[i][j] * s[j] for j in range(12)) + RC[12 * (r + 1) + i]) % P for i in range(12)]
    r = 4
    for D in sched:
        s = block([lift(x, rng) for x in s], r, D, rng)
        r += D
    assert r == 26
    for r in range(26, 30):
        s = [sbox(x % P) for x in s]
        s = [(sum(M[i][j] * s[j] for j in range(12)) + (RC[12 * (r + 1) + i] if r < 29 else 0)) % P for i in range(12)]
    return s


def test_plain_permutation_matches_kat():
    assert perm_plain(list(range(12))) == KAT


@pytest.mark.parametrize("pm", sorted(SCHEDULES))
def test_merged_schedule_equals_permutation(pm):
    rng = random.Random(pm)
    assert perm_merged(list(range(12)), SCHEDULES[pm], rng) == KAT
    for _ in range(12):
        s = [rng.randrange(P) for _ in range(12)]
        assert perm_merged(s, SCHEDULES[pm], rng) == perm_plain(s)


@pytest.mark.parametrize("D", [2, 3, 4])
def test_merged_rows_cannot_overflow(D):
    """worst case: every input representative 2^64 - 1 and the constant p - 1"""
    G, H = levels(D)
    for k in range(1, D + 1):
        rows = range(12) if k == D else [0]
        for i in rows:
            coefs = G[k][i] + [H[k][m][i] for m in range(2, k + 1)]
            row(coefs, [2**64 - 1] * len(coefs), P - 1, wide=(k == 4))
    # the D = 2 rows and the chain rows 1, 2 use the rare-carry branch form: t < 2^49
    G2, _ = levels(2)
    assert max(sum(r) for r in G2[2]) + max(M[i][0] for i in range(12)) < 2**17


def test_cpp_tables_match_model(tmp_path):
    """The tables the device code reads (csrc/poseidon.h make_pm, dumped on the host by
    tools/pm_dump.cpp) equal this model's G, H and d for every block of the default schedule:
    chain rows k = 2..D-1 at cf[k-2] (G_k row 0, then H_k[m][0] for m < k), output rows at
    cf[2 + i] (G_D row i, then H_D[m][i] for m < D), d_k[0] at d[k-1] and d_D[i] at d[4 + i]."""
    import json
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no host C++ compiler")
    root = os.path.join(os.path.dirname(__file__), "..")
    exe = str(tmp_path / "pm_dump")
    subprocess.check_call([gxx, "-std=c++17", "-O1", "-o", exe, os.path.join(root, "tools", "pm_dump.cpp")],
                          stderr=subprocess.DEVNULL)
    dump = json.loads(subprocess.check_output([exe]))
    assert dump["sched"] == SCHEDULES[4]
    r = 4
    for D, blk in zip(dump["sched"], dump["blocks"]):
        G, H = levels(D)
        d = dconsts(r, D)
        cf, dd = blk["cf"], blk["d"]
        for k in range(1, D):
            assert dd[k - 1] == d[k][0], (r, k)
        for k in range(2, D):
            assert cf[k - 2][:12] == G[k][0]
            assert cf[k - 2][12:12 + k - 2] == [H[k][m][0] for m in range(2, k)]
        for i in range(12):
            assert cf[2 + i][:12] == G[D][i], (r, i)
            assert cf[2 + i][12:12 + D - 2] == [H[D][m][i] for m in range(2, D)]
            assert dd[4 + i] == d[D][i]
        r += D
    assert r == 26
