"""The split S-box of the latency forms (lposeidon.h lp::sbox_u, qposeidon.h qp::sbox_qu) is
bit-identical to lp::sbox.

Even lanes form x^3 = mul_lat(x, x^2), odd lanes x^4 = mul_lat(x^2, x^2), they swap and multiply,
so an even lane returns mul_lat(x^3, x^4) (what lp::sbox returns) and an odd lane
mul_lat(x^4, x^3).  That is the same 64-bit word only if mul_lat's result depends on the 128-bit
product alone, not on the operand order.  mul_lat (lposeidon.h) is restated here instruction by
instruction (v_mad_u64_u32 with its carry-outs, the borrow chain, the net-wrap select), and the
claim is checked on edge values and random operands, together with its congruence to the
reference's multiply (Algebra/Goldilocks.hs: a b mod p) and the S-box x^7 (Hash/Poseidon.hs:92-96).
"""
import random

P = 0xFFFFFFFF00000001
M32 = (1 << 32) - 1
M64 = (1 << 64) - 1


def mul_lat(a, b):
    a0, a1, b0, b1 = a & M32, a >> 32, b & M32, b >> 32
    p_ = a0 * b0                                   # v_mad_u64_u32 v[4:5], a0, b0, 0
    x = a0 * b1 + (p_ >> 32)                       # v_lshrrev_b64 + v_mad_u64_u32: < 2^64, no carry
    assert x <= M64
    y_full = a1 * b0 + x                           # v_mad_u64_u32 ... carry-out cm (weight 2^96)
    cm, y = y_full >> 64, y_full & M64
    h = a1 * b1 + (y >> 32)                        # v_lshrrev_b64 + v_mad_u64_u32: < 2^64
    assert h <= M64
    h0, h1 = h & M32, h >> 32
    lo = (p_ & M32) | ((y & M32) << 32)            # v_mov_b32 v5, v6
    t_full = h0 * M32 + lo                         # v_mad_u64_u32 v8, -1, v[4:5]: carry ct
    ct, t = t_full >> 64, t_full & M64
    u_full = t - h1 - cm                           # v_subb_co (borrow-in cm), v_subb_co: borrow bw
    bw, u = (1 if u_full < 0 else 0), u_full & M64
    if ct and not bw:
        fix = M32                                  # 2^64 == 2^32 - 1 (mod p)
    elif bw and not ct:
        fix = P
    else:
        fix = 0
    return (u + fix) & M64                         # v_lshl_add_u64


def sbox(x):   # lp::sbox
    x2 = mul_lat(x, x)
    return mul_lat(mul_lat(x, x2), mul_lat(x2, x2))


def sbox_lanes(x):   # lp::sbox_u: (even lane, odd lane)
    x2 = mul_lat(x, x)
    x3, x4 = mul_lat(x, x2), mul_lat(x2, x2)
    return mul_lat(x3, x4), mul_lat(x4, x3)


EDGES = [0, 1, 2, M32, M32 + 1, 1 << 63, P - 1, P, P + 1, M64 - 1, M64, 0xFFFFFFFE00000002,
         0x00000001FFFFFFFF, 0xFFFFFFFF00000000, 0x80000000FFFFFFFF]


def test_mul_lat_is_symmetric_and_congruent():
    rng = random.Random(6)
    vals = EDGES + [rng.getrandbits(64) for _ in range(3000)]
    pairs = [(a, b) for a in EDGES for b in EDGES] + [(rng.choice(vals), rng.choice(vals)) for _ in range(20000)]
    for a, b in pairs:
        r = mul_lat(a, b)
        assert r == mul_lat(b, a), (hex(a), hex(b))
        assert r % P == (a * b) % P, (hex(a), hex(b))


def test_split_sbox_matches_sbox_on_both_lanes():
    rng = random.Random(7)
    for x in EDGES + [rng.getrandbits(64) for _ in range(5000)]:
        even, odd = sbox_lanes(x)
        ref = sbox(x)
        assert even == ref and odd == ref, hex(x)
        assert ref % P == pow(x % P, 7, P)
