"""CPU model of the shared-node Merkle paths (kernels.hip k_merkle_plan / k_merkle_cse /
k_merkle_fix / k_merkle_resolve), restated line for line in Python over a stand-in 2-to-1 hash.

The exactness argument does not depend on the hash, so a keyed stand-in is enough to hold the
planning (chain lengths e, owners, followers, roots), the checks (A) (B) (C), the re-run rule and
the ancestor walk to what the reference computes per path (Hash/Merkle.hs:27-42: every query's
path hashed on its own) on honest trees and on trees with corrupted siblings and leaves.  The
GPU suite holds the kernels themselves to the oracle (test_gpu_merkle_top_level_mutations_vs_oracle,
test_gpu_merkle_shared_nodes_many_proofs)."""
import random

import pytest

MASK = (1 << 64) - 1


def h2(a, b):   # stand-in compression: any deterministic function of the ordered pair
    x = (a * 0x9E3779B97F4A7C15 + b * 0xC2B2AE3D27D4EB4F + 0x165667B19E3779F9) & MASK
    x ^= x >> 29
    return (x * 0xBF58476D1CE4E5B9) & MASK


def plain_path_ok(leaf, sibs, idx, depth, cap):
    cur = leaf
    for l in range(depth):
        cur = h2(sibs[l], cur) if idx & 1 else h2(cur, sibs[l])
        idx >>= 1
    return cap.get(idx) == cur


def plan(idx, depth):
    """k_merkle_plan for one proof and tree class: (e, owner, same_leaf, root, fol) per query."""
    Q = len(idx)
    out = []
    for q in range(Q):
        minb, owner, root, have_root, fol = 64, q, q, False, [None] * depth
        for k in range(Q):
            b = (idx[q] ^ idx[k]).bit_length()
            if not have_root and b <= depth:
                root, have_root = k, True
            if k < q:
                if b < minb:
                    minb, owner = b, k
            elif k > q and 1 <= b <= depth and fol[b - 1] is None:
                fol[b - 1] = k
        e = depth if minb - 1 >= depth else (minb - 1 if minb >= 1 else 0)
        if e < depth:
            fol[e:] = [None] * (depth - e)
        out.append((e, owner, minb == 0, root, fol))
    return out


def cse_statuses(leaves, sibs, idx, depth, cap):
    """k_merkle_cse + k_merkle_fix + k_merkle_resolve for one proof and tree: per-query mk."""
    Q = len(idx)
    P = plan(idx, depth)
    mk, node, bad = [None] * Q, [None] * Q, [False] * Q
    for q in range(Q):   # chains are independent: any order
        e, owner, same, root, fol = P[q]
        cur, ix = leaves[q], idx[q]
        for l in range(e):
            f = fol[l]
            if f is not None and sibs[f][l] != cur:   # (B)
                bad[f] = True
            cur = h2(sibs[q][l], cur) if ix & 1 else h2(cur, sibs[q][l])
            ix >>= 1
        if e == depth:
            mk[q] = cap.get(ix) == cur
            continue
        node[q] = cur
        if same:
            fail = leaves[owner] != cur
            l0 = 0
        else:
            fail = sibs[owner][e] != cur   # (A)
            l0 = e + 1
        fail = fail or any(sibs[q][l] != sibs[owner][l] for l in range(l0, depth))   # (C)
        bad[q] = bad[q] or fail
    for q in range(Q):   # k_merkle_fix
        if not bad[q]:
            continue
        e, _, _, root, _ = P[q]
        if not mk[root]:
            mk[q] = False   # a lower query fails first
            continue
        cur, ix = node[q], idx[q] >> e
        for l in range(e, depth):
            cur = h2(sibs[q][l], cur) if ix & 1 else h2(cur, sibs[q][l])
            ix >>= 1
        mk[q] = cap.get(ix) == cur
    out = list(mk)
    for q in range(Q):   # k_merkle_resolve
        e, owner, _, _, _ = P[q]
        if e == depth or bad[q]:
            continue
        a = owner
        while not (P[a][0] == depth or bad[a]):
            a = P[a][1]
        out[q] = mk[a]
    return out, bad


def honest_tree(rnd, bits, cap_height, idx):
    leaves = {}

    def leaf(i):
        if i not in leaves:
            leaves[i] = rnd.getrandbits(64)
        return leaves[i]
    memo = {}

    def node(l, i):
        if l == 0:
            return leaf(i)
        if (l, i) not in memo:
            memo[(l, i)] = h2(node(l - 1, 2 * i), node(l - 1, 2 * i + 1))
        return memo[(l, i)]
    depth = bits - cap_height
    cap = {i: node(depth, i) for i in range(1 << cap_height)}
    sibs = [[node(l, (ix >> l) ^ 1) for l in range(depth)] for ix in idx]
    return [leaf(ix) for ix in idx], sibs, cap, depth


def first_failure(mk):
    for q, v in enumerate(mk):
        if not v:
            return q
    return None


@pytest.mark.parametrize("bits,cap_height,Q", [(15, 4, 28), (11, 4, 28), (7, 4, 28), (5, 2, 28), (9, 0, 20), (4, 4, 28)])
def test_cse_model_honest_trees_flag_nothing(bits, cap_height, Q):
    rnd = random.Random(bits * 100 + Q)
    for _ in range(40):
        idx = [rnd.randrange(1 << bits) for _ in range(Q)]
        leaves, sibs, cap, depth = honest_tree(rnd, bits, cap_height, idx)
        mk, bad = cse_statuses(leaves, sibs, idx, depth, cap)
        assert not any(bad)
        assert all(mk)
        assert sum(p[0] for p in plan(idx, depth)) <= Q * depth


@pytest.mark.parametrize("bits,cap_height", [(15, 4), (11, 4), (7, 4), (6, 2)])
def test_cse_model_corruptions_keep_the_reference_outcome(bits, cap_height):
    """Siblings, leaves and whole query paths corrupted (one or several, shared or not): the
    per-query statuses up to and including the first failing query (what k_status reads,
    Plonk/FRI.hs:105-117) equal the plain per-path statuses."""
    rnd = random.Random(bits * 7 + cap_height)
    Q = 28
    for trial in range(300):
        idx = [rnd.randrange(1 << bits) for _ in range(Q)]
        leaves, sibs, cap, depth = honest_tree(rnd, bits, cap_height, idx)
        if depth == 0:
            continue
        for _ in range(rnd.randrange(1, 4)):
            q = rnd.randrange(Q)
            kind = rnd.random()
            if kind < 0.6:
                l = rnd.randrange(depth)
                sibs[q][l] = (sibs[q][l] + rnd.randrange(1, 3)) & MASK
            elif kind < 0.8:
                leaves[q] = (leaves[q] + 1) & MASK
            else:   # the same change on a sibling two queries share
                l = depth - 1 - rnd.randrange(min(3, depth))
                for k in range(Q):
                    if idx[k] >> (l + 1) == idx[q] >> (l + 1) and (idx[k] >> l) == (idx[q] >> l):
                        sibs[k][l] = (sibs[k][l] + 5) & MASK
        ref = [plain_path_ok(leaves[q], sibs[q], idx[q], depth, cap) for q in range(Q)]
        mk, _ = cse_statuses(leaves, sibs, idx, depth, cap)
        f = first_failure(ref)
        assert first_failure(mk) == f, trial
        upto = Q if f is None else f + 1
        assert mk[:upto] == ref[:upto], trial


def test_cse_model_saves_the_expected_share():
    """Standard proof shape (LDE 2^15, cap 16, arity-16 steps: depths 11, 7, 3; 4 initial trees):
    the chains hash 86.6 % of the plain compressions."""
    rnd = random.Random(3)
    plain = cse = 0
    for _ in range(400):
        idx = [rnd.randrange(1 << 15) for _ in range(28)]
        for sh, depth, trees in ((0, 11, 4), (4, 7, 1), (8, 3, 1)):
            e = sum(p[0] for p in plan([i >> sh for i in idx], depth))
            plain += 28 * depth * trees
            cse += e * trees
    assert 0.85 < cse / plain < 0.88
