"""GPU parity tests (MI355X): libp2v's HIP path vs the ORACLE, bit-exact.

Statuses and the full debug trace (challenges, pi hash, lookup deltas, zeta, FRI
alpha/betas, PoW response, query indices, alpha-combined constraint values, quotient
values, per-query combineInitial / folded / final-polynomial values) must equal the
oracle's word for word.  Integer arithmetic: no tolerance anywhere."""
import gzip
import json
import re
import os

import numpy as np
import pytest

from support import GOLDEN, P, gen_circuit, mutate, oracle, p2v_module

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def p2v():
    # torch (its bundled HIP / HSA runtime) initialises its device context before libp2v (the
    # system ROCm runtime) is loaded, the order bench.py and smoke() use: with libp2v first, torch
    # once reported "No HIP GPUs are available" on a box (r02_probe10)
    import torch
    assert torch.cuda.is_available(), "torch sees no GPU"
    m = p2v_module()
    if m.device_count() == 0:
        pytest.fail("no GPU visible to libp2v")
    return m


def test_gpu_library_built_from_this_tree(p2v):
    """the libp2v.so this process loaded names the hash of the sources it was
    built from (p2v_version, csrc/version.cpp), and that hash equals srchash.py's recomputation
    over this tree's csrc/* and include/p2v.h: the binary the GPU tests run is HEAD's."""
    info = p2v.build_info()
    print("libp2v", info["version"], "tree", info["src_hash_tree"])
    assert info["match"], info


def _cases(gc):
    from test_oracle import _reject_cases
    out = [(gc.proof(w, s), 1) for w, s in ((1, 1), (2, 2), (1, 9))]
    return out + _reject_cases(gc)


# lk: 0 none; 1 a 256- and a 1000-entry table; 2 a 256- and a 2^16-entry table (BASELINE C3's
# tables: the baby/giant-step evalFinalRE); 3 field-sized table outputs (the generic path)
@pytest.mark.parametrize("nb,lk", [(6, 0), (6, 1), (6, 2), (6, 3), (8, 0)])
def test_gpu_matches_oracle_status_and_trace(p2v, nb, lk):
    O = oracle()
    gc = gen_circuit(nb, 4, lk)
    cases = _cases(gc)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    bv = p2v.BatchVerifier(vk, 0, len(cases))
    res, tr = bv.run(vk.pack_many([c[0] for c in cases]), trace=True)
    for i, (proof, expect) in enumerate(cases):
        st, otr = O.verify_json(gc.common, gc.vkey, proof, trace=True)
        assert st == expect
        assert res[i] == st, i
        assert np.array_equal(tr[i], otr), (i, np.nonzero(tr[i] != otr)[0][:10])


def _gpu_vs_oracle(p2v, gc, cases, ext=0, **kw):
    """Statuses and full traces of `cases` on the GPU equal the oracle's, word for word."""
    O = oracle()
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, ext)
    res, tr = p2v.BatchVerifier(vk, 0, len(cases)).run(vk.pack_many(cases), trace=True, **kw)
    sts, otrs = [], []
    for i, proof in enumerate(cases):
        st, otr = O.verify_json(gc.common, gc.vkey, proof, trace=True, ext=ext, **kw)
        assert res[i] == st, (i, int(res[i]), st)
        assert np.array_equal(tr[i], otr), (i, np.nonzero(tr[i] != otr)[0][:10])
        sts.append(st)
        otrs.append(otr)
    return sts, np.array(otrs)


@pytest.mark.parametrize("mode,nb", [(1, 6), (2, 6), (1, 8), (1, 12)])
def test_gpu_real_circuits_vs_oracle(p2v, mode, nb):
    """Real circuits (every gate on rows, selector polynomials, copy constraints with a real
    sigma, Z / partial products, a genuine quotient): every vanishing term is non-zero at zeta.
    Valid proofs accept; perturbed wire / sigma / Z / Z(omega zeta) / partial-product /
    selector openings break the identity; statuses and traces equal the oracle's."""
    from support import circuit_shape, trace_offsets
    from test_real_circuits import _real_reject_cases
    gc = gen_circuit(nb, 4, 0, 1, 28, 16, 0, mode)
    cases = _real_reject_cases(gc) if nb < 12 else _real_reject_cases(gc)[:5]
    sts, otrs = _gpu_vs_oracle(p2v, gc, [c[0] for c in cases])
    assert sts == [c[1] for c in cases]
    off = trace_offsets(*circuit_shape(gc.common))
    r = circuit_shape(gc.common)[0]
    assert (otrs[:, off["combined"]: off["combined"] + 2 * r] != 0).all()


@pytest.mark.parametrize("nb,lk,mode", [(6, 5, 1), (6, 4, 2), (8, 1, 1), (12, 2, 1), (12, 6, 2)])
def test_gpu_real_lookup_circuits_vs_oracle(p2v, nb, lk, mode):
    """valid proofs with a live lookup argument (LookupGate /
    LookupTableGate blocks on rows, lookup selectors, RE and SLDC polynomials from the
    prover's witness; 1 or 2 tables, up to a 2^16-entry range table at degree_bits 12) accept
    on the GPU with C_i and every evalFinalRE value non-zero; perturbed lookup openings,
    lookup selectors and looked-up wires break the identity.  Statuses and traces equal the
    oracle's word for word (the oracle's C_i is pinned by test_vanishing_literal.py)."""
    from support import circuit_shape, trace_offsets
    from test_real_circuits import _lookup_reject_cases
    gc = gen_circuit(nb, 4, lk, 1, 28, 16, 0, mode)
    cases = _lookup_reject_cases(gc)
    if nb >= 12:
        cases = cases[:3]
    sts, otrs = _gpu_vs_oracle(p2v, gc, [c[0] for c in cases])
    assert sts == [c[1] for c in cases]
    r, S, Q = circuit_shape(gc.common)
    off = trace_offsets(r, S, Q)
    assert (otrs[:, off["combined"]: off["combined"] + 2 * r] != 0).all()
    nl = len(json.loads(gc.common)["luts"])
    assert (otrs[:, off["lut_re"]: off["lut_re"] + r * nl] != 0).all()


@pytest.mark.parametrize("nb,mode,ext,arities", [(6, 1, 7, (3, 2)), (8, 1, 5, (1, 1, 1, 1)), (6, 2, 6, (3, 1)),
                                                  (8, 1, 7, (3, 2, 1, 1)), (6, 0, 7, (2, 2, 1)), (6, 1, 4, (1, 1, 1)),
                                                  (12, 1, 7, (4, 3, 2))])
def test_gpu_ext_conventions_vs_oracle(p2v, nb, mode, ext, arities):
    """Opt-in plonky2 conventions (include/p2v.h P2V_EXT_*; parity unpinned: the reference
    implements none of them): MinSize / fri_params arities (incl. arity-2 and arity-8 steps),
    salted leaves under hiding (hashed, then left out of combineInitial), hash_or_noop leaves
    (arity-2 step leaves are 4 elements).  Valid proofs accept, the generator's malicious
    modes reject, statuses and full traces equal the oracle's under the same flags."""
    gc = gen_circuit(nb, 4, 0, 1, 28, 16, 0, mode, ext, arities)
    cases = [gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 3, flags=1), gc.proof(1, 4, flags=2), gc.proof(2, 5, flags=4)]
    if nb >= 12:
        cases = cases[:3]
    sts, _ = _gpu_vs_oracle(p2v, gc, cases, ext=ext)
    assert sts == [1, 1, -3, 0, 0][:len(cases)]


RANDOMIZED = {
    "all": None,   # support.OPENING_KEYS
    "permutation": ("plonk_sigmas", "plonk_zs", "plonk_zs_next", "partial_products"),
    "selectors": ("constants",),
    "lookup": ("constants", "lookup_zs", "lookup_zs_next"),
}


@pytest.mark.parametrize("nb,lk,ng", [(6, 0, 1), (6, 0, 3), (6, 1, 1), (6, 1, 3), (6, 2, 3), (8, 0, 3), (8, 1, 1), (12, 0, 3), (12, 1, 3)])
def test_gpu_randomized_openings_vs_oracle(p2v, nb, lk, ng):
    """openings replaced by uniform F^2 values (gate selectors S_g(zeta) and
    lookup selectors, sigmas, Z, Z(omega zeta), partial products, lookup polynomials), on
    circuits with one and with several selector groups, with and without lookup tables.  Every
    Z(1)-boundary, partial-product, selector-weighted gate and lookup term is then a non-zero
    value; C_i must equal the oracle's bit for bit and may not be 0."""
    from support import OPENING_KEYS, circuit_shape, randomize_openings, trace_offsets
    gc = gen_circuit(nb, 4, lk, 1, 28, 16, ng, 0)
    base = [gc.proof(1, 1), gc.proof(2, 2)]
    cases = []
    for v, keys in enumerate(RANDOMIZED.values()):
        if keys == RANDOMIZED["lookup"] and not lk:
            continue
        for b, pr in enumerate(base):
            cases.append(randomize_openings(pr, 1000 * nb + 100 * lk + 10 * v + b, keys or OPENING_KEYS))
    sts, otrs = _gpu_vs_oracle(p2v, gc, cases)
    r, S, Q = circuit_shape(gc.common)
    off = trace_offsets(r, S, Q)
    comb = otrs[:, off["combined"]: off["combined"] + 2 * r]
    assert (comb != 0).all()
    assert len({tuple(c) for c in comb.tolist()}) == len(cases)
    assert set(sts) == {0}
    if lk:   # evalFinalRE of every table in every round, compared with the rest of the trace
        assert otrs[:, off["lut_re"]:].any(axis=1).all()


def test_gpu_golden_fixtures(p2v):
    exp = json.load(open(os.path.join(GOLDEN, "expected.json")))["cases"]

    def rd(n):
        with gzip.open(os.path.join(GOLDEN, n), "rb") as f:
            return f.read()
    by_circ = {}
    for c in exp:
        by_circ.setdefault(c["circuit"], []).append(c)
    for circ, cases in by_circ.items():
        vk = p2v.VerifierCircuitData.from_json(rd(circ + "_common.json.gz"), rd(circ + "_vkey.json.gz"))
        bv = p2v.BatchVerifier(vk, 0, len(cases))
        res, tr = bv.run(vk.pack_many([rd(c["name"] + "_proof.json.gz") for c in cases]), trace=True)
        for i, c in enumerate(cases):
            assert res[i] == c["status"], c["name"]
            assert [int(x) for x in tr[i]] == [int(x) for x in c["trace"]], c["name"]


def test_gpu_n12_standard_batch_vs_oracle(p2v):
    # BASELINE configs[1] shape (degree_bits 12, 28 queries); distinct proofs at random lanes
    O = oracle()
    gc = gen_circuit(12, 4, 0)
    good = [gc.proof(w, s) for w, s in ((1, 1), (1, 2), (2, 1))]

    def leaf(d):
        d["proof"]["opening_proof"]["query_round_proofs"][27]["initial_trees_proof"]["evals_proofs"][3][0][0] += 1
    bad = [mutate(good[0], leaf), gc.proof(2, 5, flags=1)]
    pool = good + bad
    expect = [O.verify_json(gc.common, gc.vkey, p) for p in pool]
    assert expect == [1, 1, 1, -1, -3]
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    packed = vk.pack_many(pool)
    rng = np.random.default_rng(7)
    idx = rng.integers(0, len(pool), 300)
    bv = p2v.BatchVerifier(vk, 0, 300)
    res, tr = bv.run(packed[idx], trace=True)
    assert list(res) == [expect[i] for i in idx]
    for k in range(len(pool)):
        lanes = np.nonzero(idx == k)[0]
        if len(lanes):
            st, otr = O.verify_json(gc.common, gc.vkey, pool[k], trace=True)
            assert np.array_equal(tr[lanes[0]], otr)
            assert (tr[lanes] == tr[lanes[0]]).all()


@pytest.mark.parametrize("form", ["row", "quad", "lane", "pair"])
@pytest.mark.parametrize("nb,mode,lk,pis", [(6, 1, 0, 4), (6, 0, 2, 0), (8, 1, 0, 19)])
def test_gpu_transcript_forms_vs_oracle(p2v, form, nb, mode, lk, pis):
    """The four transcript layouts (16, 4, 2 lanes and 1 lane per proof; api.cpp picks the
    first two by batch size, P2V_TRANSCRIPT forces any) give the oracle's challenges and statuses: real and
    degenerate circuits, lookups, 0 / 4 / 19 public inputs (19: a partial last PI block)."""
    gc = gen_circuit(nb, pis, lk, mode=mode)
    cases = [c[0] for c in _cases(gc)]
    old = os.environ.get("P2V_TRANSCRIPT")
    os.environ["P2V_TRANSCRIPT"] = form
    try:
        sts, _ = _gpu_vs_oracle(p2v, gc, cases)
    finally:
        if old is None:
            del os.environ["P2V_TRANSCRIPT"]
        else:
            os.environ["P2V_TRANSCRIPT"] = old
    assert 1 in sts and any(s != 1 for s in sts)


@pytest.mark.parametrize("nb,mode,lk", [(6, 1, 0), (6, 0, 2), (8, 1, 0)])
def test_gpu_tiled_input_matches_proof_major(p2v, nb, mode, lk):
    """P2V_FLAG_INPUT_TILED (the bench's layout): the same proofs in 64-proof tiles give the
    same statuses and full traces as the proof-major rows, host and device entry points, on a
    ragged batch (100 proofs: a partial last tile) with corrupted proofs in it."""
    import torch
    gc = gen_circuit(nb, 4, lk, 1, 28, 16, 0, mode)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    pool = [gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 3, flags=1), gc.proof(1, 4, flags=2)]
    packed = vk.pack_many(pool)
    rows = np.ascontiguousarray(packed[np.arange(100) % len(pool)])
    rows[37, vk.info.proof_words - 1] = (int(rows[37, vk.info.proof_words - 1]) + 1) % P   # last step sibling: -2
    bv = p2v.BatchVerifier(vk, 0, 100)
    r0, t0 = bv.run(rows, trace=True)
    r1, t1 = bv.run(rows, trace=True, tiled=True)
    assert np.array_equal(r0, r1) and np.array_equal(t0, t1)
    assert r0[37] == -2 and set(r0[:4].tolist()) == {1, -3, 0}
    d = torch.from_numpy(p2v.tile_proofs(rows).view(np.int64)).cuda()
    dres = torch.empty(100, dtype=torch.int8, device="cuda")
    bv.run_device(d.data_ptr(), 100, dres.data_ptr(), stream=torch.cuda.current_stream().cuda_stream, tiled=True)
    torch.cuda.synchronize()
    assert np.array_equal(dres.cpu().numpy(), r0)


def test_gpu_chained_workspaces(p2v):
    """p2v_verifier_chain: three workspaces chained cyclically on three streams, 9 batches in
    flight without host syncs (each batch a different rotation of a pool with valid and
    corrupted proofs): every batch's statuses equal the unchained verifier's; unlinking works."""
    import torch
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, 1)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    pool = [gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 3, flags=1), gc.proof(1, 4, flags=4)]
    packed = vk.pack_many(pool)
    B = 200
    batches = [np.ascontiguousarray(packed[(np.arange(B) + k) % len(pool)]) for k in range(9)]
    want = [p2v.BatchVerifier(vk, 0, B).run(b) for b in batches]
    bvs = [p2v.BatchVerifier(vk, 0, B) for _ in range(3)]
    for j in range(3):
        bvs[j].chain(bvs[j - 1])
    streams = [torch.cuda.Stream() for _ in range(3)]
    d_in = [torch.from_numpy(b.view(np.int64)).cuda() for b in batches]
    d_res = [torch.empty(B, dtype=torch.int8, device="cuda") for _ in batches]
    torch.cuda.synchronize()
    for k in range(9):   # workspace k % 3 is reused every third batch: stream order keeps them apart
        bvs[k % 3].run_device(d_in[k].data_ptr(), B, d_res[k].data_ptr(), stream=streams[k % 3].cuda_stream, sync=False)
    torch.cuda.synchronize()
    for k in range(9):
        assert np.array_equal(d_res[k].cpu().numpy(), want[k]), k
    assert set(want[0].tolist()) == {1, -3, 0}
    for bv in bvs:
        bv.chain(None)
    assert np.array_equal(bvs[0].run(batches[1]), want[1])
    # freeing the linked-to workspace first removes the link: the other one runs unchained
    import ctypes
    bvs[1].chain(bvs[0])
    assert np.array_equal(bvs[1].run(batches[2]), want[2])
    p2v.lib().p2v_verifier_free(bvs[0]._h)
    bvs[0]._h = ctypes.c_void_p()
    assert np.array_equal(bvs[1].run(batches[3]), want[3])


@pytest.mark.parametrize("B,tiled,mixed,form", [(200, False, False, None), (2048, True, False, None), (1, False, True, None),
                                                 (64, True, True, None), (2048, True, True, "lane"), (256, False, True, "pair")])
def test_gpu_transcript_lookahead(p2v, B, tiled, mixed, form):
    """P2V_FLAG_LOOKAHEAD: each batch's transcript runs on the workspace's own transcript stream
    into one of two challenge buffers, ahead of the workspace's earlier batches.  Two workspaces,
    12 different batches (rotations of a pool with valid and corrupted proofs) in flight without
    host syncs, each workspace reused every other batch (both challenge buffers cycle): every
    batch's statuses and full traces equal a plain synchronous run's.  B = 2048 runs the quad
    transcript and the tiled layout, B = 200 the row transcript; B = 1 and 64 are latency mode
    (k_fri and the coset / misc vanishing kernels on streams of their own, waiting on the
    lookahead's events), with lookahead and plain runs interleaved on each workspace (mixed;
    ADVICE r3).  form: the lane / pair transcript layouts (P2V_TRANSCRIPT) on the lookahead stream."""
    import torch
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, 1)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    pool = [gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 3, flags=1), gc.proof(1, 4, flags=4), gc.proof(2, 5, flags=2)]
    packed = vk.pack_many(pool)
    nb = 12
    batches = [np.ascontiguousarray(packed[(np.arange(B) * (k + 1) + k) % len(pool)]) for k in range(nb)]
    ref = p2v.BatchVerifier(vk, 0, B)   # the default layout, synchronous: the expected results
    want = [ref.run(b, trace=True) for b in batches]
    old = os.environ.get("P2V_TRANSCRIPT")
    if form:
        os.environ["P2V_TRANSCRIPT"] = form
    try:
        _lookahead_run(p2v, vk, batches, want, B, tiled, mixed)
    finally:
        if old is None:
            os.environ.pop("P2V_TRANSCRIPT", None)
        else:
            os.environ["P2V_TRANSCRIPT"] = old


def _lookahead_run(p2v, vk, batches, want, B, tiled, mixed):
    import torch
    nb = len(batches)
    tw = vk.info.trace_words
    bvs = [p2v.BatchVerifier(vk, 0, B) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    d_in = [torch.from_numpy((p2v.tile_proofs(b) if tiled else b).view(np.int64)).cuda() for b in batches]
    d_res = [torch.full((B,), 7, dtype=torch.int8, device="cuda") for _ in batches]
    d_tr = [torch.zeros((B, tw), dtype=torch.int64, device="cuda") for _ in batches]
    torch.cuda.synchronize()
    for k in range(nb):
        la = (k % 3 != 2) if mixed else True
        bvs[k % 2].run_device(d_in[k].data_ptr(), B, d_res[k].data_ptr(), stream=streams[k % 2].cuda_stream, sync=False,
                              tiled=tiled, lookahead=la, trace_ptr=d_tr[k].data_ptr())
    torch.cuda.synchronize()
    for k in range(nb):
        assert np.array_equal(d_res[k].cpu().numpy(), want[k][0]), k
        assert np.array_equal(d_tr[k].cpu().numpy().view(np.uint64), want[k][1]), k
    assert {1, -3, 0} <= set(np.concatenate([w[0] for w in want]).tolist()) or B == 1


def _number_paths(d, path=()):
    """Every number leaf of a JSON value, as a key path."""
    if isinstance(d, dict):
        for k, v in d.items():
            yield from _number_paths(v, path + (k,))
    elif isinstance(d, list):
        for i, v in enumerate(d):
            yield from _number_paths(v, path + (i,))
    elif isinstance(d, int) and not isinstance(d, bool):
        yield path


@pytest.mark.parametrize("nb,mode,lk", [(6, 1, 0), (6, 0, 1)])
def test_gpu_random_number_mutations_vs_oracle(p2v, nb, mode, lk):
    """Seeded campaign over the whole proof: 1-3 random numbers of a valid proof's JSON changed
    (+1 or a random field element), anywhere (caps, openings, leaves, siblings, step evals, final
    polynomial, PoW witness, public inputs).  Every status and every trace word on the GPU equals
    the oracle's, so the reference's error precedence holds wherever the damage lands."""
    import random
    gc = gen_circuit(nb, 4, lk, 1, 28, 16, 0, mode)
    base = json.loads(gc.proof(1, 1))
    paths = list(_number_paths(base))
    rnd = random.Random(1000 * nb + 10 * mode + lk)
    cases = []
    for _ in range(160):
        d = json.loads(json.dumps(base))
        for _k in range(rnd.randrange(1, 4)):
            node = d
            path = paths[rnd.randrange(len(paths))]
            for key in path[:-1]:
                node = node[key]
            node[path[-1]] = (node[path[-1]] + 1) % P if rnd.random() < 0.5 else rnd.randrange(P)
        cases.append(json.dumps(d, separators=(",", ":")).encode())
    sts, _ = _gpu_vs_oracle(p2v, gc, cases)
    assert len(set(sts)) >= 3   # the campaign reaches several outcome classes


def _merkle_top_cases(gc, base_txt, qidx, info, rnd, n_random=40):
    """Mutations aimed at the top Merkle levels, where a proof's query paths meet: siblings in
    the top min(5, depth) levels of the lowest query on a node and of another query on the same
    node, the same sibling changed identically in two queries on one node, bottom values (leaf
    evaluations), and random single / double sibling changes in those levels."""
    base = json.loads(base_txt)
    Q = len(qidx)
    lt = info.lde_bits - info.cap_height

    def trees():   # (name, shift, depth, sibling-list accessor)
        out = [(t, 0, info.lde_bits - info.cap_height) for t in range(4)]
        sh = 0
        for s, a in enumerate(info.step_arity_bits):
            sh += a
            out.append((4 + s, sh, max(0, info.lde_bits - sh - info.cap_height)))
        return out

    def sibs(d, q, t):
        qr = d["proof"]["opening_proof"]["query_round_proofs"][q]
        if t < 4:
            return qr["initial_trees_proof"]["evals_proofs"][t][1]["siblings"]
        return qr["steps"][t - 4]["merkle_proof"]["siblings"]

    def bump(d, q, t, l, w=0, by=1):
        e = sibs(d, q, t)[l]["elements"]
        e[w] = (e[w] + by) % P

    cases = []
    for t, sh, dep in trees():
        K = min(5, dep)
        for j in range(K):
            l = dep - K + j
            A = sh + l + 1
            groups = {}
            for q in range(Q):
                groups.setdefault(qidx[q] >> A, []).append(q)
            multi = [g for g in groups.values() if len(g) > 1]
            if not multi:
                continue
            g = multi[rnd.randrange(len(multi))]
            h, q = g[0], g[1 + rnd.randrange(len(g) - 1)]
            same = (qidx[h] >> (A - 1)) == (qidx[q] >> (A - 1))
            for who in ((h,), (q,), (h, q)):
                d = json.loads(base_txt)
                for x in who:
                    bump(d, x, t, l, w=j % 4)
                cases.append(d)
            if same:   # a different sibling word in each of the two
                d = json.loads(base_txt)
                bump(d, h, t, l, 0)
                bump(d, q, t, l, 1)
                cases.append(d)
        if t < 4:   # a bottom value: the leaf of one query of a shared node
            for q in range(Q):
                if any(qidx[k] >> (lt - min(5, dep)) == qidx[q] >> (lt - min(5, dep)) for k in range(Q) if k != q):
                    d = json.loads(base_txt)
                    ev = d["proof"]["opening_proof"]["query_round_proofs"][q]["initial_trees_proof"]["evals_proofs"][t][0]
                    ev[0] = (ev[0] + 1) % P
                    cases.append(d)
                    break
    tl = trees()
    for _ in range(n_random):
        d = json.loads(base_txt)
        for _k in range(rnd.randrange(1, 3)):
            t, sh, dep = tl[rnd.randrange(len(tl))]
            if dep == 0:
                continue
            K = min(5, dep)
            bump(d, rnd.randrange(Q), t, dep - K + rnd.randrange(K), rnd.randrange(4), rnd.randrange(1, P))
        cases.append(d)
    del base
    return [json.dumps(d, separators=(",", ":")).encode() for d in cases]


@pytest.mark.parametrize("cse", [1, 0])
@pytest.mark.parametrize("nb", [6, 8, 12])
def test_gpu_merkle_top_level_mutations_vs_oracle(p2v, nb, cse, monkeypatch):
    """Merkle paths near the cap against the oracle's per-path verification
    (Hash/Merkle.hs:27-42): mutations of siblings on nodes shared by several queries of one
    proof, the same change in two queries on one node, bottom values, random changes.  Every
    status and trace word equals the oracle's; the campaign reaches the Merkle failure classes.
    cse=1: the shared-node paths (kernels.hip k_merkle_plan / k_merkle_cse / k_merkle_resolve, the
    default), whose follower checks (A) (B) (C) these mutations hit on both sides of a meeting
    node; cse=0: k_merkle, one full path per lane.  The batch (> 64 proofs) takes the batch path."""
    import random
    from support import trace_offsets
    monkeypatch.setenv("P2V_MERKLE_CSE", str(cse))
    O = oracle()
    gc = gen_circuit(nb, 4, 0, 1, 28, 16, 0, 1)
    base = gc.proof(1, 1)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    info = vk.info
    st, tr = O.verify_json(gc.common, gc.vkey, base, trace=True)
    assert st == 1
    off = trace_offsets(info.num_challenges, info.num_fri_steps, info.num_query_rounds)["query_idx"]
    qidx = [int(x) for x in tr[off: off + info.num_query_rounds]]
    cases = [base] + _merkle_top_cases(gc, base, qidx, info, random.Random(nb))
    assert len(cases) > 64
    sts, _ = _gpu_vs_oracle(p2v, gc, cases)
    assert {-1, -2} <= set(sts), sorted(set(sts))


@pytest.mark.parametrize("nb,lk,mode", [(6, 0, 1), (8, 1, 1), (12, 2, 1)])
def test_gpu_merkle_shared_nodes_many_proofs(p2v, nb, lk, mode, monkeypatch):
    """The shared-node Merkle paths over many distinct valid proofs (their query indices meet at
    every level, including equal leaves in the small step trees) with a corrupted copy of each
    interleaved: statuses and traces equal the oracle's, and the plain one-path-per-lane kernel
    (P2V_MERKLE_CSE=0) returns the same words."""
    gc = gen_circuit(nb, 4, lk, 1, 28, 16, 0, mode)
    import random
    rnd = random.Random(77 * nb + lk)
    cases = []
    for i in range(40):
        good = gc.proof(1 + i % 5, 3 + i)
        cases.append(good)
        d = json.loads(good)
        qr = d["proof"]["opening_proof"]["query_round_proofs"]
        q = rnd.randrange(len(qr))
        t = rnd.randrange(4)
        sib = qr[q]["initial_trees_proof"]["evals_proofs"][t][1]["siblings"]
        if sib:
            e = sib[rnd.randrange(len(sib))]["elements"]
            e[0] = (e[0] + 1) % P
        cases.append(json.dumps(d, separators=(",", ":")).encode())
    monkeypatch.setenv("P2V_MERKLE_CSE", "1")
    sts, otr = _gpu_vs_oracle(p2v, gc, cases)
    assert sts[0::2] == [1] * 40 and -1 in sts[1::2]
    monkeypatch.setenv("P2V_MERKLE_CSE", "0")
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    res, tr = p2v.BatchVerifier(vk, 0, len(cases)).run(vk.pack_many(cases), trace=True)
    assert list(res) == sts and np.array_equal(tr, otr)


def test_gpu_merkle_fix_list_full_batch_of_garbage(p2v, monkeypatch):
    """a full batch of garbage proofs flags about half of all (tree, query, proof)
    paths as followers to re-run, many of them twice (their owner's check (B) and their own (A)/(C)).
    Each path is listed once (kernels.hip cse_flag), the list cannot overflow, and the long list runs
    in the lane form of k_merkle_fix.  A valid proof with one follower's sibling corrupted above its
    meeting level (only check (C) sees it) in the last slot, after a run in which every status of
    the workspace was 1, must still be rejected exactly as the oracle rejects it; every status and
    trace word equals the plain one-path-per-lane kernel's (P2V_MERKLE_CSE=0)."""
    from support import trace_offsets
    O = oracle()
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, 1)
    base = gc.proof(1, 1)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    info = vk.info
    st, tr = O.verify_json(gc.common, gc.vkey, base, trace=True)
    assert st == 1
    off = trace_offsets(info.num_challenges, info.num_fri_steps, info.num_query_rounds)["query_idx"]
    qidx = [int(x) for x in tr[off: off + info.num_query_rounds]]
    d = json.loads(base)
    qr = d["proof"]["opening_proof"]["query_round_proofs"]
    dep = len(qr[0]["initial_trees_proof"]["evals_proofs"][0][1]["siblings"])
    lvl = dep - 1
    # q shares its node at the top level with a lower query: it meets its owner below that level,
    # so its top sibling is compared by check (C) only
    q = next(k for k in range(1, len(qidx)) if any(qidx[h] >> lvl == qidx[k] >> lvl for h in range(k)))
    e = qr[q]["initial_trees_proof"]["evals_proofs"][2][1]["siblings"][lvl]["elements"]
    e[1] = (e[1] + 1) % P
    bad = json.dumps(d, separators=(",", ":")).encode()
    sb, tb = O.verify_json(gc.common, gc.vkey, bad, trace=True)
    assert sb == -1
    n = 4096
    good = vk.pack_many([base])
    W = good.shape[1]
    rng = np.random.default_rng(5)
    garbage = rng.integers(0, P, size=(n, W), dtype=np.uint64)
    garbage[-1] = vk.pack_many([bad])[0]
    monkeypatch.setenv("P2V_MERKLE_CSE", "1")
    bv = p2v.BatchVerifier(vk, 0, n)
    res0 = bv.run(np.repeat(good, n, axis=0))
    assert (res0 == 1).all()   # every Merkle status byte of the workspace was 1
    res, trc = bv.run(garbage, trace=True)
    assert res[-1] == sb and np.array_equal(trc[-1], tb)
    monkeypatch.setenv("P2V_MERKLE_CSE", "0")
    ref, rtr = p2v.BatchVerifier(vk, 0, n).run(garbage, trace=True)
    assert np.array_equal(res, ref) and np.array_equal(trc, rtr)


@pytest.mark.parametrize("args,ext", [((6, 4, 0, 1, 28, 16, 0, 1), 0), ((6, 0, 1, 1, 28, 16), 0),
                                      ((6, 4, 0, 1, 28, 16, 0, 1, 7, (3, 2)), 7)])
def test_gpu_bytes_ingest_matches_host_reader(p2v, args, ext):
    """Binary proofs packed on the GPU (k_bytes_pack, p2v_verifier_pack_bytes / run_bytes): words,
    codes and statuses equal the host reader's (p2v_pack_proof_bytes) and the JSON path's, for both
    public-input forms, on a batch with malformed proofs (truncated, a wrong sibling count,
    trailing bytes) that must fall back to the host reader with its exact error."""
    from support import proof_bytes
    gc = gen_circuit(*args)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, ext)
    texts = [gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 3, flags=1), gc.proof(1, 4, flags=2)]
    bins = [proof_bytes(t, pi_prefix=bool(i % 2)) for i, t in enumerate(texts)]
    bad = [bins[0][: len(bins[0]) // 3], bins[1] + b"\0" * 8, bytearray(bins[2])]
    cap_bytes = 32 * (1 << vk.info.cap_height)
    i = 3 * cap_bytes + 16 * (vk.info.num_openings_this + vk.info.num_openings_next)   # the first sibling count
    i += cap_bytes * vk.info.num_fri_steps + 8 * vk.info.leaf_widths[0]
    bad[2][i] += 1
    batch = bins * 8 + [bytes(b) for b in bad]
    bv = p2v.BatchVerifier(vk, 0, len(batch))
    words, codes = bv.pack_bytes(batch)
    assert bv.last_bytes_device == len(bins) * 8
    for k, b in enumerate(batch):
        try:
            ref, code = vk.pack_bytes(b), 0
        except p2v.P2VError as e:
            ref, code = None, e.code
        assert codes[k] == code, k
        if ref is not None:
            assert np.array_equal(words[k], ref), k
    assert list(codes[-3:]) == [p2v.E_PARSE, p2v.E_SHAPE, p2v.E_SHAPE]
    res, codes2 = bv.run_bytes(batch)
    assert np.array_equal(codes2, codes)
    ref_res = bv.run(vk.pack_many(texts))
    assert np.array_equal(res[: len(bins) * 8], np.tile(ref_res, 8))
    assert list(res[-3:]) == [-7, -5, -5]


def test_gpu_reference_intermediates(p2v):
    """proof_challenges / eval_combined_plonk_constraints / check_combined_plonk_equations (the
    sub-results src/testmain.hs:54-63 prints) equal the oracle's trace words; the identity
    holds for a valid proof and fails for a corrupted quotient opening."""
    from support import trace_offsets as toffs
    gc = gen_circuit(6, 4, 1, 1, 28, 16)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    inf = vk.info
    r, S, Q = inf.num_challenges, inf.num_fri_steps, inf.num_query_rounds
    assert p2v.trace_offsets(r, S, Q) == toffs(r, S, Q)
    good, bad = gc.proof(1, 1), gc.proof(1, 2, flags=4)
    _st, otr = oracle().verify_json(gc.common, gc.vkey, good, trace=True)
    o = toffs(r, S, Q)
    ch = p2v.proof_challenges(vk, good)
    assert list(ch.plonk_betas) == [int(x) for x in otr[o["betas"]: o["betas"] + r]]
    assert list(ch.plonk_alphas) == [int(x) for x in otr[o["alphas"]: o["alphas"] + r]]
    assert ch.plonk_zeta == (int(otr[o["zeta"]]), int(otr[o["zeta"] + 1]))
    assert len(ch.plonk_deltas) == r and ch.plonk_deltas[0] == tuple(int(x) for x in otr[o["deltas"]: o["deltas"] + 4])
    assert list(ch.fri_challenges.fri_query_indices) == [int(x) for x in otr[o["query_idx"]: o["query_idx"] + Q]]
    assert ch.fri_challenges.fri_pow_response == int(otr[o["pow"]])
    comb = p2v.eval_combined_plonk_constraints(vk, good)
    assert comb == [(int(otr[o["combined"] + 2 * i]), int(otr[o["combined"] + 2 * i + 1])) for i in range(r)]
    assert p2v.check_combined_plonk_equations(vk, good) is True
    assert p2v.check_combined_plonk_equations(vk, bad) is False


@pytest.mark.parametrize("n", [1, 63, 64, 65, 257])
def test_gpu_ragged_batch_sizes(p2v, n):
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    good = vk.pack(gc.proof(1, 1))
    bad = vk.pack(gc.proof(1, 5, flags=2))
    arr = np.stack([good if i % 5 else bad for i in range(n)])
    bv = p2v.BatchVerifier(vk, 0, 300)
    res = bv.run(arr)
    assert list(res) == [1 if i % 5 else 0 for i in range(n)]


def test_gpu_empty_and_oversized_batches(p2v):
    """n = 0 is a no-op that returns OK (no launch); n > max_batch is an argument error and
    writes nothing."""
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    bv = p2v.BatchVerifier(vk, 0, 64)
    empty = np.zeros((0, vk.info.proof_words), dtype=np.uint64)
    assert bv.run(empty).shape == (0,)
    good = vk.pack(gc.proof(1, 1))
    with pytest.raises(p2v.P2VError):
        bv.run(np.stack([good] * 65))
    assert list(bv.run(np.stack([good] * 64))) == [1] * 64


def test_gpu_full_size_properties(p2v):
    """4096 std-config proofs (BASELINE configs[1] size): every valid proof accepts, a
    single corrupted lane flips only itself (lane isolation), and re-running the same
    batch is idempotent."""
    gc = gen_circuit(12, 4, 0)
    pool = [gc.proof(w, s) for w, s in ((1, 3), (2, 4))]
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    packed = vk.pack_many(pool)
    B = 4096
    arr = np.ascontiguousarray(packed[np.arange(B) % 2])
    arr[1234, vk.info.proof_words - 7] ^= 1          # a sibling word of the last query's last step
    bv = p2v.BatchVerifier(vk, 0, B)
    r1 = bv.run(arr)
    r2 = bv.run(arr)
    assert np.array_equal(r1, r2)
    assert r1[1234] == -2
    assert (np.delete(r1, 1234) == 1).all()


def test_verify_proof_api(p2v):
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    assert p2v.verify_proof(vk, gc.proof(1, 1)) is True
    assert p2v.verify_proof(vk, gc.proof(1, 5, flags=2)) is False
    with pytest.raises(p2v.VerifierError) as e:
        p2v.verify_proof(vk, gc.proof(1, 4, flags=1))
    assert e.value.status == -3
    out = p2v.verify_proof_batch(vk, [gc.proof(1, 1), gc.proof(1, 6, flags=4)])
    assert out == [True, False]


def test_gpu_multi_device_entry_point(p2v):
    """p2v_verify_batch_devices: shards on their own host threads / streams / verifiers (here
    three shards on device 0), chunked, must equal the single-verifier statuses."""
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    pool = vk.pack_many([gc.proof(1, 1), gc.proof(1, 5, flags=2), gc.proof(1, 4, flags=1), gc.proof(2, 2)])
    idx = np.random.default_rng(3).integers(0, 4, 701)
    arr = np.ascontiguousarray(pool[idx])
    want = p2v.BatchVerifier(vk, 0, len(idx)).run(arr)
    assert sorted(set(want.tolist())) == [-3, 0, 1]
    got = p2v.verify_batch_devices(vk, arr, [0, 0, 0], chunk=100)
    assert np.array_equal(got, want)
    with pytest.raises(p2v.P2VError):
        p2v.verify_batch_devices(vk, arr, [0, 99])


def test_gpu_verify_batch_pool_reuse_and_chunks(p2v):
    """p2v_verify_batch keeps the circuit's verifier between calls and
    streams larger batches in chunks (H2D on a copy stream, three chunk buffers in flight).  One
    circuit handle, calls of 1, 64, 65, 700 (chunks of 256: three chunks, the ring wraps) and 3000
    proofs in varying order (from pageable and from pinned host memory), several threads at once:
    every call equals the single-workspace statuses."""
    import threading
    import torch
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    pool = vk.pack_many([gc.proof(1, 1), gc.proof(1, 5, flags=2), gc.proof(1, 4, flags=1), gc.proof(2, 2)])
    idx = np.random.default_rng(5).integers(0, 4, 3000)
    arr = np.ascontiguousarray(pool[idx])
    want = p2v.BatchVerifier(vk, 0, len(idx)).run(arr)
    assert sorted(set(want.tolist())) == [-3, 0, 1]
    pinned = torch.from_numpy(arr.view(np.int64)).pin_memory().numpy().view(np.uint64)
    for n in (1, 64, 65, 700, 1, 3000, 64, 2):
        src = pinned if n % 2 else arr
        assert np.array_equal(p2v.verify_batch(vk, src[:n]), want[:n]), n
    got = p2v.verify_batch_devices(vk, arr[:700], [0], chunk=256)
    assert np.array_equal(got, want[:700])
    errs = []

    def worker(k):
        try:
            for n in (1 + k, 300 + 7 * k, 64):
                if not np.array_equal(p2v.verify_batch(vk, arr[k:k + n]), want[k:k + n]):
                    errs.append((k, n))
        except Exception as e:   # noqa: BLE001
            errs.append((k, repr(e)))
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    assert p2v.verify_proof(vk, gc.proof(1, 1)) is True
    assert p2v.verify_proof(vk, gc.proof(1, 5, flags=2)) is False


def test_gpu_verify_batch_bytes_pipelined(p2v):
    """p2v_verify_batch_bytes (chunked copies, device packing and verification overlapped) equals
    p2v_verifier_run_bytes on a batch with malformed proofs spread over several chunks: statuses,
    decode codes and the device-packed count."""
    from support import proof_bytes
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    texts = [gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 3, flags=1), gc.proof(1, 4, flags=2)]
    bins = [proof_bytes(t, pi_prefix=bool(i % 2)) for i, t in enumerate(texts)]
    bad = [bins[0][: len(bins[0]) // 3], bins[1] + b"\0" * 8]
    batch = [bins[i % 4] for i in range(1100)]
    for k in (5, 400, 777, 1099):
        batch[k] = bad[k % 2]
    bv = p2v.BatchVerifier(vk, 0, len(batch))
    res_ref, codes_ref = bv.run_bytes(batch)
    ndev_ref = bv.last_bytes_device
    for chunk in (0, 256, 5000):
        res, codes, ndev = p2v.verify_batch_bytes(vk, batch, 0, chunk)
        assert np.array_equal(codes, codes_ref), chunk
        assert np.array_equal(res, res_ref), chunk
        assert ndev == ndev_ref == len(batch) - 4


def test_gpu_multi_device_distinct_devices(p2v):
    """p2v_verify_batch_devices over distinct GPUs (all visible, up to 8): each shard on its own
    device must give the single-verifier statuses.  Needs >= 2 GPUs (the driver's multi-GPU
    node); skipped on a one-GPU box."""
    n = p2v.device_count()
    if n < 2:
        pytest.skip("one GPU visible: distinct-device sharding needs >= 2")
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    pool = vk.pack_many([gc.proof(1, 1), gc.proof(1, 5, flags=2), gc.proof(1, 4, flags=1), gc.proof(2, 2)])
    idx = np.random.default_rng(4).integers(0, 4, 1001)
    arr = np.ascontiguousarray(pool[idx])
    want = p2v.BatchVerifier(vk, 0, len(idx)).run(arr)
    devs = list(range(min(n, 8)))
    assert np.array_equal(p2v.verify_batch_devices(vk, arr, devs, chunk=128), want)
    assert np.array_equal(p2v.verify_batch_devices(vk, arr, devs[::-1] + devs, chunk=64), want)


def test_gpu_verify_sharded_single_rank(p2v):
    """p2v.verify_sharded with the default per-shard BatchVerifier, world 1 (the path every
    rank of bench.py's N-GPU run takes for its shard)."""
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    pool = vk.pack_many([gc.proof(1, 1), gc.proof(1, 5, flags=2), gc.proof(1, 4, flags=1)])
    arr = np.ascontiguousarray(pool[np.arange(200) % 3])
    got = p2v.verify_sharded(vk, arr, 0, 1, 0)
    assert list(got) == [[1, 0, -3][i % 3] for i in range(200)]


def test_gpu_c3_lookup_batch_full_size(p2v):
    """BASELINE configs[2] shape: 65 536 proofs of a real lookup circuit (the recursion gate set
    plus LookupGate / LookupTableGate blocks of a 256-entry and a 2^16-entry table, every lookup
    term live) at degree_bits 12 in one batch.
    Every valid proof accepts, corrupted lanes reject with the oracle's status, and the
    full trace of sampled lanes (incl. every evalFinalRE value) equals the oracle's."""
    O = oracle()
    gc = gen_circuit(12, 4, 2, 1, 28, 16, 0, 1)   # real circuit: a live lookup argument (gen.cpp lookup blocks)
    pool = [gc.proof(1, 1), gc.proof(2, 2), gc.proof(1, 5, flags=2)]
    expect = [O.verify_json(gc.common, gc.vkey, p) for p in pool]
    assert expect == [1, 1, 0]
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    packed = vk.pack_many(pool)
    B = 65536
    idx = np.zeros(B, dtype=np.int64)
    idx[1::2] = 1
    idx[[77, 40000, 65535]] = 2
    bv = p2v.BatchVerifier(vk, 0, B)
    res, tr = bv.run(np.ascontiguousarray(packed[idx]), trace=True)
    assert np.array_equal(res, np.array(expect, dtype=np.int8)[idx])
    for k in range(len(pool)):
        st, otr = O.verify_json(gc.common, gc.vkey, pool[k], trace=True)
        lanes = np.nonzero(idx == k)[0]
        for lane in (lanes[0], lanes[-1]):
            assert np.array_equal(tr[lane], otr), (k, lane)


@pytest.mark.parametrize("mode,ext", [(1, 16), (0, 16), (1, 0)])
def test_gpu_shape_variants_vs_oracle(p2v, mode, ext):
    """proofs whose public inputs / final polynomial have other lengths than
    the circuit implies, verified as the reference verifies them (at the proof's own lengths,
    Hash/Sponge.hs:26-31, Plonk/FRI.hs:325-327) through p2v's shape variants: valid proofs that
    carry one public input more than the circuit declares (generator ext 16) and a final
    polynomial with two trailing zero coefficients (flags 8) accept; dropped / added public inputs
    and final coefficients reject.  verify_proof, verify_proof_batch and the variant's full GPU
    trace equal the oracle's."""
    from test_host import _shape_cases
    O = oracle()
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, mode, ext)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    cases = [("base", gc.proof(1, 1)), ("padded_fp_2", gc.proof(2, 3, flags=8))] + _shape_cases(gc)
    want = [O.verify_json(gc.common, gc.vkey, pj) for _, pj in cases]
    if ext & 16:
        assert want[0] == 1 and want[1] == 1   # the reference accepts them
    got = p2v.verify_proof_batch(vk, [pj for _, pj in cases])
    for (name, pj), w, g in zip(cases, want, got):
        gs = (1 if g is True else 0) if isinstance(g, bool) else g.status
        assert gs == w, (name, gs, w)
        if w >= 0:
            assert p2v.verify_proof(vk, pj) == (w == 1), name
        else:
            with pytest.raises(p2v.VerifierError):
                p2v.verify_proof(vk, pj)
        v = vk.for_proof(pj)
        res, tr = p2v.BatchVerifier(v, 0, 1).run(v.pack(pj)[None, :], trace=True)
        st, otr = O.verify_json(gc.common, gc.vkey, pj, trace=True)
        assert int(res[0]) == st and np.array_equal(tr[0], otr), name


def test_gpu_batch_shape_past_the_limit_is_false(p2v):
    """verify_proof_batch: a proof whose public-input list is longer than this
    build's shape-variant limit (2^20) is False — its transcript cannot match, as in the
    reference, which hashes the list at any length — while the rest of the batch is verified
    as usual; a proof that does not decode still raises, as aeson's decode fails."""
    gc = gen_circuit(6, 4, 0, 1, 28, 16, 0, 1)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    good, bad3 = gc.proof(1, 1), gc.proof(1, 4, flags=1)
    d = json.loads(good)
    d["public_inputs"] = [0] * ((1 << 20) + 1)
    long_pi = json.dumps(d, separators=(",", ":")).encode()
    got = p2v.verify_proof_batch(vk, [good, long_pi, bad3, good])
    assert got[0] is True and got[1] is False and got[3] is True, got
    assert isinstance(got[2], p2v.VerifierError) and got[2].status == -3, got
    with pytest.raises(p2v.P2VError):
        p2v.verify_proof_batch(vk, [good, b"{"])


def test_gpu_c5_shard_one_launch(p2v):
    """BASELINE configs[4] (C5), one GPU's shard as the bench runs it: ONE launch of 131 072
    device-resident proofs of the real n = 12 circuit in the 64-proof tiled layout.  Eight
    distinct valid proofs fill the batch; five corrupted variants (initial leaf -> -1, last step
    sibling -> -2, first FRI layer -> -3, final polynomial -> False, an opening -> False) sit at
    lanes spread over the whole batch, incl. the last.  Every other lane accepts (a corruption
    flips only its own lane), each corrupted lane has the oracle's status, and the full traces of
    sampled lanes equal the oracle's."""
    import torch
    O = oracle()
    gc = gen_circuit(12, 4, 0, 1, 28, 16, 0, 1)
    distinct = [gc.proof(1, s) for s in range(1, 9)]

    def leaf(d):
        d["proof"]["opening_proof"]["query_round_proofs"][3]["initial_trees_proof"]["evals_proofs"][1][0][5] += 1

    def last_sib(d):
        d["proof"]["opening_proof"]["query_round_proofs"][-1]["steps"][-1]["merkle_proof"]["siblings"][-1]["elements"][3] += 1

    def opening(d):
        d["proof"]["openings"]["wires"][7][0] += 1
    variants = [mutate(distinct[0], leaf), mutate(distinct[1], last_sib), gc.proof(1, 21, flags=1),
                gc.proof(1, 22, flags=2), mutate(distinct[2], opening)]
    vexp = [O.verify_json(gc.common, gc.vkey, v) for v in variants]
    assert vexp == [-1, -2, -3, 0, 0]
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    W = vk.info.proof_words
    B = 131072
    tile = p2v.tile_proofs(vk.pack_many([distinct[i % 8] for i in range(64)]))   # one 64-proof tile
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(tile.view(np.int64)).to(dev).repeat(B // 64)
    vrows = vk.pack_many(variants)
    lanes = {}
    for k in range(len(variants)):
        for lane in (1 + 26209 * k, 70001 + 9 * k, B - 1 - 2 * k):
            lanes[lane] = k
            idx = torch.from_numpy(((lane // 64) * W + np.arange(W, dtype=np.int64)) * 64 + lane % 64).to(dev)
            d[idx] = torch.from_numpy(vrows[k].view(np.int64)).to(dev)
    expect = np.ones(B, dtype=np.int8)
    for lane, k in lanes.items():
        expect[lane] = vexp[k]
    res = torch.zeros(B, dtype=torch.int8, device=dev)
    tw = vk.info.trace_words
    tr = torch.zeros((B, tw), dtype=torch.int64, device=dev)
    bv = p2v.BatchVerifier(vk, 0, B)
    bv.run_device(d.data_ptr(), B, res.data_ptr(), stream=torch.cuda.current_stream(dev).cuda_stream,
                  trace_ptr=tr.data_ptr(), sync=True, tiled=True)
    torch.cuda.synchronize(dev)
    got = res.cpu().numpy()
    assert np.array_equal(got, expect), np.nonzero(got != expect)[0][:10]
    otr = {k: O.verify_json(gc.common, gc.vkey, variants[k], trace=True)[1] for k in range(len(variants))}
    for lane in list(lanes)[::2] + [0, 63, 64, 65535, 65536, B - 2]:
        ref = otr[lanes[lane]] if lane in lanes else O.verify_json(gc.common, gc.vkey, distinct[lane % 64 % 8], trace=True)[1]
        assert np.array_equal(tr[lane].cpu().numpy().view(np.uint64), ref), lane


@pytest.mark.parametrize("nb,pis,lk,q,pw", [
    (10, 0, 0, 28, 16),    # no public inputs: PI hash = sponge [] = zero digest (Hash/Sponge.hs:26-31)
    (13, 9, 0, 28, 16),    # deeper trees (LDE 2^16), two PI sponge blocks
    (12, 4, 1, 20, 8),     # lookups, 20 queries, 8 PoW bits
    (7, 17, 0, 12, 0),     # odd degree (FRI steps 4 + final), 3 PI blocks, no proof of work
])
def test_gpu_circuit_shape_sweep_vs_oracle(p2v, nb, pis, lk, q, pw):
    O = oracle()
    gc = gen_circuit(nb, pis, lk, 1, q, pw)
    kinds = [(1, 1, 0), (2, 3, 0), (1, 4, 1), (1, 5, 2), (1, 6, 4)][: 3 if nb > 12 else 5]
    cases = [gc.proof(w, s, flags=f) for w, s, f in kinds]
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    res, tr = p2v.BatchVerifier(vk, 0, len(cases)).run(vk.pack_many(cases), trace=True)
    sts = []
    for i, proof in enumerate(cases):
        st, otr = O.verify_json(gc.common, gc.vkey, proof, trace=True)
        sts.append(st)
        assert res[i] == st, i
        assert np.array_equal(tr[i], otr), (i, np.nonzero(tr[i] != otr)[0][:10])
    assert sts == [1, 1, -3, 0, 0][: len(cases)]


@pytest.mark.parametrize("args,ext", [((10, 0, 0, 1, 28, 16), 0), ((13, 9, 0, 1, 28, 16), 0), ((12, 4, 1, 1, 20, 8), 0),
                                      ((7, 17, 0, 1, 12, 0), 0), ((8, 4, 0, 1, 28, 16, 0, 1, 5, (1, 1, 1, 1)), 5),
                                      ((6, 4, 0, 1, 28, 16, 0, 1, 7, (3, 2)), 7)])
def test_gpu_merkle_shared_nodes_shapes(p2v, args, ext, monkeypatch):
    """The shared-node Merkle paths on the shape sweep and the opt-in conventions, forced onto
    the batch path (P2V_LAT_MAX=0; small runs otherwise take the row-form k_merkle_row): no public
    inputs, LDE 2^16 (initial paths of 12 levels, the plan's limit), 20 and 12 queries, odd
    degree, four arity-2 steps (8 trees), hiding + MinSize + hash_or_noop.  Valid proofs plus
    copies with one Merkle sibling changed (initial or step tree, any level): statuses and traces
    equal the oracle's, and P2V_MERKLE_CSE=0 returns the same words."""
    import random
    gc = gen_circuit(*args)
    rnd = random.Random(sum(args[:6]) + ext)
    base = [gc.proof(1, 1), gc.proof(2, 2)]
    cases = list(base)
    for i in range(8):
        d = json.loads(base[i % 2])
        qr = d["proof"]["opening_proof"]["query_round_proofs"]
        q = rnd.randrange(len(qr))
        trees = [qr[q]["initial_trees_proof"]["evals_proofs"][t][1]["siblings"] for t in range(4)]
        trees += [st["merkle_proof"]["siblings"] for st in qr[q]["steps"]]
        sib = trees[rnd.randrange(len(trees))]
        if sib:
            e = sib[rnd.randrange(len(sib))]["elements"]
            e[rnd.randrange(4)] = (e[0] + 1) % P
        cases.append(json.dumps(d, separators=(",", ":")).encode())
    monkeypatch.setenv("P2V_LAT_MAX", "0")
    monkeypatch.setenv("P2V_MERKLE_CSE", "1")
    sts, otr = _gpu_vs_oracle(p2v, gc, cases, ext=ext)
    assert sts[:2] == [1, 1]
    monkeypatch.setenv("P2V_MERKLE_CSE", "0")
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, ext)
    res, tr = p2v.BatchVerifier(vk, 0, len(cases)).run(vk.pack_many(cases), trace=True)
    assert list(res) == sts and np.array_equal(tr, otr)


def test_gpu_c_abi_host_example_matches_golden(p2v, tmp_path):
    """examples/p2v_verify.c (plain C over include/p2v.h) on the golden fixtures, one GPU
    and the multi-device entry (--devices 1 shards nothing; the statuses must not change)."""
    import subprocess
    from test_host import _c_host_args
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plonky2-verifier_amd", "p2v_verify")
    exp = [c for c in json.load(open(os.path.join(GOLDEN, "expected.json")))["cases"] if c["circuit"] == "circuit_n6_lk0_pow16"]
    args = _c_host_args(tmp_path, "circuit_n6_lk0_pow16", [c["name"] for c in exp])
    for extra in ([], ["--devices", "1"]):
        out = subprocess.run([exe] + extra + args, capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        assert [int(ln.split()[1]) for ln in out.stdout.splitlines()] == [c["status"] for c in exp]


@pytest.mark.parametrize("nb,lk", [(6, 0), (6, 1), (6, 2), (8, 0), (12, 1)])
def test_gpu_constraint_programs_vs_oracle_unit_filters(p2v, nb, lk):
    """The generator's circuits have every gate filter and lookup selector 0 at zeta (valid
    proofs need a satisfied identity), so the statuses and C_i alone would not see a wrong
    gate program.  In parity mode (P2V_FLAG_UNIT_FILTERS / oracle full_trace bit 1) every
    filter is 1: C_i(zeta) then carries the alpha-combined vertical sum of all 14 gate kinds'
    constraints and every lookup term, and must equal the oracle's word for word."""
    O = oracle()
    gc = gen_circuit(nb, 4, lk)
    cases = [gc.proof(1, 1), gc.proof(2, 7)]
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    _, tr = p2v.BatchVerifier(vk, 0, len(cases)).run(vk.pack_many(cases), trace=True, unit_filters=True)
    _, tr0 = p2v.BatchVerifier(vk, 0, len(cases)).run(vk.pack_many(cases), trace=True)
    r, S, Q = vk.info.num_challenges, vk.info.num_fri_steps, vk.info.num_query_rounds
    o_c = 4 + 3 * r + 4 * r + 4 + 2 * S + 1 + Q   # off_combined (include/p2v.h)
    for i, proof in enumerate(cases):
        _, otr = O.verify_json(gc.common, gc.vkey, proof, trace=True, unit_filters=True)
        assert np.array_equal(tr[i], otr), (i, np.nonzero(tr[i] != otr)[0][:10])
        assert not np.array_equal(tr[i][o_c:o_c + 2 * r], tr0[i][o_c:o_c + 2 * r])   # the mode is live


def test_gpu_json_ingest_matches_host_packer(p2v):
    """p2v_verifier_run_json: JSON texts packed on the device against a template.  Proofs in
    the template's format take the device path; other formatting, exotic numbers and
    malformed texts must fall back to the host reader: statuses and decode codes must equal
    host packing (p2v_pack_proofs_json) + p2v_verifier_run on every proof."""
    from support import P
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    base = [gc.proof(1 + i % 2, 50 + i) for i in range(6)] + [gc.proof(1, 4, flags=1), gc.proof(1, 5, flags=2)]
    pw = json.loads(base[3])["proof"]["opening_proof"]["pow_witness"]
    key = b'"pow_witness":%d' % pw
    edits = [b"-%d" % pw, b"%d" % (pw + 3 * P), b"%d" % (pw + P), b"0000000000000000000000%d" % pw, b"-0", b"1e5", b"12.0", b"-", b"1-2"]
    variants = [base[3].replace(key, b'"pow_witness":' + e) for e in edits]
    variants += [json.dumps(json.loads(base[4]), indent=1).encode(), base[2][:-9], b"[]"]
    texts = base + variants + base[:3]
    codes_h = np.empty(len(texts), np.int32)
    packed = vk.pack_many(texts, codes=codes_h)
    ok = codes_h == 0
    want = np.where(ok, 0, np.where(codes_h == -3, -5, -7)).astype(np.int8)
    bv = p2v.BatchVerifier(vk, 0, len(texts))
    want[ok] = bv.run(np.ascontiguousarray(packed[ok]))
    res, codes = bv.run_json(texts)
    assert list(codes) == list(codes_h)
    assert list(res) == list(want)
    # the device packer took every proof in the template's format, numbers of <= 20 digits
    # with an optional '-' included; everything else went through the host reader
    n_fmt = len(base) + 3 + sum(1 for e in edits if re.fullmatch(rb"-?[0-9]{1,20}", e))
    assert bv.last_json_device == n_fmt
    assert sorted(set(want.tolist())) == [-7, -3, 0, 1]
    res2, _ = bv.run_json(texts[::-1])   # a second batch reuses (or rebuilds) the template
    assert list(res2) == list(want[::-1])
    words, codes3 = bv.pack_json(texts)   # the packed words themselves, bit-exact
    assert list(codes3) == list(codes_h)
    assert np.array_equal(words[ok], packed[ok]) and not words[~ok].any()


def test_gpu_json_ingest_fuzz(p2v):
    """Seeded byte-level mutations of proof texts (replace / insert / delete a byte from a
    JSON-significant alphabet, duplicate or cut a span, long digit runs): the device packer
    must flag exactly what it cannot pack, so the packed words and decode codes of
    p2v_verifier_pack_json equal the host reader's on every text."""
    rng = np.random.default_rng(1234)
    gc = gen_circuit(6, 4, 0)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    srcs = [gc.proof(1 + i % 2, 70 + i) for i in range(4)]
    alpha = b'0123456789-,:[]{}" .eE+x'
    texts = list(srcs)
    for k in range(400):
        t = bytearray(srcs[k % len(srcs)])
        for _ in range(1 + k % 3):
            op, i = int(rng.integers(6)), int(rng.integers(len(t)))
            c = alpha[int(rng.integers(len(alpha)))]
            if op == 0:
                t[i] = c
            elif op == 1:
                t.insert(i, c)
            elif op == 2:
                del t[i]
            elif op == 3:
                j = min(len(t), i + int(rng.integers(1, 40)))
                t[i:i] = t[i:j]
            elif op == 4:
                t[i:i] = b"9" * int(rng.integers(1, 25))
            else:   # a digit in a number changed: stays in the template's format
                ds = [m.start() for m in re.finditer(rb"[0-9]", bytes(t))]
                t[ds[int(rng.integers(len(ds)))]] = ord("0") + int(rng.integers(10))
        texts.append(bytes(t))
    texts.append(srcs[0][: len(srcs[0]) // 2])
    codes_h = np.empty(len(texts), np.int32)
    packed = vk.pack_many(texts, codes=codes_h)
    ok = codes_h == 0
    bv = p2v.BatchVerifier(vk, 0, len(texts))
    words, codes = bv.pack_json(texts)
    assert list(codes) == list(codes_h)
    assert np.array_equal(words[ok], packed[ok])
    print("device-packed", bv.last_json_device, "of", int(ok.sum()), "decodable")
    assert bv.last_json_device >= 80   # the device path carried the format-preserving edits
    assert ok.sum() < len(texts)                     # and the host reader saw real failures


def _edge_values():
    P = (1 << 64) - (1 << 32) + 1
    vals = {0, 1, 2, 3, P - 2, P - 1, P, P + 1, (1 << 64) - 1, (1 << 64) - 2, (1 << 32) - 1, 1 << 32, (1 << 32) + 1}
    for k in range(64):
        vals |= {1 << k, (1 << k) - 1 if k else 0, P - (1 << k) if (1 << k) < P else 0}
    return sorted(vals)


def test_gpu_field_mul_edge_values(p2v):
    """The device multiply (every S-box, every F/F^2 product of the verifier kernels) against
    exact integer arithmetic on all pairs of edge values: powers of two and their neighbours,
    p - 2^k, values >= p.  Products such as 2^48 * 2^48 = 2^96 take the rare wrap branches of
    the reduction (bits 64..95 zero, bits 0..63 below 2^32) that random inputs never reach."""
    P = (1 << 64) - (1 << 32) + 1
    ev = _edge_values()
    rng = np.random.default_rng(7)
    rnd = [int(x) for x in rng.integers(0, 1 << 63, size=64, dtype=np.uint64) * 2 + 1]
    pool = ev + rnd
    a = np.array([x for x in pool for _ in pool], dtype=np.uint64)
    b = np.array([y for _ in pool for y in pool], dtype=np.uint64)
    exp = np.array([(int(x) * int(y)) % P for x, y in zip(a.tolist(), b.tolist())], dtype=np.uint64)
    for op in (0, 3):   # the general multiply and the S-box's form (rare wrap in a branch)
        out = p2v.device_selftest(op, a, b)
        bad = np.nonzero(out != exp)[0]
        assert len(bad) == 0, [(op, hex(int(a[i])), hex(int(b[i])), hex(int(out[i])), hex(int(exp[i]))) for i in bad[:5]]
    # squares (two of the S-box's four products, Hash/Poseidon.hs:92-96): every combination of
    # extreme 32-bit halves (the chained MAD addends' bounds are tight at halves 2^32 - 1),
    # the edge values and random values
    halves = [0, 1, 2, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFE, 0xFFFFFFFF]
    sq = [h1 << 32 | h0 for h1 in halves for h0 in halves] + ev + [int(x) for x in rng.integers(0, 1 << 64, size=4096, dtype=np.uint64)]
    s = np.array(sq, dtype=np.uint64)
    exp = np.array([(x * x) % P for x in sq], dtype=np.uint64)
    for op in (0, 3):
        out = p2v.device_selftest(op, s, s)
        bad = np.nonzero(out != exp)[0]
        assert len(bad) == 0, [(op, hex(int(s[i])), hex(int(out[i])), hex(int(exp[i]))) for i in bad[:5]]


def test_gpu_poseidon_permutation_vs_oracle(p2v):
    """The device permutation and its compression form (zero capacity words, 4 output words)
    against the oracle on the reference KAT (Hash/Poseidon.hs:27-35), edge-value states
    (including words >= p, read mod p as the reference does) and random states."""
    from support import KAT_IN, KAT_OUT, P
    O = oracle()
    ev = _edge_values()
    rng = np.random.default_rng(11)
    states = [KAT_IN]
    for k in range(0, len(ev), 12):
        chunk = ev[k:k + 12]
        states.append((chunk + ev[:12])[:12])
    for v in ev[::7]:
        states.append([v] * 12)
    # 2^15 random states: the MDS row reduction's carry fix-up (a uniform branch taken with
    # probability ~2^-21 per row) is reached ~5 times in 2^15 x 360 rows
    states += [[int(x) for x in row] for row in rng.integers(0, 1 << 64, size=(1 << 15, 12), dtype=np.uint64)]
    a = np.array(states, dtype=np.uint64)
    full = p2v.device_selftest(1, a)
    comp = p2v.device_selftest(2, a)
    assert [int(x) for x in full[0]] == KAT_OUT
    for i, st in enumerate(states):
        exp = O.permute([int(x) % P for x in st])
        assert [int(x) for x in full[i]] == exp, i
        expc = O.permute([int(x) % P for x in st[:8]] + [0] * 4)
        assert [int(x) for x in comp[i][:4]] == expc[:4], i


def _mds_fixup_cases(rng, n=512):
    """States that drive the MDS row reduction's rare carry fix-up (poseidon.h reduce_rows /
    mds_group: it fires when a row's high-half accumulator has its low 32 bits above
    2^32 - 2^11, ~2^-21 per row for random data).  For each state a random subset of rows is
    aimed at low half 2^32 - 1 (the fix-up fires) or 2^32 - 2^11 (just below the threshold) by
    solving for some input words' high halves mod 2^32; the other rows stay random."""
    M32 = (1 << 32) - 1
    circ = [17, 15, 41, 16, 2, 28, 13, 13, 39, 18, 34, 20]

    def c(i, j):
        return circ[(j - i) % 12] + (8 if i == j == 0 else 0)
    kl = [int(x) for x in rng.integers(0, 1 << 32, 12, dtype=np.uint64)]
    kh = [int(x) for x in rng.integers(0, 1 << 32, 12, dtype=np.uint64)]
    states, hits = [], []
    while len(states) < n:
        rows = sorted(rng.choice(12, size=int(rng.integers(1, 4)), replace=False).tolist())
        cols = sorted(rng.choice(12, size=len(rows), replace=False).tolist())
        s = [int(x) for x in rng.integers(0, (1 << 64) - (1 << 32), 12, dtype=np.uint64)]
        target = [M32 if rng.integers(2) else (1 << 32) - (1 << 11) for _ in rows]
        # A x = b (mod 2^32) over the chosen columns' high halves; Gaussian elimination with odd pivots
        A = [[c(i, j) for j in cols] + [(target[k] - kh[i] - sum(c(i, j) * (s[j] >> 32) for j in range(12) if j not in cols)) & M32]
             for k, i in enumerate(rows)]
        m, ok = len(rows), True
        for col in range(m):
            piv = next((r for r in range(col, m) if A[r][col] & 1), None)
            if piv is None:
                ok = False
                break
            A[col], A[piv] = A[piv], A[col]
            inv = pow(A[col][col], -1, 1 << 32)
            A[col] = [(x * inv) & M32 for x in A[col]]
            for r in range(m):
                if r != col and A[r][col]:
                    f = A[r][col]
                    A[r] = [(x - f * y) & M32 for x, y in zip(A[r], A[col])]
        if not ok:
            continue
        for k, j in enumerate(cols):
            s[j] = (A[k][m] << 32) | (s[j] & M32)
        states.append(s)
        hits.append([i for i, t in zip(rows, target) if t == M32])
    return states, kl, kh, hits, c


def test_gpu_mds_layer_carry_fixup(p2v):
    """the grouped MDS carry fix-up (P2V_MDS_BRANCH 2) is reached deterministically:
    crafted states fire it in 1-3 rows of a group and leave the group's other rows alone (and
    near-misses just below the threshold); p2v_selftest op 4 runs one MDS layer exactly as the
    permutation does, compared with exact integer arithmetic."""
    P = (1 << 64) - (1 << 32) + 1
    rng = np.random.default_rng(21)
    states, kl, kh, hits, c = _mds_fixup_cases(rng)
    a = np.array(states, dtype=np.uint64)
    out = p2v.device_selftest(4, a, np.array(kl + kh, dtype=np.uint64))
    fired = 0
    for s, o in zip(states, out):
        for i in range(12):
            al = sum(c(i, j) * (s[j] & 0xFFFFFFFF) for j in range(12)) + kl[i]
            ah = sum(c(i, j) * (s[j] >> 32) for j in range(12)) + kh[i]
            assert int(o[i]) % P == (al + (ah << 32)) % P, (i, s)
            fired += ((al + (ah >> 32) * 0xFFFFFFFF) >> 32) + (ah & 0xFFFFFFFF) >= 1 << 32   # the carry of reduce_rows
    assert fired > 300   # the fix-up branch really ran (hundreds of rows, in every group)


def test_gpu_sbox_forms_edge_values(p2v):
    """every S-box form (the throughput permutation's single and grouped S-boxes, the row
    form's, the quad / pair forms') against x^7 mod p on the inputs whose products take the device
    multiply's rare -2^64 fix-up (2^48 -> 2^96, ...): 2^k, 2^k +- 1, p - 2^k, p - 1, in lanes
    mixed with random values, so the wave-uniform fix-up branch runs with some lanes needing it and
    others not."""
    from support import sbox_edge_values
    ev = sbox_edge_values()
    rng = np.random.default_rng(17)
    rnd = [int(x) for x in rng.integers(0, 1 << 64, size=3 * len(ev), dtype=np.uint64)]
    xs = ev + rnd + ev[::-1]
    rng.shuffle(xs)
    a = np.array(xs, dtype=np.uint64)
    exp = np.array([pow(x % P, 7, P) for x in xs], dtype=np.uint64)
    for op in (5, 7, 8):
        out = p2v.device_selftest(op, a)
        bad = np.nonzero(out != exp)[0]
        assert len(bad) == 0, [(op, hex(int(a[i])), hex(int(out[i])), hex(int(exp[i]))) for i in bad[:5]]
    b = a[::-1].copy()
    out = p2v.device_selftest(6, a, b)
    assert np.array_equal(out[:, 0], exp) and np.array_equal(out[:, 1], exp[::-1])


def test_gpu_permutation_forms_first_round_wrap(p2v):
    """states whose round-0 S-box inputs are exactly the wrap-taking edge values (state
    word = edge value - rc0[i], so state + rc0 = 2^48, ...), plus the KAT and random states, through
    the throughput permutation (op 1) and the transcript / small-batch latency forms (row, quad,
    pair: ops 9-11), against the oracle's permutation (Hash/Poseidon.hs:42-46)."""
    from support import KAT_IN, KAT_OUT, first_round_wrap_states
    O = oracle()
    rng = np.random.default_rng(23)
    states = [KAT_IN] + first_round_wrap_states(n_extra=200)
    states += [[int(x) for x in row] for row in rng.integers(0, 1 << 64, size=(300, 12), dtype=np.uint64)]
    a = np.array(states, dtype=np.uint64)
    exp = np.array([O.permute([int(x) % P for x in st]) for st in states], dtype=np.uint64)
    assert [int(x) for x in exp[0]] == KAT_OUT
    for op in (1, 9, 10, 11):
        out = p2v.device_selftest(op, a)
        bad = np.nonzero((out != exp).any(axis=1))[0]
        assert len(bad) == 0, (op, [int(i) for i in bad[:5]])


def test_gpu_latency_and_batch_modes_interleaved(p2v):
    """One workspace alternating between latency mode (n <= 64: row-form Merkle paths, k_fri and
    the coset / misc vanishing kernels on lazily created streams of their own) and the batch
    path (n > 64), on a lookup circuit so every vanishing class runs: each run's statuses and
    traces equal the expected ones, whatever ran before it on the workspace."""
    from test_real_circuits import _lookup_reject_cases
    gc = gen_circuit(6, 4, 5, 1, 28, 16, 0, 1)
    cases = _lookup_reject_cases(gc)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    packed = vk.pack_many([c[0] for c in cases])
    want = np.array([c[1] for c in cases])
    bv = p2v.BatchVerifier(vk, 0, 300)
    ref_tr = {}
    for n in (1, 300, 3, 64, 65, 1, 257, 2):
        sel = np.arange(n) % len(cases)
        res, tr = bv.run(np.ascontiguousarray(packed[sel]), trace=True)
        assert np.array_equal(res, want[sel]), (n, res[:8], want[sel][:8])
        for i in range(min(n, len(cases))):
            if i in ref_tr:
                assert np.array_equal(tr[i], ref_tr[i]), (n, i)
            else:
                ref_tr[i] = tr[i].copy()
