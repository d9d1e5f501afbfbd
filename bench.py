#!/usr/bin/env python3
"""bench.py — Plonky2 proofs verified/sec on MI355X (BASELINE.json metric).

One "step" = one pass of the verifier hot path (libp2v: transcript + leaf hashing ->
Merkle paths -> FRI queries -> vanishing/gates -> status) over one batch of 4 096
standard-config proofs resident in HBM (BASELINE.json configs[1], "C2"), in the 64-proof
tiled layout (P2V_FLAG_INPUT_TILED; --layout proof-major for the row-per-proof form).  By
default two batches are in flight per GPU (two verifier workspaces on two streams, the
async NO_SYNC path of the C ABI), so one batch's latency-bound transcript overlaps the
other's Merkle work; the one-at-a-time figure is reported alongside ("serial").  N GPUs =
N ranks (torchrun), each verifying its own batch (proofs shard with no data-path
collective: weak scaling); value = all proofs of all ranks / max-over-ranks time.

Workload: synthetic valid proofs from the build's prover (csrc/gen): standard recursion
config (degree_bits 12, rate_bits 3, cap_height 4, 28 queries, arity 16, PoW 16, 135 wires /
80 routed, the 14-gate recursion gate set incl. Poseidon + CosetInterpolation).  By default a
real circuit (gates on rows, selector polynomials, copy constraints, Z / partial products, a
genuine quotient: every vanishing term non-zero at zeta; with --lookups the lookup tables'
LookupGate / LookupTableGate blocks and a live lookup argument; --circuit degenerate for the
gate-filters-0 circuit).  D distinct proofs per rank repeated into distinct
HBM memory, 1/16 of them corrupted (initial Merkle leaf -> -1, last step sibling -> -2).
Every timed batch's statuses are checked against the expected vector on the device, right after
its launch on the launch's own stream (verified_steps), and a clock probe at both ends of each
timed pass gives the shader clock the chip held (clock.run_clock, valu.issue.at_run_clock).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "plonky2-verifier_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "Plonky2 proofs verified/sec (std config, 28 FRI queries) at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue roofline (measured, tools/microbench/valu_rates.hip -> profiles/r02_valu_rates.txt and
# r02_valu_rates_pmc.json): every instruction of the verifier's integer mix (v_mad_u64_u32, the
# carry-chain v_add/sub/addc_co_u32, v_cndmask_b32_e64, v_lshl_add_u64, v_mul_hi/lo_u32,
# v_cmp_*_u64, ...) issues at 4.1 SIMD cycles per wave64 instruction even with 8 waves per SIMD;
# only VOP1/VOP2 32-bit ops (v_add_u32_e32, v_xor, v_mov) pair up two per 4-cycle quad (2.1
# cycles each), and the PMC counter SQ_ACTIVE_INST_VALU2 counts exactly those quads.  So a
# launch's VALU issue cycles are 4 * (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2), against an
# available 1024 SIMDs x 2.4 GHz (the guide's "2 cycles" is the dual-issue case, which this
# instruction mix reaches for ~1 % of its instructions).
VALU_SIMDS = 256 * 4
VALU_CLOCK_GHZ = 2.4
VALU_QUAD = 4


def pmc_tag():
    """The latest profile tag (profiles/<tag>_pmc_valu.json AND <tag>_pmc_traffic.json, written
    together by tools/pmc_summary.py from one tools/profile_round.sh run), so that the line's
    `valu.issue` and `roofline.traffic` come from the same code version."""
    import glob
    tags = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "*_pmc_valu.json")):
        tag = os.path.basename(f)[: -len("_pmc_valu.json")]
        if tag.endswith("_c3"):   # the C3 circuit's passes (profile_round.sh step 5) are not the line's workload
            continue
        if os.path.exists(os.path.join(ROOT, "profiles", f"{tag}_pmc_traffic.json")):
            tags.append(tag)
    return max(tags) if tags else None


def slot_of(kernel):
    """libp2v's timing slot of a device kernel: the vanishing classes share k_vanish, and the
    shared-node Merkle kernels (plan / chains / fix / resolve) share k_merkle."""
    if kernel.startswith("k_vanish") and kernel != "k_vanish_final":
        return "k_vanish"
    if kernel.startswith("k_merkle") and kernel != "k_merkle_row":
        return "k_merkle"
    return kernel


def valu_roofline(kavg, ms_step, B, run_clock_ghz=None):
    """VALU issue utilisation from the latest committed rocprofv3 VALU pass
    (profiles/<tag>_pmc_valu.json, same 4096-proof batch): issue cycles per kernel over its
    serial launch time, and for the whole (pipelined) step.  None when no PMC summary exists."""
    tag = pmc_tag()
    if tag is None:
        return None
    vfile = os.path.join(ROOT, "profiles", f"{tag}_pmc_valu.json")
    pm = json.load(open(vfile))
    cyc = {}
    for k, v in pm.items():
        if k.startswith("_") or not v.get("SQ_INSTS_VALU"):
            continue
        kk = slot_of(k)
        cyc[kk] = cyc.get(kk, 0.0) + VALU_QUAD * (v["SQ_INSTS_VALU"] - (v.get("SQ_ACTIVE_INST_VALU2") or 0.0))
    scale = B / 4096.0   # the PMC pass ran 4096-proof batches
    peak = VALU_SIMDS * VALU_CLOCK_GHZ   # G SIMD-cycles per second
    per = {}
    for k, c in cyc.items():
        if kavg.get(k) and B == 4096:   # per-kernel fractions only at the PMC pass's own batch size
            per[k] = round(c * scale / (kavg[k] * 1e-3) / 1e9 / peak, 3)
    tot = sum(cyc.values()) * scale
    # the clock the chip held in the PMC pass's dispatches (GRBM_GUI_ACTIVE / 8 / time, the
    # MI355X guide's effective clock; present from round 4's tags on): the issue fraction of the
    # dominant kernels at that clock, next to the 2.4 GHz-priced one
    eff = {k: {"clock_ghz": v["effective_clock_ghz"], "issue_frac": v["issue_frac_at_effective_clock"]}
           for k, v in pm.items() if not k.startswith("_") and v.get("effective_clock_ghz") and (v.get("duration_s") or 0) > 3e-4}
    at_run = None
    if run_clock_ghz:
        # the same issue cycles against the capacity at the shader clock this run's own probes
        # measured (s_memtime / s_memrealtime around the timed pass)
        cap = VALU_SIMDS * run_clock_ghz
        at_run = {"clock_ghz": run_clock_ghz, "peak": round(cap, 1), "step_frac": round(tot / (ms_step * 1e-3) / 1e9 / cap, 3)}
    return {"unit": "G SIMD issue-cycles/s", "peak": peak,
            "at_run_clock": at_run,
            "at_effective_clock": eff or None,
            "step_achieved": round(tot / (ms_step * 1e-3) / 1e9, 1),
            "step_frac": round(tot / (ms_step * 1e-3) / 1e9 / peak, 3),
            "kernel_frac_serial": per, "source": os.path.relpath(vfile, ROOT),
            "model": "issue cycles = 4 x (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) per launch; peak = 1024 SIMDs x 2.4 GHz; "
                     "per-instruction costs measured in profiles/r02_valu_rates.txt",
            "note": "all kernels' VALU issue cycles per step over the pipelined step time: the binding resource"}


def host_threads(local_world=1, cap=16):
    """Host threads one rank may use (proof generation, host packing, the CPU baseline): the cores
    this process may run on -- its affinity mask, capped by the cgroup CPU quota where one is set --
    shared by the ranks of this node, at most `cap` (on the GPU box the affinity
    mask shows 256 CPUs and the quota grants 16 cores; 8 ranks x 16 threads oversubscribed them)."""
    cores = len(os.sched_getaffinity(0))
    quota = cpu_quota_cores()
    if quota:
        cores = min(cores, max(1, int(quota + 0.5)))
    return max(1, min(cap, cores // max(1, local_world)))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_workload(degree_bits, distinct, witnesses, seed_base, threads, lookups=0, real=False, ext=0, arities=()):
    """real: the generator's real circuit (every gate of the recursion set on rows, selector
    polynomials, copy constraints, a genuine quotient: every vanishing term non-zero at zeta);
    else the degenerate circuit (same shapes and the same verifier work, gate filters 0).
    ext / arities: the opt-in plonky2 conventions (P2V_EXT_*; arities under MinSize or Fixed)."""
    from support import generator
    g = generator()
    gc = g.circuit(degree_bits, 4, lookups, 1, 28, 16, 0, 1 if real else 0, ext, tuple(arities))
    wseeds = [seed_base * 1000 + i + 1 for i in range(witnesses)]
    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(gc.witness, wseeds))
        jobs = [(wseeds[i % witnesses], seed_base * 100000 + i + 1) for i in range(distinct)]
        proofs = list(ex.map(lambda a: gc.proof(a[0], a[1]), jobs))
    return gc, proofs


def kernel_bytes_model(info, trace_words):
    """Algorithmic HBM bytes per proof touched by each kernel (reads + writes), from the
    packed layout: the bytes the algorithm must move, not what it does."""
    W = info.proof_words
    Q, S, r = info.num_query_rounds, info.num_fri_steps, info.num_challenges
    widths = sum(info.leaf_widths)
    step_evals = sum(2 << a for a in info.step_arity_bits)
    depth0 = info.lde_bits - info.cap_height
    step_depths, logn = [], info.lde_bits
    for a in info.step_arity_bits:
        logn -= a
        step_depths.append(max(0, logn - info.cap_height))
    T = 4 + S
    cap = 1 << info.cap_height
    header = W - Q * (widths + 4 * 4 * depth0 + step_evals + 4 * sum(step_depths))
    chal = 4 + 7 * r + 4 + 2 * S + 1 + Q + 4
    return {
        "k_transpose": 2 * W * 8,
        "k_phase1": (header + Q * (widths + step_evals) + chal + Q * T * 4) * 8,
        "k_leaf": (Q * (widths + step_evals) + Q * T * 4) * 8,
        "k_transcript": (header + chal) * 8,
        "k_merkle": (Q * T * 4 + Q * (4 * 4 * depth0 + 4 * sum(step_depths)) + Q * T * 4 + Q) * 8 + Q * T,
        "k_fri": (Q * (widths + step_evals + 2 * info.final_poly_len + 12) + chal) * 8,
        "k_vanish": (2 * (info.num_openings_this + info.num_openings_next) + chal + 1 + 4 * r) * 8,
        "k_status": (chal + Q * T + Q * 4 + 4 * r) * 8 + 1,
    }


def kernel_bytes_detail(info):
    """Algorithmic bytes per proof of each device kernel of the default (shared-node Merkle) step,
    for the per-kernel traffic table.  k_merkle_cse: every sibling, leaf
    digest, cap word and query index read once (the plain k_merkle's bytes) plus one chain id and
    one plan / follower word per path; the follower nodes it writes for k_merkle_fix are left out
    (their number depends on the batch), so the ratio is measured against the smaller figure.
    k_merkle_plan: the query indices, the plan / follower words, the flag, status and chain-id
    slots it writes; k_merkle_resolve: one plan word, flag and status per path.  k_merkle_fix has
    no fixed figure (its list is empty for honest proofs)."""
    kb = kernel_bytes_model(info, info.trace_words)
    Q, S = info.num_query_rounds, info.num_fri_steps
    T, ncls = 4 + S, 1 + S
    return {
        "k_phase1": kb["k_phase1"],
        "k_merkle_plan": Q * 8 + ncls * Q * (4 + 8) + T * Q * (1 + 1 + 4),
        "k_merkle_cse": kb["k_merkle"] + T * Q * 4 + ncls * Q * (4 + 8),
        "k_merkle_fix": None,
        "k_merkle_resolve": T * Q * (4 + 1 + 1),
        "k_merkle": kb["k_merkle"],
        "k_fri": kb["k_fri"],
        "k_vanish": kb["k_vanish"],
        # without a trace buffer: the path statuses, the FRI check bits, the vanishing results, the status
        "k_status": T * Q + Q * 4 + (1 + 4 * info.num_challenges) * 8 + 1,
    }


def kernel_traffic_table(pt, info, B):
    """Every kernel's HBM bytes per launch from the PMC pass (profiles/<tag>_pmc_traffic.json,
    4096-proof batches, scaled to B) next to its algorithmic bytes per launch and their ratio;
    the vanishing classes are summed into k_vanish (their model is per proof, all items).  The
    step's totals compare every kernel's traffic with every kernel's algorithmic bytes."""
    det = kernel_bytes_detail(info)
    scale = B / 4096.0
    rows, van = {}, {}
    for k, v in pt.items():
        if k.startswith("_") or not isinstance(v, (int, float)) or not k.startswith("k_") or k in ("k_clock_probe", "k_count_mismatches"):
            continue
        if k.startswith("k_vanish") and k != "k_vanish_final":
            van[k] = v * scale
            continue
        alg = det.get(k)
        rows[k] = {"pmc_bytes": int(v * scale), "algorithmic_bytes": int(alg * B) if alg else None,
                   "ratio": round(v * scale / (alg * B), 3) if alg else None}
    if van:
        tot = sum(van.values())
        rows["k_vanish"] = {"pmc_bytes": int(tot), "algorithmic_bytes": int(det["k_vanish"] * B),
                            "ratio": round(tot / (det["k_vanish"] * B), 3), "parts": {k: int(v) for k, v in van.items()}}
    pmc_tot = sum(r["pmc_bytes"] for r in rows.values())
    alg_tot = sum(r["algorithmic_bytes"] or 0 for r in rows.values())
    return {"per_launch": rows, "step_pmc_bytes": pmc_tot, "step_algorithmic_bytes": alg_tot,
            "step_ratio": round(pmc_tot / alg_tot, 3) if alg_tot else None}


def mutate_batch(rows, info, every=16):
    """Corrupt every `every`-th proof of the packed batch in place; returns the expected int8
    statuses.  Alternately (a) the first leaf word of query 0's constants/sigmas tree (initial
    Merkle check fails in round 0: status -1, Plonk/FRI.hs:108) and (b) the proof's last word,
    a Merkle sibling of the last query's last FRI step (every earlier check passes: -2,
    Plonk/FRI.hs:310).  Neither word is absorbed by the transcript, so nothing earlier
    changes.  Values stay canonical (w + 1 mod p)."""
    P = 0xFFFFFFFF00000001
    W, Q = info.proof_words, info.num_query_rounds
    depth0 = info.lde_bits - info.cap_height
    qstride = sum(info.leaf_widths) + 4 * 4 * depth0
    logn = info.lde_bits
    for a in info.step_arity_bits:
        logn -= a
        qstride += (2 << a) + 4 * max(0, logn - info.cap_height)
    q0 = W - Q * qstride   # query rounds are the layout's tail: [4 leaves | 4 paths | steps] each
    expect = np.ones(rows.shape[0], dtype=np.int8)
    for k, i in enumerate(range(every // 2 - 1, rows.shape[0], every)):
        w = q0 if k % 2 == 0 else W - 1
        rows[i, w] = np.uint64((int(rows[i, w]) + 1) % P)
        expect[i] = -1 if k % 2 == 0 else -2
    return expect


def perms_per_proof(info, num_pis=4):
    """Poseidon permutations per proof (SURVEY.md §8d model; commentary/FRI.md:263-265)."""
    Q = info.num_query_rounds
    noop = bool(info.ext & 4)   # P2V_EXT_HASH_OR_NOOP: leaves of <= 4 elements are not hashed
    sponge = lambda w: 0 if noop and w <= 4 else (w + 7) // 8   # noqa: E731
    leaf = sum(sponge(w) for w in info.leaf_widths) + sum(sponge(2 << a) for a in info.step_arity_bits)
    depth0 = info.lde_bits - info.cap_height
    paths, logn = 4 * depth0, info.lde_bits
    for a in info.step_arity_bits:
        logn -= a
        paths += max(0, logn - info.cap_height)
    return Q * (leaf + paths)   # + transcript (~114) + ceil(#PI/8), counted separately


def cpu_model():
    """The host CPU's model string (/proc/cpuinfo), for the baseline's record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_quota_cores():
    """The cgroup CPU quota of this process in cores (cgroup v2 cpu.max), or None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(gc, proofs, threads, target_s=10.0, target_1_s=6.0, target_all_s=10.0):
    """ORACLE (C restatement) timed on this host: the CPU path beside the GPU number, on bounded
    samples of about `target_s` seconds of CPU work on `threads` threads, `target_1_s` on one
    thread and `target_all_s` on every core this process may run on (os.sched_getaffinity, at
    most 256 threads) -- SURVEY.md §8(d): single-thread and all-cores, core count and CPU model
    stated.  The top-level value is the all-cores row."""
    from support import oracle
    O = oracle()
    c = O.circuit(gc.common, gc.vkey)
    ps = [O.proof(p) for p in proofs]

    def run(k, th):
        sel = [ps[i % len(ps)] for i in range(k)]
        arr = (ctypes.c_void_p * k)(*sel)
        res = np.zeros(k, dtype=np.int8)
        t = time.perf_counter()
        acc = O.L.or_verify_many(c, arr, k, res.ctypes.data, th)
        dt = time.perf_counter() - t
        assert acc == k, f"oracle rejected {k - acc} generated proofs"
        return dt
    # calibrate on one pass over the distinct proofs, then time a sample of ~target_s seconds
    dt0 = run(len(ps), threads)
    k = max(len(ps), min(64 * len(ps), int(len(ps) * target_s / max(dt0, 1e-3))))
    dt = run(k, threads)
    rate = k / dt
    # one thread: calibrated from the multi-thread rate, at least the distinct proofs once
    k1 = max(8, min(len(ps) * 4, int(target_1_s * rate / max(1, threads))))
    dt1 = run(k1, 1)
    # all cores: one thread per core this process may use -- its affinity mask, capped by the
    # cgroup's CPU quota where one is set (on the GPU box the mask shows 256 CPUs and the quota
    # grants 16 cores: 256 threads there ran at 124 proofs/s against 180 on 16, gpurun_out/r05a)
    affinity = len(os.sched_getaffinity(0))
    quota = cpu_quota_cores()
    n_all = max(1, min(256, affinity, int(quota + 0.5) if quota else affinity))
    if n_all == threads:   # the multi-thread row already ran on all of them
        k_all, dt_all = k, dt
    else:
        k_all = max(len(ps), min(256 * len(ps), int(target_all_s * rate / max(1, threads) * n_all)))
        dt_all = run(k_all, n_all)
    for p in ps:
        O.L.or_proof_free(p)
    O.L.or_circuit_free(c)
    return {"value": round(k_all / dt_all, 2), "unit": "proofs/s", "cores": n_all, "kind": "port",
            "cpu_model": cpu_model(), "affinity_cpus": affinity, "cpu_quota_cores": quota,
            "sample": f"{k_all} std-config proofs ({len(ps)} distinct, degree_bits 12) verified by oracle/oracle.c "
                      f"on {n_all} host threads (all cores this process may use: affinity {affinity} CPUs, "
                      f"cgroup quota {quota if quota else 'none'}) in {dt_all:.2f}s",
            "threads_16": {"value": round(rate, 2), "cores": threads,
                           "sample": f"{k} proofs on {threads} threads in {dt:.2f}s"},
            "single_thread": {"value": round(k1 / dt1, 2), "cores": 1,
                              "sample": f"{k1} proofs on 1 thread in {dt1:.2f}s"}}


def ingest_rate(vk, proofs, threads):
    """Host JSON -> packed words (p2v_pack_proofs_json, template-guided scan): proofs/s on
    1 thread and on `threads` threads, over the bench's proof texts (reported
    separately, not part of the device-resident value)."""
    texts = [bytes(p) for p in proofs] * max(1, 512 // max(1, len(proofs)))
    out = {}
    for th, sample in ((1, texts[:96]), (threads, texts)):
        vk.pack_many(sample[:4], threads=1)
        t = time.perf_counter()
        vk.pack_many(sample, threads=th)
        dt = time.perf_counter() - t
        out[f"threads_{th}"] = round(len(sample) / dt, 1)
    mb = sum(len(x) for x in texts) / len(texts) / 1e6
    return {"unit": "proofs/s", **out, "json_MB_per_proof": round(mb, 3), "cores": threads,
            "note": "host JSON->packed (template-guided scan; DOM reader for anything else)"}


def json_rate(bvs, proofs, B, steps=3):
    """End to end from JSON: B proof texts (the distinct ones repeated) in pinned host memory,
    copied to the device and packed there (p2v_verifier_run_json), then verified.  Serial:
    one batch at a time; pipelined: one host thread per verifier workspace, each on its own
    stream, so one batch's H2D copy overlaps another's packing and verification.  Reported
    next to the host packer's rate, never as the bench value."""
    import threading
    import torch
    texts = [bytes(proofs[i % len(proofs)]) for i in range(B)]
    offs = np.zeros(B + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(t) for t in texts])
    blob = torch.from_numpy(np.frombuffer(b"".join(texts), dtype=np.uint8).copy()).pin_memory().numpy()
    streams = [torch.cuda.Stream() for _ in bvs]
    for bv, st in zip(bvs, streams):
        res, codes = bv.run_json((blob, offs), stream=st.cuda_stream)
        assert (codes == 0).all() and (res == 1).all() and bv.last_json_device == B
    t = time.perf_counter()
    for _ in range(steps):
        res, codes = bvs[0].run_json((blob, offs), stream=streams[0].cuda_stream)
    dt = (time.perf_counter() - t) / steps
    assert (res == 1).all()
    out = {"value": round(B / dt, 1), "unit": "proofs/s", "ms_per_step": round(dt * 1e3, 3),
           "note": f"{B} JSON proofs ({blob.nbytes / 1e6:.0f} MB, pinned) per step: H2D + device packing (k_json_pack) + verify, one batch at a time"}
    if len(bvs) > 1:
        bad = []

        def worker(bv, st):
            for _ in range(steps):
                r, _c = bv.run_json((blob, offs), stream=st.cuda_stream)
                if not (r == 1).all():
                    bad.append(1)
        ths = [threading.Thread(target=worker, args=(bv, st)) for bv, st in zip(bvs, streams)]
        t = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t
        assert not bad
        out["pipelined"] = {"value": round(B * steps * len(bvs) / dt, 1), "inflight": len(bvs),
                            "h2d_GBps_equiv": round(blob.nbytes * steps * len(bvs) / dt / 1e9, 1)}
    return out


def bytes_rate(bvs, proofs, B, steps=3, local=0, expect=None):
    """End to end from plonky2's binary proofs: B proofs (the distinct ones repeated) in pinned
    host memory, copied to the device, packed there through the circuit's byte map (k_bytes_pack),
    then verified.  Serial: p2v_verifier_run_bytes, one batch at a time.  Pipelined:
    p2v_verify_batch_bytes on 16 384 proofs per call (chunked copies on a copy stream, device
    packing and verification overlapped).  Reported next to the JSON and packed-word legs, never as
    the bench value."""
    import torch
    import p2v
    from support import proof_bytes
    bins = [proof_bytes(p) for p in proofs]

    def pinned_blob(m):
        texts = [bins[i % len(bins)] for i in range(m)]
        offs = np.zeros(m + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(t) for t in texts])
        blob = torch.from_numpy(np.frombuffer(b"".join(texts), dtype=np.uint8).copy()).pin_memory()
        return blob, offs
    tblob, offs = pinned_blob(B)
    blob = tblob.numpy()
    st = torch.cuda.Stream()
    res, codes = bvs[0].run_bytes((blob, offs), stream=st.cuda_stream)
    assert (codes == 0).all() and (res == 1).all() and bvs[0].last_bytes_device == B
    t = time.perf_counter()
    for _ in range(steps):
        res, codes = bvs[0].run_bytes((blob, offs), stream=st.cuda_stream)
    dt = (time.perf_counter() - t) / steps
    assert (res == 1).all()
    out = {"value": round(B / dt, 1), "unit": "proofs/s", "ms_per_step": round(dt * 1e3, 3),
           "note": f"{B} binary proofs ({blob.nbytes / 1e6:.0f} MB, pinned) per step: H2D + device packing (k_bytes_pack) + verify, one batch at a time"}
    m = max(B, STREAM_PROOFS // B * B)
    tbig, boffs = pinned_blob(m)
    big = tbig.numpy()
    vk = bvs[0].circuit
    res, codes, ndev = p2v.verify_batch_bytes(vk, (big, boffs), local)   # warm: creates the pooled pipe
    assert (codes == 0).all() and (res == 1).all() and ndev == m
    t = time.perf_counter()
    for _ in range(steps):
        res, codes, ndev = p2v.verify_batch_bytes(vk, (big, boffs), local)
        assert (codes == 0).all() and (res == 1).all() and ndev == m
    dt = time.perf_counter() - t
    out["pipelined"] = {"value": round(m * steps / dt, 1), "proofs_per_call": m,
                        "h2d_GBps_equiv": round(big.nbytes * steps / dt / 1e9, 1),
                        "note": "p2v_verify_batch_bytes: chunked H2D on a copy stream, device packing + verification overlapped, "
                                "statuses and codes of every call checked"}
    del tbig, tblob
    return out


STREAM_PROOFS = 16384   # proofs per call of the pipelined from-host legs (4 x the C2 batch)


def h2d_rate(bvs, rows, B, expect, steps=3, local=0):
    """PCIe-inclusive: packed proofs in pinned host memory, H2D copy inside the timed run.
    Serial: one 4096-proof batch at a time on a workspace (copy, then verify, then D2H).
    Pipelined: p2v_verify_batch (the circuit's pooled pipeline) on 16 384 pinned proofs per call,
    in chunks whose copies run on a copy stream of their own, overlapped with the verification
    of the chunks before them (three in flight); every call's statuses checked."""
    import torch
    import p2v
    host = torch.from_numpy(rows.view(np.int64)).pin_memory()
    arr = host.numpy().view(np.uint64)
    assert np.array_equal(bvs[0].run(arr), expect)
    t = time.perf_counter()
    for _ in range(steps):
        res = bvs[0].run(arr)
    dt = (time.perf_counter() - t) / steps
    assert np.array_equal(res, expect)
    out = {"value": round(B / dt, 1), "unit": "proofs/s", "ms_per_step": round(dt * 1e3, 3),
           "note": f"{B} proofs from pinned host memory per step, H2D {rows.nbytes / 1e6:.0f} MB + verify + D2H, one batch at a time"}
    reps = max(1, STREAM_PROOFS // B)
    big = torch.from_numpy(np.tile(rows, (reps, 1)).view(np.int64)).pin_memory()
    barr = big.numpy().view(np.uint64)
    bexp = np.tile(expect, reps)
    vk = bvs[0].circuit
    assert np.array_equal(p2v.verify_batch(vk, barr, local), bexp)   # warm: creates the pooled pipe
    t = time.perf_counter()
    for _ in range(steps):
        res = p2v.verify_batch(vk, barr, local)
        assert np.array_equal(res, bexp)
    dt = time.perf_counter() - t
    out["pipelined"] = {"value": round(barr.shape[0] * steps / dt, 1), "proofs_per_call": barr.shape[0],
                        "h2d_GBps_equiv": round(barr.nbytes * steps / dt / 1e9, 1),
                        "note": "p2v_verify_batch: chunked H2D on a copy stream overlapped with verification, statuses of every call checked"}
    del big
    return out


def dropin_leg(p2v, gc, proofs, packed, expect, local, reps=30):
    """The reference's API is one proof per call (verifyProof, Plonk/Verifier.hs:56): the cost a
    drop-in caller pays through the C-ABI.  cold = a fresh circuit handle's
    first p2v_verify_batch (its pooled verifier is created then); warm = the median of later calls
    on the same handle; workspace = the same proofs on a pre-created BatchVerifier (the batch-1
    latency figure of DESIGN.md); verify_proof = p2v.verify_proof on the JSON text (pack + verify)."""
    import ctypes as ct
    out = {"unit": "ms"}
    L = p2v.lib()
    for n in (1, 64):
        rows = np.ascontiguousarray(packed[:n])
        res = np.empty(n, dtype=np.int8)
        t = time.perf_counter()
        vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
        t_circ = time.perf_counter() - t
        t = time.perf_counter()
        rc = L.p2v_verify_batch(vk.handle, rows.ctypes.data, n, res.ctypes.data, local)
        cold = time.perf_counter() - t
        assert rc == 0 and np.array_equal(res, expect[:n])
        warm = []
        for _ in range(reps):
            t = time.perf_counter()
            rc = L.p2v_verify_batch(vk.handle, rows.ctypes.data, n, res.ctypes.data, local)
            warm.append(time.perf_counter() - t)
            assert rc == 0 and np.array_equal(res, expect[:n])
        bv = p2v.BatchVerifier(vk, local, n)
        ws = []
        for _ in range(reps):
            t = time.perf_counter()
            r = bv.run(rows)
            ws.append(time.perf_counter() - t)
            assert np.array_equal(r, expect[:n])
        del bv
        out[f"n{n}"] = {"circuit_from_json": round(t_circ * 1e3, 3), "cold": round(cold * 1e3, 3),
                        "warm": round(float(np.median(warm)) * 1e3, 3), "warm_min": round(min(warm) * 1e3, 3),
                        "workspace": round(float(np.median(ws)) * 1e3, 3),
                        "warm_over_workspace": round(float(np.median(warm)) / float(np.median(ws)), 3)}
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    text = bytes(proofs[0])
    assert p2v.verify_proof(vk, text, device=local) is True
    vp = []
    for _ in range(reps):
        t = time.perf_counter()
        ok = p2v.verify_proof(vk, text, device=local)
        vp.append(time.perf_counter() - t)
        assert ok is True
    out["verify_proof"] = {"warm": round(float(np.median(vp)) * 1e3, 3), "json_MB": round(len(text) / 1e6, 3)}
    out["note"] = ("C-ABI p2v_verify_batch through ctypes, host proofs in pageable memory; cold includes creating the "
                   "circuit's pooled verifier; median of %d warm calls" % reps)
    return out


C5_PROOFS = 1 << 20       # BASELINE.json configs[4]: 1M proofs over the node's GPUs
C5_CHUNK = 131072         # per launch: C5's per-GPU share on 8 GPUs


def max_over_ranks(dt, world, cpu_grp):
    """The step time of the slowest rank: an all-reduce MAX of one float64 over the gloo side
    group (CPU tensor), so the multi-GPU number depends on no RCCL call."""
    if world == 1:
        return dt
    import torch
    import torch.distributed as dist
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=cpu_grp)
    return float(t.item())


def gather_over_ranks(x, world, cpu_grp):
    """Every rank's value of one float (all_gather over the gloo side group, CPU tensors): the
    per-rank figures behind the max-over-ranks time."""
    if world == 1:
        return [x]
    import torch
    import torch.distributed as dist
    mine = torch.tensor([x], dtype=torch.float64)
    parts = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(parts, mine, group=cpu_grp)
    return [float(p.item()) for p in parts]


def per_rank_summary(proofs, own_s, world, cpu_grp, clock_ghz=None):
    """Per-rank throughput (each rank's own proofs over its own time, before the closing barrier),
    min / max and the imbalance 1 - min/max; with clock_ghz, every rank's shader clock over its pass."""
    rates = [proofs / t if t > 0 else 0.0 for t in gather_over_ranks(own_s, world, cpu_grp)]
    out = {"proofs_per_s": [round(r, 1) for r in rates], "min": round(min(rates), 1), "max": round(max(rates), 1),
           "imbalance": round(1.0 - min(rates) / max(rates), 4) if max(rates) > 0 else None}
    if clock_ghz is not None:
        out["clock_ghz"] = [round(c, 4) for c in gather_over_ranks(float(clock_ghz), world, cpu_grp)]
    return out


def c5_leg(p2v, vk, info, d_proofs, d_expect, B, world, local, dev, cpu_grp, streams, tiled, steps=1, stagger=0,
           total=C5_PROOFS, chunk=C5_CHUNK, note=None, warm=1):
    """BASELINE.json configs[4] (C5): 1 048 576 std proofs sharded over the ranks (contiguous
    shards, p2v.shard_bounds), each rank verifying its shard in launches of up to 131 072 proofs
    (the per-GPU share at 8 GPUs) on two workspaces in flight.  The shard is device-resident:
    the C2 batch repeated on the device to 131 072 distinct HBM rows, reused by every launch of
    the shard.  Statuses of every launch are checked: the result buffers are cleared before the
    timed pass and each launch's statuses are compared with the expected vector on its own
    stream, folded into a per-stream device flag.  Time = max over ranks.
    total / chunk / note: the same leg for another configuration (C3: 65 536 lookup proofs).
    warm: untimed passes before the timed ones (the clock ramps back up after the host-side gap)."""
    import torch
    s, e = p2v.shard_bounds(total, world, int(os.environ.get("RANK", "0")))
    n = e - s
    rows = min(chunk, n)
    reps = (rows + B - 1) // B
    if tiled:   # whole 64-proof tiles of the tiled batch, repeated (proof order is preserved)
        big = d_proofs.repeat(reps)[: (rows + 63) // 64 * 64 * info.proof_words].contiguous()
    else:
        big = d_proofs.repeat(reps, 1)[:rows].contiguous()
    exp = d_expect.repeat(reps)[:rows]
    bvs = [p2v.BatchVerifier(vk, local, rows) for _ in range(2)]
    if stagger:
        bvs[0].chain(bvs[1])
        bvs[1].chain(bvs[0])
    import torch.distributed as dist
    res = [torch.empty(rows, dtype=torch.int8, device=dev) for _ in range(2)]
    chunks = [min(rows, n - k) for k in range(0, n, rows)]
    sts = [streams[j % len(streams)] for j in range(2)]
    okf = [torch.ones((), dtype=torch.bool, device=dev) for _ in range(2)]

    def one_pass(check):
        for i, c in enumerate(chunks):
            j = i % 2
            bvs[j].run_device(big.data_ptr(), c, res[j].data_ptr(), stream=sts[j].cuda_stream, sync=False, tiled=tiled)
            if check:   # this launch's statuses, on its stream, before the buffer is reused
                with torch.cuda.stream(sts[j]):
                    okf[j] &= (res[j][:c] == exp[:c]).all()
    for _ in range(warm):   # warm-up
        one_pass(False)
    torch.cuda.synchronize(dev)
    for r in res:
        r.zero_()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier(group=cpu_grp)
    t = time.perf_counter()
    for _ in range(steps):
        one_pass(True)
    torch.cuda.synchronize(dev)
    own = time.perf_counter() - t   # this rank's own time (before the closing barrier)
    if world > 1:
        dist.barrier(group=cpu_grp)
    dt = time.perf_counter() - t
    ok = bool(okf[0].item()) and bool(okf[1].item())
    dt = max_over_ranks(dt, world, cpu_grp)
    per_rank = per_rank_summary(n * steps, own, world, cpu_grp)
    ok_all = all(v > 0 for v in gather_over_ranks(1.0 if ok else 0.0, world, cpu_grp))
    del big, bvs, res
    torch.cuda.empty_cache()
    return {"proofs": total * steps, "value": round(total * steps / dt, 1), "unit": "proofs/s",
            "per_gpu": round(total * steps / dt / world, 1), "seconds": round(dt, 4), "n_gpus": world,
            "per_rank": per_rank, "shard_per_gpu": n, "launch_proofs": rows, "verified_all": ok_all,
            "note": note or ("BASELINE configs[4]: 1M std proofs sharded over the ranks (no data-path collective), "
                             "launches of <= 131072 device-resident proofs, two in flight per GPU, every launch's statuses checked on "
                             "the device; time = max over ranks")}


C3_PROOFS = 65536   # BASELINE.json configs[2]
C3_CHUNK = 16384
C3_PASSES = 3   # timed passes over the 65 536 proofs (one pass is ~56 ms: a clock dip after the workload's
                # generation on the host read 0.66 M once, profiles/r04q_vanish_items_merge.txt)
C3_WARM = 4     # untimed passes first.  The first bench process on a fresh box reads ~0.97 M against
                # ~1.20 M for every later one, whichever library runs, with 2 warm passes and with 4:
                # host-side time inside the bracket, not device time (profiles/r06t_c3_ab_rev.txt,
                # r06z2_first_process.txt)


def c3_leg(p2v, args, threads, dev, local, streams):
    """BASELINE.json configs[2] (C3): 65 536 proofs of the real circuit with LookupGate /
    LookupTableGate blocks and a live lookup argument (a 256-entry and a 2^16-entry table,
    Plonk/Lookups.hs:45-132), on one GPU: 64 distinct generated proofs, 1/16 corrupted, tiled
    and repeated on the device to 65 536 rows, verified in launches of 16 384 on two workspaces
    in flight, every launch's statuses checked on the device.  Per-kernel times (k_lut and the
    vanishing kernels, which include the lookup items) from one serial 4 096-proof run."""
    import torch
    t0 = time.time()
    gc, proofs = make_workload(args.degree_bits, args.distinct, args.witnesses, 7, threads, 2, True)
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey)
    info = vk.info
    rows = np.ascontiguousarray(vk.pack_many(proofs)[np.arange(args.batch) % len(proofs)])
    expect = mutate_batch(rows, info)
    d_proofs = torch.from_numpy(p2v.tile_proofs(rows).view(np.int64)).to(dev)
    d_expect = torch.from_numpy(expect).to(dev)
    gen_s = time.time() - t0
    out = c5_leg(p2v, vk, info, d_proofs, d_expect, args.batch, 1, local, dev, None, streams, True,
                 total=C3_PROOFS, chunk=C3_CHUNK, steps=C3_PASSES, warm=C3_WARM,
                 note="BASELINE configs[2]: 65536 proofs of the real circuit with LookupGate/LookupTableGate (256 + 65536-entry "
                      "tables, live lookup argument), device-resident, launches of 16384, two in flight, statuses checked on the device; "
                      f"timed over {C3_PASSES} passes after {C3_WARM} untimed ones ('proofs' counts all three)")
    bv = p2v.BatchVerifier(vk, local, args.batch)
    res = torch.empty(args.batch, dtype=torch.int8, device=dev)
    kt = {}
    for _ in range(3):   # serial 4096-proof runs: per-kernel times of the lookup circuit
        bv.run_device(d_proofs.data_ptr(), args.batch, res.data_ptr(), stream=streams[0].cuda_stream, sync=True, tiled=True)
        for k, v in bv.last_timings().items():
            kt.setdefault(k, []).append(v)
    out["verified_all"] = out["verified_all"] and bool((res == d_expect).all())
    out["kernel_ms_serial_4096"] = {k: round(float(np.mean(v[1:])), 4) for k, v in kt.items()}
    out["workload"] = f"{len(proofs)} distinct proofs generated in {gen_s:.1f}s, degree_bits {info.degree_bits}, {info.proof_words} words per proof"
    del d_proofs, bv
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks). Under torchrun it must equal WORLD_SIZE; without torchrun and N > 1 "
                         "bench.py starts the N ranks itself (torch.distributed.run child process)")
    ap.add_argument("--steps", type=int, default=300)   # ~1.1 s pipelined + ~1.4 s serial timed: long enough for an external utilisation sampler
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="proofs per GPU per step")
    ap.add_argument("--distinct", type=int, default=64, help="distinct generated proofs per rank (repeated to the batch)")
    ap.add_argument("--witnesses", type=int, default=8)
    ap.add_argument("--circuit", choices=("real", "degenerate"), default="real",
                    help="real: gates on rows, copy constraints, genuine quotient (C4's recursion gate set; with --lookups "
                         "also LookupGate / LookupTableGate blocks with a live lookup argument); degenerate: gate filters 0")
    ap.add_argument("--degree-bits", type=int, default=12)
    ap.add_argument("--inflight", type=int, default=2, help="batches in flight per GPU (workspaces/streams)")
    ap.add_argument("--stagger", type=int, default=0, choices=(0, 1),
                    help="1: chain the in-flight workspaces (p2v_verifier_chain) so their phase 1 alternate")
    ap.add_argument("--lookahead", type=int, default=0, choices=(0, 1),
                    help="1: P2V_FLAG_LOOKAHEAD (each batch's transcript on its own stream, ahead of the workspace's earlier batches)")
    ap.add_argument("--layout", choices=("tiled", "proof-major"), default="tiled",
                    help="device-resident batch layout: 64-proof tiles (P2V_FLAG_INPUT_TILED, coalesced loads) or proof-major rows")
    ap.add_argument("--ext", type=int, default=0, help="P2V_EXT_* flags of the workload circuit (1 MinSize arities, 2 hiding, 4 hash_or_noop)")
    ap.add_argument("--arities", default="", help="comma-separated FRI arity bits (with --ext 1: MinSize; else Fixed)")
    ap.add_argument("--lookups", type=int, default=0,
                    help="0: standard recursion circuit (C2); 2: + LookupGate/LookupTableGate with a 256-entry and a 2^16-entry table (C3 circuit)")
    ap.add_argument("--transcript", choices=("auto", "row", "quad", "pair", "lane"), default="auto",
                    help="transcript layout (P2V_TRANSCRIPT): auto = row below 4096 proofs per launch, quad from 4096 "
                         "(P2V_QUAD_MIN), lane from 16384 (P2V_LANE_MIN)")
    ap.add_argument("--single-stream", action="store_true", help="P2V_SINGLE_STREAM=1: each workspace on one stream (no side stream)")
    ap.add_argument("--hw-queues", type=int, default=0, help="GPU_MAX_HW_QUEUES for this process (0: the runtime's default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="gloo",
                    help="the default process group: gloo (the bench's cross-rank operations are CPU-side barriers and "
                         "reductions; no data-path collective) or nccl (= RCCL, with a gloo side group for those operations)")
    ap.add_argument("--quick", action="store_true", help="device-resident figure only (no ingest / PCIe / CPU / C5 legs)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 leg (1M proofs sharded over the ranks)")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 leg (65536 lookup-circuit proofs, one GPU)")
    ap.add_argument("--no-host-legs", action="store_true",
                    help="skip the drop-in, ingest, from-host and CPU-baseline legs (device-resident C2 / C5 / C3 only)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus and args.gpus > 1:
        # N GPUs requested without a launcher: start the N ranks as a child torch.distributed.run
        # (before anything touches the GPU; no exec) and exit with its status
        import socket
        import subprocess
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
        log("[bench] launching", args.gpus, "ranks:", " ".join(cmd))
        sys.exit(subprocess.call(cmd))
    world = int(env_world or "1")
    cpu_grp = None
    if args.gpus is not None and args.gpus != world:
        log(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a mislabelled number")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # read by libp2v when a workspace is created / by the HIP runtimes at initialisation: set
    # before anything touches the GPU
    if args.transcript != "auto":
        os.environ["P2V_TRANSCRIPT"] = args.transcript
    if args.single_stream:
        os.environ["P2V_SINGLE_STREAM"] = "1"
    if args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import torch.distributed as dist
    if world > 1:
        # stdout carries exactly one JSON line: the backends' own start-up chatter (gloo prints
        # its peer count to fd 1) goes to stderr
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            # the default group is gloo: the proofs shard with no data-path collective, and the bench's
            # only cross-rank operations (barriers, the max-over-ranks time, the per-rank figures) are
            # on CPU tensors, so RCCL initialisation is not a failure point of the multi-GPU run
            # (VERDICT r5 item 2); --dist-backend nccl adds the RCCL group and keeps gloo beside it
            backend = args.dist_backend if torch.cuda.is_available() else "gloo"
            dist.init_process_group(backend)
            cpu_grp = dist.group.WORLD if backend == "gloo" else dist.new_group(backend="gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    # one rank per GPU; ranks beyond the visible GPUs (gloo rehearsal only) share devices
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    import p2v
    build = p2v.check_build()   # refuse a libp2v.so built from other sources than this tree

    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    threads = host_threads(local_world)
    t0 = time.time()
    real = args.circuit == "real"
    arities = tuple(int(a) for a in args.arities.split(",") if a)
    gc, proofs = make_workload(args.degree_bits, args.distinct, args.witnesses, rank + 1, threads, args.lookups, real, args.ext, arities)
    log(f"[rank {rank}] generated {len(proofs)} distinct proofs in {time.time() - t0:.1f}s")
    vk = p2v.VerifierCircuitData.from_json(gc.common, gc.vkey, args.ext)
    info = vk.info
    packed = vk.pack_many(proofs)
    B = args.batch
    rows = np.ascontiguousarray(packed[np.arange(B) % len(proofs)])
    # 1/16 of the batch is corrupted: the GPU does the same work for them, and
    # the statuses of every timed batch are checked against the expected vector
    expect = mutate_batch(rows, info)
    dev = torch.device("cuda", local)
    lay_tiled = args.layout == "tiled"
    d_proofs = torch.from_numpy((p2v.tile_proofs(rows) if lay_tiled else rows).view(np.int64)).to(dev)
    d_expect = torch.from_numpy(expect).to(dev)
    nv = max(1, args.inflight)
    d_res = [torch.empty(B, dtype=torch.int8, device=dev) for _ in range(nv)]
    bvs = [p2v.BatchVerifier(vk, local, B) for _ in range(nv)]
    if args.stagger and nv > 1:   # workspace j's phase 1 follows workspace j-1's (cyclically)
        for j in range(nv):
            bvs[j].chain(bvs[j - 1])
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(nv - 1)]

    NPROBE = 256   # one-wave clock-probe workgroups (spread over every XCD)

    def timed(k, pipelined):
        """k steps; pipelined: batch i goes to workspace/stream i % nv without host sync, so
        up to nv batches are in flight (batch i+1's transcript overlaps batch i's Merkle
        work); serial: one workspace, synchronous, per-kernel times recorded.  Every step's
        statuses are compared with the expected vector on the device, on the launch's own stream,
        right after it (p2v_count_mismatches: a per-stream mismatch counter and check count), and
        a clock probe at each end of the pass gives the shader clock the chip held over it."""
        ktimes = {}
        # device-side clock of the same pass: one timing event per stream
        # before its first launch and one after every launch, on the launch's own stream
        nst = nv if pipelined else 1
        ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(nst)]
        ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(k)]
        cnt = torch.zeros((nst, 2), dtype=torch.int64, device=dev)   # per stream: mismatches, checks run
        stamps = torch.zeros((2, NPROBE, 3), dtype=torch.int64, device=dev)
        host_enq = []
        if world > 1:
            dist.barrier(group=cpu_grp)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for j in range(nst):
            ev0[j].record(streams[j])
        p2v.clock_probe(stamps[0].data_ptr(), NPROBE, streams[0].cuda_stream)
        for i in range(k):
            j = i % nv if pipelined else 0
            bvs[j].run_device(d_proofs.data_ptr(), B, d_res[j].data_ptr(), stream=streams[j].cuda_stream, sync=not pipelined,
                              tiled=lay_tiled, lookahead=bool(args.lookahead))
            p2v.count_mismatches(d_res[j].data_ptr(), d_expect.data_ptr(), B, cnt[j].data_ptr(), streams[j].cuda_stream)
            ev1[i].record(streams[j])
            host_enq.append(time.perf_counter() - t)
            if not pipelined:
                for name, v in bvs[0].last_timings().items():
                    ktimes.setdefault(name, []).append(v)
        for j in range(1, nst):
            streams[0].wait_stream(streams[j])
        p2v.clock_probe(stamps[1].data_ptr(), NPROBE, streams[0].cuda_stream)
        torch.cuda.synchronize(dev)
        own = time.perf_counter() - t   # this rank's own time, before the closing barrier
        if world > 1:
            dist.barrier(group=cpu_grp)
        dt = time.perf_counter() - t
        # completion time of every step on the device clock, from the first stream's start event
        done = [ev0[0].elapsed_time(e) for e in ev1]
        starts = [ev0[0].elapsed_time(e) for e in ev0]
        dev_ms = max(done) - min(starts)
        gaps = np.diff(np.array([min(starts)] + done))
        st = stamps.cpu().numpy().view(np.uint64)
        run_clock = p2v.clock_from_probes(st[0], st[1])
        c = cnt.cpu().numpy()
        check = {"steps": int(c[:, 1].sum()), "mismatches": int(c[:, 0].sum())}
        clock = {"host_ms": round(dt * 1e3, 3), "device_ms": round(dev_ms, 3),
                 "device_over_host": round(dev_ms / (dt * 1e3), 4),
                 "step_ms": {"mean": round(float(gaps.mean()), 4), "min": round(float(gaps.min()), 4),
                             "max": round(float(gaps.max()), 4), "std": round(float(gaps.std()), 4),
                             "first": [round(float(x), 4) for x in gaps[:4]], "last": [round(float(x), 4) for x in gaps[-4:]]},
                 "host_enqueue_ms": {"mean": round(float(np.mean(np.diff([0.0] + host_enq))) * 1e3, 4),
                                     "max": round(float(np.max(np.diff([0.0] + host_enq))) * 1e3, 4),
                                     "last_enqueued_at": round(host_enq[-1] * 1e3, 3)},
                 "run_clock": run_clock}
        return max_over_ranks(dt, world, cpu_grp), ktimes, clock, own, check

    # Order: the W warm-up steps run immediately before the headline
    # (pipelined) pass, with no host work between them, because the GPU's clock drops within
    # milliseconds of idling and takes ~35 ms of load to come back (profiles/r04b_*: a 15 ms
    # host gap before the pipelined pass cost its first pair of steps ~2 ms).  Statuses are
    # checked after the timed pass; torch's compare kernels are loaded here, before any timing.
    assert bool((d_res[0] == d_res[0]).all())
    for r in d_res:
        r.zero_()
    for i in range(args.warmup):
        bvs[i % nv].run_device(d_proofs.data_ptr(), B, d_res[i % nv].data_ptr(), stream=streams[i % nv].cuda_stream, sync=False,
                               tiled=lay_tiled, lookahead=bool(args.lookahead))
    if nv > 1:
        dt, _, clock, own, check = timed(args.steps, True)
        ok = all(bool((r == d_expect).all()) for r in d_res[:min(nv, args.steps)])
        for r in d_res:
            r.zero_()
    # serial pass: per-kernel durations (HIP events recorded on the run's streams inside libp2v)
    dt_serial, ktimes, clock_serial, own_serial, check_serial = timed(args.steps, False)
    if nv > 1:
        ok = ok and bool((d_res[0] == d_expect).all())
    else:
        dt, clock, own, check = dt_serial, clock_serial, own_serial, check_serial
        ok = bool((d_res[0] == d_expect).all())
    # every timed step of both passes checked on the device, on every rank
    ok = ok and check["mismatches"] == 0 and check["steps"] == args.steps
    ok = ok and check_serial["mismatches"] == 0 and check_serial["steps"] == args.steps
    ok = all(v > 0 for v in gather_over_ranks(1.0 if ok else 0.0, world, cpu_grp))
    verified_steps = int(min(gather_over_ranks(float(check["steps"] if check["mismatches"] == 0 else 0), world, cpu_grp)))
    run_clock = (clock.get("run_clock") or {}).get("clock_ghz")
    per_rank = per_rank_summary(B * args.steps, own, world, cpu_grp, run_clock)
    total = B * args.steps * world
    value = total / dt
    kavg = {k: float(np.mean(v)) for k, v in ktimes.items()}
    c5 = None
    if not args.quick and not args.no_c5:
        c5 = c5_leg(p2v, vk, info, d_proofs, d_expect, B, world, local, dev, cpu_grp, streams, lay_tiled,
                    stagger=args.stagger)
    c3 = None
    if world == 1 and not args.quick and not args.no_c3 and not args.lookups and real:
        c3 = c3_leg(p2v, args, threads, dev, local, streams)
    if rank == 0:
        kb = kernel_bytes_model(info, info.trace_words)
        # dominant kernel: the longest launch on the main stream (k_transcript / k_vanish / k_fri /
        # k_lut run on the side stream under k_leaf / k_merkle and do not set the step time)
        main_stream = [k for k in ("k_transpose", "k_phase1", "k_leaf", "k_merkle", "k_status") if k in kavg]
        dom = max(main_stream, key=kavg.get)
        achieved = kb[dom] * B / (kavg[dom] * 1e-3) / 1e9
        # HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes
        # (profiles/<tag>_pmc_traffic.json, corrected per MI355X_MICROARCH.md §HBM; the same tag
        # as valu.issue), as GB/s over this run's measured launch time; null if no PMC summary.
        traffic, traffic_bytes, ktable = None, None, None
        tag = pmc_tag()
        pmc = os.path.join(ROOT, "profiles", f"{tag}_pmc_traffic.json") if tag else ""
        if tag:
            try:
                pt = json.load(open(pmc))
                if real and info.degree_bits == 12 and not args.lookups and not args.ext and not arities:
                    ktable = kernel_traffic_table(pt, info, B)   # the PMC pass's own workload only
                traffic_bytes = sum(v for k, v in pt.items() if not k.startswith("_") and slot_of(k) == dom and isinstance(v, (int, float))) or None
                if traffic_bytes:
                    traffic_bytes = int(traffic_bytes * B / 4096)   # the PMC passes ran 4096-proof batches
                    traffic = round(traffic_bytes / (kavg[dom] * 1e-3) / 1e9, 2)
            except Exception:
                traffic = None
        ppp = perms_per_proof(info) + 114 + 1
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "proofs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64 (Goldilocks mod-p integer)", "data": "synthetic",
            "config": {"workload": f"{'C3' if args.lookups else 'C2'}: {B} std-config Plonky2 proofs per GPU per step (degree_bits {info.degree_bits}, "
                                   f"{'real circuit of the recursion gate set, ' if real else 'degenerate circuit, '}"
                                   f"28 FRI queries, {'arity bits ' + str(list(info.step_arity_bits)) if arities else 'arity 16'}, deg-2 ext{', lookups: 256 + 65536-entry tables' if args.lookups > 1 else (', lookups' if args.lookups else '')}), "
                                   f"{len(proofs)} distinct repeated, 1/16 corrupted, device-resident"
                                   f"{' in 64-proof tiles' if lay_tiled else ' proof-major'}",
                       "global_batch": B * world, "degree_bits": info.degree_bits, "parallelism": f"proof-sharded x{world}",
                       **({"ext": args.ext} if args.ext else {}),
                       "inflight": nv, "stagger": bool(args.stagger and nv > 1), "lookahead": bool(args.lookahead),
                       **({"transcript": args.transcript} if args.transcript != "auto" else {}),
                       **({"single_stream": True} if args.single_stream else {}),
                       **({"hw_queues": args.hw_queues} if args.hw_queues else {})},
            "clock": {**clock, "note": "the timed pass on the device clock: HIP events on each workspace stream (start before its "
                                       "first launch, one after every launch); step_ms = intervals between successive completions"},
            "serial": {"value": round(total / dt_serial, 1), "ms_per_step": round(dt_serial / args.steps * 1e3, 4),
                       "clock": clock_serial,
                       "note": "one batch at a time, host-synchronised per step; kernel_ms and roofline come from this pass"},
            # bound: the binding resource is the integer VALU issue rate (valu.issue, from the PMC
            # pass); achieved / peak / frac stay the HBM form the metric asks for
            "roofline": {"bound": "valu", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic,
                         "traffic_bytes_per_launch": traffic_bytes, "algorithmic_bytes_per_launch": kb[dom] * B,
                         "traffic_source": os.path.relpath(pmc, ROOT) if pmc else None,
                         "kernels": ktable,
                         "valu_issue_frac": None,
                         "note": "binding resource: integer VALU issue (Poseidon), valu_issue_frac = valu.issue.step_frac; "
                                 "achieved/peak/frac: the dominant kernel's algorithmic HBM bytes over its launch time"},
            "valu": {"perms_per_proof": ppp, "perm_rate_G": round(value / world * ppp / 1e9, 3),
                     "perms_note": "perms_per_proof counts every query path in full (the reference's work); the shared-node "
                                   "Merkle kernels hash each node several queries share once, ~86.6 % of the compressions "
                                   "(DESIGN.md 5.6), so perm_rate_G is reference-equivalent permutations/s",
                     "issue": valu_roofline(kavg, dt / args.steps * 1e3, B, run_clock)
                     if (real and info.degree_bits == 12 and not args.lookups and not args.ext and not arities) else None},   # the PMC pass's own workload only
            "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
            "verified_all": ok,
            "verified_steps": verified_steps,
            "verification": {"pipelined": check, "serial": check_serial,
                             "note": "every timed step's statuses compared with the expected vector on the device, on the "
                                     "launch's stream right after it (p2v_count_mismatches); steps = checks that ran, min over ranks"},
            "per_rank": per_rank,
            "build": {**build, "host_threads_per_rank": threads, "local_world": local_world},
        }
        if out["valu"]["issue"]:
            out["roofline"]["valu_issue_frac"] = out["valu"]["issue"]["step_frac"]
        if c5 is not None:
            out["c5"] = c5
        if c3 is not None:
            out["c3"] = c3
        if world == 1 and not args.quick and not args.no_host_legs:
            out["dropin"] = dropin_leg(p2v, gc, proofs, rows, expect, local)
            out["ingest"] = ingest_rate(vk, proofs, threads)
            out["h2d_end_to_end"] = h2d_rate(bvs, rows, B, expect, local=local)
            out["json_end_to_end"] = json_rate(bvs, proofs, B)
            out["bytes_end_to_end"] = bytes_rate(bvs, proofs, B, local=local)
        if world == 1 and not args.no_cpu_baseline and not args.quick and not args.no_host_legs:
            out["cpu_baseline"] = cpu_baseline(gc, proofs, threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
