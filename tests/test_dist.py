"""Multi-process sharding (gloo, world_size 2, CPU): the proof-sharding and result
gathering used for N GPUs (embarrassingly parallel, no data-path
collective).  The per-shard verification here is the ORACLE (CPU) so the test runs
without a GPU; on GPUs each rank runs libp2v on its own device.  The second test drives the
product's own p2v.verify_sharded (packing, shard bounds, padded all_gather) with the ORACLE
injected as the per-shard verifier."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from support import gen_circuit, oracle, p2v_module


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, proofs, common, vkey, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p2v = p2v_module()
    s, e = p2v.shard_bounds(len(proofs), world, rank)
    O = oracle()
    local = [O.verify_json(common, vkey, proofs[i]) for i in range(s, e)]
    parts = [None] * world
    dist.all_gather_object(parts, local)
    flat = [x for p in parts for x in p]
    if rank == 0:
        out.put(flat)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover_exactly():
    p2v = p2v_module()
    for n in (0, 1, 7, 64, 4097):
        for w in (1, 2, 3, 8):
            spans = [p2v.shard_bounds(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gloo_sharded_verification():
    gc = gen_circuit(6, 4, 0)
    proofs = [gc.proof(1, 1), gc.proof(1, 5, flags=2), gc.proof(2, 2), gc.proof(1, 4, flags=1), gc.proof(2, 3)]
    expect = [oracle().verify_json(gc.common, gc.vkey, p) for p in proofs]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, proofs, gc.common, gc.vkey, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == expect == [1, 0, 1, -3, 1]


def _worker_product(rank, world, port, proofs, common, vkey, out, side=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    side_grp = dist.new_group(backend="gloo") if side else None
    p2v = p2v_module()
    vk = p2v.VerifierCircuitData.from_json(common, vkey)   # host-only: no GPU needed
    packed = vk.pack_many(proofs)
    O = oracle()
    seen = []

    def shard(rows, s, e):
        assert rows.shape[0] == e - s and np.array_equal(rows, packed[s:e])
        seen.append((s, e))
        return np.array([O.verify_json(common, vkey, proofs[i]) for i in range(s, e)], dtype=np.int8)
    got = p2v.verify_sharded(vk, packed, rank, world, 0, verify_shard=shard, gather_group=side_grp)
    out.put((rank, seen, got.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,side", [(2, False), (3, False), (2, True)])
def test_product_verify_sharded_gather_gloo(world, side):
    """p2v.verify_sharded itself (the per-rank path of bench.py / multi-GPU hosts) on gloo:
    every rank verifies exactly its contiguous shard, and every rank ends with the full status
    vector in batch order (uneven shards: 7 proofs over 2 or 3 ranks)."""
    gc = gen_circuit(6, 4, 0)
    kinds = [(1, 1, 0), (1, 5, 2), (2, 2, 0), (1, 4, 1), (2, 3, 0), (1, 6, 4), (2, 9, 0)]
    proofs = [gc.proof(w, s, flags=f) for w, s, f in kinds]
    expect = [oracle().verify_json(gc.common, gc.vkey, p) for p in proofs]
    assert expect == [1, 0, 1, -3, 1, 0, 1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_product, args=(r, world, port, proofs, gc.common, gc.vkey, q, side)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    p2v = p2v_module()
    for rank, seen, got in res:
        assert seen == [p2v.shard_bounds(len(proofs), world, rank)]
        assert got == expect


def _worker_max(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.new_group(backend="gloo")
    dist.barrier(group=grp)
    out.put((rank, bench.max_over_ranks(0.5 + rank, world, grp)))
    dist.destroy_process_group()


def test_bench_max_over_ranks_on_gloo_side_group():
    """bench.py's step time is the slowest rank's, reduced over a gloo side group on CPU
    tensors (the 8-GPU run needs no RCCL call for its number): 3 ranks timing 0.5 / 1.5 /
    2.5 s all report 2.5 s."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_max, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(3))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [v for _, v in res] == [2.5, 2.5, 2.5]


def _worker_per_rank(rank, world, port, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.new_group(backend="gloo")
    # rank r verified 4096 proofs in (1 + r) seconds at a shader clock of 2.0 + 0.1 r GHz
    summ = bench.per_rank_summary(4096, 1.0 + rank, world, grp, clock_ghz=2.0 + 0.1 * rank)
    out.put((rank, summ, bench.gather_over_ranks(float(rank), world, grp)))
    dist.barrier(group=grp)
    dist.destroy_process_group()


def test_bench_per_rank_summary_on_gloo_side_group():
    """the bench reports every rank's own throughput (its proofs over its own
    time before the closing barrier), min / max, the imbalance and every rank's shader clock, all
    gathered over the gloo side group; every rank holds the same summary, in rank order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_per_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(2)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, summ, ranks in res:
        assert ranks == [0.0, 1.0]
        assert summ["proofs_per_s"] == [4096.0, 2048.0]
        assert summ["min"] == 2048.0 and summ["max"] == 4096.0
        assert summ["imbalance"] == 0.5
        assert summ["clock_ghz"] == [2.0, 2.1]


def test_bench_host_threads_shared_by_local_ranks(monkeypatch):
    """each rank's host threads are the cores this process may use -- the
    affinity mask, capped by the cgroup CPU quota -- divided among the node's ranks, at most 16.
    On the GPU box the mask shows 256 CPUs and the quota grants 16 cores: one rank gets 16
    threads, each of 8 ranks gets 2 (not 16 each, 128 in all)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(bench, "cpu_quota_cores", lambda: 16.0)
    assert [bench.host_threads(w) for w in (1, 2, 4, 8)] == [16, 8, 4, 2]
    assert bench.host_threads(32) == 1
    monkeypatch.setattr(bench, "cpu_quota_cores", lambda: None)   # no quota: the mask
    assert [bench.host_threads(w) for w in (1, 8)] == [16, 16]
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)))
    assert [bench.host_threads(w) for w in (1, 2, 8, 16)] == [8, 4, 1, 1]
    monkeypatch.setattr(bench, "cpu_quota_cores", lambda: 2.5)   # a fractional quota rounds to the nearest core
    assert bench.host_threads(1) == 3


def _worker_default_group(rank, world, port, out):
    """bench.py's process-group setup path: the default group is gloo and is the side group."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.group.WORLD
    out.put((rank, dist.get_backend(), bench.max_over_ranks(1.0 + rank, world, grp),
             bench.gather_over_ranks(float(rank), world, grp)))
    dist.barrier(group=grp)
    dist.destroy_process_group()


def test_bench_default_group_is_gloo():
    """the bench's default process group is gloo (--dist-backend default), and
    its cross-rank operations run on it directly -- no RCCL group is created for the number."""
    import inspect
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    src = inspect.getsource(bench.main)
    assert 'ap.add_argument("--dist-backend", default="gloo"' in src
    assert 'dist.group.WORLD if backend == "gloo"' in src
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_worker_default_group, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, backend, mx, ranks in res:
        assert backend == "gloo" and mx == 4.0 and ranks == [0.0, 1.0, 2.0, 3.0]
