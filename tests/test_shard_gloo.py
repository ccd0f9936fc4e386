"""Multi-process (gloo, world_size 2, CPU) checks of the node-sharded protocol (koordinator_amd.shard):
every rank derives the same disjoint 512-aligned node partition, the RCCL unique id reaches every
rank through the control plane, and per-shard top-k_j candidate lists merged after an all-gather
equal the global top-k_j of the oracle's framework totals for every pod of a batch."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from koordinator_amd import shard, synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_nodes, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.binding import Oracle  # checker

        # 1. partition: disjoint, covering, aligned, identical on every rank
        lo, hi = shard.node_range(n_nodes, rank, world)
        ranges = [None] * world
        dist.all_gather_object(ranges, (lo, hi))
        # 2. unique-id exchange through the control plane (fake id: no device on CPU)
        uid = shard.exchange_unique_id(rank, lambda: bytes(range(128)))
        # 3. sharded candidate lists: this rank's range only, then all-gather + merge
        cl = synth.make_cluster(n_nodes, synth.BASE_SEED + 71)
        pods = synth.make_pods(64, synth.BASE_SEED + 72)
        cfg = synth.config(n_nodes)
        o = Oracle(cfg, n_nodes)
        synth.load_into(o, cl)
        total = o.eval(pods, synth.T0)["total"]
        keys = shard.make_keys(total[:, lo:hi], first_node=lo)
        mine = [shard.topk_keys(keys[j], j + 1) for j in range(len(pods))]
        allk = [None] * world
        dist.all_gather_object(allk, mine)
        full = shard.make_keys(total)
        ok = all(np.array_equal(shard.merge_candidate_lists([allk[r][j] for r in range(world)], j + 1),
                                shard.topk_keys(full[j], j + 1)) for j in range(len(pods)))
        out_q.put((rank, ranges, uid, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_protocol_gloo(world):
    n_nodes = 1700
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_nodes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    ranges = res[0][1]
    assert all(r[1] == ranges for r in res)
    assert ranges[0][0] == 0 and ranges[-1][1] == n_nodes
    for (a, b), (c, d) in zip(ranges, ranges[1:]):
        assert b == c and a % shard.SHARD_ALIGN == 0
    assert all(r[2] == bytes(range(128)) for r in res)
    assert all(r[3] for r in res), "merged per-shard top-k differs from the global top-k"


def test_node_range_edges():
    for n in (0, 1, 511, 512, 513, 50_000):
        for world in (1, 2, 3, 8):
            rs = [shard.node_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(b == c for (_, b), (c, _) in zip(rs, rs[1:]))
            assert all(lo % shard.SHARD_ALIGN == 0 or lo == n for lo, _ in rs)
