"""Node sharding across GPUs: one process per GPU, every rank a full replica of the node state.

The reference fans the per-node Filter/Score calls of one pod over 16 goroutines (upstream
Parallelizer, passed through at cmd/koord-scheduler/app/server.go:417).  Here the fan-out is over
GPUs: rank r evaluates the contiguous node range `node_range(N, r, world)`; per speculative batch
the ranks exchange their per-pod top-k_j candidate lists with one RCCL all-gather inside
libkoordeval (ke_shard_init / ke_schedule) and resolve the batch identically.  torch.distributed
(any backend; gloo is enough) is only the control plane: it broadcasts the RCCL unique id.
"""
import numpy as np

KEY_IDX_BITS = 23
KEY_IDX_MASK = (1 << KEY_IDX_BITS) - 1
SHARD_ALIGN = 512  # k_select reads 8 scores per lane with 16-B loads: ranges start 512-aligned


def node_range(n_nodes, rank, world):
    """[lo, hi) of shard `rank` (mirror of shard_range in ke_kernels.hip)."""
    chunk = ((n_nodes + world - 1) // world + SHARD_ALIGN - 1) // SHARD_ALIGN * SHARD_ALIGN
    lo = min(rank * chunk, n_nodes)
    return lo, min(lo + chunk, n_nodes)


def make_keys(total, first_node=0):
    """Packed candidate keys (ke_types.h make_key): higher is better, ties -> lowest node index."""
    total = np.asarray(total, np.int64)
    idx = first_node + np.arange(total.shape[-1], dtype=np.int64)
    key = ((total + 1) << KEY_IDX_BITS) | (KEY_IDX_MASK - idx)
    return np.where(total < 0, 0, key).astype(np.uint32)


def topk_keys(keys, k):
    """The k largest non-zero keys, best first."""
    keys = np.asarray(keys, np.uint32)
    keys = keys[keys != 0]
    return np.sort(keys)[::-1][:k]


def merge_candidate_lists(lists, k):
    """Global top-k of the union of per-shard top-k lists (what k_merge computes on the device)."""
    return topk_keys(np.concatenate([np.asarray(x, np.uint32) for x in lists] or [np.zeros(0, np.uint32)]), k)


def exchange_unique_id(rank, make_id, group=None):
    """Rank 0 creates the RCCL unique id, every rank returns the same bytes."""
    import torch.distributed as dist

    obj = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def init_node_sharding(ev, rank, world, group=None):
    """Collective: give Evaluator `ev` its shard of a `world`-rank job (one process per GPU)."""
    from .evaluator import comm_unique_id

    if world == 1:
        ev.shard_init(0, 1, None)
        return
    uid = exchange_unique_id(rank, lambda: comm_unique_id(ev.lib), group)
    ev.shard_init(rank, world, uid)


def gloo_collective(group=None):
    """A host collective for Evaluator.shard_init_host over a torch.distributed process group (gloo: CPU
    tensors): all-gather of uint32 words (as int32 bits), all-reduce MAX / MIN of 32 / 64-bit integers (as int64;
    the library's 64-bit words stay below 2^63)."""
    import torch
    import torch.distributed as dist

    def collective(op, dt, send, world):
        if op == 0:  # all-gather, rank-major
            t = torch.from_numpy(send.view(np.int32).copy())
            outs = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(outs, t, group=group)
            return np.concatenate([o.numpy() for o in outs]).view(np.int32).view(dt)
        if dt == np.uint64 and (send >> np.uint64(63)).any():
            raise ValueError("64-bit word beyond int64")
        t = torch.from_numpy(send.astype(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == 1 else dist.ReduceOp.MIN, group=group)
        return t.numpy().astype(dt)

    return collective
