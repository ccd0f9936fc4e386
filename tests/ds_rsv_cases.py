"""Clusters of reservations whose reserve pods hold GPU / RDMA instances, for DeviceShare's allocate-from-reservation
path (deviceshare/reservation.go:99-450) on the oracle and the GPU.  Every name a pod or a reservation holds beyond
cpu / memory has a resource id (the Reservation plugin reads them by name): the device resources too -- the node's
Allocatable / Requested of them (ke_node_resource rows), the reservations' allocatable (ke_reservation_resource
entries) and the pods' requests (ke_pod.xres)."""
import numpy as np

from koordinator_amd import abi, synth

GI = synth.GI
GPU_MEM = synth.GPU_MEM
# (device type, device key) -> resource id (synth.DEVICE_XRES; synth.XRES keeps 0..6)
KEY_ID = synth.DEVICE_KEY_XRES
PDR_ID = {abi.PDR["koordinator.sh/gpu-core"]: 10, abi.PDR["koordinator.sh/gpu-memory"]: 12,
          abi.PDR["koordinator.sh/gpu-memory-ratio"]: 11, abi.PDR["koordinator.sh/rdma"]: 13,
          abi.PDR["nvidia.com/gpu"]: 5}


def _used(d, j, k):
    return int(d["used"][j, k]) if d["has_used"][j, k] else 0


def _hold(d, j, amt, a, owner_amt=None):
    """the reserve pod's (and its owners') allocation on instance j: into the alloc record and the device cache"""
    ty, mi = int(d["type"][j]), int(d["minor"][j])
    bit = np.uint64(1) << np.uint64(16 * ty + mi)
    a["device_minors"] |= bit
    for k, v in enumerate(amt):
        a["device"][ty, mi, k] += v
        d["used"][j, k] = _used(d, j, k) + v
        d["has_used"][j, k] = 1
    if owner_amt is not None and any(owner_amt):
        a["owner_device_minors"] |= bit
        for k, v in enumerate(owner_amt):
            a["owner_device"][ty, mi, k] += v
            d["used"][j, k] += v


def make_ds_reservations(cl, devices, seed, n_groups=10, per_group=(2, 7), owner_fraction=0.5, policies=(0, 1, 2)):
    """Owner-grouped reservations on nodes with a device cache whose reserve pods hold a slice of one GPU (25 / 50 /
    100 % of core and memory), two whole GPUs, or an RDMA share next to either; owner pods hold part of the first
    instance on `owner_fraction` of them.  Mutates cl.nodes (NodeInfo Requested / pod count) and the device cache.
    Returns (reservations, allocs, resources, group per reservation)."""
    rng = np.random.default_rng(seed)
    nodes = [i for i in range(cl.n_nodes) if devices[i] is not None]
    rs, al, res, grp = [], [], [], []
    for g in range(n_groups):
        for _ in range(int(rng.integers(*per_group))):
            i = int(rng.choice(nodes))
            d = devices[i]
            r = np.zeros((), abi.RESERVATION_DTYPE)
            a = np.zeros((), abi.RESERVATION_ALLOC_DTYPE)
            r["node"], r["available"] = i, int(rng.random() < 0.95)
            r["allocate_once"] = int(rng.random() < 0.1)
            r["allocate_policy"] = int(rng.choice(policies))
            r["order"] = int(rng.choice([0, 0, 0, 5, 9, 3]))
            owners = rng.random() < owner_fraction
            r["allocated_pods"] = int(rng.integers(1, 3)) if owners else 0
            gpus = [j for j in range(len(d)) if d["type"][j] == abi.DEV_GPU and d["health"][j]]
            kind = rng.random()
            held = False
            if kind < 0.55:  # a slice of one GPU
                share = int(rng.choice([25, 50, 100]))
                cand = [j for j in gpus if _used(d, j, 0) <= 100 - share]
                if cand:
                    j = int(rng.choice(cand))
                    amt = [share, GPU_MEM * share // 100, share]
                    own = [share // 2, GPU_MEM * share // 200, share // 2] if owners and rng.random() < 0.7 else None
                    _hold(d, j, amt, a, own)
                    held = True
            else:  # two whole GPUs
                cand = [j for j in gpus if _used(d, j, 0) == 0]
                if len(cand) >= 2:
                    for q, j in enumerate(rng.choice(cand, 2, replace=False)):
                        own = [100, GPU_MEM, 100] if owners and q == 0 and rng.random() < 0.5 else None
                        _hold(d, int(j), [100, GPU_MEM, 100], a, own)
                    held = True
            if rng.random() < 0.3:  # an RDMA share
                rd = [j for j in range(len(d)) if d["type"][j] == abi.DEV_RDMA and _used(d, j, 0) <= 50]
                if rd:
                    j = int(rng.choice(rd))
                    _hold(d, j, [50], a, [25] if owners and rng.random() < 0.5 else None)
                    held = True
            if not held:
                continue
            r["holds"] = abi.RSV_HOLDS_DEVICES | abi.RSV_OTHER_ALLOCATABLE
            r["allocatable"][:] = [int(rng.choice([2000, 4000, 8000])), int(rng.choice([4, 8, 16])) * GI]
            if owners:
                r["allocated"][:] = [r["allocatable"][0] // 2, r["allocatable"][1] // 4]
            # the reservation's allocatable beyond cpu / memory: its device resources (the reserve pod's requests)
            e = synth.device_resource_entries(a)
            cl.nodes["requested"][i, 0] += r["allocatable"][0] + (r["allocated"][0] if owners else 0)
            cl.nodes["requested"][i, 1] += r["allocatable"][1] + (r["allocated"][1] if owners else 0)
            cl.nodes["pod_count"][i] += 1 + int(r["allocated_pods"])
            rs.append(r)
            al.append(a)
            res.append(e)
            grp.append(g)
    return (np.array(rs, abi.RESERVATION_DTYPE), np.array(al, abi.RESERVATION_ALLOC_DTYPE), res, np.array(grp))


def node_tables(cl, devices):
    """per node the ke_node_resource rows: cpu / memory, and the device resources' Allocatable (the healthy and
    unhealthy devices the node reports) and Requested (the device cache's used)"""
    tables = []
    for i in range(cl.n_nodes):
        rows = [(abi.XRES_CPU, int(cl.nodes["allocatable"][i, 0]), int(cl.nodes["requested"][i, 0])),
                (abi.XRES_MEMORY, int(cl.nodes["allocatable"][i, 1]), int(cl.nodes["requested"][i, 1]))]
        d = devices[i]
        if d is not None:
            for (ty, k), rid in KEY_ID.items():
                m = d["type"] == ty
                tot = int(d["total"][m, k].sum())
                used = int((d["used"][m, k] * d["has_used"][m, k]).sum())
                if tot:
                    rows.append((rid, tot, used))
        t = np.zeros(len(rows), abi.NODE_RESOURCE_DTYPE)
        for e, (rid, av, rq) in enumerate(rows):
            t[e]["id"], t[e]["allocatable"], t[e]["requested"] = rid, av, rq
        tables.append(t)
    return tables


def add_device_xres(pods):
    """ke_pod.xres entries of the device requests (the names PodRequests holds)"""
    for p in range(len(pods)):
        n = int(pods["n_xres"][p])
        for pdr, rid in PDR_ID.items():
            v = int(pods["device_requests"][p, pdr])
            if v > 0 and n < abi.MAX_POD_XRES:
                pods["xres_id"][p, n], pods["xres_value"][p, n] = rid, v
                pods["xres_request_mask"][p] |= 1 << rid
                n += 1
        pods["n_xres"][p] = n
    return pods


def setup(handles_factory, n, seed, n_pods, affinity=0.2, ignored=0.1, match=0.5, topology=True, strategy=None):
    """A cluster of n nodes (device caches, GPU topology), owner-grouped device-holding reservations, and a queue of
    DeviceShare pods (half of them) of which `match` are KE_RSV_MATCHED (or AFFINITY for `affinity` of those) with one
    group's reservations and `ignored` KE_RSV_IGNORED.  handles_factory(cfg, n) -> the handles to load.  Returns
    (handles, pods, matches, reservations)."""
    rng = np.random.default_rng(seed)
    cl = synth.make_cluster(n, synth.BASE_SEED + seed)
    devices = synth.make_devices(n, synth.BASE_SEED + seed + 1, no_cache_fraction=0.1)
    if topology:
        synth.add_gpu_topology(devices, synth.BASE_SEED + seed + 2)
    rs, al, res, grp = make_ds_reservations(cl, devices, synth.BASE_SEED + seed + 3)
    tables = node_tables(cl, devices)
    cfg = synth.config(n)
    if strategy is not None:
        cfg.deviceshare.strategy = strategy
    hs = handles_factory(cfg, n)
    for h in hs:
        synth.load_into(h, cl)
        synth.load_devices(h, devices)
        for i, t in enumerate(tables):
            h.set_resources(i, t)
        h.reservations_load(rs, al, res)
    pods = synth.make_ds_pods(n_pods, synth.BASE_SEED + seed + 4, device_fraction=0.6)
    pods = synth.add_pod_xres(pods, synth.BASE_SEED + seed + 5, gpu_fraction=0.0, storage_fraction=0.0,
                              scarce_fraction=0.0)
    pods = add_device_xres(pods)
    pods["numa_topology_policy"] = 0
    matches = [[] for _ in range(n_pods)]
    for p in range(n_pods):
        u = rng.random()
        if u < match:
            pods["reservation_matched"][p] = abi.RSV_AFFINITY if rng.random() < affinity else abi.RSV_MATCHED
            matches[p] = np.flatnonzero(grp == rng.integers(0, grp.max() + 1)).tolist()
            if pods["reservation_matched"][p] == abi.RSV_AFFINITY and rng.random() < 0.2:
                matches[p] = matches[p][:1]
        elif u < match + ignored:
            pods["reservation_matched"][p] = abi.RSV_IGNORED
    return hs, pods, matches, rs
