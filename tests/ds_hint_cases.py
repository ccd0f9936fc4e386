"""Builds the DeviceShare hint golden cases (tests/golden/ds_hints.json) on a cluster handle (Oracle or Evaluator):
the case's Device object through the product's decoder (ke_decode_device), its flags, an assigned pod's device
usage, and the pod with its DeviceAllocateHints / DeviceJointAllocate record."""
import numpy as np

import cases
from koordinator_amd import abi, decode, model

HINTS = cases.load("ds_hints.json")
GPU_RES = {"koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory": "80Gi", "koordinator.sh/gpu-memory-ratio": "100"}


def vf_rank(device_cr, minor, bus):
    d = [x for x in device_cr["spec"]["devices"] if x["type"] == "rdma" and x["minor"] == minor][0]
    buses = sorted(v["busID"] for g in d.get("vfGroups", []) for v in g["vfs"])
    return buses.index(bus)


def build(h, case, node=0):
    devs, (has_table, honor, parts) = decode.decode_device(case["device"])
    devs = devs.copy()
    a = case.get("assigned")
    if a:  # an assigned pod's allocations (the pod informer's updateCacheUsed)
        for d in devs:
            if d["type"] == abi.DEV_GPU and d["minor"] in a["gpu"]:
                d["has_used"][:] = d["has_total"]
                d["used"][:] = d["total"]
            for m, bus in a["rdma"]:
                if d["type"] == abi.DEV_RDMA and d["minor"] == m:
                    d["has_used"][0], d["used"][0] = 1, 1
                    d["vf_allocated"] |= np.uint64(1 << vf_rank(case["device"], m, bus))
    h.set_devices(node, devs)
    h.set_gpu_partitions(node, has_table, honor, parts)
    h.set_device_flags(node, case.get("secondary_well_planned", False), 0)


def pod_and_hints(case, index=1):
    pod = model.make_pod(requests=case["requests"])
    hint = model.make_device_hints(case.get("hints"), case.get("joint"))
    pod.device_hint = index
    return pod, hint


def node_cluster(h, n=1):
    for i in range(n):
        h.upsert_node(i, model.make_node(allocatable={"cpu": "96", "memory": "512Gi"}))


# ---- randomized clusters for the GPU-vs-oracle comparison ------------------------------------------------------
LABEL_TYPES = ["fakeW", "fakeS", "fast", None]


def random_device_cr(rng, n_gpu=8, n_rdma=4, vf_fraction=0.7):
    devs = []
    for m in range(n_gpu):
        devs.append({"type": "gpu", "minor": m, "health": bool(rng.random() > 0.02), "resources": GPU_RES,
                     "labels": {"model": str(rng.choice(["A100", "H100"]))} if rng.random() < 0.3 else {},
                     "topology": {"socketID": m * 2 // n_gpu, "nodeID": m * 2 // n_gpu, "pcieID": str(m // 2)}})
    for k in range(n_rdma):
        m = k + 1
        lt = LABEL_TYPES[int(rng.integers(0, len(LABEL_TYPES)))]
        d = {"type": "rdma", "minor": m, "health": True, "resources": {"koordinator.sh/rdma": "100"},
             "labels": {"type": lt} if lt else {},
             "topology": {"socketID": k * 2 // n_rdma, "nodeID": k * 2 // n_rdma, "pcieID": str(k * n_gpu // 2 // n_rdma)}}
        if rng.random() < vf_fraction:
            groups = []
            for g in range(int(rng.integers(1, 3))):
                groups.append({"labels": {"type": str(rng.choice(["general", "fakeG", "fakeC"]))},
                               "vfs": [{"minor": v, "busID": f"0000:{16 * m + g:02x}:{v // 8:02x}.{v % 8}"}
                                       for v in range(int(rng.integers(2, 9)))]})
            d["vfGroups"] = groups
        devs.append(d)
    return {"metadata": {"name": "n"}, "spec": {"devices": devs}}


def random_hint_pod(rng):
    """(requests, DeviceAllocateHints, DeviceJointAllocate) drawn over the modelled hint space"""
    req, hints, joint = {}, {}, None
    g = int(rng.choice([0, 1, 1, 2, 4, 8]))
    if g:
        req["nvidia.com/gpu"] = str(g)
    kind = rng.random()
    rdma = {}
    if kind < 0.35:
        req["koordinator.sh/rdma"] = "1"
        rdma["vfSelector"] = {"matchExpressions": [{"key": "type", "operator": "In",
                                                    "values": ["general", str(rng.choice(["fakeG", "fakeC"]))]}]}
    elif kind < 0.5:
        req["koordinator.sh/rdma"] = "1"
        rdma["allocateStrategy"] = "ApplyForAll"
    elif kind < 0.65:
        req["koordinator.sh/rdma"] = str(int(rng.integers(1, 4)))
        rdma["allocateStrategy"] = "RequestsAsCount"
        if rng.random() < 0.5:
            rdma["exclusivePolicy"] = "DeviceLevel"
    else:
        req["koordinator.sh/rdma"] = str(int(rng.choice([50, 100, 200])))
    if rng.random() < 0.6:
        rdma["selector"] = rng.choice([{"matchLabels": {"type": "fakeW"}},
                                       {"matchExpressions": [{"key": "type", "operator": "Exists"}]},
                                       {"matchExpressions": [{"key": "type", "operator": "NotIn", "values": ["fakeS"]}]}])
    hints["rdma"] = rdma
    if g and rng.random() < 0.3:
        hints["gpu"] = {"selector": {"matchExpressions": [{"key": "model", "operator": "DoesNotExist"}]}}
    if g and rng.random() < 0.6:
        joint = {"deviceTypes": ["gpu", "rdma"]}
        if rng.random() < 0.4:
            joint["requiredScope"] = "SamePCIe"
    return req, hints, joint


def random_hint_queue(rng, n, key_base):
    pods, table = [], []
    for i in range(n):
        req, hints, joint = random_hint_pod(rng)
        req["cpu"] = str(int(rng.choice([1, 2, 4])))
        req["memory"] = f"{int(rng.choice([2, 4, 8]))}Gi"
        p = model.make_pod(name=f"h{key_base + i}", requests=req)
        p.uid = key_base + i
        table.append(model.make_device_hints(hints, joint))
        p.device_hint = len(table)
        pods.append(p)
    return pods, table
