"""A cluster as the apiserver serves it: Node, NodeMetric, NodeResourceTopology and Device objects plus bound and
pending Pods, all JSON.  `ingest` runs every object through the product's decoders
(ke_decode_* over the C ABI) and replays the informer events a koord-scheduler would deliver into a cluster
handle (Evaluator or Oracle — the same calls):

  Node add            -> ke_decode_node, ke_decode_nrt (patches the NRT-side fields), ke_node_upsert,
                         ke_node_numa_set, ke_node_cpus_set
  NodeMetric add      -> ke_decode_node_metric, ke_nodemetric_upsert (absent NodeMetric: lister NotFound)
  Device add          -> ke_decode_device, ke_node_devices_set, ke_node_gpu_partitions
  Pod add (bound)     -> ke_decode_pod, ke_pod_assign at its PodScheduled time (pod_assign_cache.go:89-124),
                         NodeInfo.Requested += its requests (the framework's NodeInfo)
  Pod (pending)       -> ke_decode_pod -> the scheduling queue

Objects are generated from a seed with the shapes of BASELINE configs 3-5 (LoadAware metrics and thresholds,
NUMA zones with CPU topologies and policies, GPUs / RDMA with PCIe topology, LS/LSR/BE pods, cpuset and device
requests).  Nothing here computes a plugin result: the oracle and the product both consume the decoded structs.
"""
import json

import numpy as np

from koordinator_amd import abi, decode

T0 = 1_760_000_000  # seconds; every time below is relative to it
GI = 2**30


def ts(sec):
    """RFC 3339 of T0 + sec (UTC, whole seconds)."""
    import datetime
    return datetime.datetime.fromtimestamp(T0 + sec, datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _rl(cpu_m, mem):
    return {"cpu": f"{cpu_m}m", "memory": str(mem)}


def make_objects(n_nodes, n_bound, n_pending, seed, devices=True, numa=True):
    rng = np.random.default_rng(seed)
    nodes, metrics, nrts, devs = [], [], [], []
    for i in range(n_nodes):
        name = f"node-{i}"
        cpus = int(rng.choice([32, 64, 96, 128]))
        mem = int(rng.choice([128, 256, 512])) * GI
        labels, ann = {}, {}
        if numa and rng.random() < 0.5:
            labels["node.koordinator.sh/numa-topology-policy"] = str(rng.choice(["BestEffort", "Restricted",
                                                                                 "SingleNUMANode"]))
        if rng.random() < 0.15:
            ann["node.koordinator.sh/resource-amplification-ratio"] = json.dumps({"cpu": float(rng.choice([1.5, 2.0]))})
        if rng.random() < 0.1:
            ann["scheduling.koordinator.sh/usage-thresholds"] = json.dumps(
                {"usageThresholds": {"cpu": int(rng.integers(50, 90)), "memory": int(rng.integers(70, 95))}})
        if rng.random() < 0.1:
            ann["node.koordinator.sh/raw-allocatable"] = json.dumps({"cpu": str(cpus), "memory": f"{mem // GI}Gi"})
        nodes.append({"apiVersion": "v1", "kind": "Node",
                      "metadata": {"name": name, "labels": labels, "annotations": ann},
                      "status": {"allocatable": {"cpu": str(cpus), "memory": f"{mem // GI}Gi", "pods": "110"},
                                 "capacity": {"cpu": str(cpus), "memory": f"{mem // GI}Gi"}}})
        r = rng.random()
        if r < 0.96:
            up = -30 if r < 0.94 else -1_000_000
            nm = {"apiVersion": "slo.koordinator.sh/v1alpha1", "kind": "NodeMetric", "metadata": {"name": name},
                  "spec": {"metricCollectPolicy": {"reportIntervalSeconds": 60}},
                  "status": {"updateTime": ts(up), "nodeMetric": {"nodeUsage": {"resources": _rl(
                      int(rng.integers(0, cpus * 750)), int(rng.uniform(0.1, 0.8) * mem) // 2**20 * 2**20)}},
                             "podsMetric": []}}
            if rng.random() < 0.3:
                nm["status"]["nodeMetric"]["aggregatedNodeUsages"] = [
                    {"duration": "5m0s", "usage": {"p95": {"resources": _rl(int(rng.integers(0, cpus * 800)),
                                                                            int(0.5 * mem))}}}]
            metrics.append(nm)
        else:
            metrics.append(None)
        nrt = None
        if numa:
            nz = int(rng.choice([1, 2, 4]))
            tpc = 2
            cores = cpus // tpc
            rows = [{"id": c * tpc + t, "core": c, "socket": (c * nz // cores) * 2 // max(nz, 2) if nz > 1 else 0,
                     "node": c * nz // cores} for c in range(cores) for t in range(tpc)]
            nann = {"node.koordinator.sh/cpu-topology": json.dumps({"detail": rows})}
            if rng.random() < 0.2:
                nann["node.koordinator.sh/reservation"] = json.dumps({"reservedCPUs": "0-1"})
            zones = [{"name": f"node-{z}", "type": "Node", "resources": [
                {"name": "cpu", "capacity": str(cpus // nz), "allocatable": str(cpus // nz), "available": str(cpus // nz)},
                {"name": "memory", "capacity": str(mem // nz), "allocatable": str(mem // nz), "available": str(mem // nz)}]}
                for z in range(nz)]
            nrt = {"apiVersion": "topology.node.k8s.io/v1alpha1", "kind": "NodeResourceTopology",
                   "metadata": {"name": name, "annotations": nann}, "topologyPolicies": ["None"], "zones": zones}
        nrts.append(nrt)
        dev = None
        if devices and rng.random() < 0.6:
            gpu = {"koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory": "80Gi",
                   "koordinator.sh/gpu-memory-ratio": "100"}
            n_gpu = int(rng.choice([4, 8]))
            dl = [{"type": "gpu", "minor": m, "health": bool(rng.random() > 0.03), "resources": gpu,
                   "topology": {"socketID": 0, "nodeID": m * 2 // n_gpu, "pcieID": str(m // 2), "busID": f"0000:{m:02x}"}}
                  for m in range(n_gpu)]
            dl += [{"type": "rdma", "minor": m, "health": True, "resources": {"koordinator.sh/rdma": "100"},
                    "topology": {"socketID": 0, "nodeID": m, "pcieID": str(10 + m)}} for m in range(2)]
            dev = {"apiVersion": "scheduling.koordinator.sh/v1alpha1", "kind": "Device", "metadata": {"name": name},
                   "spec": {"devices": dl}}
        devs.append(dev)
    bound, pending = [], []
    for k in range(n_bound + n_pending):
        is_bound = k < n_bound
        kind = rng.random()
        labels, ann = {}, {}
        cpu = int(rng.choice([1, 2, 4, 8])) * 1000
        mem = int(rng.choice([2, 4, 8, 16])) * GI
        req = {"cpu": f"{cpu}m", "memory": f"{mem // GI}Gi"}
        lim = dict(req) if rng.random() < 0.5 else {"cpu": f"{2 * cpu}m", "memory": f"{2 * mem // GI}Gi"}
        if kind < 0.45:
            labels["koordinator.sh/qosClass"] = "LS"
        elif kind < 0.6 and not is_bound:
            labels["koordinator.sh/qosClass"] = str(rng.choice(["LSR", "LSE"]))
            labels["koordinator.sh/priority-class"] = "koord-prod"
            lim = dict(req)
            if rng.random() < 0.3:
                ann["scheduling.koordinator.sh/resource-spec"] = json.dumps(
                    {"preferredCPUBindPolicy": str(rng.choice(["FullPCPUs", "SpreadByPCPUs"]))})
        elif kind < 0.85:
            labels["koordinator.sh/qosClass"] = "BE"
            labels["koordinator.sh/priority-class"] = "koord-batch"
            req = {"kubernetes.io/batch-cpu": str(cpu), "kubernetes.io/batch-memory": f"{mem // GI}Gi"}
            lim = dict(req)
        if devices and not is_bound and rng.random() < 0.25:
            g = int(rng.choice([25, 50, 100, 200]))
            req["koordinator.sh/gpu-core"] = str(g)
            req["koordinator.sh/gpu-memory-ratio"] = str(g)
            lim["koordinator.sh/gpu-core"] = str(g)
            lim["koordinator.sh/gpu-memory-ratio"] = str(g)
            if rng.random() < 0.3:
                req["koordinator.sh/rdma"] = "100"
                lim["koordinator.sh/rdma"] = "100"
        if numa and not is_bound and rng.random() < 0.1:
            ann["scheduling.koordinator.sh/numa-topology-spec"] = json.dumps(
                {"numaTopologyPolicy": str(rng.choice(["BestEffort", "Restricted", "SingleNUMANode"]))})
        owner = "DaemonSet" if rng.random() < 0.02 else "ReplicaSet"
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": f"pod-{k}", "namespace": "wire", "uid": f"uid-{seed}-{k}", "labels": labels,
                            "annotations": ann, "ownerReferences": [{"kind": owner, "name": "o"}]},
               "spec": {"containers": [{"name": "c", "resources": {"requests": req, "limits": lim}}]},
               "status": {"phase": "Pending"}}
        if is_bound:
            node = int(rng.integers(0, n_nodes))
            pod["spec"]["nodeName"] = f"node-{node}"
            pod["status"] = {"phase": "Running", "conditions": [
                {"type": "PodScheduled", "status": "True", "lastTransitionTime": ts(-3600 - int(rng.integers(0, 600)))}]}
            nm = metrics[node]
            if nm is not None and rng.random() < 0.9:
                nm["status"]["podsMetric"].append(
                    {"namespace": "wire", "name": f"pod-{k}", "priority": labels.get("koordinator.sh/priority-class", ""),
                     "podUsage": {"resources": _rl(int(cpu * rng.uniform(0.1, 1.0)), int(mem * rng.uniform(0.1, 1.0)))}})
            bound.append(pod)
        else:
            pending.append(pod)
    return {"nodes": nodes, "nodemetrics": metrics, "nrts": nrts, "devices": devs, "bound": bound,
            "pending": pending}


def ingest(handles, objs, now_ns):
    """Decode every object and replay the informer events into each handle; returns the decoded pending pods
    (POD_DTYPE array, queue order)."""
    names = {o["metadata"]["name"]: i for i, o in enumerate(objs["nodes"])}
    n = len(objs["nodes"])
    requested = np.zeros((n, 2), np.int64)
    bound = []
    for p in objs["bound"]:
        d = decode.decode_pod(p)
        i = names[p["spec"]["nodeName"]]
        bound.append((i, d))
        requested[i] += [d.requests[abi.RES_CPU], d.requests[abi.RES_MEMORY]]
    for i, nd in enumerate(objs["nodes"]):
        node = decode.decode_node(nd)
        zones = cpus = None
        if objs["nrts"][i] is not None:
            zones, cpus = decode.decode_nrt(objs["nrts"][i], node)
        node.requested[:] = list(requested[i])
        nm = None
        if objs["nodemetrics"][i] is not None:
            nm = decode.decode_node_metric(objs["nodemetrics"][i])
        dev = None
        if objs["devices"][i] is not None:
            dev = decode.decode_device(objs["devices"][i])
        for h in handles:
            h.upsert_node(i, node)
            if zones is not None:
                h.set_numa(i, zones)
                if len(cpus):
                    h.set_cpus(i, cpus)
            if nm is not None:
                h.set_nodemetric(i, nm)
            else:
                h.delete_nodemetric(i)
            if dev is not None:
                devices, (has_table, honor, parts) = dev
                h.set_devices(i, devices)
                h.set_gpu_partitions(i, has_table, honor, parts)
    for i, d in bound:
        for h in handles:
            h.assign(i, d, int(d.scheduled_transition_ns))
    pods = np.zeros(len(objs["pending"]), abi.POD_DTYPE)
    for k, p in enumerate(objs["pending"]):
        d = decode.decode_pod(p)
        pods[k] = np.frombuffer(bytes(d), abi.POD_DTYPE)[0]
    return pods
