"""Synthetic clusters for the bench and the parity tests (BASELINE.md "CPU baseline plan").

Seeds: 20251015 + config id.  Quantities are exact integers (cpu in milli, memory a multiple of 1 MiB)
so that resource.Quantity rounding never enters.  Node mix: allocatable cpu {32,64,96,128} cores,
memory {128,256,512,1024} GiB; NodeMetric 96% fresh (t0-30s) / 2% expired (t0-1e6 s) / 2% absent with
NodeMetricExpirationSeconds = 3600; NodeUsage cpu ~ U[0, .75 alloc], memory ~ U[.1, .9] alloc; 30% of
nodes carry a 5-minute p95 AggregatedUsage; 10% carry custom usage thresholds; U{0..20} pre-existing
pods per node with PodMetrics and PodScheduled at t0-3600s (never "estimated").  Pod queue: 60% LS
koord-prod, 38% BE koord-batch, 2% DaemonSet-owned.
"""
from dataclasses import dataclass

import numpy as np

from . import abi, model

BASE_SEED = 20251015
NS = 1_000_000_000
GI = 1 << 30
MI = 1 << 20
T0 = 1_760_000_000 * NS  # "now" of the synthetic cluster

CONFIGS = {
    1: dict(nodes=1_000, pods=1_000, name="1k nodes x 1k pods, LoadAwareScheduling + NodeNUMAResource"),
    2: dict(nodes=5_000, pods=10_000, name="5k nodes x 10k pods, mixed LS/BE with NodeMetric usage"),
    3: dict(nodes=50_000, pods=100_000, name="50k nodes x 100k pods"),
    5: dict(nodes=20_000, pods=20_000, name="20k nodes x 8 GPU + 2 RDMA, DeviceShare partial-device pods"),
}


@dataclass
class Cluster:
    n_nodes: int
    nodes: np.ndarray          # NODE_DTYPE
    nm: np.ndarray             # NODE_METRIC_DTYPE
    has_nm: np.ndarray         # bool: NodeMetric exists (lister Get succeeds)
    pm_offsets: np.ndarray
    pod_metrics: np.ndarray    # POD_METRIC_DTYPE
    agg_offsets: np.ndarray
    aggregated: np.ndarray     # AGG_DTYPE
    asg_nodes: np.ndarray      # int32
    asg_pods: np.ndarray       # POD_DTYPE
    asg_ts: np.ndarray         # int64
    now: int = T0


def config(node_capacity, pod_batch=64, global_node_offset=0, device_ordinal=0):
    """bench args: v1beta3 defaults except NodeMetricExpirationSeconds = 3600."""
    cfg = abi.default_config(node_capacity, pod_batch=pod_batch, device_ordinal=device_ordinal,
                             global_node_offset=global_node_offset)
    cfg.loadaware.node_metric_expiration_seconds = 3600
    return cfg


def _rmap_fill(arr, cpu, mem, n_keys=2):
    arr["value"][:, 0] = cpu
    arr["value"][:, 1] = mem
    arr["present"][:, 0] = 1
    arr["present"][:, 1] = 1
    arr["n_keys"] = n_keys


def make_cluster(n_nodes, seed, amplified_fraction=0.0, max_pods_per_node=20, key_base=1_000_000):
    rng = np.random.default_rng(seed)
    N = n_nodes
    nodes = np.zeros(N, abi.NODE_DTYPE)
    cpu_cores = rng.choice([32, 64, 96, 128], N)
    mem_gib = rng.choice([128, 256, 512, 1024], N)
    nodes["allocatable"][:, 0] = cpu_cores * 1000
    nodes["allocatable"][:, 1] = mem_gib * GI
    nodes["raw_allocatable"][:] = abi.ABSENT
    nodes["cpu_amplification_ratio"] = -1.0
    nodes["nrt_cpu_amplification_ratio"] = -2.0
    for f in ("custom_usage_thresholds", "custom_prod_usage_thresholds", "custom_agg_thresholds"):
        nodes[f][:] = abi.ABSENT
    custom = rng.random(N) < 0.10
    nodes["has_custom_thresholds"][custom] = 1
    nodes["custom_usage_thresholds"][custom, 0] = rng.choice([50, 60, 70, 80], custom.sum())
    nodes["custom_usage_thresholds"][custom, 1] = rng.choice([80, 90, 95], custom.sum())
    if amplified_fraction > 0:
        amp = rng.random(N) < amplified_fraction
        ratio = rng.choice([1.5, 2.0, 2.5], amp.sum())
        nodes["cpu_amplification_ratio"][amp] = ratio
        nodes["raw_allocatable"][amp, 0] = nodes["allocatable"][amp, 0]
        nodes["allocatable"][amp, 0] = np.ceil(nodes["allocatable"][amp, 0] * ratio).astype(np.int64)
        nodes["cpuset_allocated_cpus"][amp] = rng.integers(0, 8, amp.sum()) * 2

    # NodeMetric headers
    kind = rng.random(N)
    has_nm = kind < 0.98
    expired = (kind >= 0.96) & has_nm
    nm = np.zeros(N, abi.NODE_METRIC_DTYPE)
    nm["has_update_time"] = 1
    nm["update_time_ns"] = np.where(expired, T0 - 10**6 * NS, T0 - 30 * NS)
    nm["report_interval_seconds"] = 60
    nm["has_node_metric"] = 1
    alloc_cpu = nodes["allocatable"][:, 0]
    alloc_mem = nodes["allocatable"][:, 1]
    use_cpu = (rng.random(N) * 0.75 * alloc_cpu).astype(np.int64)
    use_mem = ((0.1 + 0.8 * rng.random(N)) * alloc_mem).astype(np.int64) // MI * MI
    _rmap_fill(nm["node_usage"], use_cpu, use_mem)

    # aggregated usages: 30% carry a 5-minute p95
    has_agg = rng.random(N) < 0.30
    n_agg = has_agg.astype(np.int64)
    agg_offsets = np.zeros(N + 1, np.int64)
    agg_offsets[1:] = np.cumsum(n_agg)
    aggregated = np.zeros(int(agg_offsets[-1]), abi.AGG_DTYPE)
    aggregated["duration_ns"] = 300 * NS
    idx = np.nonzero(has_agg)[0]
    p95 = aggregated["usage"][:, abi.AGG_P95]
    _rmap_fill(p95, np.minimum(alloc_cpu[idx], (use_cpu[idx] * 1.1).astype(np.int64)),
               np.minimum(alloc_mem[idx], use_mem[idx] + 4 * GI))
    aggregated["usage"][:, abi.AGG_P95] = p95

    # pre-existing pods + their pod metrics
    per_node = rng.integers(0, max_pods_per_node + 1, N)
    P0 = int(per_node.sum())
    asg_nodes = np.repeat(np.arange(N, dtype=np.int32), per_node)
    asg = np.zeros(P0, abi.POD_DTYPE)
    asg["pod_key"] = key_base + np.arange(P0)
    asg["uid"] = key_base + np.arange(P0)
    prod = rng.random(P0) < 0.6
    req_cpu = rng.choice([500, 1000, 2000, 4000], P0)
    req_mem = rng.choice([1, 2, 4, 8], P0) * GI
    asg["requests"][prod, abi.RES_CPU] = req_cpu[prod]
    asg["requests"][prod, abi.RES_MEMORY] = req_mem[prod]
    asg["limits"][prod, abi.RES_CPU] = req_cpu[prod]
    asg["limits"][prod, abi.RES_MEMORY] = req_mem[prod]
    asg["requests"][~prod, abi.RES_BATCH_CPU] = req_cpu[~prod]
    asg["requests"][~prod, abi.RES_BATCH_MEMORY] = req_mem[~prod]
    asg["priority_class"] = np.where(prod, abi.PRIORITY_PROD, abi.PRIORITY_BATCH)
    asg["qos_class"] = np.where(prod, abi.QOS_LS, abi.QOS_BE)
    asg["custom_scaling_factors"][:] = abi.ABSENT
    asg["custom_seconds_after_scheduled"] = abi.ABSENT
    asg["custom_seconds_after_initialized"] = abi.ABSENT
    asg["has_scheduled"] = 1
    asg["scheduled_transition_ns"] = T0 - 3600 * NS
    asg_ts = np.full(P0, T0 - 3600 * NS, np.int64)
    # NodeInfo.Requested = Σ requests of the pods on the node (cpu/memory); len(NodeInfo.Pods); kubelet's
    # default max-pods as AllowedPodNumber (NodeResourcesFit's Filter)
    nodes["pod_count"] = per_node
    nodes["allowed_pods"] = 110
    np.add.at(nodes["requested"][:, 0], asg_nodes, asg["requests"][:, abi.RES_CPU])
    np.add.at(nodes["requested"][:, 1], asg_nodes, asg["requests"][:, abi.RES_MEMORY])
    # pod metrics (only nodes that have a NodeMetric)
    pm_mask = has_nm[asg_nodes]
    pm_per_node = np.bincount(asg_nodes[pm_mask], minlength=N)
    pm_offsets = np.zeros(N + 1, np.int64)
    pm_offsets[1:] = np.cumsum(pm_per_node)
    pms = np.zeros(int(pm_mask.sum()), abi.POD_METRIC_DTYPE)
    pms["pod_key"] = asg["pod_key"][pm_mask]
    pms["priority_class"] = asg["priority_class"][pm_mask]
    frac = rng.random(len(pms))
    pcpu = np.where(prod[pm_mask], req_cpu[pm_mask], req_cpu[pm_mask])
    _rmap_fill(pms["usage"], (pcpu * frac).astype(np.int64), (req_mem[pm_mask] * frac).astype(np.int64) // MI * MI)
    return Cluster(N, nodes, nm, has_nm, pm_offsets, pms, agg_offsets, aggregated, asg_nodes, asg, asg_ts)


def make_pods(n_pods, seed, key_base=1_000_000_000):
    """The pending-pod queue: 60% LS koord-prod, 38% BE koord-batch, 2% DaemonSet-owned."""
    rng = np.random.default_rng(seed)
    P = n_pods
    pods = np.zeros(P, abi.POD_DTYPE)
    pods["pod_key"] = key_base + np.arange(P)
    pods["uid"] = key_base + np.arange(P)
    u = rng.random(P)
    ls = u < 0.60
    be = (u >= 0.60) & (u < 0.98)
    ds = u >= 0.98
    cpu = rng.choice([1, 2, 4, 8], P) * 1000
    mem = rng.choice([2, 4, 8, 16], P) * GI
    lim_mult = rng.choice([1, 2], P)
    pods["requests"][ls | ds, abi.RES_CPU] = cpu[ls | ds]
    pods["requests"][ls | ds, abi.RES_MEMORY] = mem[ls | ds]
    pods["limits"][ls | ds, abi.RES_CPU] = (cpu * lim_mult)[ls | ds]
    pods["limits"][ls | ds, abi.RES_MEMORY] = (mem * lim_mult)[ls | ds]
    bcpu = rng.integers(1, 9, P) * 1000
    bmem = rng.integers(1, 9, P) * GI
    pods["requests"][be, abi.RES_BATCH_CPU] = bcpu[be]
    pods["requests"][be, abi.RES_BATCH_MEMORY] = bmem[be]
    pods["limits"][be, abi.RES_BATCH_CPU] = bcpu[be]
    pods["limits"][be, abi.RES_BATCH_MEMORY] = bmem[be]
    pods["priority_class"] = np.where(be, abi.PRIORITY_BATCH, abi.PRIORITY_PROD)
    pods["qos_class"] = np.where(be, abi.QOS_BE, abi.QOS_LS)
    pods["is_daemonset"] = ds.astype(np.uint8)
    pods["custom_scaling_factors"][:] = abi.ABSENT
    pods["custom_seconds_after_scheduled"] = abi.ABSENT
    pods["gpu_ring_bus_bandwidth"] = abi.ABSENT
    pods["custom_seconds_after_initialized"] = abi.ABSENT
    return pods


def load_into(handle, cl):
    """Ingest a synthetic cluster into an Evaluator or an Oracle (same informer-event calls)."""
    handle.nodes_load(cl.nodes)
    hm = np.nonzero(cl.has_nm)[0]
    # nodemetrics_load covers [0, N): load all, then delete the absent ones (lister NotFound)
    handle.nodemetrics_load(cl.nm, cl.pm_offsets, cl.pod_metrics, cl.agg_offsets, cl.aggregated)
    for i in np.nonzero(~cl.has_nm)[0]:
        handle.delete_nodemetric(int(i))
    handle.assign_bulk(cl.asg_nodes, cl.asg_pods, cl.asg_ts)
    return len(hm)


def shard(cl, rank, world):
    """Contiguous node shard [rank*N/world, (rank+1)*N/world) of a cluster."""
    N = cl.n_nodes
    lo, hi = rank * N // world, (rank + 1) * N // world
    pm0, pm1 = cl.pm_offsets[lo], cl.pm_offsets[hi]
    ag0, ag1 = cl.agg_offsets[lo], cl.agg_offsets[hi]
    am = (cl.asg_nodes >= lo) & (cl.asg_nodes < hi)
    return lo, Cluster(hi - lo, cl.nodes[lo:hi].copy(), cl.nm[lo:hi].copy(), cl.has_nm[lo:hi].copy(),
                       cl.pm_offsets[lo:hi + 1] - pm0, cl.pod_metrics[pm0:pm1].copy(),
                       cl.agg_offsets[lo:hi + 1] - ag0, cl.aggregated[ag0:ag1].copy(),
                       (cl.asg_nodes[am] - lo).astype(np.int32), cl.asg_pods[am].copy(), cl.asg_ts[am].copy(), cl.now)


# ---- DeviceShare (BASELINE config 5) -------------------------------------------------------------
GPU_MEM = 192 * GI


def make_devices(n_nodes, seed, gpus=8, rdmas=2, no_cache_fraction=0.05, unhealthy_fraction=0.02):
    """Per node a DeviceShare cache entry (or None): `gpus` GPUs (gpu-core 100, gpu-memory-ratio 100,
    gpu-memory 192Gi) and `rdmas` RDMA NICs (rdma 100) with random partial usage."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_nodes):
        if rng.random() < no_cache_fraction:
            out.append(None)
            continue
        devs = np.zeros(gpus + rdmas, abi.DEVICE_DTYPE)
        frac = rng.choice([0, 0, 0, 25, 50, 75, 100], gpus)
        for m in range(gpus):
            d = devs[m]
            d["type"], d["minor"] = abi.DEV_GPU, m
            d["health"] = 0 if rng.random() < unhealthy_fraction else 1
            d["has_total"][:] = 1
            d["total"][:] = [100, GPU_MEM, 100]
            if frac[m]:
                d["has_used"][:] = 1
                d["used"][:] = [frac[m], GPU_MEM * frac[m] // 100, frac[m]]
        for r in range(rdmas):
            d = devs[gpus + r]
            d["type"], d["minor"] = abi.DEV_RDMA, r
            d["health"] = 1
            d["has_total"][0] = 1
            d["total"][0] = 100
            u = rng.choice([0, 25, 50, 100])
            if u:
                d["has_used"][0] = 1
                d["used"][0] = u
        out.append(devs)
    return out


def load_devices(handle, devices):
    for i, d in enumerate(devices):
        if d is not None:
            handle.set_devices(i, d)


def add_gpu_topology(devices, seed, nil_fraction=0.05):
    """Give the GPUs of each device cache entry a DeviceInfo.Topology (in place): NUMA nodes of 2-4 GPUs
    (NodeID possibly non-contiguous), PCIe switches of 1-2 GPUs, PCIEID strings whose Go order differs from
    their numeric order ("10" < "9").  A `nil_fraction` of the entries leave one GPU without topology
    (GetGPUTopologyScope -> nil).  RDMA NICs get topologies too (unused by the GPU tree)."""
    rng = np.random.default_rng(seed)
    for devs in devices:
        if devs is None:
            continue
        g = np.nonzero(devs["type"] == abi.DEV_GPU)[0]
        per_numa = int(rng.choice([2, 4, 4, 8]))
        per_pcie = int(rng.choice([1, 2, 2]))
        numa_ids = rng.permutation(4)[: (len(g) + per_numa - 1) // per_numa] if len(g) else []
        names = []
        for j, i in enumerate(g):
            m = int(devs[i]["minor"])
            devs[i]["has_topology"] = 1
            devs[i]["numa_node"] = int(numa_ids[j // per_numa])
            names.append((i, str(7 + m // per_pcie)))  # "7", "8", "9", "10", ...
        for i in np.nonzero(devs["type"] != abi.DEV_GPU)[0]:
            devs[i]["has_topology"] = 1
            devs[i]["numa_node"] = int(numa_ids[0]) if len(numa_ids) else 0
            names.append((i, str(7 + int(devs[i]["minor"]))))
        order = sorted({n for _, n in names}, key=lambda x: x.encode())
        for i, n in names:
            devs[i]["pcie_rank"] = order.index(n)
        if len(g) and rng.random() < nil_fraction:
            devs[g[rng.integers(len(g))]]["has_topology"] = 0
    return devices


def add_device_numa(devices, zones, seed, off_zone_fraction=0.05, no_topology_fraction=0.05):
    """Give each device cache entry NUMA node ids consistent with the node's NRT zones (in place), for
    DeviceShare's NUMA hints: 8 GPUs over the zones (2 or 4 zones: spread evenly; 8 zones: two zones,
    so a BestEffort merge stays within the permutation budget), the RDMA NICs on the GPUs' zones.  An
    `off_zone_fraction` of the entries put a GPU on a NUMA id the node has no zone for, a
    `no_topology_fraction` leave one GPU without topology (filtered out under an affinity)."""
    rng = np.random.default_rng(seed)
    for devs, z in zip(devices, zones):
        if devs is None:
            continue
        nz = len(z) if z is not None else 2
        ids = list(range(nz)) if nz <= 4 else sorted(rng.choice(nz, 2, replace=False).tolist())
        g = np.nonzero(devs["type"] == abi.DEV_GPU)[0]
        r = np.nonzero(devs["type"] != abi.DEV_GPU)[0]
        for j, i in enumerate(g):
            devs[i]["has_topology"] = 1
            devs[i]["numa_node"] = ids[j * len(ids) // len(g)]
            devs[i]["pcie_rank"] = j // 2
        for j, i in enumerate(r):
            devs[i]["has_topology"] = 1
            devs[i]["numa_node"] = ids[j * len(ids) // len(r)]
            devs[i]["pcie_rank"] = (len(g) + 1) // 2 + j
        if len(g) and rng.random() < off_zone_fraction:
            devs[g[-1]]["numa_node"] = min(nz, 7)
        if len(g) and rng.random() < no_topology_fraction:
            k = g[rng.integers(len(g))]
            devs[k]["has_topology"] = 0
            devs[k]["numa_node"] = -1
    return devices


def make_ds_numa_pods(n_pods, seed, policy_fraction=0.3, key_base=2_500_000_000):
    """make_ds_pods (device requests on half of the queue) where `policy_fraction` of the pods also carry a
    NUMA topology spec (BestEffort / Restricted / SingleNUMANode, SingleNUMANodeExclusive unset /
    Preferred / Required)."""
    rng = np.random.default_rng(seed)
    pods = make_ds_pods(n_pods, seed + 1, key_base=key_base)
    pol = rng.random(n_pods) < policy_fraction
    pods["numa_topology_policy"] = np.where(pol, rng.integers(1, 4, n_pods), 0)
    pods["numa_exclusive"] = np.where(pol, rng.integers(0, 3, n_pods), 0)
    return pods


def make_partition_states(n_nodes, seed, gpus=8):
    """Per node (has_table, honor, partitions) for ke_node_gpu_partitions: the designated Hopper table
    (40 %), a custom table with two allocation-score groups and ring bus bandwidths (15 %), an empty table
    (5 %), or none; Honor on half of the nodes."""
    from . import model
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_nodes):
        u, honor = rng.random(), bool(rng.random() < 0.5)
        if u < 0.40:
            out.append((True, honor, model.gpu_partition_state(
                node_labels={"node.koordinator.sh/gpu-model": "H800"})[2]))
        elif u < 0.55:
            table = {}
            for n in (1, 2, 4):
                parts = []
                for start in range(0, gpus - n + 1, n):
                    parts.append({"minors": list(range(start, start + n)), "allocationScore": int(rng.choice([1, 2])),
                                  "ringBusBandwidth": None if rng.random() < 0.2 else int(rng.choice([100, 200, 400]))})
                table[n] = parts
            table[3] = [{"minors": [0, 1, 2], "allocationScore": 1}, {"minors": [4, 5, 6], "allocationScore": 1}]
            out.append((True, honor, model.make_gpu_partitions(table)))
        elif u < 0.60:
            out.append((True, honor, None))
        else:
            out.append((False, honor, None))
    return out


def load_partition_states(handle, states):
    for i, (has, honor, parts) in enumerate(states):
        if has or honor:
            handle.set_gpu_partitions(i, has, honor, parts)


def make_gpu_alloc_pods(n_pods, seed, key_base=5_000_000_000):
    """Pods exercising GPUAllocator.Allocate: whole GPUs (1, 2, 3, 4, 8), shared slices (gpu.shared 1 or 2),
    GPU hints with a required topology scope, GPUPartitionSpec (Restricted, ring bus bandwidth)."""
    rng = np.random.default_rng(seed)
    pods = make_pods(n_pods, seed + 1, key_base=key_base)
    for i in range(n_pods):
        r = pods["device_requests"][i]
        k = rng.random()
        if k < 0.55:
            r[abi.PDR["nvidia.com/gpu"]] = rng.choice([1, 1, 2, 2, 3, 4, 8])
        elif k < 0.8:
            r[abi.PDR["koordinator.sh/gpu.shared"]] = 1
            r[abi.PDR["koordinator.sh/gpu-core"]] = rng.choice([25, 50])
            r[abi.PDR["koordinator.sh/gpu-memory-ratio"]] = rng.choice([25, 50])
        elif k < 0.9:
            sh = int(rng.choice([1, 2]))
            r[abi.PDR["koordinator.sh/gpu.shared"]] = sh
            r[abi.PDR["koordinator.sh/gpu-memory-ratio"]] = 50 * sh
        else:
            r[abi.PDR["koordinator.sh/gpu-core"]] = 200
            r[abi.PDR["koordinator.sh/gpu-memory-ratio"]] = 200
        pods["has_other_requests"][i] = 1
        pods["gpu_ring_bus_bandwidth"][i] = abi.ABSENT
        if rng.random() < 0.3:
            pods["gpu_required_topology_scope"][i] = rng.choice([abi.SCOPE_NODE, abi.SCOPE_NUMA, abi.SCOPE_PCIE,
                                                                 abi.SCOPE_PCIE, abi.SCOPE_DEVICE, abi.SCOPE_UNKNOWN])
        if rng.random() < 0.25:
            pods["gpu_partition_spec"][i] = 1
            pods["gpu_partition_restricted"][i] = int(rng.random() < 0.4)
            if rng.random() < 0.5:
                pods["gpu_ring_bus_bandwidth"][i] = rng.choice([50, 200, 300])
    return pods


def make_ds_pods(n_pods, seed, device_fraction=0.5, key_base=2_000_000_000):
    """Queue for config 5: the config-2 mix, of which `device_fraction` also request devices:
    gpu-core = gpu-memory-ratio in {25,50,100,200,400,800}, nvidia.com/gpu in {1,2}, or a shared
    gpu-memory slice; 30% of them also RDMA {50,100}; 1% carry an invalid request."""
    rng = np.random.default_rng(seed)
    pods = make_pods(n_pods, seed + 1, key_base=key_base)
    dev = rng.random(n_pods) < device_fraction
    kind = rng.random(n_pods)
    pct = rng.choice([25, 50, 100, 200, 400, 800], n_pods)
    for i in np.nonzero(dev)[0]:
        r = pods["device_requests"][i]
        if kind[i] < 0.6:
            r[abi.PDR["koordinator.sh/gpu-core"]] = pct[i]
            r[abi.PDR["koordinator.sh/gpu-memory-ratio"]] = pct[i]
        elif kind[i] < 0.8:
            r[abi.PDR["nvidia.com/gpu"]] = rng.choice([1, 2])
        elif kind[i] < 0.99:
            r[abi.PDR["koordinator.sh/gpu-memory"]] = rng.choice([16, 48, 96]) * GI
        else:
            r[abi.PDR["koordinator.sh/gpu-memory-ratio"]] = 150  # invalid: > 100 and not a multiple
        if rng.random() < 0.3:
            r[abi.PDR["koordinator.sh/rdma"]] = rng.choice([50, 100])
        pods["has_other_requests"][i] = 1
    return pods


# ---- NUMA topology policies (BASELINE config 4, non-cpuset part) ----------------------------------
def make_numa(cl, seed, zone_counts=(8,), policy_weights=(0.1, 0.3, 0.3, 0.3), no_zone_fraction=0.02,
              missing_memory_fraction=0.03, allocated_fraction=0.7, status_fraction=0.0):
    """Give the nodes of cluster `cl` a NUMA topology policy (None / BestEffort / Restricted /
    SingleNUMANode by `policy_weights`) and NodeResourceTopology zones: the node's allocatable split
    evenly over `zone_counts` zones (cpu in whole cores), a few zones without a memory key, and a
    random resource-manager allocation on most zones (cpuset CPUs on a quarter of the allocated zones
    of amplified nodes).  Mutates cl.nodes; returns the per-node zone arrays (None = no NRT zones)."""
    rng = np.random.default_rng(seed)
    N = cl.n_nodes
    pol = rng.choice(4, N, p=np.asarray(policy_weights) / np.sum(policy_weights))
    cl.nodes["numa_topology_policy"] = pol
    out = []
    for i in range(N):
        if rng.random() < no_zone_fraction:
            out.append(None)
            continue
        nz = int(rng.choice(zone_counts))
        cores = int(cl.nodes["allocatable"][i, 0]) // 1000
        mem = int(cl.nodes["allocatable"][i, 1])
        z = np.zeros(nz, abi.NUMA_ZONE_DTYPE)
        amplified = cl.nodes["cpu_amplification_ratio"][i] > 1.0
        for k in range(nz):
            z[k]["id"] = k
            z[k]["has"][0] = 1
            z[k]["capacity"][0] = (cores // nz) * 1000
            if rng.random() >= missing_memory_fraction:
                z[k]["has"][1] = 1
                z[k]["capacity"][1] = mem // nz // MI * MI
            if rng.random() < allocated_fraction:
                f = rng.choice([0.0, 0.25, 0.5, 0.75, 0.9, 1.0])
                z[k]["allocated"][0] = int(z[k]["capacity"][0] * f) // 1000 * 1000
                z[k]["allocated"][1] = int(z[k]["capacity"][1] * rng.choice([0.0, 0.3, 0.6, 0.95])) // MI * MI
                # the entry's keys: those allocated (zero amounts keep their key after a release)
                keys = abi.NUMA_ALLOC_ENTRY
                if z[k]["allocated"][0] or rng.random() < 0.5:
                    keys |= abi.NUMA_ALLOC_CPU
                if z[k]["allocated"][1] or rng.random() < 0.5:
                    keys |= abi.NUMA_ALLOC_MEMORY
                z[k]["has_allocated"] = keys
                if amplified and rng.random() < 0.25:
                    z[k]["cpuset_cpus"] = int(rng.integers(1, 4))
            # NUMANodeSharedStatus from cpuset pods already on the node (the Go path placed them)
            if rng.random() < status_fraction:
                z[k]["numa_status"] = rng.choice([abi.NUMA_STATUS_SINGLE, abi.NUMA_STATUS_SHARED])
        out.append(z)
    return out


def make_numa_pods(n_pods, seed, policy_fraction=0.3, key_base=3_000_000_000):
    """The config-2 queue where `policy_fraction` of the pods carry a numa-topology-spec annotation:
    a policy (BestEffort / Restricted / SingleNUMANode) and SingleNUMANodeExclusive unset (Required by
    default) / Preferred / Required."""
    rng = np.random.default_rng(seed)
    pods = make_pods(n_pods, seed + 1, key_base=key_base)
    pol = rng.random(n_pods) < policy_fraction
    pods["numa_topology_policy"] = np.where(pol, rng.integers(1, 4, n_pods), 0)
    pods["numa_exclusive"] = np.where(pol, rng.integers(0, 3, n_pods), 0)
    return pods


def load_numa(handle, zones):
    for i, z in enumerate(zones):
        if z is not None:
            handle.set_numa(i, z)


# ---- CPU tables + cpuset pods (NodeNUMAResource, NUMA policy None) ----------------------------------
def make_cpus(cl, seed, no_table_fraction=0.03, invalid_fraction=0.02, bind_weights=(0.7, 0.15, 0.15),
              max_ref_choices=(1, 1, 1, 2), allocated_choices=(0.0, 0.1, 0.3, 0.6, 0.9), reserved_fraction=0.3):
    """Give the nodes of `cl` a CPU topology table (kubelet-style: the node's logical CPUs over 1-2
    sockets x 1-2 NUMA nodes, 1 or 2 threads per core, sibling ids adjacent or split by half), cpuset
    allocations of earlier pods (RefCount up to MaxRefCount, PCPU / NUMA-level exclusivity), a few
    reserved CPUs, a node CPU bind policy (None / FullPCPUsOnly / SpreadByPCPUs by `bind_weights`) and
    a NUMA allocate strategy label.  Mutates cl.nodes; returns [(table or None, max_ref)] per node."""
    rng = np.random.default_rng(seed)
    N = cl.n_nodes
    cl.nodes["cpu_bind_policy"] = rng.choice(3, N, p=np.asarray(bind_weights) / np.sum(bind_weights))
    cl.nodes["numa_allocate_strategy"] = rng.choice(3, N)
    out = []
    for i in range(N):
        u = rng.random()
        if u < no_table_fraction:
            out.append((None, 1))
            continue
        if u < no_table_fraction + invalid_fraction:
            cl.nodes["cpu_topology_invalid"][i] = 1
            out.append((None, 1))
            continue
        cap = cl.nodes["raw_allocatable"][i, 0]
        ncpu = int((cap if cap != abi.ABSENT else cl.nodes["allocatable"][i, 0]) // 1000)
        ncpu = min(ncpu, abi.MAX_CPUS)
        sockets = int(rng.choice([1, 2]))
        nps = int(rng.choice([1, 2]))
        tpc = int(rng.choice([1, 2, 2]))
        cores = ncpu // (sockets * nps * tpc)
        n_all = sockets * nps * cores * tpc
        split = rng.random() < 0.5  # Linux numbering: thread t of core k is cpu k + t*(n_all/tpc)
        rows = []
        core = 0
        for s in range(sockets):
            for q in range(nps):
                for _ in range(cores):
                    for t in range(tpc):
                        cpu = core + t * (n_all // tpc) if split else core * tpc + t
                        rows.append((cpu, 1000 + 7 * core, s * nps + q, 10 + s))
                    core += 1
        max_ref = int(rng.choice(max_ref_choices))
        f = float(rng.choice(allocated_choices))
        allocated = {}
        for cpu, _, _, _ in rows:
            if rng.random() < f:
                excl = rng.choice([None, None, "PCPULevel", "NUMANodeLevel"])
                allocated[cpu] = (int(rng.integers(1, max_ref + 1)), excl)
        reserved = ()
        if rng.random() < reserved_fraction:
            reserved = tuple(int(c) for c in rng.choice([r[0] for r in rows], int(rng.integers(1, 5)), replace=False))
        out.append((model.make_cpus(rows, allocated, reserved), max_ref))
    return out


def load_cpus(handle, tables):
    for i, (t, max_ref) in enumerate(tables):
        if t is not None:
            handle.set_cpus(i, t, max_ref)


def make_cpuset_pods(n_pods, seed, cpuset_fraction=0.5, key_base=4_000_000_000):
    """The config-2 queue where `cpuset_fraction` of the pods are LSE/LSR koord-prod with whole-CPU
    requests (a few fractional) and a ResourceSpec: required / preferred bind policy (unset, Default,
    FullPCPUs, SpreadByPCPUs, ConstrainedBurst) and preferred CPU exclusivity."""
    rng = np.random.default_rng(seed)
    pods = make_pods(n_pods, seed + 1, key_base=key_base)
    cs = rng.random(n_pods) < cpuset_fraction
    k = int(cs.sum())
    pods["priority_class"][cs] = abi.PRIORITY_PROD
    pods["qos_class"][cs] = rng.choice([abi.QOS_LSE, abi.QOS_LSR], k)
    cpu = rng.choice([1000, 2000, 3000, 4000, 6000, 8000, 16000, 1500], k, p=[.15, .2, .1, .2, .1, .1, .1, .05])
    pods["requests"][cs, abi.RES_CPU] = cpu
    pods["limits"][cs, abi.RES_CPU] = cpu
    pods["requests"][cs, abi.RES_MEMORY] = rng.choice([2, 4, 8], k) * GI
    pods["limits"][cs, abi.RES_MEMORY] = pods["requests"][cs, abi.RES_MEMORY]
    pods["requests"][cs, abi.RES_BATCH_CPU] = 0
    pods["requests"][cs, abi.RES_BATCH_MEMORY] = 0
    pods["is_daemonset"][cs] = 0
    pods["cpu_bind_required"][cs] = rng.choice(5, k, p=[.6, .1, .12, .12, .06])
    pods["cpu_bind_preferred"][cs] = rng.choice(5, k, p=[.4, .15, .2, .2, .05])
    pods["cpu_exclusive"][cs] = rng.choice(3, k, p=[.6, .2, .2])
    return pods


def make_numa_cpus(cl, seed, zone_counts=(2, 4, 8), policy_weights=(0.1, 0.3, 0.3, 0.3), bind_weights=(0.8, 0.1, 0.1),
                   cpuset_fraction=(0.0, 0.1, 0.3, 0.6), max_ref_choices=(1, 1, 2), threads=None, sockets=None):
    """Config 4 (NUMA-aware cpuset binding, BASELINE.json configs[3]): per node a NUMA topology policy
    (None / BestEffort / Restricted / SingleNUMANode by `policy_weights`), NRT zones over `zone_counts`
    NUMA nodes with a CPU table consistent with them (1-2 sockets, 1-2 threads per core), cpusets of
    earlier LSR/LSE pods (RefCount, exclusivity) whose CPUs also sit in the zones' allocation entries
    (plus shared cpu / memory allocations), the zones' single / shared status from those cpusets, a
    node CPU bind policy and a NUMA allocate strategy label.  Mutates cl.nodes; returns
    (zones, tables) as make_numa / make_cpus do."""
    rng = np.random.default_rng(seed)
    N = cl.n_nodes
    cl.nodes["numa_topology_policy"] = rng.choice(4, N, p=np.asarray(policy_weights) / np.sum(policy_weights))
    cl.nodes["cpu_bind_policy"] = rng.choice(3, N, p=np.asarray(bind_weights) / np.sum(bind_weights))
    cl.nodes["numa_allocate_strategy"] = rng.choice(3, N)
    zones_out, tables = [], []
    excl_codes = np.array([abi.CPU_EXCL_NONE, abi.CPU_EXCL_NONE, abi.CPU_EXCL_PCPU_LEVEL, abi.CPU_EXCL_NUMA_NODE_LEVEL])
    for i in range(N):
        cap = cl.nodes["raw_allocatable"][i, 0]
        ncpu = min(int((cap if cap != abi.ABSENT else cl.nodes["allocatable"][i, 0]) // 1000), abi.MAX_CPUS)
        nz = int(rng.choice([z for z in zone_counts if ncpu % z == 0] or [1]))
        cpz = ncpu // nz
        tpc = threads if threads else (int(rng.choice([1, 2])) if cpz % 2 == 0 else 1)
        n_sock = sockets if sockets else (2 if nz % 2 == 0 and rng.random() < 0.7 else 1)
        split = rng.random() < 0.5
        # CPU rows in (zone, core, thread) order: core k of the node, thread t
        core = np.repeat(np.arange(ncpu // tpc), tpc)
        thread = np.tile(np.arange(tpc), ncpu // tpc)
        zone = core // (cpz // tpc)
        t = np.zeros(ncpu, abi.CPU_DTYPE)
        t["cpu_id"] = core + thread * (ncpu // tpc) if split else core * tpc + thread
        t["core_id"] = 500 + 3 * core
        t["numa_id"] = zone
        t["socket_id"] = zone * n_sock // nz
        max_ref = int(rng.choice(max_ref_choices))
        frac = float(rng.choice(cpuset_fraction))
        busy = rng.random(ncpu) < frac
        t["ref_count"] = np.where(busy, rng.integers(1, max_ref + 1, ncpu), 0)
        t["exclusive"] = np.where(busy, excl_codes[rng.integers(0, 4, ncpu)], 0)
        per_zone = np.bincount(zone[busy], minlength=nz)
        mem = int(cl.nodes["allocatable"][i, 1])
        amplified = cl.nodes["cpu_amplification_ratio"][i] > 1.0
        z_arr = np.zeros(nz, abi.NUMA_ZONE_DTYPE)
        z_arr["id"] = np.arange(nz)
        z_arr["has"][:] = 1
        z_arr["capacity"][:, 0] = cpz * 1000
        z_arr["capacity"][:, 1] = mem // nz // MI * MI
        shared = np.where(rng.random(nz) < 0.6, rng.choice([0, 0, 1000, 2500, 4000], nz), 0)
        mem_al = (z_arr["capacity"][:, 1] * rng.choice([0.0, 0.2, 0.5, 0.8], nz)).astype(np.int64) // MI * MI
        entry = (per_zone > 0) | (shared > 0) | (mem_al > 0) | (amplified & (rng.random(nz) < 0.3))
        z_arr["has_allocated"] = np.where(entry, abi.NUMA_ALLOC_ENTRY | abi.NUMA_ALLOC_CPU | abi.NUMA_ALLOC_MEMORY, 0)
        z_arr["allocated"][:, 0] = np.where(entry, per_zone * 1000 + shared, 0)
        z_arr["allocated"][:, 1] = np.where(entry, mem_al, 0)
        z_arr["numa_status"] = np.where(per_zone > 0, np.where(rng.random(nz) < 0.7, abi.NUMA_STATUS_SINGLE,
                                                                   abi.NUMA_STATUS_SHARED), 0)
        zones_out.append(z_arr)
        tables.append((t, max_ref))
    return zones_out, tables


def make_c4_cluster(n_nodes, seed, policy_weights=(0.0, 0.3, 0.3, 0.4)):
    """128-CPU hosts (2 sockets x 4 NUMA x 8 cores x 2 threads), NUMA policy labels
    SingleNUMANode / Restricted / BestEffort 40/30/30, earlier cpusets on part of the CPUs."""
    cl = make_cluster(n_nodes, seed)
    cl.nodes["allocatable"][:, 0] = 128_000
    zones, tables = make_numa_cpus(cl, seed + 1, zone_counts=(8,), policy_weights=policy_weights,
                                   bind_weights=(1.0, 0.0, 0.0), threads=2, sockets=2)
    return cl, zones, tables


def make_c4_pods(n_pods, seed, key_base=8_000_000_000):
    """SURVEY.md §8d C4 queue: LSR/LSE koord-prod pods, cpu in {2,4,8,16} cores, the FullPCPUs default
    (no ResourceSpec annotation)."""
    rng = np.random.default_rng(seed)
    pods = make_pods(n_pods, seed + 1, key_base=key_base)
    cpu = rng.choice([2, 4, 8, 16], n_pods) * 1000
    pods["priority_class"] = abi.PRIORITY_PROD
    pods["qos_class"] = rng.choice([abi.QOS_LSE, abi.QOS_LSR], n_pods)
    pods["is_daemonset"] = 0
    pods["requests"][:] = 0
    pods["limits"][:] = 0
    pods["requests"][:, abi.RES_CPU] = cpu
    pods["limits"][:, abi.RES_CPU] = cpu
    mem = rng.choice([4, 8, 16, 32], n_pods) * GI
    pods["requests"][:, abi.RES_MEMORY] = mem
    pods["limits"][:, abi.RES_MEMORY] = mem
    return pods


def make_numa_cpuset_pods(n_pods, seed, cpuset_fraction=0.6, policy_fraction=0.2, key_base=6_000_000_000):
    """Config 4's queue: make_cpuset_pods (LSR/LSE koord-prod binding pods, bind / exclusive policies)
    where `policy_fraction` of the pods also carry a NUMA topology spec."""
    rng = np.random.default_rng(seed)
    pods = make_cpuset_pods(n_pods, seed + 1, cpuset_fraction=cpuset_fraction, key_base=key_base)
    pol = rng.random(n_pods) < policy_fraction
    pods["numa_topology_policy"] = np.where(pol, rng.integers(1, 4, n_pods), 0)
    pods["numa_exclusive"] = np.where(pol, rng.integers(0, 3, n_pods), 0)
    return pods


# ---- ElasticQuota (config 5: "ElasticQuota tree of 64 leaves") ----------------------------------
def make_quota_tree(seed, n_leaves=64, fanout=8, total_cpu=None, total_mem=None, lent_fraction=0.8):
    """A 3-level tree: root children (n_leaves / fanout parents) -> leaves.  Max / Min / shared weight
    in cpu milli and memory bytes; about a fifth of the quotas do not lend (allow-lent-resource
    false).  Returns the ke_quota array; leaves are the last n_leaves entries."""
    rng = np.random.default_rng(seed)
    n_par = max(1, n_leaves // fanout)
    q = np.zeros(n_par + n_leaves, abi.QUOTA_DTYPE)
    total_cpu = total_cpu or 1_000_000 * 1000
    total_mem = total_mem or 4_000_000 * GI

    def fill(i, parent, scale):
        q[i]["parent"] = parent
        cpu_max = int(rng.integers(1, 4) * scale[0])
        mem_max = int(rng.integers(1, 4) * scale[1])
        q[i]["has_max"] = (1, 1)
        q[i]["max"] = (cpu_max, mem_max)
        q[i]["has_min"] = (1, 1)
        q[i]["min"] = (int(cpu_max * rng.uniform(0.1, 0.6)) // 1000 * 1000, int(mem_max * rng.uniform(0.1, 0.6)) // MI * MI)
        q[i]["shared_weight"] = q[i]["max"]
        q[i]["allow_lent_resource"] = 1 if rng.random() < lent_fraction else 0

    for p in range(n_par):
        fill(p, -1, (total_cpu // n_par, total_mem // n_par))
    for l in range(n_leaves):
        fill(n_par + l, l // fanout if n_par > 1 else 0, (total_cpu // n_leaves, total_mem // n_leaves))
    return q


def quota_args(total_cpu, total_mem, runtime=True, check_parent=False, scale_min=True):
    a = abi.QuotaArgs()
    a.total[0], a.total[1] = total_cpu, total_mem
    a.enable_runtime_quota = 1 if runtime else 0
    a.enable_check_parent_quota = 1 if check_parent else 0
    a.disable_scale_min_quota = 0 if scale_min else 1
    return a


def assign_quotas(pods, quotas, seed, no_quota_fraction=0.1, non_preemptible_fraction=0.2):
    """Pods -> leaf quotas (ke_pod.quota = 1 + index); the quotas' self requests are the masked
    requests of their pods (the whole queue is pending: GroupQuotaManager counts pending pods)."""
    rng = np.random.default_rng(seed)
    parents = set(int(x) for x in quotas["parent"] if x >= 0)
    leaves = np.array([i for i in range(len(quotas)) if i not in parents], np.int64)
    pods = pods.copy()
    for p in range(len(pods)):
        if rng.random() < no_quota_fraction:
            pods[p]["quota"] = 0
            continue
        qi = int(leaves[rng.integers(0, len(leaves))])
        pods[p]["quota"] = qi + 1
        pods[p]["quota_non_preemptible"] = 1 if rng.random() < non_preemptible_fraction else 0
        for r, res in enumerate((abi.RES_CPU, abi.RES_MEMORY)):
            if quotas[qi]["has_max"][r]:
                quotas[qi]["self_request"][r] += pods[p]["requests"][res]
    return pods


# ---- NodeResourcesFitPlus / ScarceResourceAvoidance -------------------------------
# Resource ids of the synthetic profile: the KE_RES_* names plus ephemeral storage and two extended resources
# (a GPU count and a scarce device that most pods never request).
XRES = {"cpu": abi.XRES_CPU, "memory": abi.XRES_MEMORY, "kubernetes.io/batch-cpu": 2, "kubernetes.io/batch-memory": 3,
        "ephemeral-storage": 4, "nvidia.com/gpu": 5, "example.com/scarce": 6}
_POD_RES = ((abi.RES_CPU, 0), (abi.RES_MEMORY, 1), (abi.RES_BATCH_CPU, 2), (abi.RES_BATCH_MEMORY, 3))


def ext_config(cfg, w_fitplus=1, w_sra=1, fitplus=None, sra=("nvidia.com/gpu", "example.com/scarce")):
    """The profile of config/manager/scheduler-config.yaml's resource scorer (cpu, memory, batch-cpu,
    batch-memory at weight 1) as NodeResourcesFitPlus args, GPUs MostAllocated, plus ScarceResourceAvoidance."""
    x = cfg.ext
    x.weight_fitplus, x.weight_sra = w_fitplus, w_sra
    fitplus = fitplus if fitplus is not None else [("cpu", abi.STRATEGY_LEAST_ALLOCATED, 1),
                                                   ("memory", abi.STRATEGY_LEAST_ALLOCATED, 1),
                                                   ("kubernetes.io/batch-cpu", abi.STRATEGY_LEAST_ALLOCATED, 1),
                                                   ("nvidia.com/gpu", abi.STRATEGY_MOST_ALLOCATED, 2)]
    x.n_fitplus = len(fitplus)
    for q, (name, typ, w) in enumerate(fitplus):
        x.fitplus[q].id, x.fitplus[q].type, x.fitplus[q].weight = XRES[name], typ, w
    x.sra_resources = sum(1 << XRES[n] for n in sra)
    return cfg


def fit_config(cfg, weight=1, filter=True, strategy=abi.STRATEGY_LEAST_ALLOCATED,
               resources=(("cpu", 1), ("memory", 1), ("kubernetes.io/batch-cpu", 1), ("kubernetes.io/batch-memory", 1)),
               scalars=("kubernetes.io/batch-cpu", "kubernetes.io/batch-memory", "ephemeral-storage", "nvidia.com/gpu",
                        "example.com/scarce")):
    """NodeResourcesFit as the shipped profile configures it (config/manager/scheduler-config.yaml:17-31: LeastAllocated
    over cpu, memory, batch-cpu, batch-memory at weight 1) with its Filter over the synthetic scalar resources."""
    f = cfg.fit
    f.weight, f.filter, f.strategy = weight, int(filter), strategy
    f.n_resources = len(resources)
    for q, (name, w) in enumerate(resources):
        f.resources[q].id, f.resources[q].weight = XRES[name], w
    f.n_scalars = len(scalars)
    for q, name in enumerate(scalars):
        f.scalars[q] = XRES[name]
    return cfg


def add_fit_defaults(pods):
    """calculatePodResourceRequest's 100m / 200Mi container defaults for pods whose containers request no cpu /
    memory (one container): xres entries for ids 0 / 1 without a requested-name bit."""
    for p in range(len(pods)):
        n = int(pods["n_xres"][p])
        have = set(pods["xres_id"][p, :n].tolist())
        for rid, v in ((abi.XRES_CPU, 100), (abi.XRES_MEMORY, 200 * 2**20)):
            if rid not in have and n < abi.MAX_POD_XRES:
                pods["xres_id"][p, n], pods["xres_value"][p, n] = rid, v
                n += 1
        pods["n_xres"][p] = n
    return pods


def make_node_resources(cl, seed, gpu_fraction=0.3, scarce_fraction=0.15):
    """Per node a ke_node_resource table consistent with the cluster: Allocatable cpu / memory of the node,
    NonZeroRequested = Requested (+ the 100m / 200Mi defaults of a few zero-request pods), batch resources,
    ephemeral storage, and on some nodes GPUs / a scarce device with random usage."""
    rng = np.random.default_rng(seed)
    tables = []
    for i in range(cl.n_nodes):
        n = cl.nodes[i]
        rows = [(XRES["cpu"], int(n["allocatable"][0]), int(n["requested"][0]) + 100 * int(rng.integers(0, 3))),
                (XRES["memory"], int(n["allocatable"][1]), int(n["requested"][1]) + 200 * 2**20 * int(rng.integers(0, 3)))]
        if rng.random() < 0.8:
            bc = int(rng.integers(8, 65)) * 1000
            rows.append((2, bc, int(rng.integers(0, bc // 1000 + 8)) * 1000))
            bm = int(rng.integers(32, 257)) * GI
            rows.append((3, bm, int(rng.integers(0, bm // GI + 8)) * GI))
        if rng.random() < 0.9:
            rows.append((4, int(rng.integers(100, 1000)) * GI, int(rng.integers(0, 100)) * GI))
        if rng.random() < gpu_fraction:
            g = int(rng.choice([4, 8]))
            rows.append((5, g, int(rng.integers(0, g + 1))))
        if rng.random() < scarce_fraction:
            rows.append((6, int(rng.integers(1, 4)), 0))
        if rng.random() < 0.03:  # a listed resource with zero allocatable: not a name of the node
            free = [r for r in (6, 5) if r not in {x[0] for x in rows}]
            if free:
                rows.append((free[0], 0, 0))
        t = np.zeros(len(rows), abi.NODE_RESOURCE_DTYPE)
        for e, (rid, a, r) in enumerate(rows):
            t[e]["id"], t[e]["allocatable"], t[e]["requested"] = rid, a, r
        tables.append(t)
    return tables


def load_node_resources(handle, tables):
    for i, t in enumerate(tables):
        handle.set_resources(i, t)


def add_pod_xres(pods, seed, gpu_fraction=0.2, storage_fraction=0.5, scarce_fraction=0.03):
    """ke_pod.xres_*: the requested names of each pod (PodRequests > 0) and calculatePodResourceRequest; a few
    pods request GPUs, ephemeral storage or the scarce device, a few have a container without a cpu / memory
    request (the 100m / 200Mi nonzero defaults)."""
    rng = np.random.default_rng(seed)
    for p in range(len(pods)):
        mask, ids, vals = 0, [], []
        for r, rid in _POD_RES:
            v = int(pods["requests"][p, r])
            if v > 0:
                mask |= 1 << rid
                extra = 0
                if rid in (0, 1) and rng.random() < 0.1:  # a second container without this request
                    extra = 100 if rid == 0 else 200 * 2**20
                ids.append(rid), vals.append(v + extra)
        for rid, frac, lo, hi in ((5, gpu_fraction, 1, 5), (4, storage_fraction, 1, 50), (6, scarce_fraction, 1, 2)):
            if rng.random() < frac:
                v = int(rng.integers(lo, hi)) * (GI if rid == 4 else 1)
                mask |= 1 << rid
                ids.append(rid), vals.append(v)
        pods["xres_request_mask"][p] = mask
        pods["n_xres"][p] = len(ids)
        pods["xres_id"][p, :len(ids)] = ids
        pods["xres_value"][p, :len(ids)] = vals
    return pods


# ---- reservations whose reserve pods hold NUMA resources, cpusets and devices ------------------------------------
# resource ids of the device resource names (after XRES's 0..6): a reservation's allocatable names them when its
# reserve pod holds devices (ReservationInfo.Allocatable = the reserve pod's requests)
DEVICE_XRES = {"koordinator.sh/gpu-core": 10, "koordinator.sh/gpu-memory-ratio": 11, "koordinator.sh/gpu-memory": 12,
               "koordinator.sh/rdma": 13}
DEVICE_KEY_XRES = {(abi.DEV_GPU, 0): 10, (abi.DEV_GPU, 1): 12, (abi.DEV_GPU, 2): 11, (abi.DEV_RDMA, 0): 13}


def device_resource_entries(a, owners=True):
    """a reservation's allocatable entries of the device resources its reserve pod holds (RESERVATION_ALLOC record
    `a`): per resource id the Σ over instances, allocated = the owners' Σ (ke_reservation_resource array)"""
    sums = {}
    for (ty, k), rid in DEVICE_KEY_XRES.items():
        v = int(a["device"][ty, :, k].sum())
        if v:
            sums[rid] = (v, int(a["owner_device"][ty, :, k].sum()) if owners else 0)
    e = np.zeros(len(sums), abi.RESERVATION_RESOURCE_DTYPE)
    for q, rid in enumerate(sorted(sums)):
        e[q]["id"], e[q]["allocatable"], e[q]["allocated"] = rid, sums[rid][0], sums[rid][1]
    return e


def make_reservation_holdings(cl, seed, zones=None, tabs=None, devices=None, frac=0.3, owner_fraction=0.6,
                              policies=(0, 1, 2)):
    """Reservations on a `frac` of the nodes whose reserve pods hold, where the node has them, a NUMA allocation on
    one or two zones, a cpuset out of the zones' free CPUs and a share of one GPU / RDMA instance, with owner pods
    (allocated_pods > 0 for `owner_fraction` of them) holding part of each.  Both are added to the node state the way
    the resource manager and the device cache count them (zone allocation, CPU ref counts, device used, NodeInfo
    Requested / pod count).  A reservation holding devices names their resources in its allocatable (the reserve
    pod requests them): entries by DEVICE_XRES id, KE_RSV_OTHER_ALLOCATABLE.  Mutates cl.nodes, zones, tabs and
    devices; returns (RESERVATION_DTYPE array, RESERVATION_ALLOC_DTYPE array, per reservation its
    RESERVATION_RESOURCE_DTYPE entries)."""
    rng = np.random.default_rng(seed)
    rs, al, res = [], [], []
    for i in range(cl.n_nodes):
        if rng.random() >= frac:
            continue
        for _ in range(int(rng.integers(1, 3))):
            r = np.zeros((), abi.RESERVATION_DTYPE)
            a = np.zeros((), abi.RESERVATION_ALLOC_DTYPE)
            r["node"], r["available"] = i, int(rng.random() < 0.95)
            r["allocate_policy"] = int(rng.choice(policies))
            r["order"] = int(rng.choice([0, 0, 0, 5, 9]))
            owners = rng.random() < owner_fraction
            r["allocated_pods"] = int(rng.integers(1, 3)) if owners else 0
            holds = 0
            cpu_total = mem_total = cpu_owned = mem_owned = 0
            z = zones[i] if zones is not None else None
            t = tabs[i][0] if tabs is not None and tabs[i] is not None else None
            if z is not None and len(z):
                picked = rng.choice(len(z), int(min(len(z), rng.integers(1, 3))), replace=False)
                for zi in picked:
                    zid = int(z["id"][zi])
                    ko = 0
                    if t is not None and rng.random() < 0.6:  # a cpuset on this zone
                        free = np.flatnonzero((t["numa_id"] == zid) & (t["ref_count"] == 0) & (t["reserved"] == 0))
                        k = int(min(len(free), rng.choice([2, 4, 6])))
                        if k == 0:
                            continue
                        cpus = t["cpu_id"][free[:k]]
                        t["ref_count"][free[:k]] += 1
                        for c in cpus:
                            a["cpuset"][c >> 6] |= np.uint64(1) << np.uint64(c & 63)
                        cpu = k * 1000
                        if z["single_pods"][zi] == 0 and z["shared_pods"][zi] == 0:  # a status without counts: one pod
                            z["single_pods"][zi] = int(z["numa_status"][zi] == abi.NUMA_STATUS_SINGLE)
                            z["shared_pods"][zi] = int(z["numa_status"][zi] == abi.NUMA_STATUS_SHARED)
                        z["single_pods"][zi] += 1
                        z["numa_status"][zi] = abi.NUMA_STATUS_SHARED if z["shared_pods"][zi] else abi.NUMA_STATUS_SINGLE
                        if owners:
                            ko = int(rng.integers(1, k + 1))
                            t["ref_count"][free[:ko]] += 1
                            for c in cpus[:ko]:
                                a["owner_cpuset"][c >> 6] |= np.uint64(1) << np.uint64(c & 63)
                            a["owner_numa"][2 * zid] += ko * 1000
                            z["allocated"][zi, 0] += ko * 1000
                            cpu_owned += ko * 1000
                            z["single_pods"][zi] += 1
                    else:
                        cpu = int(rng.choice([1000, 2000, 2500, 4000]))
                    mem = int(rng.choice([1, 2, 4])) * GI
                    a["numa"][2 * zid] += cpu
                    a["numa"][2 * zid + 1] += mem
                    cpu_total += cpu
                    mem_total += mem
                    z["has_allocated"][zi] = abi.NUMA_ALLOC_ENTRY | abi.NUMA_ALLOC_CPU | abi.NUMA_ALLOC_MEMORY
                    z["allocated"][zi, 0] += cpu
                    z["allocated"][zi, 1] += mem
                    if owners:
                        oc = 0 if ko else cpu // 2 // 1000 * 1000  # (a cpuset zone's owners hold CPUs above)
                        om = mem // 2
                        a["owner_numa"][2 * zid] += oc
                        a["owner_numa"][2 * zid + 1] += om
                        z["allocated"][zi, 0] += oc
                        z["allocated"][zi, 1] += om
                        cpu_owned += oc
                        mem_owned += om
                if a["numa"].any():
                    holds |= abi.RSV_HOLDS_NUMA
                if a["cpuset"].any():
                    holds |= abi.RSV_HOLDS_CPUSET
            d = devices[i] if devices is not None else None
            if d is not None and len(d) and rng.random() < 0.7:
                cand = [j for j in range(len(d)) if d["health"][j] and
                        (d["used"][j, 0] if d["has_used"][j, 0] else 0) <= d["total"][j, 0] - 50]
                if cand:
                    j = int(rng.choice(cand))
                    ty, mi = int(d["type"][j]), int(d["minor"][j])
                    nk = 3 if ty == abi.DEV_GPU else 1
                    share = 50
                    amt = [share, int(d["total"][j, 1]) * share // 100, share][:nk] if ty == abi.DEV_GPU else [share]
                    a["device_minors"] |= np.uint64(1) << np.uint64(16 * ty + mi)
                    for k in range(nk):
                        a["device"][ty, mi, k] = amt[k]
                        d["used"][j, k] = (d["used"][j, k] if d["has_used"][j, k] else 0) + amt[k]
                        d["has_used"][j, k] = 1
                    if owners:
                        a["owner_device_minors"] |= np.uint64(1) << np.uint64(16 * ty + mi)
                        for k in range(nk):
                            o = amt[k] // 2
                            a["owner_device"][ty, mi, k] = o
                            d["used"][j, k] += o
                    holds |= abi.RSV_HOLDS_DEVICES
            if holds == 0 and rng.random() < 0.5:
                continue
            cpu_total = cpu_total or int(rng.choice([2000, 4000]))
            mem_total = mem_total or int(rng.choice([2, 4])) * GI
            e = device_resource_entries(a)
            r["holds"] = holds | (abi.RSV_OTHER_ALLOCATABLE if len(e) else 0)
            r["allocatable"][:] = [cpu_total, mem_total]
            if owners:
                r["allocated"][:] = [max(cpu_owned, 1000), max(mem_owned, GI)]
            # the reserve pod and its owners are pods of the node (NodeInfo.Requested / Pods)
            cl.nodes["requested"][i, 0] += cpu_total + (r["allocated"][0] if owners else 0)
            cl.nodes["requested"][i, 1] += mem_total + (r["allocated"][1] if owners else 0)
            cl.nodes["pod_count"][i] += 1 + int(r["allocated_pods"])
            rs.append(r)
            al.append(a)
            res.append(e)
    return np.array(rs, abi.RESERVATION_DTYPE), np.array(al, abi.RESERVATION_ALLOC_DTYPE), res
