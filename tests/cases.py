"""Turn the JSON golden fixtures (tests/golden/*.json) into calls on a cluster handle — the oracle
(oracle.binding.Oracle) or the product (koordinator_amd.Evaluator); both expose the same methods."""
import json
import os

from koordinator_amd import abi, model

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NOW = 1_760_000_000 * model.NS  # the instant the plugin method runs (fixture offsets are relative)
S = model.NS


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)["cases"]


def t(offset_s):
    return None if offset_s is None else NOW + int(round(offset_s * S))


def make_cfg(case, n_nodes=1):
    """v1beta3-defaulted args with the case's overrides (the Go tests call SetDefaults_* first)."""
    cfg = abi.default_config(n_nodes)
    a = cfg.loadaware
    args = case.get("args", {})
    if "filter_expired_node_metrics" in args:
        a.filter_expired_node_metrics = int(args["filter_expired_node_metrics"])
    if "enable_schedule_when_node_metrics_expired" in args:
        a.enable_schedule_when_node_metrics_expired = int(args["enable_schedule_when_node_metrics_expired"])
    if "score_according_prod_usage" in args:
        a.score_according_prod_usage = int(args["score_according_prod_usage"])
    if "allow_customize_estimation" in args:
        a.allow_customize_estimation = int(args["allow_customize_estimation"])
    if "usage_thresholds" in args:  # SetDefaults only fills an empty map
        a.usage_thresholds[:] = [abi.ABSENT, abi.ABSENT]
        for k, v in args["usage_thresholds"].items():
            a.usage_thresholds[model.RESOURCE_INDEX[k]] = v
    if "prod_usage_thresholds" in args:
        for k, v in args["prod_usage_thresholds"].items():
            a.prod_usage_thresholds[model.RESOURCE_INDEX[k]] = v
    if "estimated_scaling_factors" in args:  # merged with the defaults (defaults.go:105-113)
        for k, v in args["estimated_scaling_factors"].items():
            a.estimated_scaling_factors[model.RESOURCE_INDEX[k]] = v
    agg = args.get("aggregated")
    if agg is not None:
        a.has_aggregated = 1
        for k, v in agg.get("usage_thresholds", {}).items():
            a.agg_usage_thresholds[model.RESOURCE_INDEX[k]] = v
        a.agg_usage_type = model.AGG_BY_NAME[agg.get("usage_aggregation_type", "")]
        a.agg_usage_duration_ns = int(agg.get("usage_aggregated_duration_s", 0) * S)
        a.agg_score_type = model.AGG_BY_NAME[agg.get("score_aggregation_type", "")]
        a.agg_score_duration_ns = int(agg.get("score_aggregated_duration_s", 0) * S)
    na = case.get("numa_args")
    if na:
        cfg.numa.strategy = abi.STRATEGY_MOST_ALLOCATED if na["strategy"] == "MostAllocated" else abi.STRATEGY_LEAST_ALLOCATED
        cfg.numa.weights[:] = [abi.ABSENT, abi.ABSENT]
        for k, v in na["weights"].items():
            cfg.numa.weights[model.RESOURCE_INDEX[k]] = v
    return cfg


def make_pod(spec):
    spec = dict(spec)
    kw = {}
    for k in ("name", "namespace", "requests", "limits", "containers", "priority", "labels", "owner_kind",
              "custom_factors"):
        if k in spec:
            kw[k] = spec[k]
    return model.make_pod(**kw)


def make_la_node(spec):
    ca = spec.get("custom_aggregated")
    if ca is not None:
        ca = {"thresholds": ca.get("thresholds"), "type": ca.get("type", ""),
              "duration_ns": int(ca.get("duration_s", 0) * S)}
    return model.make_node(allocatable=spec.get("allocatable"),
                           custom_usage_thresholds=spec.get("custom_usage_thresholds"),
                           custom_prod_usage_thresholds=spec.get("custom_prod_usage_thresholds"),
                           custom_aggregated=ca)


def make_nm(spec):
    aggs = [{"duration_ns": int(a["duration_s"] * S), "usage": a["usage"]} for a in spec.get("aggregated", [])]
    return model.make_node_metric(update_time=t(spec.get("update_time_s")),
                                  report_interval_seconds=spec.get("report_interval_seconds"),
                                  node_usage=spec.get("node_usage"), has_node_metric=spec.get("has_node_metric", True),
                                  pods=spec.get("pods", []), aggregated=aggs)


def setup_loadaware(handle, case):
    """One-node cluster of a LoadAware case on `handle`; returns the pod under test."""
    handle.upsert_node(0, make_la_node(case["node"]))
    if case.get("node_metric") is not None:
        handle.set_nodemetric(0, make_nm(case["node_metric"]))
    for ap in case.get("assigned_pods", []):
        spec = dict(ap["pod"])
        pod = make_pod(spec)
        if "scheduled_at_s" in ap:
            pod.has_scheduled = 1
            pod.scheduled_transition_ns = t(ap["scheduled_at_s"])
        handle.assign(0, pod, t(ap.get("timestamp_s", -0.001)))
    return make_pod(case.get("pod", {}))


def make_numa_nodes(case):
    """makeNode (plugin_test.go:123-129) + existing pods folded into NodeInfo.Requested and the
    resource manager's cpuset allocation (only recorded on nodes with NRT)."""
    nodes = []
    nrt = case.get("nrt", [False] * len(case["nodes"]))
    for i, spec in enumerate(case["nodes"]):
        cpu_m = model.milli_value(spec["capacity_cpu"])
        ratio = spec["amplification_ratio"]
        amp_cpu = cpu_m if ratio <= 1 else int(-(-cpu_m * ratio // 1))
        n = model.make_node(allocatable={"cpu": f"{amp_cpu}m", "memory": spec["memory"]},
                            raw_allocatable={"cpu": spec["capacity_cpu"], "memory": spec["memory"]},
                            amplification_ratio=ratio)
        req_cpu = req_mem = cpus = 0
        for e in case.get("existing", []):
            if e["node"] != i:
                continue
            req_cpu += model.milli_value(e.get("cpu", "0"))
            req_mem += model.value(e.get("memory", "0"))
            if e.get("cpuset") and nrt[i]:
                cpus += model.milli_value(e["cpu"]) // 1000
        n.requested[:] = [req_cpu, req_mem]
        n.cpuset_allocated_cpus = cpus
        nodes.append(n)
    return nodes


# ---- DeviceShare -----------------------------------------------------------------------------------
def ds_cfg(case, n_nodes=1):
    cfg = abi.default_config(n_nodes)
    if case.get("strategy") == "MostAllocated":
        cfg.deviceshare.strategy = abi.STRATEGY_MOST_ALLOCATED
    return cfg


def ds_pod(case):
    """A pod whose only requests are the case's device requests (the Go tests build the pod from
    preFilterState.podRequests, plugin_test.go:2614-2629)."""
    return model.make_pod(requests=dict(case["pod"]["requests"]))


def setup_ds(handle, case, node=0):
    """Node `node` of `handle` gets the case's device cache (or none) and a big allocatable so that the
    LoadAware / NodeNUMAResource filters pass; returns the pod."""
    handle.upsert_node(node, model.make_node(allocatable={"cpu": "96", "memory": "512Gi"}))
    if case.get("cache", True):
        handle.set_devices(node, model.make_devices(case["devices"]))
    return ds_pod(case)


def rl3(dev_type, rl):
    vals, has = [0, 0, 0], [0, 0, 0]
    for k, v in rl.items():
        key = model.DEVICE_KEYS[dev_type][k]
        vals[key] = model.value(v)
        has[key] = 1
    return vals, has


# ---- NodeNUMAResource non-cpuset NUMA vectors (numa_policy.json ops affinity/distribute/hints/available)
NUMA_POLICY_ID = {"None": 0, "BestEffort": 1, "Restricted": 2, "SingleNUMANode": 3}


def numa_case_cfg(case):
    cfg = abi.default_config(1)
    if case.get("numa_strategy") == "MostAllocated":
        cfg.numa.numa_strategy = abi.STRATEGY_MOST_ALLOCATED
    return cfg


def numa_case_zones(case):
    """The case's zones (+ allocation entries and cpusets) as model.make_zones input."""
    if case["op"] == "affinity":
        n = case["zones"]
        cpu_m = model.milli_value(case["node"]["cpu"]) // n
        mem = model.value(case["node"]["memory"]) // n
        zones = []
        for k in range(n):
            z = {"id": k, "cpu": f"{cpu_m}m", "memory": str(mem)}
            ex = case["existing"].get(str(k), case["existing"].get(k, []))
            if ex:
                z["allocated"] = {"cpu": f"{sum(model.milli_value(p['cpu']) for p in ex)}m",
                                  "memory": str(sum(model.value(p["memory"]) for p in ex))}
            zones.append(z)
        return zones
    zones = []
    for k, z in enumerate(case["zones"]):
        z = dict(z)
        al = (case.get("allocated") or [None] * len(case["zones"]))[k]
        if al is not None:
            z["allocated"] = dict(al)
        cs = (case.get("cpusets") or [0] * len(case["zones"]))[k]
        if cs:
            z["cpuset_cpus"] = cs
        zones.append(z)
    return zones


def setup_numa_case(handle, case):
    """Node 0 of `handle` with the case's policy, amplification ratio and zones; returns the pod."""
    n = model.make_node(allocatable=case["node"], amplification_ratio=case.get("ratio"),
                        nrt_amplification_ratio=case.get("nrt_ratio"))
    n.numa_topology_policy = NUMA_POLICY_ID[case.get("policy", "BestEffort")]
    handle.upsert_node(0, n)
    handle.set_numa(0, model.make_zones(numa_case_zones(case)))
    return model.make_pod(requests=dict(case.get("pod", {})))


def quantity_vec(rl):
    """{'cpu': q, 'memory': q} -> [cpu milli, memory bytes]"""
    return [model.milli_value(rl.get("cpu", 0)), model.value(rl.get("memory", 0))]


# ---- CPU accumulator vectors (cpu_accumulator.json) ---------------------------------------------
BIND_ID = {"": 0, "None": 0, "FullPCPUs": 1, "SpreadByPCPUs": 2}
CPU_EXCL_ID = {"": 0, "None": 0, "PCPULevel": 1, "NUMANodeLevel": 2}


def test_topology(sockets, nodes_per_socket, cores_per_node, cpus_per_core, core_shift=False):
    """buildCPUTopologyForTest (cpu_accumulator_test.go:30-57): rows [cpu, core, node, socket]."""
    rows, node, core, cpu = [], 0, 0, 0
    for s in range(sockets):
        for _ in range(nodes_per_socket):
            for _ in range(cores_per_node):
                for _ in range(cpus_per_core):
                    rows.append([cpu, (s << 16 | core) if core_shift else core, node, s])
                    cpu += 1
                core += 1
            node += 1
    return rows


def parse_cpuset(s):
    """cpuset.MustParse: '0-3,8' -> sorted list"""
    out = []
    for part in filter(None, (s or "").split(",")):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(out)


def cpu_bits(cpus):
    import numpy as np
    b = np.zeros(4, np.uint64)
    for c in cpus:
        b[c >> 6] |= np.uint64(1) << np.uint64(c & 63)
    return b


def bits_cpus(b):
    return [c for c in range(256) if (int(b[c >> 6]) >> (c & 63)) & 1]


# ---- cpuset Filter / Reserve vectors (cpuset.json) ------------------------------------------------
def cpuset_pod(spec):
    kind = spec["kind"]
    if kind == "be":
        return model.make_pod(requests={"kubernetes.io/batch-cpu": "4000"}, priority=5500)
    labels = {"koordinator.sh/qosClass": "LSR" if kind == "cpuset" else "LS"}
    return model.make_pod(requests={"cpu": spec["cpu"]}, labels=labels, priority=9500,
                          cpu_bind_required=spec.get("required") or None,
                          cpu_bind_preferred=spec.get("preferred") or None)


def setup_cpuset_case(handle, case):
    n = model.make_node(allocatable={"cpu": "96", "memory": "512Gi"}, amplification_ratio=case.get("ratio"),
                        cpu_topology_invalid=case.get("invalid_topology", False))
    n.cpu_bind_policy = model.NODE_CPU_BIND_BY_NAME[case["node_bind"]]
    n.numa_allocate_strategy = {"": 0, "MostAllocated": 1, "LeastAllocated": 2}[case.get("numa_allocate_strategy", "")]
    handle.upsert_node(0, n)
    if not case.get("invalid_topology"):
        rows = test_topology(*case["topology"])
        allocated = {c: (1, None) for c in parse_cpuset(case.get("allocated", ""))}
        handle.set_cpus(0, model.make_cpus(rows, allocated))
    return cpuset_pod(case["pod"])


# ---- cpusets under NUMA policies (numa_cpuset.json) ----------------------------------------------
def numa_cpuset_pod(spec):
    """A binding pod (LSR koord-prod with a required bind policy) or a plain cpu pod."""
    if spec.get("bind"):
        return cpuset_pod({"kind": "cpuset", "cpu": spec["cpu"], "required": spec["bind"]})
    p = model.make_pod(requests={"cpu": spec["cpu"]})
    if spec.get("other"):
        p.has_other_requests = 1
    return p


def setup_numa_cpuset_case(handle, case):
    """Node 0: the resource-manager tests' node, zones with the case's allocation entries, CPU table
    with the allocated CPUs (RefCount 1)."""
    n = model.make_node(allocatable=case["node"], amplification_ratio=case.get("ratio"))
    handle.upsert_node(0, n)
    zones = [dict(z) for z in case["zones"]]
    allocated = case.get("allocated")
    if allocated:
        for e in allocated["numa"]:
            zones[e["id"]]["allocated"] = {"cpu": e["cpu"]}
    handle.set_numa(0, model.make_zones(zones))
    busy = {c: (1, None) for c in parse_cpuset(allocated["cpuset"])} if allocated else {}
    handle.set_cpus(0, model.make_cpus(test_topology(*case["topology"]), busy))
    return numa_cpuset_pod(case["pod"])


def setup_numa_score_case(handle, case):
    """TestNUMANodeScore nodes: zones = allocatable / count, existing pods' requests on NUMA 0, their
    cpusets 0..cpu-1 for LSR koord-prod pods; returns the pod."""
    for i, nd in enumerate(case["nodes"]):
        n = model.make_node(allocatable={"cpu": nd["cpu"], "memory": nd["memory"]})
        n.numa_topology_policy = NUMA_POLICY_ID[nd["policy"]]
        handle.upsert_node(i, n)
        cnt = nd["numa"]
        cpu_m, mem = model.milli_value(nd["cpu"]), model.value(nd["memory"])
        zones = [{"id": k, "cpu": f"{cpu_m // cnt}m", "memory": str(mem // cnt)} for k in range(cnt)]
        ex = [e for e in case["existing"] if e["node"] == i]
        if ex:
            zones[0]["allocated"] = {"cpu": f"{sum(model.milli_value(e['cpu']) for e in ex)}m",
                                     "memory": str(sum(model.value(e["memory"]) for e in ex))}
        refs = {}
        for e in ex:
            if e["lsr"]:
                for c in range(model.milli_value(e["cpu"]) // 1000):
                    refs[c] = refs.get(c, 0) + 1
        if refs:  # addPodAllocation: the LSR pods' CPUs (NUMA 0) make it a single-NUMA node
            zones[0]["status"] = "single"
        handle.set_numa(i, model.make_zones(zones))
        rows = test_topology(cnt, 1, cpu_m // 1000 // 2 // cnt, 2)
        handle.set_cpus(i, model.make_cpus(rows, {c: (r, None) for c, r in refs.items()}), max(refs.values(), default=1))
    p = case["pod"]
    if p["lsr"]:
        return model.make_pod(requests={"cpu": p["cpu"], "memory": p["memory"]},
                              labels={"koordinator.sh/qosClass": "LSR"}, priority=9500)
    return model.make_pod(requests={"cpu": p["cpu"], "memory": p["memory"]})
