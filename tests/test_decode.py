"""Wire-format decoders, CPU only: the product's C++ decoders (ke_decode_* through the
C ABI) against the reference's own apis/extension test vectors (tests/golden/decode.json) and, field by field,
against model.py — the independent Python statement of the same apimachinery / apis/extension rules the tests
have used since round 1 — on generated objects."""
import ctypes as C
import json
from fractions import Fraction

import numpy as np
import pytest

import cases
from koordinator_amd import abi, decode, model

DEC = cases.load("decode.json")


@pytest.mark.parametrize("case", [c for c in DEC if c["kind"] == "nrt"], ids=lambda c: c["name"])
def test_decode_nrt_golden(lib, case):
    node = decode.decode_node({"metadata": {"name": "n"}})
    zones, cpus = decode.decode_nrt(case["object"], node)
    w = case["want"]
    assert [[int(z["id"]), int(z["capacity"][0])] for z in zones] == w["zone_cpu"], case["source"]
    assert all(z["has"][0] == 1 and z["has"][1] == 0 for z in zones)
    assert [[int(c["cpu_id"]), int(c["core_id"]), int(c["numa_id"]), int(c["socket_id"])] for c in cpus] == w["cpus"]
    assert [int(c["cpu_id"]) for c in cpus if c["reserved"]] == w["reserved"]
    assert node.cpu_topology_invalid == 0 and node.nrt_cpu_amplification_ratio == -2.0
    # options {"static": "true"} is not full-pcpus-only: the node keeps no CPU bind policy
    assert node.cpu_bind_policy == 0


def test_decode_nrt_policy_and_kubelet(lib):
    node = decode.decode_node({"metadata": {"name": "n"}})
    nrt = {"topologyPolicies": ["None", "SingleNUMANodePodLevel"],
           "metadata": {"annotations": {"kubelet.koordinator.sh/cpu-manager-policy":
                                        '{"policy":"static","options":{"full-pcpus-only":"true"}}',
                                        "node.koordinator.sh/resource-amplification-ratio": '{"memory":1.5}'}},
           "zones": [{"name": "node-1", "type": "Node", "resources": [{"name": "memory", "allocatable": "64Gi"}]},
                     {"name": "node-0", "type": "Node", "resources": [{"name": "memory", "allocatable": "64Gi"}]},
                     {"name": "socket-0", "type": "Socket"}, {"name": "node-x", "type": "Node"}]}
    zones, cpus = decode.decode_nrt(nrt, node)
    assert [int(z["id"]) for z in zones] == [0, 1] and len(cpus) == 0
    assert int(zones[0]["capacity"][1]) == 64 * 2**30 and zones[0]["has"][0] == 0
    assert node.numa_topology_policy == abi.NUMA_POLICY_SINGLE_NUMA_NODE
    assert node.cpu_bind_policy == 1 and node.cpu_topology_invalid == 1
    assert node.nrt_cpu_amplification_ratio == 0.0  # a ratio map without cpu: Go's zero value
    labelled = decode.decode_node({"metadata": {"labels": {"node.koordinator.sh/numa-topology-policy": "Restricted"}}})
    decode.decode_nrt(nrt, labelled)
    assert labelled.numa_topology_policy == abi.NUMA_POLICY_RESTRICTED  # the label wins (getNUMATopologyPolicy)


@pytest.mark.parametrize("case", [c for c in DEC if c["kind"] == "device"], ids=lambda c: c["name"])
def test_decode_device_golden(lib, case):
    w = case["want"]
    if w.get("error"):
        with pytest.raises(decode.DecodeError):
            decode.decode_device(case["object"])
        return
    _, (has_table, honor, parts) = decode.decode_device(case["object"])
    if "has_table" in w:
        assert int(has_table) == w["has_table"], case["source"]
        got = [[int(p["minors"]), int(p["number_of_gpus"]), int(p["allocation_score"]), int(p["ring_bus_bandwidth"])]
               for p in parts]
        assert got == w["partitions"], case["source"]
    if "honor" in w:
        assert int(honor) == w["honor"], case["source"]


@pytest.mark.parametrize("case", [c for c in DEC if c["kind"] in ("node", "pod")], ids=lambda c: c["name"])
def test_decode_golden(lib, case):
    obj = decode.decode_node(case["object"]) if case["kind"] == "node" else decode.decode_pod(case["object"])
    for k, v in case["want"].items():
        assert getattr(obj, k) == v, (case["source"], k)


# ---- resource.Quantity ----------------------------------------------------------------------------------
QUANTITIES = ["0", "1", "100m", "1.5", "0.5", "512Gi", "1Ki", "1k", "1M", "1G", "1T", "1P", "1e3", "1E3",
              "1e-3", "2.5e2", "+3", "1n", "1u", "0.1m", "1500m", "0.0001", "123456789", "3.14159", "1.0Gi", "007",
              "16Gi", "0.25Ki", "1e+2", "10Mi", "96", "0.000000001", "1.000000001", "4.5G"]
INVALID = ["", "abc", "1.2.3", " 1", "1 ", "Ki", "1e", "1Qi", "1KiB", ".", "1..2", "--1", "1e3.5", "m"]


@pytest.mark.parametrize("q", QUANTITIES)
def test_quantity(lib, q):
    assert decode.parse_quantity(q) == (model.value(q), model.milli_value(q))


@pytest.mark.parametrize("q", INVALID)
def test_quantity_invalid(lib, q):
    with pytest.raises(decode.DecodeError) as e:
        decode.parse_quantity(q)
    assert e.value.code == abi.ERR_INVALID


def test_quantity_out_of_range(lib):
    for q in ("-1", "9Ei", "1e30", "99999999999999999999", "1E", "2Ei"):  # MilliValue beyond int64
        with pytest.raises(decode.DecodeError) as e:
            decode.parse_quantity(q)
        assert e.value.code == abi.ERR_UNSUPPORTED


def test_quantity_random(lib):
    rng = np.random.default_rng(7)
    sufs = ["", "m", "k", "M", "G", "Ki", "Mi", "Gi", "e2", "e-2", "n", "u"]
    for _ in range(400):
        whole = int(rng.integers(0, 10**int(rng.integers(1, 8))))
        frac = "" if rng.random() < 0.5 else "." + str(int(rng.integers(0, 10**int(rng.integers(1, 6))))).zfill(3)
        q = f"{whole}{frac}{sufs[int(rng.integers(0, len(sufs)))]}"
        if model.milli_value(q) >= 2**63:  # MilliValue beyond int64: refused (KE_ERR_UNSUPPORTED)
            with pytest.raises(decode.DecodeError):
                decode.parse_quantity(q)
            continue
        assert decode.parse_quantity(q) == (model.value(q), model.milli_value(q)), q


# ---- Node ---------------------------------------------------------------------------------------------------
def node_doc(allocatable, annotations=None, labels=None):
    return {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n", "annotations": annotations or {},
                                                           "labels": labels or {}},
            "status": {"allocatable": allocatable, "capacity": allocatable}}


def same(a, b, skip=()):
    for name, _ in a._fields_:
        if name in skip or name.startswith("pad"):
            continue
        x, y = getattr(a, name), getattr(b, name)
        if hasattr(x, "_length_"):
            x, y = list(x), list(y)
        if isinstance(x, C.Structure):
            same(x, y)
            continue
        if x and hasattr(x[0] if isinstance(x, list) else None, "_fields_"):
            for u, v in zip(x, y):
                same(u, v)
            continue
        assert x == y, (name, x, y)


def test_node_thresholds_ratio_raw_labels(lib):
    th = {"usageThresholds": {"cpu": 60, "memory": 80}, "prodUsageThresholds": {"cpu": 50},
          "aggregatedUsage": {"usageThresholds": {"memory": 70}, "usageAggregationType": "p95",
                              "usageAggregatedDuration": "5m"}}
    doc = node_doc({"cpu": "96", "memory": "512Gi", "pods": "110"},
                   {"scheduling.koordinator.sh/usage-thresholds": json.dumps(th),
                    "node.koordinator.sh/resource-amplification-ratio": '{"cpu":1.5}',
                    "node.koordinator.sh/raw-allocatable": '{"cpu":"64","memory":"500Gi"}'},
                   {"node.koordinator.sh/numa-topology-policy": "SingleNUMANode",
                    "node.koordinator.sh/cpu-bind-policy": "FullPCPUsOnly",
                    "node.koordinator.sh/numa-allocate-strategy": "MostAllocated"})
    got = decode.decode_node(doc)
    want = model.make_node(allocatable={"cpu": "96", "memory": "512Gi", "pods": "110"},
                           raw_allocatable={"cpu": "64", "memory": "500Gi"},
                           amplification_ratio=1.5, custom_usage_thresholds={"cpu": 60, "memory": 80},
                           custom_prod_usage_thresholds={"cpu": 50},
                           custom_aggregated=dict(thresholds={"memory": 70}, type="p95", duration_ns=300 * 10**9))
    want.numa_topology_policy = abi.NUMA_POLICY_SINGLE_NUMA_NODE
    want.cpu_bind_policy = 1
    want.numa_allocate_strategy = 1
    same(got, want)


def test_node_annotation_errors(lib):
    got = decode.decode_node(node_doc({"cpu": "8"}, {"scheduling.koordinator.sh/usage-thresholds": '{"usageThresholds":{"cpu":"60"}}',
                                                     "node.koordinator.sh/raw-allocatable": "{bad"}))
    assert got.custom_thresholds_error == 1 and got.has_custom_thresholds == 0
    assert list(got.raw_allocatable) == [abi.ABSENT, abi.ABSENT]  # EstimateNode falls back to Allocatable
    got = decode.decode_node(node_doc({"cpu": "8"}, {"scheduling.koordinator.sh/usage-thresholds": '{"UsageThresholds":{"cpu":61}}'}))
    assert got.has_custom_thresholds == 1 and list(got.custom_usage_thresholds) == [61, abi.ABSENT]  # Go: case-insensitive
    got = decode.decode_node(node_doc({"cpu": "8"}, {"scheduling.koordinator.sh/usage-thresholds": '{"usageThresholds":{"cpu":61.5}}'}))
    assert got.custom_thresholds_error == 1
    for ann, lab in (({"scheduling.koordinator.sh/usage-thresholds": '{"usageThresholds":{"nvidia.com/gpu":50}}'}, {}),
                     ({}, {"node.koordinator.sh/numa-topology-policy": "Whatever"})):
        with pytest.raises(decode.DecodeError) as e:
            decode.decode_node(node_doc({"cpu": "8"}, ann, lab))
        assert e.value.code == abi.ERR_UNSUPPORTED
    for bad in ("{", "[]", '{"metadata": {"labels": {"a": 1}}}', '{"status": {"allocatable": {"cpu": "x"}}}'):
        with pytest.raises(decode.DecodeError) as e:
            decode.decode_node(bad)
        assert e.value.code == abi.ERR_INVALID


# ---- NodeMetric ---------------------------------------------------------------------------------------------
def test_node_metric(lib):
    doc = {"apiVersion": "slo.koordinator.sh/v1alpha1", "kind": "NodeMetric", "metadata": {"name": "n"},
           "spec": {"metricCollectPolicy": {"reportIntervalSeconds": 60}},
           "status": {"updateTime": "2025-10-15T12:00:00Z",
                      "nodeMetric": {"nodeUsage": {"resources": {"cpu": "12500m", "memory": "64Gi"}},
                                     "aggregatedNodeUsages": [
                                         {"usage": {"p95": {"resources": {"cpu": "20", "memory": "100Gi"}},
                                                    "avg": {"resources": {"cpu": "10"}}}, "duration": "5m0s"}]},
                      "podsMetric": [{"namespace": "default", "name": "a", "priority": "koord-prod",
                                      "podUsage": {"resources": {"cpu": "1", "memory": "1Gi", "nvidia.com/gpu": "1"}}},
                                     None,
                                     {"namespace": "x", "name": "b", "podUsage": {"resources": {"memory": "2Gi"}}}]}}
    nm, pms, n_pm, aggs, n_agg = decode.decode_node_metric(doc)
    t = 1760529600 * 10**9  # 2025-10-15T12:00:00Z
    want, wpm, wn, wagg, wna = model.make_node_metric(
        update_time=t, report_interval_seconds=60, node_usage={"cpu": "12500m", "memory": "64Gi"},
        pods=[dict(namespace="default", name="a", priority="koord-prod", usage={"cpu": "1", "memory": "1Gi",
                                                                              "nvidia.com/gpu": "1"}),
              dict(namespace="x", name="b", usage={"memory": "2Gi"})],
        aggregated=[dict(duration_ns=300 * 10**9, usage={"p95": {"cpu": "20", "memory": "100Gi"}, "avg": {"cpu": "10"}})])
    same(nm, want)
    assert (n_pm, n_agg) == (wn, wna)
    for i in range(n_pm):
        same(pms[i], wpm[i], skip=("pod_key",))
    assert pms[0].pod_key == decode.pod_key("default", "a") and pms[1].pod_key == decode.pod_key("x", "b")
    same(aggs[0], wagg[0])


@pytest.mark.parametrize("ts,ns", [("1970-01-01T00:00:00Z", 0), ("2024-02-29T23:59:59+01:00", 1709247599 * 10**9),
                                   ("2025-10-15T12:00:00.5Z", 1760529600 * 10**9 + 5 * 10**8)])
def test_rfc3339(lib, ts, ns):
    nm = decode.decode_node_metric({"status": {"updateTime": ts}})[0]
    assert nm.has_update_time == 1 and nm.update_time_ns == ns


@pytest.mark.parametrize("d,ns", [("5m", 300 * 10**9), ("1h30m", 5400 * 10**9), ("1.5s", 1500 * 10**6), ("300ms", 3 * 10**8),
                                  ("0", 0), ("2h45m30.5s", (2 * 3600 + 45 * 60 + 30) * 10**9 + 5 * 10**8)])
def test_duration(lib, d, ns):
    th = {"aggregatedUsage": {"usageThresholds": {"cpu": 50}, "usageAggregationType": "avg", "usageAggregatedDuration": d}}
    got = decode.decode_node(node_doc({}, {"scheduling.koordinator.sh/usage-thresholds": json.dumps(th)}))
    assert got.custom_agg_duration_ns == ns


# ---- Pod ----------------------------------------------------------------------------------------------------
def _q(rng, kind):
    if kind == "cpu":
        return rng.choice(["100m", "250m", "1", "2", "4", "1500m"])
    if kind == "memory":
        return rng.choice(["128Mi", "1Gi", "2Gi", "512M", "1.5Gi"])
    return rng.choice(["1", "2", "1000", "4Gi"])


def random_pod(rng, i):
    names = ["cpu", "memory", "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory", "nvidia.com/gpu",
             "ephemeral-storage", "koordinator.sh/rdma", "dcu.com/gpu", "huawei.com/npu-core"]
    def rl():
        return {n: str(_q(rng, n)) for n in names if rng.random() < (0.6 if n in ("cpu", "memory") else 0.15)}
    cs = [{"name": f"c{k}", "resources": {"requests": rl(), "limits": rl()}} for k in range(int(rng.integers(0, 3)))]
    ics = [{"name": f"i{k}", "resources": {"requests": rl()}} for k in range(int(rng.integers(0, 2)))]
    labels, ann = {}, {}
    if rng.random() < 0.4:
        labels["koordinator.sh/priority-class"] = str(rng.choice(["koord-prod", "koord-batch", "koord-mid", "koord-free", "x"]))
    if rng.random() < 0.4:
        labels["koordinator.sh/qosClass"] = str(rng.choice(["LSE", "LSR", "LS", "BE", "SYSTEM"]))
    if rng.random() < 0.2:
        labels["quota.scheduling.koordinator.sh/preemptible"] = "false"
    factors = None
    if rng.random() < 0.2:
        factors = {"cpu": int(rng.integers(50, 100)), "memory": int(rng.integers(50, 100))}
        ann["scheduling.koordinator.sh/load-estimated-scaling-factors"] = json.dumps(factors)
    bind = excl = None
    if rng.random() < 0.3:
        bind = str(rng.choice(["FullPCPUs", "SpreadByPCPUs", "Default"]))
        excl = str(rng.choice(["PCPULevel", "NUMANodeLevel", "None"]))
        ann["scheduling.koordinator.sh/resource-spec"] = json.dumps({"preferredCPUBindPolicy": bind,
                                                                     "preferredCPUExclusivePolicy": excl})
    numa = None
    if rng.random() < 0.2:
        numa = str(rng.choice(["BestEffort", "Restricted", "SingleNUMANode"]))
        ann["scheduling.koordinator.sh/numa-topology-spec"] = json.dumps({"numaTopologyPolicy": numa})
    spec = {"containers": cs, "initContainers": ics}
    prio = None
    if rng.random() < 0.5:
        prio = int(rng.choice([9500, 7500, 5500, 3500, 100]))
        spec["priority"] = prio
    overhead = None
    if rng.random() < 0.1:
        overhead = {"cpu": "100m", "memory": "64Mi"}
        spec["overhead"] = overhead
    status_qos = None
    if rng.random() < 0.3:  # Status.QOSClass as the apiserver reports it (may disagree with the containers)
        status_qos = str(rng.choice(["Guaranteed", "Burstable", "BestEffort"]))
    owner = "DaemonSet" if rng.random() < 0.1 else "ReplicaSet"
    sched = 1_700_000_000 * 10**9 + i * 10**9
    doc = {"metadata": {"name": f"p{i}", "namespace": "ns", "uid": f"uid-{i}", "labels": labels, "annotations": ann,
                        "ownerReferences": [{"kind": owner, "name": "o"}]},
           "spec": spec,
           "status": {"phase": "Running", "conditions": [{"type": "PodScheduled", "status": "True",
                                                          "lastTransitionTime": "2023-11-14T22:13:%02dZ" % (20 + i % 40)}]}}
    if status_qos:
        doc["status"]["qosClass"] = status_qos
    kw = dict(containers=[{"requests": c["resources"]["requests"], "limits": c["resources"]["limits"]} for c in cs],
              init_containers=[{"requests": c["resources"]["requests"]} for c in ics], overhead=overhead,
              priority=prio, labels=labels, owner_kind=owner, custom_factors=factors, numa_policy=numa,
              cpu_bind_preferred=bind, cpu_exclusive=excl, status_qos=status_qos)
    return doc, kw


def test_pod_random_vs_model(lib):
    rng = np.random.default_rng(11)
    xres = ["cpu", "memory", "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory", "nvidia.com/gpu", "ephemeral-storage",
            "koordinator.sh/rdma", "dcu.com/gpu", "huawei.com/npu-core"]
    for name in xres:
        model.xres_id(name)
    table = sorted(model.XRES_IDS, key=model.XRES_IDS.get)
    for i in range(300):
        doc, kw = random_pod(rng, i)
        if kw["overhead"]:  # calculatePodResourceRequest's Overhead term (PodOverhead gate): refused
            with pytest.raises(decode.DecodeError) as e:
                decode.decode_pod(doc, table)
            assert e.value.code == abi.ERR_UNSUPPORTED
            continue
        got = decode.decode_pod(doc, table)
        want = model.make_pod(**kw)
        want.quota_non_preemptible = 1 if kw["labels"].get("quota.scheduling.koordinator.sh/preemptible") == "false" else 0
        same(got, want, skip=("pod_key", "uid", "has_scheduled", "scheduled_transition_ns", "xres_id", "xres_value"))
        assert got.has_scheduled == 1
        # the FitPlus request list: same (id, value) pairs in any order
        g = sorted(zip(got.xres_id[:got.n_xres], got.xres_value[:got.n_xres]))
        w = sorted(zip(want.xres_id[:want.n_xres], want.xres_value[:want.n_xres]))
        assert g == w, i
        assert got.pod_key == decode.pod_key("ns", f"p{i}")


def test_pod_conditions_phase_and_errors(lib):
    doc = {"metadata": {"name": "a", "namespace": "b"}, "spec": {"containers": [{"resources": {"requests": {"cpu": "1"}}}]},
           "status": {"phase": "Succeeded", "conditions": [
               {"type": "Initialized", "status": "True", "lastTransitionTime": "2023-11-14T22:13:20Z"},
               {"type": "PodScheduled", "status": "False", "lastTransitionTime": "2023-11-14T22:13:20Z"}]}}
    p = decode.decode_pod(doc)
    assert p.is_terminated == 1 and p.has_scheduled == 0 and p.has_initialized == 1
    assert p.initialized_transition_ns == 1_700_000_000 * 10**9
    doc["metadata"]["annotations"] = {"scheduling.koordinator.sh/resource-spec": "{bad"}
    assert decode.decode_pod(doc).has_resource_spec == 1  # PreFilter's unmarshal error, refused by ke_schedule
    doc["metadata"]["annotations"] = {"scheduling.koordinator.sh/load-estimated-seconds-after-pod-scheduled": "30",
                                      "scheduling.koordinator.sh/load-estimated-seconds-after-initialized": "x"}
    p = decode.decode_pod(doc)
    assert p.custom_seconds_after_scheduled == 30 and p.custom_seconds_after_initialized == abi.ABSENT
    sidecar = {"spec": {"initContainers": [{"restartPolicy": "Always", "resources": {"requests": {"cpu": "1"}}}]}}
    with pytest.raises(decode.DecodeError) as e:
        decode.decode_pod(sidecar)
    assert e.value.code == abi.ERR_UNSUPPORTED


def test_pod_device_annotations(lib):
    doc = {"metadata": {"name": "a", "namespace": "b", "annotations": {
        "scheduling.koordinator.sh/gpu-partition-spec": '{"allocatePolicy":"Restricted","ringBusBandwidth":"200Gi"}',
        "scheduling.koordinator.sh/device-allocate-hint": '{"gpu":{"requiredTopologyScope":"PCIe"},"rdma":{"vfSelector":{}}}',
        "scheduling.koordinator.sh/device-joint-allocate": '{"deviceTypes":["gpu","rdma"]}'}},
        "spec": {"containers": [{"resources": {"requests": {"nvidia.com/gpu": "2", "koordinator.sh/rdma": "100"}}}]}}
    got = decode.decode_pod(doc)
    want = model.make_pod(containers=[{"requests": {"nvidia.com/gpu": "2", "koordinator.sh/rdma": "100"}}],
                          gpu_partition_spec={"allocatePolicy": "Restricted", "ringBusBandwidth": "200Gi"},
                          device_hints={"gpu": {"requiredTopologyScope": "PCIe"}, "rdma": {"vfSelector": {}}},
                          device_joint_allocate={"deviceTypes": ["gpu", "rdma"]})
    same(got, want, skip=("pod_key", "uid", "xres_request_mask", "n_xres", "xres_id", "xres_value", "has_other_requests"))
    # without a resource-name table the device names have no id (2); with one (the model's interning) they do (1)
    assert (got.has_other_requests, want.has_other_requests) == (2, 1)
    assert decode.decode_pod(doc, ["cpu", "memory", "nvidia.com/gpu", "koordinator.sh/rdma"]).has_other_requests == 1


# ---- Device -------------------------------------------------------------------------------------------------
def test_device_vs_model(lib):
    gpu = {"koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory": "80Gi", "koordinator.sh/gpu-memory-ratio": "100"}
    devs = [{"type": "gpu", "minor": m, "health": m != 3, "resources": gpu,
             "topology": {"socketID": 0, "nodeID": m // 4, "pcieID": str(m // 2), "busID": f"0000:{m}"}} for m in range(8)]
    devs += [{"type": "rdma", "minor": 1, "health": True, "resources": {"koordinator.sh/rdma": "100"},
              "topology": {"nodeID": 0, "pcieID": "10"}}]
    table = {"1": [{"minors": [m], "allocationScore": 1} for m in range(8)],
             "2": [{"minors": [0, 1], "allocationScore": 2, "ringBusBandwidth": "400Gi"}]}
    doc = {"metadata": {"name": "n", "labels": {"node.koordinator.sh/gpu-partition-policy": "Honor"},
                        "annotations": {"scheduling.koordinator.sh/gpu-partitions": json.dumps(table)}},
           "spec": {"devices": devs}}
    got, (has_table, honor, parts) = decode.decode_device(doc)
    want = model.make_devices([{"type": d["type"], "minor": d["minor"], "health": d["health"],
                                "total": d["resources"] if d["health"] else {}, "topology": d["topology"]} for d in devs])
    assert got.tobytes() == want.tobytes()
    assert has_table and honor
    wt = model.make_gpu_partitions({int(k): v for k, v in table.items()})
    assert parts.tobytes() == wt.tobytes()
    with pytest.raises(decode.DecodeError) as e:
        decode.decode_device({"spec": {"devices": [{"type": "npu", "minor": 0, "health": True}]}})
    assert e.value.code == abi.ERR_UNSUPPORTED


def test_pod_status_qos_class_first(lib):
    """GetKubeQosClass reads Status.QOSClass before computing it (qos_utils.go:72-78): a Burstable-looking pod
    reported Guaranteed defaults to LSR -> koord-prod; reported BestEffort -> koord-batch."""
    base = {"metadata": {"name": "q", "namespace": "n"},
            "spec": {"containers": [{"resources": {"requests": {"cpu": "1"}}}]}}
    assert decode.decode_pod(base).priority_class == abi.PRIORITY_PROD  # computed Burstable -> LS -> prod
    doc = dict(base, status={"qosClass": "BestEffort"})
    assert decode.decode_pod(doc).priority_class == abi.PRIORITY_BATCH
    with pytest.raises(decode.DecodeError):
        decode.decode_pod(dict(base, status={"qosClass": "Platinum"}))


def test_pod_fitplus_request_rounding_and_names(lib):
    """calculatePodResourceRequest (node_resource_fit_plus_utils.go:140-203): each container's value is
    rounded (MilliValue / Value) before the sum; a name that is not a scalar resource counts 0."""
    names = ["cpu", "memory", "pods", "example.com/dev", "ephemeral-storage"]
    doc = {"metadata": {"name": "r", "namespace": "n"}, "spec": {"containers": [
        {"resources": {"requests": {"cpu": "100100u", "memory": "1500m", "pods": "1", "example.com/dev": "1"}}},
        {"resources": {"requests": {"cpu": "100100u", "memory": "1500m", "example.com/dev": "2"}}}]}}
    p = decode.decode_pod(doc, names)
    got = dict(zip(p.xres_id[:p.n_xres], p.xres_value[:p.n_xres]))
    assert got[0] == 202  # ceil(100.1m) = 101m per container (the PodRequests total would round to 201m)
    assert got[1] == 4    # ceil(1.5) = 2 bytes per container
    assert got[2] == 0    # "pods" is not a scalar resource
    assert got[3] == 3
    assert p.xres_request_mask == 0b1111
    want = model.make_pod(containers=[{"requests": {"cpu": "100100u", "memory": "1500m", "pods": "1", "example.com/dev": "1"}},
                                      {"requests": {"cpu": "100100u", "memory": "1500m", "example.com/dev": "2"}}])
    assert sorted(want.xres_value[:want.n_xres]) == sorted(got.values())
    with pytest.raises(decode.DecodeError) as e:  # overhead on a requested name: refused
        decode.decode_pod({"spec": {"containers": [{"resources": {"requests": {"cpu": "1"}}}],
                                    "overhead": {"cpu": "100m"}}}, names)
    assert e.value.code == abi.ERR_UNSUPPORTED
