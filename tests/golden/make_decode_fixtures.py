"""Transcription of the reference's apis/extension tests whose inputs are wire-format objects into
tests/golden/decode.json (the decoders' golden vectors).

Same rules as make_fixtures.py: the Go tests cannot run here; every case restates one test case's
object and expected result by hand.  Only data is written.

  * node_resource_amplification_test.go:27-151  GetNodeResourceAmplificationRatio(annotations, cpu)
    (-1 unset, 1.22 set, error on an unparsable annotation)
  * priority_utils_test.go:86-196  GetPodPriorityClassWithDefault (spec.priority ranges, the priority-class label,
    QoS labels, kube QoS of the containers)
  * nodenumaresource/topology_options_test.go:36-176  NewTopologyOptions from a NodeResourceTopology (CPU topology,
    reserved CPUs from four annotations, zone cpu less the reserved CPUs)

  * device_share_test.go:174-251  GetGPUPartitionSpec (pod annotation gpu-partition-spec: absent, {}, BestEffort,
    Restricted, Restricted + ringBusBandwidth 200Gi)
  * device_share_test.go:253-311  GetGPUPartitionTable (Device annotation gpu-partitions: a valid table, none,
    invalid JSON -> error)
  * device_share_test.go:313-359  GetGPUPartitionPolicy (Device label gpu-partition-policy Honor / Prefer / none)
  * qos_utils_test.go:27-111  GetPodQoSClassRaw / GetQoSClassByAttrs (the koordinator.sh/qosClass label)
  * node_reservation_test.go:37-153  GetReservedCPUs: the node.koordinator.sh/reservation annotation's reservedCPUs
    (the string NewTopologyOptions parses with cpuset.Parse, topology_options.go:108-112), observed as the
    NodeResourceTopology's reserved CPUs ("-1" does not parse: nothing reserved)

Run:  python tests/golden/make_decode_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
AMP = "apis/extension/node_resource_amplification_test.go"
PRI = "apis/extension/priority_utils_test.go"
RATIO = "node.koordinator.sh/resource-amplification-ratio"
PROD, BATCH, NONE = 1, 3, 0  # KE_PRIORITY_*

cases = []
for name, lines, ann, want, err in (
        ("ratio_no_annotation", "100-108", None, -1.0, False),
        ("ratio_no_ratio_annotation", "109-123", {"a": "b"}, -1.0, False),
        ("ratio_cpu_set", "124-139", {"a": "b", RATIO: '{"cpu":1.22}'}, 1.22, False),
        ("ratio_cpu_unset", "140-155", {"a": "b", RATIO: '{"memory":1.22}'}, -1.0, False),
        ("ratio_invalid", "156-171", {"a": "b", RATIO: "invalid"}, -1.0, True)):
    node = {"metadata": {"name": "test-node"}}
    if ann is not None:
        node["metadata"]["annotations"] = ann
    cases.append({"name": name, "source": f"{AMP}:{lines}", "kind": "node", "object": node,
                  "want": {"cpu_amplification_ratio": want, "amplification_error": int(err)}})


def pod(labels=None, priority=None, containers=None):
    p = {"metadata": {"name": "p", "namespace": "default"}, "spec": {}}
    if labels:
        p["metadata"]["labels"] = labels
    if priority is not None:
        p["spec"]["priority"] = priority
    if containers is not None:
        p["spec"]["containers"] = containers
    return p


PC, QOS = "koordinator.sh/priority-class", "koordinator.sh/qosClass"
for i, (obj, want) in enumerate((
        (pod(priority=(9000 + 9999) // 2), PROD),
        (pod(labels={PC: "koord-prod"}, priority=(5000 + 5999) // 2), PROD),
        (pod(labels={QOS: "LSR"}, priority=(5000 + 5999) // 2), BATCH),
        (pod(labels={QOS: "LSR"}), PROD),
        (pod(labels={QOS: "BE"}), BATCH),
        (pod(containers=[{"resources": {"requests": {"cpu": "100"}, "limits": {"cpu": "200"}}}]), PROD),
        (pod(containers=[{"resources": {"requests": {"cpu": "100"}, "limits": {"cpu": "100"}}}]), PROD),
        (pod(containers=[{"name": "abc"}]), BATCH))):
    cases.append({"name": f"priority_with_default_{i}", "source": f"{PRI}:86-196", "kind": "pod", "object": obj,
                  "want": {"priority_class": want}})

# TestTopologyOptionsManager (nodenumaresource/topology_options_test.go:36-185): buildCPUTopologyForTest(2, 1, 4, 2)
# reported as the cpu-topology annotation (raw core ids), kubelet static policy with reservedCPUs 0-1, a kubelet-managed
# pod-cpu-alloc 0-3, system QoS cpuset 4-5 (exclusive by default), node reservation 6-7; zones node-0 / node-1 with
# 8 cpus each.  Expected: reserved 0-7, zone cpu 0 and 8000 milli, core ids socket<<16|core; after the pod allocs
# are removed the reserved set is 0-1,4-7 (zone node-0: 8000 - 6000).
NRT_SRC = "pkg/scheduler/plugins/nodenumaresource/topology_options_test.go"
rows, core, cpu = [], 0, 0
for sock in range(2):
    for _ in range(4):
        for _ in range(2):
            rows.append({"id": cpu, "core": core, "socket": sock, "node": sock})
            cpu += 1
        core += 1
nrt_ann = {
    "node.koordinator.sh/cpu-topology": json.dumps({"detail": rows}),
    "kubelet.koordinator.sh/cpu-manager-policy": json.dumps({"policy": "static", "options": {"static": "true"},
                                                             "reservedCPUs": "0-1"}),
    "node.koordinator.sh/pod-cpu-allocs": json.dumps([{"namespace": "default", "name": "pod-1", "uid": "0b6a3c5e",
                                                       "cpuset": "0-3", "managedByKubelet": True}]),
    "node.koordinator.sh/system-qos-resource": json.dumps({"cpuset": "4-5"}),
    "node.koordinator.sh/reservation": json.dumps({"reservedCPUs": "6-7"}),
}
zone = lambda n: {"name": f"node-{n}", "type": "Node", "resources": [{"name": "cpu", "capacity": "8", "allocatable": "8",
                                                                      "available": "8"}]}
nrt = {"metadata": {"name": "test-node-1", "annotations": nrt_ann}, "zones": [zone(0), zone(1)]}
want_cpus = [[r["id"], r["socket"] << 16 | r["core"], r["node"], r["socket"]] for r in rows]
cases.append({"name": "nrt_topology_options", "source": f"{NRT_SRC}:36-167", "kind": "nrt", "object": nrt,
              "want": {"reserved": list(range(8)), "zone_cpu": [[0, 0], [1, 8000]], "cpus": want_cpus}})
nrt2 = json.loads(json.dumps(nrt))
del nrt2["metadata"]["annotations"]["node.koordinator.sh/pod-cpu-allocs"]
cases.append({"name": "nrt_topology_options_no_pod_allocs", "source": f"{NRT_SRC}:169-176", "kind": "nrt",
              "object": nrt2, "want": {"reserved": [0, 1, 4, 5, 6, 7], "zone_cpu": [[0, 2000], [1, 8000]],
                                       "cpus": want_cpus}})

# ---- apis/extension/device_share_test.go -------------------------------------------------------------------
DS = "apis/extension/device_share_test.go"
SPEC = "scheduling.koordinator.sh/gpu-partition-spec"
ABSENT = -1
for name, lines, ann, want in (
        ("gpu_partition_spec_nil", "185-192", None, (0, 0, ABSENT)),
        ("gpu_partition_spec_empty", "193-203", "{}", (1, 0, ABSENT)),
        ("gpu_partition_spec_best_effort", "204-214", '{"allocatePolicy":"BestEffort"}', (1, 0, ABSENT)),
        ("gpu_partition_spec_restricted", "215-225", '{"allocatePolicy":"Restricted"}', (1, 1, ABSENT)),
        ("gpu_partition_spec_restricted_bw", "226-237", '{"allocatePolicy":"Restricted", "ringBusBandwidth":"200Gi"}',
         (1, 1, 200 * 2**30))):
    obj = {"metadata": {"name": "p", "namespace": "default", "annotations": {SPEC: ann} if ann else {}},
           "spec": {"containers": []}}
    cases.append({"name": name, "source": f"{DS}:{lines}", "kind": "pod", "object": obj,
                  "want": {"gpu_partition_spec": want[0], "gpu_partition_restricted": want[1],
                           "gpu_ring_bus_bandwidth": want[2]}})
PARTS = "scheduling.koordinator.sh/gpu-partitions"
cases.append({"name": "gpu_partition_table_valid", "source": f"{DS}:259-279", "kind": "device",
              "object": {"metadata": {"annotations": {PARTS: '{"0": [{"minors": [0,1], "gpuLinkType": "NVLink",'
                                                             '"ringBusBandwidth": "200Gi", "allocationScore": 10}]}'}},
                         "spec": {"devices": []}},
              "want": {"has_table": 1, "partitions": [[0b11, 0, 10, 200 * 2**30]]}})
cases.append({"name": "gpu_partition_table_none", "source": f"{DS}:280-285", "kind": "device",
              "object": {"spec": {"devices": []}}, "want": {"has_table": 0, "partitions": []}})
cases.append({"name": "gpu_partition_table_invalid_json", "source": f"{DS}:286-296", "kind": "device",
              "object": {"metadata": {"annotations": {PARTS: "Invalid JSON format"}}, "spec": {"devices": []}},
              "want": {"error": True}})
POLICY = "node.koordinator.sh/gpu-partition-policy"
for name, lines, labels, honor in (("gpu_partition_policy_honor", "321-331", {POLICY: "Honor"}, 1),
                                   ("gpu_partition_policy_prefer", "332-342", {POLICY: "Prefer"}, 0),
                                   ("gpu_partition_policy_unset", "343-351", {}, 0)):
    cases.append({"name": name, "source": f"{DS}:{lines}", "kind": "device",
                  "object": {"metadata": {"labels": labels}, "spec": {"devices": []}}, "want": {"honor": honor}})

# ---- apis/extension/qos_utils_test.go ----------------------------------------------------------------------
QU = "apis/extension/qos_utils_test.go"
QOS_NONE, QOS_LS, QOS_BE = 0, 3, 4  # KE_QOS_*
for name, lines, labels, want in (("qos_not_specified", "33-37", None, QOS_NONE),
                                  ("qos_not_specified_1", "38-46", {}, QOS_NONE),
                                  ("qos_ls", "47-56", {QOS: "LS"}, QOS_LS),
                                  ("qos_be", "57-66", {QOS: "BE"}, QOS_BE),
                                  ("qos_by_attrs_not_specified", "88-94", {}, QOS_NONE),
                                  ("qos_by_attrs_be", "95-103", {QOS: "BE"}, QOS_BE)):
    obj = {"metadata": {"name": "p", "namespace": "default"}, "spec": {}}
    if labels is not None:
        obj["metadata"]["labels"] = labels
    cases.append({"name": name, "source": f"{QU}:{lines}", "kind": "pod", "object": obj, "want": {"qos_class": want}})

# ---- apis/extension/node_reservation_test.go ---------------------------------------------------------------
NR = "apis/extension/node_reservation_test.go"
small_rows = [{"id": c, "core": c // 2, "socket": 0, "node": c // 4} for c in range(8)]
small_zone = lambda n: {"name": f"node-{n}", "type": "Node", "resources": [
    {"name": "cpu", "capacity": "4", "allocatable": "4", "available": "4"}]}
for name, lines, reservation, reserved in (
        ("reserved_cpus_nil_annotation", "47-54", None, []),
        ("reserved_cpus_empty", "55-66", {}, []),
        ("reserved_cpus_quantity_only", "67-77", {"resources": {"cpu": "10"}}, []),
        ("reserved_cpus_quantity_not_integer", "78-88", {"resources": {"cpu": "2500m"}}, []),
        ("reserved_cpus_quantity_negative", "89-99", {"resources": {"cpu": "-2"}}, []),
        ("reserved_cpus_specific", "100-110", {"reservedCPUs": "0-1"}, [0, 1]),
        ("reserved_cpus_unavailable_id", "111-121", {"reservedCPUs": "-1"}, []),
        ("reserved_cpus_specific_and_quantity", "122-133", {"resources": {"cpu": "10"}, "reservedCPUs": "0-1"}, [0, 1])):
    ann = {"node.koordinator.sh/cpu-topology": json.dumps({"detail": small_rows})}
    if reservation is not None:
        ann["node.koordinator.sh/reservation"] = json.dumps(reservation)
    zone_cpu = [[z, 4000 - 1000 * sum(1 for c in reserved if c // 4 == z)] for z in range(2)]
    cases.append({"name": name, "source": f"{NR}:{lines}", "kind": "nrt",
                  "object": {"metadata": {"name": "n", "annotations": ann}, "zones": [small_zone(0), small_zone(1)]},
                  "want": {"reserved": reserved, "zone_cpu": zone_cpu,
                           "cpus": [[r["id"], r["socket"] << 16 | r["core"], r["node"], r["socket"]] for r in small_rows]}})

if __name__ == "__main__":
    with open(os.path.join(HERE, "decode.json"), "w") as f:
        json.dump({"source": "make_decode_fixtures.py", "cases": cases}, f, indent=1)
    print(len(cases), "cases")
