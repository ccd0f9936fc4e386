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

if __name__ == "__main__":
    with open(os.path.join(HERE, "decode.json"), "w") as f:
        json.dump({"source": "make_decode_fixtures.py", "cases": cases}, f, indent=1)
    print(len(cases), "cases")
