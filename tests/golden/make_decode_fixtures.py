"""Transcription of the reference's apis/extension tests whose inputs are wire-format objects into
tests/golden/decode.json (the decoders' golden vectors).

Same rules as make_fixtures.py: the Go tests cannot run here; every case restates one test case's
object and expected result by hand.  Only data is written.

  * node_resource_amplification_test.go:27-151  GetNodeResourceAmplificationRatio(annotations, cpu)
    (-1 unset, 1.22 set, error on an unparsable annotation)
  * priority_utils_test.go:86-196  GetPodPriorityClassWithDefault (spec.priority ranges, the priority-class label,
    QoS labels, kube QoS of the containers)

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

if __name__ == "__main__":
    with open(os.path.join(HERE, "decode.json"), "w") as f:
        json.dump({"source": "make_decode_fixtures.py", "cases": cases}, f, indent=1)
    print(len(cases), "cases")
