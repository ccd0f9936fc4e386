"""Transcription of NodeResourcesFitPlus's and ScarceResourceAvoidance's Score tests into
tests/golden/ext_plugins.json.

Same rules as make_fixtures.py: the reference is Go and cannot run here, so every case restates
the inputs of the Go test it cites (paths relative to haoyann/koordinator).  The two TestPlugin_Score functions
assert only an ORDER between their two nodes (`scoreNode1 > scoreNode2` / `scoreNode1 < scoreNode2`); the
`want` scores here are the published algorithm applied by hand to the test's inputs (arithmetic in the
comments), and the order the Go test asserts is kept as `order` so the tests check both.  The remaining cases
exercise the branches of node_resource_fit_plus_utils.go:35-89 and scarce_resource_avoidance.go:70-90,159-161
(weight sum 0, zero capacity, request above capacity, no diff / no intersection).

Node tables hold what calculateResourceAllocatableRequest reads: Allocatable and NodeInfo.NonZeroRequested
(cpu / memory) or Requested (other resources).  Pods list their requests per container.

Run:  python tests/golden/make_ext_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
FP = "pkg/scheduler/plugins/noderesourcefitplus/node_resources_fit_plus_test.go"
SRA = "pkg/scheduler/plugins/scarceresourceavoidance/scarce_resource_avoidance_test.go"
MOST, LEAST = 1, 0
GI = 2**30

cases = []

# TestPlugin_Score (node_resources_fit_plus_test.go:116-266): args gpu MostAllocated w2, cpu / memory
# LeastAllocated w1; testNode1 (96 cpu, 512Gi, 8 GPUs) carries test-pod-0 (16 cpu, 32Gi, 4 GPUs); testNode2 adds
# "xx.xx/xx": 8 and has no pods; the pod requests 16 cpu, 32Gi, 2 GPUs.
#   node1: cpu (96000-32000)*100/96000 = 66, memory (512-64)Gi*100/512Gi = 87, gpu 6*100/8 = 75
#          (66 + 87 + 2*75) / 4 = 303/4 = 75
#   node2: cpu 80000*100/96000 = 83, memory 480*100/512 = 93, gpu 2*100/8 = 25 -> (83 + 93 + 50)/4 = 56
fp_args = [("nvidia.com/gpu", MOST, 2), ("cpu", LEAST, 1), ("memory", LEAST, 1)]
fp_pod = {"containers": [{"requests": {"cpu": "16", "memory": "32Gi", "nvidia.com/gpu": "2"}}]}
cases.append({
    "name": "fitplus_test_plugin_score", "source": f"{FP}:116-266", "plugin": "fitplus", "args": fp_args,
    "nodes": [
        {"allocatable": {"cpu": "96", "memory": "512Gi", "nvidia.com/gpu": "8"},
         "requested": {"cpu": "16", "memory": "32Gi", "nvidia.com/gpu": "4"}},
        {"allocatable": {"cpu": "96", "memory": "512Gi", "nvidia.com/gpu": "8", "xx.xx/xx": "8"}, "requested": {}},
    ],
    "pod": fp_pod, "want": [75, 56], "order": "gt"})

# TestPlugin_Score (scarce_resource_avoidance_test.go:107-218): args [nvidia.com/gpu]; testNode1 has cpu, memory,
# nvidia.com/gpu, xx.xx/xx; testNode2 cpu, memory; the pod requests cpu + memory.
#   node1: diff = {gpu, xx}, intersect = {gpu} -> (2-1)*100/2 = 50;  node2: diff empty -> 100
cases.append({
    "name": "sra_test_plugin_score", "source": f"{SRA}:107-218", "plugin": "sra", "args": ["nvidia.com/gpu"],
    "nodes": [
        {"allocatable": {"cpu": "96", "memory": "512Gi", "nvidia.com/gpu": "8", "xx.xx/xx": "8"}, "requested": {}},
        {"allocatable": {"cpu": "96", "memory": "512Gi"}, "requested": {}},
    ],
    "pod": {"containers": [{"requests": {"cpu": "16", "memory": "32Gi"}}]}, "want": [50, 100], "order": "lt"})

# branch cases (algorithm of the cited lines, no Go assertion)
cases.append({
    "name": "fitplus_weight_sum_zero", "source": f"{FP.replace('_test', '_utils').replace('node_resources_fit_plus_utils', 'node_resource_fit_plus_utils')}:79-81",
    "plugin": "fitplus", "args": [("nvidia.com/gpu", MOST, 2)],
    "nodes": [{"allocatable": {"cpu": "8", "memory": "16Gi", "nvidia.com/gpu": "4"}, "requested": {}}],
    "pod": {"containers": [{"requests": {"cpu": "1", "memory": "1Gi"}}]}, "want": [100]})
cases.append({
    "name": "fitplus_zero_capacity_and_over_request", "source": "pkg/scheduler/plugins/noderesourcefitplus/node_resource_fit_plus_utils.go:35-55",
    "plugin": "fitplus", "args": [("cpu", LEAST, 3), ("nvidia.com/gpu", MOST, 1), ("memory", MOST, 1)],
    # cpu: 7+2 > 8 -> 0 (least); gpu: not on the node -> capacity 0 -> 0; memory: min(20Gi,16Gi)*100/16Gi = 100
    "nodes": [{"allocatable": {"cpu": "8", "memory": "16Gi"}, "requested": {"cpu": "7", "memory": "12Gi"}}],
    "pod": {"containers": [{"requests": {"cpu": "2", "memory": "8Gi", "nvidia.com/gpu": "1"}}]},
    "want": [(0 * 3 + 0 * 1 + 100 * 1) // 5]})
cases.append({
    "name": "fitplus_nonzero_defaults", "source": "pkg/scheduler/plugins/noderesourcefitplus/node_resource_fit_plus_utils.go:138-203",
    "plugin": "fitplus", "args": [("cpu", LEAST, 1), ("memory", LEAST, 1)],
    # PodRequests cpu 1000 > 0 and memory 1Gi > 0: both names scored; the second container has no requests, so
    # calculatePodResourceRequest adds the 100m / 200Mi defaults: cpu 1100, memory 1Gi + 200Mi.
    #   cpu (10000-1100)*100/10000 = 89; memory (8Gi - 1Gi - 200Mi)*100/8Gi = 85 -> (89 + 85)/2 = 87
    "nodes": [{"allocatable": {"cpu": "10", "memory": "8Gi"}, "requested": {}}],
    "pod": {"containers": [{"requests": {"cpu": "1", "memory": "1Gi"}}, {"requests": {}}]},
    "want": [(89 + 85) // 2]})
cases.append({
    "name": "sra_no_intersection_and_pod_requests_scarce", "source": f"{SRA.replace('_test', '')}:76-90",
    "plugin": "sra", "args": ["nvidia.com/gpu", "example.com/fpga"],
    # node1: diff {storage} has no scarce name -> 100; node2: the pod requests the GPU: diff {fpga, storage},
    # intersect {fpga} -> (2-1)*100/2 = 50; node3: the same names listed in another order -> 50
    "nodes": [
        {"allocatable": {"cpu": "8", "memory": "8Gi", "ephemeral-storage": "100Gi"}, "requested": {}},
        {"allocatable": {"cpu": "8", "memory": "8Gi", "nvidia.com/gpu": "2", "example.com/fpga": "1",
                         "ephemeral-storage": "100Gi"}, "requested": {}},
        {"allocatable": {"nvidia.com/gpu": "2", "example.com/fpga": "1", "ephemeral-storage": "100Gi",
                         "cpu": "8", "memory": "8Gi"}, "requested": {}},
    ],
    "pod": {"containers": [{"requests": {"cpu": "1", "memory": "1Gi", "nvidia.com/gpu": "1"}}]},
    "want": [100, 50, 50]})
cases.append({
    "name": "sra_zero_allocatable_is_not_a_name", "source": f"{SRA.replace('_test', '')}:109-150",
    "plugin": "sra", "args": ["nvidia.com/gpu"],
    "nodes": [{"allocatable": {"cpu": "8", "memory": "8Gi", "nvidia.com/gpu": "0"}, "requested": {}}],
    "pod": {"containers": [{"requests": {"cpu": "1"}}]}, "want": [100]})

if __name__ == "__main__":
    with open(os.path.join(HERE, "ext_plugins.json"), "w") as f:
        json.dump({"source": "make_ext_fixtures.py", "cases": cases}, f, indent=1)
    print(len(cases), "cases")
