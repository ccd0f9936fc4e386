"""Transcription of NUMA topology known-answer tests into tests/golden/numa_policy.json.

Same rules as make_fixtures.py (hand transcription, each case cites its Go test lines; paths relative to
haoyann/koordinator).  Cases:

* topologymanager Policy.Merge cases (frameworkext/topologymanager/policy_test.go): provider hint lists
  -> merged hint (NUMANodeAffinity, Preferred) and admit.  The Go tables leave `Unsatisfied` and `Score`
  unset in their expectations; only the affinity, Preferred and admit are compared.
* NodeNUMAResource for pods without CPU binding: the NUMA affinity Filter stores under SingleNUMANode /
  Restricted with NUMA-scope hint scoring (plugin_test.go), tryBestToDistributeEvenly on a fixed hint
  and hint generation (resource_manager_test.go), getAvailableNUMANodeResources (node_allocation_test.go).
  Cases that need CPU binding (cpusets), hugepages or reservations are not transcribed.

Hint: [bits or None, preferred].  Provider: None (no hints) | {} (empty map) | {resource: None | [] | [hints]}.

Run:  python tests/golden/make_numa_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
POLICY = "pkg/scheduler/frameworkext/topologymanager/policy_test.go"

ALL = "all"  # NewTestBitMask(numaNodes...)


def H(bits, pref=True):
    return [bits, pref]


# commonPolicyMergeTestCases (policy_test.go:63-346): one expectation for every policy
COMMON = [
    ("Two providers, 1 hint each, same mask, both preferred 1/2", 66, [{"resource1": [H([0])]}, {"resource2": [H([0])]}], [0], True),
    ("Two providers, 1 hint each, same mask, both preferred 2/2", 95, [{"resource1": [H([1])]}, {"resource2": [H([1])]}], [1], True),
    ("Two providers, 1 no hints, 1 single hint preferred 1/2", 124, [None, {"resource": [H([0])]}], [0], True),
    ("Two providers, 1 no hints, 1 single hint preferred 2/2", 144, [None, {"resource": [H([1])]}], [1], True),
    ("Two providers, 1 with 2 hints, 1 with single hint matching 1/2", 164,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0])]}], [0], True),
    ("Two providers, 1 with 2 hints, 1 with single hint matching 2/2", 197,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([1])]}], [1], True),
    ("Two providers, both with 2 hints, matching narrower preferred hint from both", 230,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0]), H([0, 1], False)]}], [0], True),
    ("Ensure less narrow preferred hints are chosen over narrower non-preferred hints", 267,
     [{"resource1": [H([1]), H([0, 1], False)]}, {"resource2": [H([0]), H([1]), H([0, 1], False)]}], [1], True),
    ("Multiple resources, same provider", 308,
     [{"resource1": [H([1]), H([0, 1], False)], "resource2": [H([0]), H([1]), H([0, 1], False)]}], [1], True),
]

# per-policy mergeTestCases: (name, line, providers, expected bits (ALL / None = nil), preferred, admit)
BEST_EFFORT = [
    ("Two providers, 2 hints each, same mask (some with different bits), same preferred", 350,
     [{"resource1": [H([0, 1]), H([0, 2])]}, {"resource2": [H([0, 1]), H([0, 2])]}], [0, 1], True),
    ("NUMATopologyHint not set", 387, [], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map", 395, [{}], ALL, True),
    ("NUMATopologyHintProvider returns -nil map from provider", 407, [{"resource": None}], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map from provider", 421, [{"resource": []}], ALL, False),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil", 435,
     [{"resource": [H(None, True)]}], ALL, True),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil", 455,
     [{"resource": [H(None, False)]}], ALL, False),
    ("Two providers, 1 hint each, no common mask", 475, [{"resource1": [H([0])]}, {"resource2": [H([1])]}], ALL, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2", 505,
     [{"resource1": [H([0])]}, {"resource2": [H([0], False)]}], [0], False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2", 535,
     [{"resource1": [H([1])]}, {"resource2": [H([1], False)]}], [1], False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 1/2", 565,
     [{"resource1": [H([0])]}, {"resource2": [H([0, 1])]}], ALL, False),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching", 595,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0, 1], False)]}], ALL, False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 2/2", 629,
     [{"resource1": [H([1])]}, {"resource2": [H([0, 1])]}], ALL, False),
]
RESTRICTED = [
    ("Two providers, 2 hints each, same mask (some with different bits), same preferred", 664,
     [{"resource1": [H([0, 1]), H([0, 2])]}, {"resource2": [H([0, 1]), H([0, 2])]}], [0, 1], True),
    ("NUMATopologyHint not set", 701, [], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map", 709, [{}], ALL, True),
    ("NUMATopologyHintProvider returns -nil map from provider", 721, [{"resource": None}], ALL, True),
    ("NUMATopologyHintProvider returns empty non-nil map from provider", 735, [{"resource": []}], ALL, False),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil", 749,
     [{"resource": [H(None, True)]}], ALL, True),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil", 768,
     [{"resource": [H(None, False)]}], ALL, False),
    ("Two providers, 1 hint each, no common mask", 788, [{"resource1": [H([0])]}, {"resource2": [H([1])]}], ALL, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2", 818,
     [{"resource1": [H([0])]}, {"resource2": [H([0], False)]}], [0], False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2", 848,
     [{"resource1": [H([1])]}, {"resource2": [H([1], False)]}], [1], False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 1/2", 878,
     [{"resource1": [H([0])]}, {"resource2": [H([0, 1])]}], [0], False),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching", 909,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0, 1], False)]}], [0], False),
    ("Two providers, 1 hint each, 1 wider mask, both preferred 2/2", 944,
     [{"resource1": [H([1])]}, {"resource2": [H([0, 1])]}], [1], False),
]
SINGLE = [
    ("NUMATopologyHint not set", 980, [], None, True),
    ("NUMATopologyHintProvider returns empty non-nil map", 988, [{}], None, True),
    ("NUMATopologyHintProvider returns -nil map from provider", 1000, [{"resource": None}], None, True),
    ("NUMATopologyHintProvider returns empty non-nil map from provider", 1014, [{"resource": []}], None, False),
    ("Single NUMATopologyHint with Preferred as true and NUMANodeAffinity as nil", 1028,
     [{"resource": [H(None, True)]}], None, True),
    ("Single NUMATopologyHint with Preferred as false and NUMANodeAffinity as nil", 1047,
     [{"resource": [H(None, False)]}], None, False),
    ("Two providers, 1 hint each, no common mask", 1067, [{"resource1": [H([0])]}, {"resource2": [H([1])]}], None, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 1/2", 1097,
     [{"resource1": [H([0])]}, {"resource2": [H([0], False)]}], None, False),
    ("Two providers, 1 hint each, same mask, 1 preferred, 1 not 2/2", 1127,
     [{"resource1": [H([1])]}, {"resource2": [H([1], False)]}], None, False),
    ("Two providers, 1 with 2 hints, 1 with single non-preferred hint matching", 1157,
     [{"resource1": [H([0]), H([1])]}, {"resource2": [H([0, 1], False)]}], None, False),
    ("Single NUMA hint generation", 1191,
     [{"resource1": [H([0, 1])], "resource2": [H([0]), H([1]), H([0, 1], False)]}], None, False),
    ("One no-preference provider", 1225, [{"resource1": [H([0]), H([1]), H([0, 1], False)]}, None], [0], True),
]

cases = []
for policy, numa_nodes, table, src_end in (
        ("BestEffort", [0, 1, 2, 3], BEST_EFFORT, 660),
        ("Restricted", [0, 1, 2, 3], RESTRICTED, 976),
        ("SingleNUMANode", [0, 1], SINGLE, 1256)):
    for name, line, providers, bits, pref in COMMON:
        exp = bits
        if policy == "SingleNUMANode" and bits == numa_nodes:
            exp = None
        cases.append({"name": f"{policy}: {name}", "source": f"{POLICY}:{line}", "op": "merge", "policy": policy,
                      "numa_nodes": numa_nodes, "providers": providers,
                      "want": {"bits": exp, "preferred": pref, "admit": pref or policy == "BestEffort"}})
    for name, line, providers, bits, pref in table:
        exp = numa_nodes if bits == ALL else bits
        admit = True if policy == "BestEffort" else pref
        cases.append({"name": f"{policy}: {name}", "source": f"{POLICY}:{line}", "op": "merge", "policy": policy,
                      "numa_nodes": numa_nodes, "providers": providers,
                      "want": {"bits": exp, "preferred": pref, "admit": admit}})

# ---- NodeNUMAResource non-cpuset NUMA path ----------------------------------------------------------
PLUGIN = "pkg/scheduler/plugins/nodenumaresource/plugin_test.go"
RM = "pkg/scheduler/plugins/nodenumaresource/resource_manager_test.go"
NA = "pkg/scheduler/plugins/nodenumaresource/node_allocation_test.go"

# TestFilterWithNUMANodeScoring (plugin_test.go:1969-2190): node cpu 104 / memory 256Gi split evenly over
# `zones` NUMA nodes, existing pods' requests allocated per zone (resourceManager.Update), the pod
# requests cpu 4 / memory 40Gi; Filter succeeds and stores `want` as the NUMA affinity.
def affinity(name, lines, policy, zones, existing, strategy, want):
    cases.append({"name": f"{policy}: {name}", "source": f"{PLUGIN}:{lines}", "op": "affinity", "policy": policy,
                  "numa_strategy": strategy, "node": {"cpu": "104", "memory": "256Gi"}, "zones": zones,
                  "existing": existing, "pod": {"cpu": "4", "memory": "40Gi"}, "want": {"bits": want}})


E2 = {0: [{"cpu": "4", "memory": "8Gi"}], 1: [{"cpu": "40", "memory": "8Gi"}]}
E4 = {0: [{"cpu": "24", "memory": "8Gi"}], 1: [{"cpu": "23", "memory": "8Gi"}], 2: [{"cpu": "4", "memory": "8Gi"}],
      3: [{"cpu": "8", "memory": "8Gi"}]}
affinity("single numa nodes and select most allocated", "2006-2026", "SingleNUMANode", 2, E2, "MostAllocated", [1])
affinity("single numa nodes and select least allocated", "2028-2048", "SingleNUMANode", 2, E2, "LeastAllocated", [0])
affinity("single numa nodes and only one node can be used", "2050-2070", "SingleNUMANode", 2,
         {0: [{"cpu": "4", "memory": "8Gi"}], 1: [{"cpu": "52", "memory": "8Gi"}]}, "LeastAllocated", [0])
affinity("restricted numa nodes and select most allocated and preferred", "2072-2098", "Restricted", 4, E4,
         "MostAllocated", [3])
affinity("restricted numa nodes and select least allocated and preferred", "2100-2126", "Restricted", 4, E4,
         "LeastAllocated", [2])

# resource manager on buildCPUTopologyForTest(2, 1, 26, 2): NUMA 0 = CPUs 0-51, NUMA 1 = CPUs 52-103,
# NUMANodeResources cpu 52 / memory 128Gi each (resource_manager_test.go:1213-1231, 1617-1637).
RM_ZONES = [{"id": 0, "cpu": "52", "memory": "128Gi"}, {"id": 1, "cpu": "52", "memory": "128Gi"}]
CPUSHARE_ALLOC = [{"cpu": "50"}, {"cpu": "50"}]  # PodAllocation CPUSet 0-49,52-101 + NUMANodeResources
CPUSHARE_CPUSETS = [50, 50]


def distribute(name, lines, requests, hint, want, ratio=None, allocated=None, cpusets=None):
    """TestAllocateDistributeEvenly cases without CPU binding: Allocate with a fixed hint."""
    cases.append({"name": name, "source": f"{RM}:{lines}", "op": "distribute", "node": {"cpu": "104", "memory": "256Gi"},
                  "ratio": ratio, "zones": RM_ZONES, "allocated": allocated, "cpusets": cpusets,
                  "pod": requests, "hint": hint, "want": want})


distribute("allocate with non-existing resources in NUMA", "611-644", {"cpu": "4"}, [0, 1],
           {"ok": True, "alloc": {"0": {"cpu": "2"}, "1": {"cpu": "2"}}})  # gpu-memory is not a NUMA resource
distribute("allocate with insufficient resources", "645-662", {"cpu": "108"}, [0, 1], {"ok": False})
distribute("allocate with CPU Share and allocated and amplified ratios", "1154-1210", {"cpu": "3.5"}, [0, 1],
           {"ok": True, "alloc": {"0": {"cpu": "1.75"}, "1": {"cpu": "1.75"}}}, ratio=1.5,
           allocated=CPUSHARE_ALLOC, cpusets=CPUSHARE_CPUSETS)

# TestResourceManagerGetTopologyHint (resource_manager_test.go:1279-1668), BestEffort, no CPU binding
cases.append({"name": "failed to allocate with CPU Share and allocated and amplified ratios",
              "source": f"{RM}:1532-1580", "op": "hints", "policy": "BestEffort", "node": {"cpu": "104", "memory": "256Gi"},
              "ratio": 1.5, "zones": RM_ZONES, "allocated": CPUSHARE_ALLOC, "cpusets": CPUSHARE_CPUSETS,
              "pod": {"cpu": "4"}, "want": {"hints": {"cpu": [[[0, 1], True]]}}})

# Test_getAvailableNUMANodeResources (node_allocation_test.go:171-300): CPU topology (2, 1, 8, 2), so
# allocatedCPUSets = 4 are CPUs 0-3 on NUMA 0.  `nrt_ratio`: TopologyOptions.AmplificationRatios (the
# NUMANodeResources are already amplified).
R16 = {"cpu": "16", "memory": "32Gi"}
R24 = {"cpu": "24", "memory": "32Gi"}
for name, lines, res, ratio, alloc, cpusets, want in [
    ("normal node", "190-205", R16, None, None, None, [R16, R16]),
    ("normal node with amplification ratios", "206-223", R24, 1.5, None, None, [R24, R24]),
    ("normal node with amplification ratios and allocated CPUSets", "224-256", R24, 1.5, [{"cpu": "4"}, None], [4, 0],
     [{"cpu": "18", "memory": "32Gi"}, R24]),
    ("normal node with amplification ratios and allocated CPUSets and CPU Shares", "257-289", R24, 1.5,
     [{"cpu": "8"}, None], [4, 0], [{"cpu": "14", "memory": "32Gi"}, R24]),
]:
    cases.append({"name": name, "source": f"{NA}:{lines}", "op": "available", "node": {"cpu": "32", "memory": "64Gi"},
                  "nrt_ratio": ratio, "zones": [dict(id=k, **res) for k in range(2)], "allocated": alloc,
                  "cpusets": cpusets, "want": {"available": want}})


# Test_checkExclusivePolicy (frameworkext/topologymanager/policy_test.go:1278-1400)
POLICY_T = "pkg/scheduler/frameworkext/topologymanager/policy_test.go"
for name, line, bits, excl, status, want in [
    ("preferred policy 1", 1291, [0], "Preferred", ["shared", "shared"], True),
    ("preferred policy 2", 1300, [0, 1], "Preferred", ["shared", "shared"], True),
    ("preferred policy 3", 1309, [0], "Preferred", ["idle", "single"], True),
    ("preferred policy 4", 1318, [0, 1], "Preferred", ["idle", "single"], True),
    ("required policy 1", 1327, [0], "Required", ["idle", "single"], True),
    ("required policy 2", 1336, [0], "Required", ["shared", "single"], False),
    ("required policy 3", 1345, [0], "Required", ["shared", "shared"], False),
    ("required policy 4", 1354, [0], "Required", ["single", "shared"], True),
    ("required policy 5", 1363, [0, 1], "Required", ["shared", "single"], False),
    ("required policy 6", 1372, [0, 1], "Required", ["shared", "idle"], True),
    ("required policy 7", 1381, [0, 1], "Required", ["shared", "shared"], True),
]:
    cases.append({"name": f"checkExclusivePolicy {name}", "source": f"{POLICY_T}:{line}", "op": "exclusive",
                  "bits": bits, "exclusive": excl, "status": status, "want": {"ok": want}})


def main():
    with open(os.path.join(HERE, "numa_policy.json"), "w") as f:
        json.dump({"source": "haoyann/koordinator topologymanager / nodenumaresource tests, transcribed by "
                             "make_numa_fixtures.py", "cases": cases}, f, indent=1)
    print(f"numa_policy.json: {len(cases)} cases")


if __name__ == "__main__":
    main()
