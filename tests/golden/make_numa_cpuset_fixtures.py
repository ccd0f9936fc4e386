"""Golden vectors for cpusets under NUMA topology policies, transcribed by hand from the reference's
own tests (values copied from the Go test tables; no reference code is executed):

  * resource_manager_test.go:35-597    TestResourceManagerAllocate       -> op "allocate" (Allocate, one hint)
  * resource_manager_test.go:600-1277  TestAllocateDistributeEvenly      -> op "allocate" (the cpuset cases)
  * resource_manager_test.go:1279-1680 TestResourceManagerGetTopologyHint -> op "hints" (BestEffort)
  * scoring_test.go:47-255             TestNUMANodeScore                 -> op "node_score" (Filter + Score)

Common node of the resource-manager tests (resource_manager_test.go:540-575, 1216-1260, 1640-1665): CPU
topology buildCPUTopologyForTest(2, 1, 26, 2) (104 CPUs, NUMA 0 = CPUs 0-51, NUMA 1 = 52-103), NUMA
zones of 52 cpu / 128Gi each, node allocatable 104 / 256Gi, amplification ratios from the node
annotation.  A case's `allocated` PodAllocation = allocated CPUs (RefCount 1) + NUMA allocation entries.

Transcription notes:
  * Allocated cpusets written "...-104" name CPU 104, which the 104-CPU topology lacks; the reference
    records it with a zero CPUInfo (NUMA 0).  It only changes NUMA 0's cpuset count under an
    amplification ratio, and no such case names it; it is dropped here.
  * The hugepages hint case (resource_manager_test.go:1581-1620) needs a resource outside cpu/memory
    and is not transcribed.
  * GetTopologyHint's expectations carry Score 0 (no numaScorer in that test): masks and Preferred are
    compared.

Run: python tests/golden/make_numa_cpuset_fixtures.py  (writes tests/golden/numa_cpuset.json)
"""
import json
import os

RM = "pkg/scheduler/plugins/nodenumaresource/resource_manager_test.go"
SC = "pkg/scheduler/plugins/nodenumaresource/scoring_test.go"

RM_NODE = {"cpu": "104", "memory": "256Gi"}
RM_TOPOLOGY = [2, 1, 26, 2]
RM_ZONES = [{"id": 0, "cpu": "52", "memory": "128Gi"}, {"id": 1, "cpu": "52", "memory": "128Gi"}]


def alloc(c0, c1):
    return [{"id": 0, "cpu": c0}, {"id": 1, "cpu": c1}]


cases = []


def rm_case(op, name, lines, pod, want, hint=None, ratio=None, allocated=None):
    c = {"name": name, "source": f"{RM}:{lines}", "op": op, "node": RM_NODE, "topology": RM_TOPOLOGY,
         "zones": RM_ZONES, "ratio": ratio, "pod": pod, "want": want}
    if hint is not None:
        c["hint"] = hint
    if allocated is not None:
        c["allocated"] = {"cpuset": allocated[0], "numa": allocated[1]}
    cases.append(c)


def pod(cpu, bind="", other=False):
    """cpu request; bind = the required bind policy of a binding (LSR koord-prod) pod, "" = no binding;
    other = a requested resource outside the NUMA resources (gpu-memory)"""
    return {"cpu": cpu, "bind": bind, "other": other}


def ok(cpuset, **numa):
    return {"error": False, "cpuset": cpuset, "numa": {k[1:]: {"cpu": v} for k, v in numa.items()}}


ERR = {"error": True}


def allocate():
    rm_case("allocate", "allocate with non-existing resources in NUMA", "45-72", pod("4", other=True),
            ok("", z0="4"), hint=[0])
    rm_case("allocate", "allocate with insufficient resources", "73-90", pod("54"), ERR, hint=[0])
    rm_case("allocate", "allocate with required CPUBindPolicyFullPCPUs", "91-121", pod("4", "FullPCPUs"),
            ok("0-3", z0="4"), hint=[0])
    rm_case("allocate", "allocate with required CPUBindPolicyFullPCPUs and allocated", "122-171",
            pod("4", "FullPCPUs"), ok("0-3", z0="4"), hint=[0], allocated=("4-103", alloc("48", "52")))
    rm_case("allocate", "failed to allocate with required CPUBindPolicyFullPCPUs and allocated", "172-215",
            pod("4", "FullPCPUs"), ERR, hint=[0], allocated=("1,3,5,7-103", alloc("48", "52")))
    rm_case("allocate", "allocate with required CPUBindPolicySpreadByPCPUs", "216-246", pod("4", "SpreadByPCPUs"),
            ok("0,2,4,6", z0="4"), hint=[0])
    rm_case("allocate", "allocate with required CPUBindPolicySpreadByPCPUs and allocated", "247-297",
            pod("4", "SpreadByPCPUs"), ok("0,2,4,6", z0="4"), hint=[0], allocated=("1,3,5,7-103", alloc("48", "52")))
    rm_case("allocate", "failed to allocate with required CPUBindPolicySpreadByPCPUs and allocated", "298-338",
            pod("4", "SpreadByPCPUs"), ERR, hint=[0], allocated=("4-103", alloc("48", "52")))
    rm_case("allocate", "allocate with required CPUBindPolicySpreadByPCPUs and amplified requests", "339-375",
            pod("4", "SpreadByPCPUs"), ok("0,2,4,6", z0="4"), hint=[0], ratio=1.5)
    rm_case("allocate", "allocate with required CPUBindPolicySpreadByPCPUs and allocated and amplified requests",
            "376-432", pod("4", "SpreadByPCPUs"), ok("0,2,4,6", z0="4"), hint=[0], ratio=1.5,
            allocated=("1,3,5,7-103", alloc("48", "52")))
    rm_case("allocate", "failed to allocate with CPU Share and allocated and amplified ratios", "433-478",
            pod("4"), ERR, hint=[0], ratio=1.5, allocated=("0-49,52-101", alloc("50", "50")))
    rm_case("allocate", "allocate by numa hint on mixed cpuset/share node", "479-535", pod("8", "FullPCPUs"),
            ok("44-47,98-101", z0="4", z1="4"), hint=[0, 1], allocated=("0-43,53-96", alloc("48", "48")))
    # TestAllocateDistributeEvenly: hints over both NUMA nodes
    rm_case("allocate", "distribute: allocate with required CPUBindPolicyFullPCPUs", "664-700",
            pod("4", "FullPCPUs"), ok("0-1,52-53", z0="2", z1="2"), hint=[0, 1])
    rm_case("allocate", "distribute: allocate with required CPUBindPolicyFullPCPUs and allocated", "701-757",
            pod("4", "FullPCPUs"), ok("0-1,102-103", z0="2", z1="2"), hint=[0, 1],
            allocated=("4-101", alloc("48", "50")))
    rm_case("allocate", "distribute: failed to allocate with required CPUBindPolicyFullPCPUs and allocated",
            "758-798", pod("4", "FullPCPUs"), ERR, hint=[0], allocated=("1,3,5,7-103", alloc("48", "52")))
    rm_case("allocate", "distribute: allocate with required CPUBindPolicySpreadByPCPUs", "799-835",
            pod("4", "SpreadByPCPUs"), ok("0,2,52,54", z0="2", z1="2"), hint=[0, 1])
    rm_case("allocate", "distribute: SpreadByPCPUs and allocated, plural numCPUsNeeded, not balanced", "836-892",
            pod("4", "SpreadByPCPUs"), ok("0,2,4,102", z0="3", z1="1"), hint=[0, 1],
            allocated=("1,3,5,7-101,103", alloc("48", "50")))
    rm_case("allocate", "distribute: SpreadByPCPUs and allocated, plural numCPUsNeeded, balanced", "893-949",
            pod("4", "SpreadByPCPUs"), ok("0,2,101-102", z0="2", z1="2"), hint=[0, 1],
            allocated=("4-100", alloc("48", "49")))
    rm_case("allocate", "distribute: SpreadByPCPUs and allocated, singular num cpus needed", "950-1006",
            pod("5", "SpreadByPCPUs"), ok("0,2,4,98,100", z0="3", z1="2"), hint=[0, 1],
            allocated=("1,3,5,7-97,103", alloc("48", "47")))
    rm_case("allocate", "distribute: failed to allocate with required CPUBindPolicySpreadByPCPUs and allocated",
            "1007-1047", pod("4", "SpreadByPCPUs"), ERR, hint=[0, 1], allocated=("4-103", alloc("48", "52")))
    rm_case("allocate", "distribute: SpreadByPCPUs and amplified requests", "1048-1090", pod("4", "SpreadByPCPUs"),
            ok("0,2,52,54", z0="2", z1="2"), hint=[0, 1], ratio=1.5)
    rm_case("allocate", "distribute: SpreadByPCPUs and allocated and amplified requests", "1091-1153",
            pod("4", "SpreadByPCPUs"), ok("0,2,4,102", z0="3", z1="1"), hint=[0, 1], ratio=1.5,
            allocated=("1,3,5,7-101", alloc("48", "50")))


def hints():
    both = [{"bits": [0], "preferred": True}, {"bits": [1], "preferred": True}, {"bits": [0, 1], "preferred": False}]
    rm_case("hints", "allocate with required CPUBindPolicyFullPCPUs", "1289-1326", pod("4", "FullPCPUs"),
            {"cpu": both})
    rm_case("hints", "allocate with required CPUBindPolicyFullPCPUs and allocated", "1327-1371",
            pod("4", "FullPCPUs"), {"cpu": [{"bits": [0], "preferred": True}]}, allocated=("4-103", alloc("48", "52")))
    rm_case("hints", "failed to allocate with required CPUBindPolicyFullPCPUs and allocated", "1372-1408",
            pod("4", "FullPCPUs"), {"cpu": []}, allocated=("1,3,5,7-103", alloc("48", "52")))
    rm_case("hints", "allocate with required CPUBindPolicySpreadByPCPUs", "1409-1446", pod("4", "SpreadByPCPUs"),
            {"cpu": both})
    rm_case("hints", "allocate with required CPUBindPolicySpreadByPCPUs and allocated", "1447-1491",
            pod("4", "SpreadByPCPUs"), {"cpu": [{"bits": [0], "preferred": True}]},
            allocated=("1,3,5,7-103", alloc("48", "52")))
    rm_case("hints", "failed to allocate with required CPUBindPolicySpreadByPCPUs and allocated", "1492-1528",
            pod("4", "SpreadByPCPUs"), {"cpu": []}, allocated=("4-103", alloc("48", "52")))
    rm_case("hints", "failed to allocate with CPU Share and allocated and amplified ratios", "1529-1580", pod("4"),
            {"cpu": [{"bits": [0, 1], "preferred": True}]}, ratio=1.5, allocated=("0-49,52-101", alloc("50", "50")))


def node_score():
    """TestNUMANodeScore: NUMA zones = node allocatable / count, CPU topology
    buildCPUTopologyForTest(count, 1, cpu/2/count, 2) (scoring_test.go:263-283); existing pods are
    allocations on NUMA 0 (their requests; cpusets 0..cpu-1 for LSR koord-prod pods, :285-305); the
    snapshot holds no pods (NodeInfo.Requested = 0).  Node scorer MostAllocated, NUMA scorer the
    default (LeastAllocated)."""
    def node(name, cpu, mem, count, policy):
        return {"name": name, "cpu": cpu, "memory": mem, "numa": count, "policy": policy}

    def existing(node_i, cpu, mem, lsr=False):
        return {"node": node_i, "cpu": cpu, "memory": mem, "lsr": lsr}

    def case(name, lines, nodes, pod_spec, want, existing_pods=()):
        cases.append({"name": name, "source": f"{SC}:{lines}", "op": "node_score", "nodes": nodes,
                      "pod": pod_spec, "existing": list(existing_pods), "strategy": "MostAllocated",
                      "want": {"scores": want}})

    case("single numa nodes score", "57-97",
         [node("test-node-1", "104", "256Gi", 2, "SingleNUMANode"),
          node("test-node-2", "64", "128Gi", 1, "SingleNUMANode")],
         {"cpu": "21", "memory": "40Gi", "lsr": False}, [35, 31])
    case("restricted numa nodes score", "98-138",
         [node("test-node-1", "104", "256Gi", 2, "Restricted"), node("test-node-2", "64", "128Gi", 1, "Restricted")],
         {"cpu": "50", "memory": "40Gi", "lsr": False}, [63, 54])
    three = [node(f"test-node-{k}", "104", "256Gi", 2, "SingleNUMANode") for k in (1, 2, 3)]
    case("single numa nodes score with same capacity but different requested", "139-193", three,
         {"cpu": "4", "memory": "40Gi", "lsr": False}, [19, 19, 19],
         [existing(0, "4", "8Gi"), existing(1, "8", "32Gi"), existing(2, "32", "40Gi")])
    case("single numa nodes score with same capacity but different requested and LSR", "194-253", three,
         {"cpu": "4", "memory": "40Gi", "lsr": True}, [23, 27, 34],
         [existing(0, "4", "8Gi"), existing(0, "4", "8Gi", True), existing(1, "8", "32Gi"),
          existing(1, "8", "32Gi", True), existing(2, "16", "40Gi"), existing(2, "16", "40Gi", True)])


def main():
    allocate()
    hints()
    node_score()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "numa_cpuset.json")
    with open(out, "w") as f:
        json.dump({"source": "koordinator nodenumaresource tests (cpusets under NUMA policies)", "cases": cases}, f,
                  indent=1)
    print(f"{len(cases)} cases -> {out}")


if __name__ == "__main__":
    main()
