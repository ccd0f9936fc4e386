"""Transcription of NodeNUMAResource cpuset Filter / Reserve known-answer tests into
tests/golden/cpuset.json (same rules as make_fixtures.py; paths relative to haoyann/koordinator).

Source: pkg/scheduler/plugins/nodenumaresource/plugin_test.go, TestPlugin_Filter (:564-911) and
TestPlugin_Reserve (:1086-1558), the cases without NUMA topology policy and without reservations.
The Go tests write the preFilterState directly; here the equivalent pod is given: `cpuset` = a
koord-prod LSR pod (AllowUseCPUSet) with the ResourceSpec bind policies, `ls` = a koord-prod LS pod.
A state with requestCPUBind and no requested cpus has no pod equivalent; "succeed with valid cpu
topology" (Filter :589) is restated with 4 cpus.  Node: allocatable cpu 96 / memory 512Gi,
buildCPUTopologyForTest CPU topology, labels / kubelet policy as node cpu bind policy.

Run:  python tests/golden/make_cpuset_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/plugins/nodenumaresource/plugin_test.go"
UU, U = 3, 2
INVALID_TOPO, INVALID_CPUS, CONFLICT, SMT = 18, 23, 24, 25
cases = []


def filt(name, line, pod, want=(0, 0), node_bind="None", topology=(2, 1, 4, 2), invalid_topology=False, ratio=None):
    cases.append({"name": name, "source": f"{SRC}:{line}", "op": "filter", "pod": pod, "node_bind": node_bind,
                  "topology": list(topology), "invalid_topology": invalid_topology, "ratio": ratio,
                  "want": {"code": want[0], "reason": want[1]}})


def cs(cpu, required="", preferred="", kind="cpuset"):
    return {"kind": kind, "cpu": cpu, "required": required, "preferred": preferred}


filt("error with invalid cpu topology", "580-587", cs("4"), (UU, INVALID_TOPO), invalid_topology=True)
filt("succeed with valid cpu topology", "589-596", cs("4"))
filt("failed to verify Node FullPCPUsOnly with SMTAlignmentError", "605-617", cs("5", preferred="FullPCPUs"),
     (UU, SMT), node_bind="FullPCPUsOnly")
filt("LS Pod failed to verify Node FullPCPUsOnly with SMTAlignmentError", "619-633", cs("5", kind="ls"), (UU, SMT),
     node_bind="FullPCPUsOnly")
filt("LS Pod failed to verify Node FullPCPUsOnly with non-integer request", "635-649", cs("5200m", kind="ls"),
     (UU, INVALID_CPUS), node_bind="FullPCPUsOnly")
filt("verify Node FullPCPUsOnly", "651-663", cs("4", preferred="FullPCPUs"), node_bind="FullPCPUsOnly")
filt("failed to verify required FullPCPUs SMTAlignmentError", "665-674", cs("5", required="FullPCPUs"), (UU, SMT))
filt("verify required FullPCPUs", "676-685", cs("4", required="FullPCPUs"))
filt("verify FullPCPUsOnly with preferred SpreadByPCPUs", "687-699", cs("4", preferred="SpreadByPCPUs"),
     node_bind="FullPCPUsOnly")
filt("failed to verify FullPCPUsOnly with required SpreadByPCPUs", "701-713", cs("4", required="FullPCPUs"),
     (UU, CONFLICT), node_bind="SpreadByPCPUs")
filt("verify FullPCPUsOnly with required FullPCPUs", "715-727", cs("4", required="FullPCPUs"), node_bind="FullPCPUsOnly")
# kubelet static policy with full-pcpus-only=true: GetNodeCPUBindPolicy -> FullPCPUsOnly
filt("verify Kubelet FullPCPUsOnly with SMTAlignmentError", "729-744", cs("5", preferred="FullPCPUs"), (UU, SMT),
     node_bind="FullPCPUsOnly")
filt("verify Kubelet FullPCPUsOnly with required SpreadByPCPUs", "746-761", cs("4", required="SpreadByPCPUs"),
     (UU, CONFLICT), node_bind="FullPCPUsOnly")
filt("verify Kubelet FullPCPUsOnly with required FullPCPUs", "763-778", cs("4", required="FullPCPUs"),
     node_bind="FullPCPUsOnly")
filt("verify required FullPCPUs with none NUMA topology policy", "780-789", cs("4", required="FullPCPUs",
                                                                             preferred="FullPCPUs"))
filt("verify FullPCPUs with None NUMA Topology Policy and amplification ratio", "822-837",
     cs("4", required="FullPCPUs", preferred="FullPCPUs"), ratio=1.5)


def reserve(name, line, pod, want_cpus, node_bind="None", topology=(2, 1, 4, 2), allocated="", strategy="",
            fails=False):
    cases.append({"name": name, "source": f"{SRC}:{line}", "op": "reserve", "pod": pod, "node_bind": node_bind,
                  "topology": list(topology), "allocated": allocated, "numa_allocate_strategy": strategy,
                  "want": {"fails": fails, "cpuset": want_cpus}})


reserve("succeed with valid cpu topology", "1126-1137", cs("4", preferred="FullPCPUs"), "0-3")
reserve("allocated by node cpu bind policy", "1138-1154", cs("4", kind="ls"), "0,2,4,6", node_bind="SpreadByPCPUs")
reserve("BE Pod reserves with node cpu bind policy", "1155-1169", cs("0", kind="be"), "", node_bind="SpreadByPCPUs")
reserve("error with big request cpu", "1170-1179", cs("24"), "", fails=True)
reserve("succeed with valid cpu topology and node numa least allocate strategy", "1180-1195",
        cs("4", preferred="FullPCPUs"), "16-19", topology=(2, 1, 8, 2), allocated="0-3", strategy="LeastAllocated")
reserve("succeed with valid cpu topology and node numa most allocate strategy", "1196-1211",
        cs("4", preferred="FullPCPUs"), "4-7", topology=(2, 1, 8, 2), allocated="0-3", strategy="MostAllocated")


def main():
    with open(os.path.join(HERE, "cpuset.json"), "w") as f:
        json.dump({"source": "haoyann/koordinator nodenumaresource plugin_test.go, transcribed by "
                             "make_cpuset_fixtures.py", "cases": cases}, f, indent=1)
    print(f"cpuset.json: {len(cases)} cases")


if __name__ == "__main__":
    main()
