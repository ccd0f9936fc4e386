"""Transcription of the CPU accumulator known-answer tests into tests/golden/cpu_accumulator.json.

Same rules as make_fixtures.py (hand transcription; each case cites its Go test lines, relative to
haoyann/koordinator).  Source: pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go.
Topologies are buildCPUTopologyForTest(sockets, nodesPerSocket, coresPerNode, cpusPerCore)
(:30-57): CPU ids, NUMA node ids and core ids numbered in that nesting order; `core_shift` = the test
rewrites CoreID to SocketID<<16 | CoreID.

Run:  python tests/golden/make_cpu_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go"
cases = []


def take(name, line, topo, needed, want, bind, strategy="MostAllocated", allocated="", alloc_excl="",
         excl="", max_ref=1, preferred=None):
    cases.append({"name": name, "source": f"{SRC}:{line}", "op": "take", "topology": topo, "max_ref": max_ref,
                  "allocated": allocated, "alloc_excl": alloc_excl, "needed": needed, "bind": bind, "excl": excl,
                  "strategy": strategy, "preferred": preferred, "want": want})


FULL, SPREAD = "FullPCPUs", "SpreadByPCPUs"
# TestTakeFullPCPUs (:59-173), NUMAMostAllocated
for name, line, topo, alloc, n, want in [
    ("allocate on non-NUMA node", 70, [1, 1, 4, 2], "", 2, "0-1"),
    ("with allocated cpus", 77, [1, 1, 4, 2], "0-1", 2, "2-3"),
    ("allocate whole socket", 85, [2, 1, 4, 2], "", 8, "0-7"),
    ("allocate across socket", 92, [2, 1, 4, 2], "", 12, "0-11"),
    ("allocate whole socket with partially-allocated socket", 99, [2, 1, 4, 2], "0-1", 8, "8-15"),
    ("allocate in the smallest idle socket", 107, [2, 2, 4, 2], "0-5,16-23", 6, "24-29"),
    ("allocate the most of CPUs on the same socket", 115, [2, 2, 4, 2], "0-5,16-23", 12, "6-15,24-25"),
    ("allocate from first socket", 123, [2, 2, 4, 2], "0-3,8-11", 4, "4-7"),
    ("allocate with less spread cpus", 131, [2, 2, 2, 2], "0,2,4,8,12", 4, "10-11,14-15"),
    ("allocate with the most spread cpus", 139, [2, 2, 2, 2], "0,2,4,8,10,12", 6, "5-7,13-15"),
    ("allocate with the most spread cpus on the smallest idle cpus socket", 147, [2, 2, 2, 2], "0,2,4,8-10,12", 6,
     "6-7,11,13-15"),
]:
    take(f"FullPCPUs MostAllocated: {name}", line, topo, n, want, FULL, allocated=alloc)
# TestTakeFullPCPUsWithNUMALeastAllocated (:175-289)
for name, line, topo, alloc, n, want in [
    ("allocate on non-NUMA node", 186, [1, 1, 4, 2], "", 2, "0-1"),
    ("with allocated cpus", 193, [1, 1, 4, 2], "0-1", 2, "2-3"),
    ("allocate whole socket", 201, [2, 1, 4, 2], "", 8, "0-7"),
    ("allocate across socket", 208, [2, 1, 4, 2], "", 12, "0-11"),
    ("allocate whole socket with partially-allocated socket", 215, [2, 1, 4, 2], "0-1", 8, "8-15"),
    ("allocate in the most idle socket", 223, [2, 2, 4, 2], "0-5,16-23", 6, "8-13"),
    ("allocate the most of CPUs on the same socket", 231, [2, 2, 4, 2], "0-5,16-23", 12, "6-15,24-25"),
    ("allocate from second socket", 239, [2, 2, 4, 2], "0-3,8-11", 4, "16-19"),
    ("allocate with less spread cpus", 247, [2, 2, 2, 2], "0,2,4,8,12", 4, "10-11,14-15"),
    ("allocate with the less spread cpus 2", 255, [2, 2, 2, 2], "0,2,4,8,10,12", 6, "1,3,6-7,14-15"),
    ("allocate with the most spread cpus on the most idle cpus socket 3", 263, [2, 2, 4, 2], "0,2,4,8-10,12", 6,
     "16-21"),
]:
    take(f"FullPCPUs LeastAllocated: {name}", line, topo, n, want, FULL, strategy="LeastAllocated", allocated=alloc)
# TestTakeSpreadByPCPUs (:301-361) / WithNUMALeastAllocated (:373-433)
for strategy, rows in [("MostAllocated", [
        ("allocate on non-NUMA node", 312, [1, 1, 4, 2], "", 4, "0,2,4,6"),
        ("allocate satisfied the partially-allocated socket", 319, [2, 1, 4, 2], "0,2", 4, "1,3-4,6"),
        ("allocate cpus on full-free socket", 327, [2, 1, 4, 2], "0-3", 4, "8,10,12,14"),
        ("allocate most of CPUs in the same socket and overlapped-cores", 335, [2, 1, 4, 2], "0,2", 6, "1,3-7")]),
        ("LeastAllocated", [
        ("allocate on non-NUMA node", 384, [1, 1, 4, 2], "", 4, "0,2,4,6"),
        ("allocate satisfied the partially-allocated socket", 391, [2, 1, 4, 2], "0,2", 4, "8,10,12,14"),
        ("allocate cpus on full-free socket", 399, [2, 1, 4, 2], "0-3", 4, "8,10,12,14"),
        ("allocate most of CPUs in the same socket and overlapped-cores", 407, [2, 1, 4, 2], "0,2", 6,
         "8-12,14")])]:
    for name, line, topo, alloc, n, want in rows:
        take(f"SpreadByPCPUs {strategy}: {name}", line, topo, n, want, SPREAD, strategy=strategy, allocated=alloc)
# TestTakeCPUsWithExclusivePolicy (:435-558): allocated CPUs carry PCPULevel unless stated; the pod's
# exclusive policy defaults to PCPULevel and its bind policy to SpreadByPCPUs
for name, line, topo, alloc, alloc_excl, excl, bind, n, want in [
    ("allocate cpus on full-free socket with PCPULevel", 449, [2, 1, 4, 2], "0,2", "PCPULevel", "PCPULevel", SPREAD,
     4, "8,10,12,14"),
    ("allocate overlapped cpus with PCPULevel", 457, [2, 1, 4, 2], "", "PCPULevel", "PCPULevel", SPREAD, 10,
     "0-4,6,8,10,12,14"),
    ("allocate cpus on large-size partially-allocated socket with PCPULevel", 464, [2, 1, 8, 2], "0,2", "PCPULevel",
     "PCPULevel", SPREAD, 4, "4,6,8,10"),
    ("allocate cpus with none exclusive policy", 472, [2, 1, 8, 2], "0,2", "PCPULevel", "None", SPREAD, 4, "1,3-4,6"),
    ("allocate cpus on full-free socket with NUMANodeLevel", 481, [2, 1, 4, 2], "0,2", "NUMANodeLevel", "NUMANodeLevel",
     SPREAD, 4, "8,10,12,14"),
    ("allocate cpus on partially-allocated socket without NUMANodeLevel", 491, [2, 1, 4, 2], "0,2", "NUMANodeLevel",
     "None", SPREAD, 4, "1,3-4,6"),
    ("allocate cpus on full-free socket with NUMANodeLevel with PCPUs", 501, [2, 1, 4, 2], "0,2", "NUMANodeLevel",
     "NUMANodeLevel", FULL, 4, "8-11"),
    ("allocate cpus on partially-allocated socket without NUMANodeLevel with PCPUs", 512, [2, 1, 4, 2], "0,2",
     "NUMANodeLevel", "None", FULL, 4, "4-7"),
]:
    take(f"ExclusivePolicy: {name}", line, topo, n, want, bind, allocated=alloc, alloc_excl=alloc_excl, excl=excl)
# TestTakePreferredCPUs (:758-777): topology (2, 1, 16, 2), all CPUs available
take("TakePreferredCPUs: takeCPUs spread 2", 761, [2, 1, 16, 2], 2, "0,2", SPREAD)
take("TakePreferredCPUs: preferred 0,2", 765, [2, 1, 16, 2], 2, "0,2", SPREAD, preferred="0,2")
take("TakePreferredCPUs: without 0,2", 769, [2, 1, 16, 2], 2, "1,3", SPREAD, allocated="0,2", preferred="")
take("TakePreferredCPUs: preferred 11,13,15,17", 773, [2, 1, 16, 2], 2, "11,13", SPREAD, preferred="11,13,15,17")

# sequences with resource-manager state (NodeAllocation.addCPUs, PCPULevel) between pods, maxRefCount 2
cases.append({"name": "TakeCPUsWithMaxRefCount", "source": f"{SRC}:560-599", "op": "sequence",
              "topology": [1, 1, 4, 2], "core_shift": True, "max_ref": 2, "strategy": "MostAllocated",
              "steps": [[4, FULL, "0-3"], [5, FULL, "0,4-7"], [4, FULL, "2-5"]]})
cases.append({"name": "TakeCPUsSortByRefCount", "source": f"{SRC}:601-653", "op": "sequence",
              "topology": [1, 1, 16, 2], "core_shift": True, "max_ref": 2, "strategy": "MostAllocated",
              "steps": [[16, SPREAD, "0,2,4,6,8,10,12,14,16,18,20,22,24,26,28,30"], [16, FULL, "0-15"],
                        [16, SPREAD, "1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31"], [16, FULL, "16-31"]],
              "final_available": ""})
# TestCPUSpreadByPCPUs (:291-299) / WithNUMALeastAllocated (:363-371): freeCPUs + spreadCPUs order
ORDER = [0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30, 1, 3, 5, 7, 9, 11, 13, 15, 17, 19, 21, 23, 25, 27,
         29, 31]
for strategy, line in (("MostAllocated", "291-299"), ("LeastAllocated", "363-371")):
    cases.append({"name": f"CPUSpreadByPCPUs {strategy}", "source": f"{SRC}:{line}", "op": "spread",
                  "topology": [2, 2, 4, 2], "strategy": strategy, "want": ORDER})


def main():
    with open(os.path.join(HERE, "cpu_accumulator.json"), "w") as f:
        json.dump({"source": "haoyann/koordinator cpu_accumulator_test.go, transcribed by make_cpu_fixtures.py",
                   "cases": cases}, f, indent=1)
    print(f"cpu_accumulator.json: {len(cases)} cases")


if __name__ == "__main__":
    main()
