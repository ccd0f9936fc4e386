"""Transcription of DeviceShare's NUMA hint-provider tests into tests/golden/ds_numa.json.

Same rules as make_fixtures.py: the reference is Go and cannot run here, so every case is
restated by hand from the Go test it cites (paths relative to haoyann/koordinator).  Only data is written:
the node's devices (fakeDeviceCR: 8 GPUs and 4 RDMA NICs on two NUMA nodes), the pod's device requests, the
assigned allocations (as `used`), and the expected hints / status.

Cases whose pods carry an RDMA VFSelector, an AllocateStrategy or a DeviceJointAllocate are not transcribed:
those paths are refused at the boundary (KE_ERR_UNSUPPORTED, koord_eval.h KE_DHINT_*).

Run:  python tests/golden/make_ds_numa_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "pkg/scheduler/plugins/deviceshare/topology_hint_test.go"
CORE, MEM, RATIO, RDMA = ("koordinator.sh/gpu-core", "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio",
                          "koordinator.sh/rdma")
GPU_TOTAL = {CORE: "100", MEM: "83201216Ki", RATIO: "100"}
UNRESOLVABLE = 3

# fakeDeviceCR (device_allocator_test.go:63-...): type, minor, NUMA node, PCIe id
FAKE = ([("rdma", m, n, p) for m, n, p in ((1, 0, "0"), (2, 0, "1"), (3, 1, "2"), (4, 1, "3"))] +
        [("gpu", m, m // 4, str(m // 2)) for m in range(8)])


def devices(used=None):
    used = used or {}
    out = []
    for t, m, n, p in FAKE:
        total = GPU_TOTAL if t == "gpu" else {RDMA: "100"}
        out.append({"type": t, "minor": m, "total": total, "used": used.get((t, m), {}),
                    "topology": {"nodeID": n, "pcieID": p}})
    return out


def bits(*ids):
    return sum(1 << i for i in ids)


cases = []


def hints(name, lines, requests, want=None, copies=0, code=0, reason=0, used=None):
    cases.append({"name": name, "source": f"{SRC}:{lines}", "op": "hints", "devices": devices(used),
                  "pod": {"requests": requests},
                  "want": {"code": code, "reason": reason, "copies": copies,
                           "hints": [list(h) for h in (want or [])]}})


def allocate(name, lines, requests, affinity, code=0):
    cases.append({"name": name, "source": f"{SRC}:{lines}", "op": "allocate", "devices": devices(),
                  "pod": {"requests": requests}, "affinity": affinity, "want": {"code": code}})


G1 = {CORE: "100", RATIO: "100"}  # gpuRequests, :47-50
R2 = {RDMA: "2"}                  # rdmaRequests, :55-57
# ---- TestPlugin_GetPodTopologyHints (topology_hint_test.go:40-269); want: (mask, preferred, score) per hint
hints("generate gpu&rdma hints", "67-85", dict(G1, **R2),
      [(bits(0), True, 500), (bits(1), True, 0), (bits(0, 1), False, 500)], copies=2)
hints("generate gpu&rdma hints but large gpu requests", "86-94", dict({CORE: "1700", RATIO: "1700"}, **R2),
      code=UNRESOLVABLE, reason=43)
hints("generate gpu hints with assigned devices", "95-117", {CORE: "400", RATIO: "400"},
      [(bits(1), True, 500), (bits(0, 1), False, 500)], copies=1, used={("gpu", 0): G1})
hints("generate fpga empty hints", "118-127", {"koordinator.sh/fpga": "100"}, code=UNRESOLVABLE, reason=35)

# ---- TestPlugin_Allocate (topology_hint_test.go:271-418)
allocate("allocate gpu&rdma by affinity", "293-302", {CORE: "100", MEM: "8Gi", RDMA: "2"}, bits(0))
allocate("generate fpga empty hints", "303-312", {"koordinator.sh/fpga": "100"}, 0, code=UNRESOLVABLE)

if __name__ == "__main__":
    path = os.path.join(HERE, "ds_numa.json")
    with open(path, "w") as f:
        json.dump({"source": "haoyann/koordinator DeviceShare NUMA hint tests, transcribed by make_ds_numa_fixtures.py",
                   "cases": cases}, f, indent=1)
    print(f"{len(cases)} cases -> {path}")
