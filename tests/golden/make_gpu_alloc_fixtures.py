"""Transcription of the GPUAllocator known-answer tests into tests/golden/gpu_allocator.json.

Same rules as make_fixtures.py: the reference is Go and cannot run here, so every case is
restated by hand from the Go test table it cites (paths relative to haoyann/koordinator).  Only data is
written: the node's GPU devices (total, used, topology), the partition indexer + policy the allocator
resolves for the node, the pod's GPU request and annotations, and the expected status or GPU minors.

The Go tables allocate GPUs jointly with RDMA virtual functions (DeviceJointAllocate + VFSelector hints).
Those parts are outside the modelled path and refused at the boundary; the joint allocation allocates
the primary GPU type first through the same GPUAllocator.Allocate (device_allocator.go:252-262), so the
GPU minors of each expected allocation are what a GPU-only request yields.  The RDMA devices and the
assigned pod's RDMA allocations are therefore left out.  Assigned GPU allocations become `used` on the
devices (updateCacheUsed).

Run:  python tests/golden/make_gpu_alloc_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ALLOC = "pkg/scheduler/plugins/deviceshare/allocator_gpu_test.go"
CR = "pkg/scheduler/plugins/deviceshare/device_allocator_test.go"

CORE, MEM, RATIO = "koordinator.sh/gpu-core", "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio"
FULL = {CORE: "100", RATIO: "100", MEM: "85198045184"}  # gpuResourceList, device_allocator_test.go:43-47
HALF = {CORE: "50", RATIO: "50", MEM: "42599022592"}    # gpuSharedResourceList, :49-53
TOTAL = {CORE: "100", MEM: "83201216Ki", RATIO: "100"}

UNSCHED, UNRESOLVABLE = 2, 3
R_UNSUPPORTED_NUMBER, R_INSUFFICIENT_SCOPED = 37, 41

# fakeH800DeviceCR (allocator_gpu_test.go:40-47): GPU minor -> (NUMA node, PCIe id)
H800_TOPO = {0: (0, "0"), 1: (0, "2"), 2: (0, "3"), 3: (0, "4"), 4: (1, "5"), 5: (1, "6"), 6: (1, "7"), 7: (1, "8")}
# fakeDeviceCR (device_allocator_test.go:63-...): two GPUs per PCIe switch, two switches per NUMA node
FAKE_TOPO = {0: (0, "0"), 1: (0, "0"), 2: (0, "1"), 3: (0, "1"), 4: (1, "2"), 5: (1, "2"), 6: (1, "3"), 7: (1, "3")}


def gpus(topo, used):
    return [{"type": "gpu", "minor": m, "total": TOTAL, "used": used.get(m, {}),
             "topology": {"nodeID": n, "pcieID": p}} for m, (n, p) in sorted(topo.items())]


cases = []


def case(name, src, topo, node_labels, requests, used, want=None, code=0, reason=0, hints=None, shared_scorer=False):
    cases.append({"name": name, "source": src, "devices": gpus(topo, used), "node_labels": node_labels,
                  "pod": {"requests": requests, "device_hints": hints},
                  "weights": [1, None, None, None] if shared_scorer else None,
                  "strategy": "MostAllocated" if shared_scorer else "LeastAllocated",
                  "want": {"code": code, "reason": reason, "minors": want}})


def whole(n):
    return {"nvidia.com/gpu": str(n)}


# ---- TestAllocateByPartition (allocator_gpu_test.go:54-964): node labels gpu-model H800/H100 and
# gpu-partition-policy Honor unless the case overrides it (:852-862); the Device has no partition table, so
# the designated Hopper indexer applies (allocator_gpu_helper.go:146-162).
def honor(model, policy="Honor"):
    return {"node.koordinator.sh/gpu-model": model, "node.koordinator.sh/gpu-partition-policy": policy}


P = ALLOC
case("partition: 1 GPU", f"{P}:91-120", H800_TOPO, honor("H800"), whole(1), {}, want=[0])
case("partition: 2 GPUs", f"{P}:121-168", H800_TOPO, honor("H800"), whole(2), {}, want=[0, 1])
case("partition: 3 GPUs unsupported", f"{P}:169-175", H800_TOPO, honor("H800"), whole(3), {},
     code=UNRESOLVABLE, reason=R_UNSUPPORTED_NUMBER)
case("partition: 4 GPUs", f"{P}:176-259", H800_TOPO, honor("H800"), whole(4), {}, want=[0, 1, 2, 3])
case("partition: 6 GPUs unsupported", f"{P}:260-266", H800_TOPO, honor("H800"), whole(6), {},
     code=UNRESOLVABLE, reason=R_UNSUPPORTED_NUMBER)
case("partition: 8 GPUs", f"{P}:267-422", H800_TOPO, honor("H800"), whole(8), {}, want=list(range(8)))
case("partition: 2 GPUs with 2,3 assigned", f"{P}:423-513", H800_TOPO, honor("H800"), whole(2),
     {2: FULL, 3: FULL}, want=[0, 1])
case("partition: 2 GPUs with 4 assigned, binpack", f"{P}:514-586", H800_TOPO, honor("H800"), whole(2),
     {4: FULL}, want=[6, 7])
case("partition: 1 GPU with 4 assigned, binpack", f"{P}:587-641", H800_TOPO, honor("H800"), whole(1),
     {4: FULL}, want=[5])
case("partition: H100 2 GPUs with 2,3 assigned", f"{P}:642-732", H800_TOPO, honor("H100"), whole(2),
     {2: FULL, 3: FULL}, want=[0, 1])
case("partition: H100 Prefer 3 GPUs falls back to topology", f"{P}:733-842", H800_TOPO,
     honor("H100", "Prefer"), whole(3), {2: FULL, 3: FULL}, want=[4, 5, 6])

# ---- TestAllocateByTopology (allocator_gpu_test.go:965-1404): fakeDeviceCR, no partition table
T = ALLOC
case("topology: 1 GPU with 5 assigned", f"{T}:978-1031", FAKE_TOPO, {}, whole(1), {5: FULL}, want=[4])
case("topology: 2 GPUs with 5 assigned", f"{T}:1032-1089", FAKE_TOPO, {}, whole(2), {5: FULL}, want=[6, 7])
case("topology: 2 GPUs required PCIe", f"{T}:1090-1148", FAKE_TOPO, {}, whole(2), {5: FULL}, want=[6, 7],
     hints={"gpu": {"requiredTopologyScope": "PCIe"}})
case("topology: 4 GPUs required NUMANode", f"{T}:1149-1229", FAKE_TOPO, {}, whole(4), {5: FULL},
     want=[0, 1, 2, 3], hints={"gpu": {"requiredTopologyScope": "NUMANode"}})
case("topology: 4 GPUs required NUMANode, insufficient", f"{T}:1230-1278", FAKE_TOPO, {}, whole(4),
     {5: FULL, 0: FULL}, code=UNSCHED, reason=R_INSUFFICIENT_SCOPED,
     hints={"gpu": {"requiredTopologyScope": "NUMANode"}})

# ---- TestAllocateSharedGPU (allocator_gpu_test.go:1405-1668): gpu.shared 1, ratio 50, core 50 per pod;
# scorer MostAllocated over gpu-memory-ratio weight 1 (:1630-1640)
S = ALLOC
SHARED = {"koordinator.sh/gpu.shared": "1", RATIO: "50", CORE: "50"}
case("shared: 1 GPU with 5 assigned", f"{S}:1418-1471", FAKE_TOPO, {}, SHARED, {5: FULL}, want=[4],
     shared_scorer=True)
case("shared: two non-empty scopes, binpack takes precedence", f"{S}:1472-1529", FAKE_TOPO, {}, SHARED,
     {5: FULL, 7: HALF}, want=[7], shared_scorer=True)

if __name__ == "__main__":
    path = os.path.join(HERE, "gpu_allocator.json")
    with open(path, "w") as f:
        json.dump({"source": "haoyann/koordinator GPUAllocator tests, transcribed by make_gpu_alloc_fixtures.py",
                   "cases": cases}, f, indent=1)
    print(f"{len(cases)} cases -> {path}")
