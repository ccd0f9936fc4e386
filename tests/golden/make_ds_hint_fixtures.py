"""Transcription of the reference's DeviceShare hint tests into tests/golden/ds_hints.json.

Same rules as make_fixtures.py: the Go tests cannot run here; each case restates one test case's
objects and expectations by hand.  Only data is written.

  * deviceshare/device_allocator_test.go:63-92  fakeDeviceCR: 4 RDMA NICs (minors 1-4, label type=fakeW, PCIe
    0-3, NUMA 0,0,1,1) with one VF group (label type=general) of 30 VFs each, 8 GPUs (2 per PCIe switch)
  * device_allocator_test.go:94-165  the tests' hints: an RDMA Selector type=fakeW, a VFSelector type In
    [general, <vfType>], ApplyForAll on RDMA, the joint allocation [gpu, rdma]
  * device_allocator_test.go:167-1180  TestAutopilotAllocator (Allocate outside Reserve, no scorer): the fakeDeviceCR
    cases — 0/1/2/3/4/6/8 GPUs with VFs, with assigned devices, and with secondary devices well planned
  * devicehandler_default_test.go:32-183  DefaultDeviceHandler.CalcDesiredRequestsAndCount on fakeDeviceCR plus an
    RDMA minor 5 labelled type=fakeS: ApplyForAll with matchLabels / Exists selectors, RequestsAsCount with and
    without the DeviceLevel exclusive policy (observed as the RDMA minors allocated and their per-device amount)

Run:  python tests/golden/make_ds_hint_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
DA = "pkg/scheduler/plugins/deviceshare/device_allocator_test.go"
DH = "pkg/scheduler/plugins/deviceshare/devicehandler_default_test.go"
GPU_RES = {"koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory": "83201216Ki",
           "koordinator.sh/gpu-memory-ratio": "100"}
PREFIX = {1: "0000:1f", 2: "0000:90", 3: "0000:51", 4: "0000:b9"}


def vf_bus(minor, k):
    """the k-th VF of RDMA `minor` in fakeDeviceCR: functions .2 .. .7 of device 00, then 01.0 ..."""
    flat = k + 2
    return f"{PREFIX[minor]}:{flat // 8:02x}.{flat % 8}"


def fake_device_cr(extra_rdma5=False):
    devs = []
    for m in range(1, 5):
        devs.append({"type": "rdma", "labels": {"type": "fakeW"}, "minor": m, "health": True,
                     "resources": {"koordinator.sh/rdma": "100"},
                     "topology": {"socketID": (m - 1) // 2, "nodeID": (m - 1) // 2, "pcieID": str(m - 1)},
                     "vfGroups": [{"labels": {"type": "general"},
                                   "vfs": [{"minor": k, "busID": vf_bus(m, k)} for k in range(30)]}]})
    for m in range(8):
        devs.append({"type": "gpu", "minor": m, "health": True, "resources": GPU_RES,
                     "topology": {"socketID": m // 4, "nodeID": m // 4, "pcieID": str(m // 2)}})
    if extra_rdma5:  # devicehandler_default_test.go:33-50
        devs.append({"type": "rdma", "labels": {"type": "fakeS"}, "minor": 5, "health": True,
                     "resources": {"koordinator.sh/rdma": "100"},
                     "topology": {"socketID": 1, "nodeID": 1, "pcieID": "4"}})
    return {"metadata": {"name": "test-node-1"}, "spec": {"devices": devs}}


def hints(vf_type=None, apply_for_all=False):
    rdma = {"selector": {"matchLabels": {"type": "fakeW"}}}  # setDefaultTestAllocateHints
    if vf_type:
        rdma["vfSelector"] = {"matchExpressions": [{"key": "type", "operator": "In", "values": ["general", vf_type]}]}
    if apply_for_all:
        rdma["allocateStrategy"] = "ApplyForAll"
    return {"rdma": rdma}


JOINT = {"deviceTypes": ["gpu", "rdma"]}
cases = []


def autopilot(name, lines, gpu, want_gpu, want_rdma, assigned=None, well_planned=False, host_network=False):
    """want_rdma: [(minor, vf BusID or None)]"""
    if host_network:
        h, joint = hints(apply_for_all=True), JOINT
    elif gpu > 0:
        h, joint = hints("fakeG"), JOINT
    else:
        h, joint = hints("fakeC"), None
    req = {"koordinator.sh/rdma": "1"}
    if gpu:
        req["nvidia.com/gpu"] = str(gpu)
    cases.append({"name": name, "source": f"{DA}:{lines}", "kind": "autopilot", "device": fake_device_cr(),
                  "secondary_well_planned": well_planned, "assigned": assigned, "requests": req, "hints": h,
                  "joint": joint, "want": {"gpu": want_gpu, "rdma": want_rdma}})


ASSIGNED = {"gpu": [0], "rdma": [[1, "0000:1f:00.2"]]}  # an assigned pod: GPU 0 whole, RDMA 1 with one VF (rdma 1)
autopilot("allocate_0_gpu_1_vf", "193-215", 0, [], [[1, "0000:1f:00.2"]])
autopilot("allocate_1_gpu_1_vf", "216-244", 1, [0], [[1, "0000:1f:00.2"]])
autopilot("allocate_2_gpu_1_vf", "245-277", 2, [0, 1], [[1, "0000:1f:00.2"]])
autopilot("allocate_3_gpu_2_vf", "278-328", 3, [0, 1, 2], [[1, "0000:1f:00.2"], [2, "0000:90:00.2"]])
autopilot("allocate_4_gpu_2_vf", "329-383", 4, [0, 1, 2, 3], [[1, "0000:1f:00.2"], [2, "0000:90:00.2"]])
autopilot("allocate_6_gpu_3_vf", "384-460", 6, [0, 1, 2, 3, 4, 5],
          [[1, "0000:1f:00.2"], [2, "0000:90:00.2"], [3, "0000:51:00.2"]])
autopilot("allocate_8_gpu_4_vf", "461-559", 8, list(range(8)),
          [[1, "0000:1f:00.2"], [2, "0000:90:00.2"], [3, "0000:51:00.2"], [4, "0000:b9:00.2"]])
autopilot("allocate_2_gpu_1_vf_assigned", "560-616", 2, [2, 3], [[2, "0000:90:00.2"]], assigned=ASSIGNED)
autopilot("allocate_3_gpu_2_vf_assigned", "617-691", 3, [1, 2, 3], [[1, "0000:1f:00.3"], [2, "0000:90:00.2"]],
          assigned=ASSIGNED)
autopilot("allocate_8_gpu_4_vf_well_planned", "1016-1058", 8, list(range(8)), [], well_planned=True)

# DefaultDeviceHandler.CalcDesiredRequestsAndCount (devicehandler_default_test.go:62-156): pod requests rdma only
for name, lines, q, hint, want_count, want_per, ok in (
        ("general_one_nic", "63-69", "100", None, 1, 100, True),
        ("apply_for_all_fakeW", "70-84", "1", {"selector": {"matchLabels": {"type": "fakeW"}},
                                                "allocateStrategy": "ApplyForAll"}, 4, 1, True),
        ("apply_for_all_fakeS", "85-99", "1", {"selector": {"matchLabels": {"type": "fakeS"}},
                                                "allocateStrategy": "ApplyForAll"}, 1, 1, True),
        ("apply_for_all_exists", "100-118", "1", {"selector": {"matchExpressions": [{"key": "type", "operator": "Exists"}]},
                                                   "allocateStrategy": "ApplyForAll"}, 5, 1, True),
        ("apply_for_all_unmatched", "119-136", "1", {"selector": {"matchExpressions": [{"key": "non-exists-label",
                                                                                         "operator": "Exists"}]},
                                                      "allocateStrategy": "ApplyForAll"}, 0, 0, False),
        ("requests_as_count", "137-149", "4", {"allocateStrategy": "RequestsAsCount"}, 4, 1, True),
        ("requests_as_count_exclusive", "150-163", "4", {"allocateStrategy": "RequestsAsCount",
                                                          "exclusivePolicy": "DeviceLevel"}, 4, 100, True)):
    cases.append({"name": name, "source": f"{DH}:{lines}", "kind": "handler", "device": fake_device_cr(True),
                  "requests": {"koordinator.sh/rdma": q}, "hints": {"rdma": hint} if hint else None,
                  "want": {"count": want_count, "per_device": want_per, "ok": ok}})

# DeviceShare's NUMA hints (topology_hint_test.go:128-212, fakeDeviceCR): [mask, preferred, score] per hint,
# one list per requested type (copies); GPU requests gpu-core 100 + gpu-memory-ratio 100, RDMA requests rdma 2
TH = "pkg/scheduler/plugins/deviceshare/topology_hint_test.go"
ONE, TWO, BOTH = 1, 2, 3
for name, lines, req, hint, joint, copies, want in (
        ("numa_hints_2_rdma", "128-145", {"koordinator.sh/rdma": "2"}, {"rdma": {"allocateStrategy": "RequestsAsCount"}},
         None, 1, [[ONE, True, 500], [TWO, True, 500], [BOTH, False, 500]]),
        ("numa_hints_rdma_2_vf", "146-164", {"koordinator.sh/rdma": "2"},
         {"rdma": {"vfSelector": {}, "allocateStrategy": "RequestsAsCount"}}, None, 1,
         [[ONE, True, 500], [TWO, True, 500], [BOTH, False, 500]]),
        ("numa_hints_rdma_4_vf", "165-183", {"koordinator.sh/rdma": "4"},
         {"rdma": {"vfSelector": {}, "allocateStrategy": "RequestsAsCount"}}, None, 1, [[BOTH, True, 500]]),
        ("numa_hints_joint_gpu_rdma", "184-208", {"koordinator.sh/rdma": "2", "koordinator.sh/gpu-core": "100",
                                                  "koordinator.sh/gpu-memory-ratio": "100"},
         {"rdma": {"vfSelector": {}}}, {"deviceTypes": ["gpu", "rdma"]}, 2,
         [[ONE, True, 500], [TWO, True, 0], [BOTH, False, 500]])):
    cases.append({"name": name, "source": f"{TH}:{lines}", "kind": "numa_hints", "device": fake_device_cr(),
                  "requests": req, "hints": hint, "joint": joint, "want": {"copies": copies, "hints": want}})

if __name__ == "__main__":
    with open(os.path.join(HERE, "ds_hints.json"), "w") as f:
        json.dump({"source": "make_ds_hint_fixtures.py", "cases": cases}, f, indent=1)
    print(len(cases), "cases")
