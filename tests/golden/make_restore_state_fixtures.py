"""Transcription of the reference's RestoreReservation tests of NodeNUMAResource and DeviceShare (SURVEY.md §8f
rank 3: the reservation holdings) into tests/golden/reservation_restore.json.  Same rules as make_fixtures.py: the
Go tests cannot run here; each case restates one test's objects and expectations by hand.  Only data is written.

  * pkg/scheduler/plugins/nodenumaresource/plugin_test.go:1748-1851 TestRestoreReservation: the reserve pod of
    test-reservation holds cpuset 6-9 (resourceManager.Update, :1773-1777); pod-a holds 6-7, pod-b 8-9
    (:1799-1808).  With pod-a assigned the matched state's remainedCPUs is 8-9 (:1841); with pod-b too it is empty
    and allocatedCPUs is 6-9 (:1846-1850).
  * pkg/scheduler/plugins/deviceshare/reservation_test.go:38-210 Test_Plugin_ReservationRestore: two GPUs (minors
    1, 2; gpu-core 100, gpu-memory 8Gi, gpu-memory-ratio 100); the reserve pod of reservation-1 uses all of minor
    1 (:105-124), allocated-pod-1 (assigned to it) 50 / 4Gi / 50 of minor 1 (:126-143).  The matched state
    (:157-209): allocatable = minor 1 100 / 8Gi / 100, allocated = 50 / 4Gi / 50, remained = 50 / 4Gi / 50, and
    mergedMatchedAllocatable / mergedMatchedAllocated the same two lists.
  * pkg/scheduler/plugins/nodenumaresource/plugin_test.go:1086-1500 TestPlugin_Reserve, its allocate-from-reservation
    cases without a NUMA affinity (:1226-1280): CPU topology buildCPUTopologyForTest(2, 1, 4, 2) -- CPU c in core
    c / 2, NUMA node = socket = c / 8 -- MaxRefCount 1, the matched reservation's remainedCPUs added to the node
    allocation under its UID (:1449-1466; the hand-built restore state holds no merged CPUs, so preferredCPUs =
    remainedCPUs), a 4-CPU pod preferring FullPCPUs, the reservation nominated (:1480):
    Default, remained 4-10 -> 4-7; Restricted, remained 4-10 -> 4-7; Restricted, remained 4-5, with a reservation
    affinity -> Unschedulable "Reservation(s) not enough cpus available to satisfy request".
  * the same test's cases under a pod NUMA policy with a stored affinity (:1268-1398) and its reservation-ignored
    cpuset case (:1399-1433) -- policy_cases / ignored_cases below.
Encoding: cpusets as CPU id lists; device amounts as [gpu-core, gpu-memory, gpu-memory-ratio] of GPU minors;
reserve cases: policy 0 Default / 2 Restricted, want_code 1 (from the reservation) / -1 (Unschedulable).

Run:  python tests/golden/make_restore_state_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GI = 2**30

cases = [
    {"name": "numa_cpuset_one_owner", "source": "pkg/scheduler/plugins/nodenumaresource/plugin_test.go:1748-1841",
     "reserve_cpuset": [6, 7, 8, 9], "owner_cpusets": [[6, 7]],
     "want": {"allocatable_cpus": [6, 7, 8, 9], "allocated_cpus": [6, 7, 8, 9], "remained_cpus": [8, 9]}},
    {"name": "numa_cpuset_two_owners", "source": "pkg/scheduler/plugins/nodenumaresource/plugin_test.go:1843-1850",
     "reserve_cpuset": [6, 7, 8, 9], "owner_cpusets": [[6, 7], [8, 9]],
     "want": {"allocatable_cpus": [6, 7, 8, 9], "allocated_cpus": [6, 7, 8, 9], "remained_cpus": []}},
    {"name": "deviceshare_gpu_half_owned", "source": "pkg/scheduler/plugins/deviceshare/reservation_test.go:38-210",
     "devices": [{"minor": 1, "total": [100, 8 * GI, 100]}, {"minor": 2, "total": [100, 8 * GI, 100]}],
     "reserve_gpu": {"1": [100, 8 * GI, 100]}, "owner_gpu": {"1": [50, 4 * GI, 50]},
     "want": {"gpu_allocatable": {"1": [100, 8 * GI, 100]}, "gpu_allocated": {"1": [50, 4 * GI, 50]},
              "gpu_remained": {"1": [50, 4 * GI, 50]},
              "merged_matched_allocatable": {"1": [100, 8 * GI, 100]},
              "merged_matched_allocated": {"1": [50, 4 * GI, 50]}}},
]

SRC = "pkg/scheduler/plugins/nodenumaresource/plugin_test.go"
reserve_cases = [
    {"name": "reserve_from_reservation_default", "source": f"{SRC}:1226-1242", "topology": [2, 1, 4, 2],
     "remained": [4, 5, 6, 7, 8, 9, 10], "policy": 0, "affinity": False, "num_cpus": 4, "want_code": 1,
     "want_cpus": [4, 5, 6, 7]},
    {"name": "reserve_from_reservation_restricted", "source": f"{SRC}:1243-1259", "topology": [2, 1, 4, 2],
     "remained": [4, 5, 6, 7, 8, 9, 10], "policy": 2, "affinity": False, "num_cpus": 4, "want_code": 1,
     "want_cpus": [4, 5, 6, 7]},
    {"name": "reserve_from_reservation_restricted_fails", "source": f"{SRC}:1260-1277", "topology": [2, 1, 4, 2],
     "remained": [4, 5], "policy": 2, "affinity": True, "num_cpus": 4, "want_code": -1, "want_cpus": []},
]

# TestPlugin_Reserve's allocate-from-reservation cases under the pod's NUMA policy (Restricted) with a stored affinity
# (:1268-1398) and its reservation-ignored case (:1399-1433).  Node: NUMANodeResources cpu = CPUsPerNode per socket
# (no memory key, :1466-1471); the reservation's reserve pod holds remainedCPUs and its `allocatable` NUMA amounts
# (addCPUs + addPodAllocation, :1476-1494).  The hand-built restore state of the test carries no merged lists; the
# holdings model restates it with the owners holding allocatable - remained (none where the test gives no remained) --
# the amounts Reserve reads are the same.  Encoding: numa maps {id: cpu milli}; bind = requestCPUBind (a 4-CPU LSR
# pod preferring FullPCPUs) else a LS pod; affinity_mask = the stored NUMANodeAffinity; required = the reservation
# affinity; want_code 1 / 0 (from the node) / -1 (Unschedulable); want_numa {id: cpu milli}.
policy_cases = [
    {"name": "numa_cpuset_restricted", "source": f"{SRC}:1268-1297", "topology": [2, 1, 8, 2], "bind": True,
     "remained_cpus": [4, 5, 6, 7, 8, 9, 10], "allocatable": {"0": 7000}, "remained": None, "policy": 2,
     "required": True, "affinity_mask": 1, "want_code": 1, "want_cpus": [4, 5, 6, 7], "want_numa": {"0": 4000}},
    {"name": "numa_cpuset_restricted_fails", "source": f"{SRC}:1299-1330", "topology": [2, 1, 4, 2], "bind": True,
     "remained_cpus": [4, 5], "allocatable": {"0": 2000}, "remained": {"0": 2000}, "policy": 2,
     "required": True, "affinity_mask": 1, "want_code": -1, "want_cpus": [], "want_numa": {}},
    {"name": "numa_restricted", "source": f"{SRC}:1331-1364", "topology": [2, 1, 4, 2], "bind": False,
     "remained_cpus": [], "allocatable": {"1": 7000}, "remained": {"1": 7000}, "policy": 2,
     "required": True, "affinity_mask": 2, "want_code": 1, "want_cpus": [], "want_numa": {"1": 4000}},
    {"name": "numa_restricted_fails", "source": f"{SRC}:1366-1397", "topology": [2, 1, 4, 2], "bind": False,
     "remained_cpus": [], "allocatable": {"0": 2000}, "remained": {"0": 2000}, "policy": 2,
     "required": True, "affinity_mask": 1, "want_code": -1, "want_cpus": [], "want_numa": {}},
]
ignored_cases = [
    {"name": "ignored_pod_cpuset", "source": f"{SRC}:1399-1433", "topology": [2, 1, 4, 2],
     "remained_cpus": [4, 5, 6, 7, 8, 9, 10], "num_cpus": 4, "want_code": 1, "want_cpus": [4, 5, 6, 7]},
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "reservation_restore.json"), "w") as f:
        json.dump({"cases": cases, "reserve_cases": reserve_cases, "policy_cases": policy_cases,
                   "ignored_cases": ignored_cases}, f, indent=1)
    print(f"wrote {len(cases)} cases")
