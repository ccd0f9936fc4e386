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
Encoding: cpusets as CPU id lists; device amounts as [gpu-core, gpu-memory, gpu-memory-ratio] of GPU minors.

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

if __name__ == "__main__":
    with open(os.path.join(HERE, "reservation_restore.json"), "w") as f:
        json.dump({"cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} cases")
