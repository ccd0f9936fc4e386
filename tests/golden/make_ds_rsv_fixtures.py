"""Transcription of the reference's DeviceShare allocate-from-reservation tests into
tests/golden/ds_reservation.json.  Same rules as make_fixtures.py: the Go tests cannot run here; each case restates one
test's objects and expectations by hand.  Only data is written.

  * pkg/scheduler/plugins/deviceshare/reservation_test.go:225-888 Test_tryAllocateFromReservation: two healthy GPUs
    (minors 0, 1: gpu-core 100, gpu-memory-ratio 100, gpu-memory 8Gi), the node's deviceUsed per case, a pod requesting
    gpu-core 50 / gpu-memory 4Gi per GPU (or 60 / 5Gi, 30 / 1Gi), the restore state written by hand (matched
    reservations with allocatable / allocated / remained, mergedUnmatchedUsed, mergedMatchedAllocatable,
    mergedMatchedAllocated), no scorer; the result's minors or the status.
  * pkg/scheduler/plugins/deviceshare/scoring_test.go:670-1240 TestScoreReservation: one GPU (minor 0: 100 / 100 /
    16Gi) and one RDMA device (100); the reservation's reserve pod is added to the cache (updatePod), so the GPU's used
    is the case's deviceUsed plus the reservation's allocation; RestoreReservation gives allocatable = remained = that
    allocation (no owners); the node's preemptibleDevices join basicPreemptible; Least / MostAllocated;
    ScoreReservation's value (and NormalizeReservationScore 95 -> 100 for the one list).
  * pkg/scheduler/plugins/deviceshare/plugin_test.go:2681-2800 Test_Plugin_FilterNominateReservation: GPUs 1, 2
    (100 / 8Gi / 100); reservation-1's reserve pod holds GPU 1 whole: FilterNominateReservation (tryAllocateFromReservation
    over it alone, required) of a koordinator.sh/gpu 100 pod succeeds; after allocated-pod-1 (assigned to it) takes
    GPUs 1 and 2, the owners' part on the reservation's GPU is all of it, nothing remains: "Reservation(s) Insufficient
    gpu devices".
Encoding: a deviceResources map as {"gpu": {minor: [core, memory, ratio] or null per absent key}, "rdma": {minor: v}};
pod device requests by KE_PDR name; want_code 0 success (want_minors), 1 nil result, 2 Unschedulable (want_reason
"rsv" = Reservation(s) ..., "gpu" = Insufficient gpu devices).

Run:  python tests/golden/make_ds_rsv_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GI = 2**30
RT = "pkg/scheduler/plugins/deviceshare/reservation_test.go"
ST = "pkg/scheduler/plugins/deviceshare/scoring_test.go"
PT = "pkg/scheduler/plugins/deviceshare/plugin_test.go"
DEFAULT, ALIGNED, RESTRICTED = 0, 1, 2


def g(core, mem, ratio):
    return [core, mem, ratio]


ONE = {"gpu": {"0": g(100, 8 * GI, 100), "1": g(100, 8 * GI, 100)}}
HALF = {"gpu": {"0": g(50, 4 * GI, 50)}}
P75 = {"gpu": {"0": g(75, 6 * GI, 75)}}
P25 = {"gpu": {"0": g(25, 2 * GI, 25)}}
P25_1 = {"gpu": {"0": g(25, 2 * GI, 25), "1": g(100, 8 * GI, 100)}}
EMPTY = {}
HALF_POD = {"gpu_core": 50, "gpu_memory": 4 * GI}

try_devices = {"gpu": {"0": g(100, 8 * GI, 100), "1": g(100, 8 * GI, 100)}}


def tcase(name, lines, pod, matched, used, m_alloc, m_allocd, required=False, ignored=False, want_code=0,
          want_minors=None, want_reason=None):
    return {"name": name, "source": f"{RT}:{lines}", "devices": try_devices, "used": used, "pod": pod,
            "matched": matched, "basic": EMPTY, "matched_allocatable": m_alloc, "matched_allocated": m_allocd,
            "required": required, "ignored": ignored, "want_code": want_code, "want_minors": want_minors,
            "want_reason": want_reason}


def m(policy, allocatable, allocated, remained):
    return {"policy": policy, "allocatable": allocatable, "allocated": allocated, "remained": remained}


try_cases = [
    tcase("no_matched_reservations", "345-357", HALF_POD, [], EMPTY, EMPTY, EMPTY, want_code=1),
    tcase("default_policy", "358-390", HALF_POD, [m(DEFAULT, P25, EMPTY, P25)], EMPTY, P25, EMPTY,
          want_minors={"gpu": [0]}),
    tcase("default_policy_required", "391-434", HALF_POD, [m(DEFAULT, HALF, P25, HALF)],
          {"gpu": {"0": g(50, 4 * GI, 50)}}, HALF, P25, required=True, want_minors={"gpu": [0]}),
    tcase("default_policy_required_reservation_empty", "435-478", HALF_POD, [m(DEFAULT, HALF, HALF, EMPTY)],
          {"gpu": {"0": g(150, 12 * GI, 150)}}, HALF, HALF, required=True, want_minors={"gpu": [1]}),
    tcase("aligned_policy", "479-524", HALF_POD, [m(ALIGNED, HALF, EMPTY, HALF)],
          {"gpu": {"0": g(100, 8 * GI, 100), "1": g(100, 8 * GI, 100)}}, HALF, EMPTY, want_minors={"gpu": [0]}),
    tcase("aligned_bigger_request_no_node_remaining", "525-565", {"gpu_core": 60, "gpu_memory": 5 * GI},
          [m(ALIGNED, HALF, EMPTY, HALF)], {"gpu": {"0": g(100, 8 * GI, 100), "1": g(100, 8 * GI, 100)}}, HALF, EMPTY,
          required=True, want_code=2, want_reason="rsv"),
    tcase("aligned_remaining_too_little", "566-608", {"gpu_core": 30, "gpu_memory": 1 * GI},
          [m(ALIGNED, HALF, P25, P25)], {"gpu": {"0": g(125, 10 * GI, 125), "1": g(100, 8 * GI, 100)}}, HALF, P25,
          required=True, want_code=2, want_reason="rsv"),
    tcase("restricted_policy", "609-654", HALF_POD, [m(RESTRICTED, HALF, EMPTY, HALF)],
          {"gpu": {"0": g(100, 8 * GI, 100), "1": g(100, 8 * GI, 100)}}, HALF, EMPTY, want_minors={"gpu": [0]}),
    tcase("restricted_node_remains_reservation_not", "655-692", HALF_POD, [m(RESTRICTED, HALF, P25, P25)],
          {"gpu": {"0": g(75, 6 * GI, 75), "1": g(100, 8 * GI, 100)}}, HALF, P25, required=True, want_code=2,
          want_reason="rsv"),
    tcase("restricted_with_ignored_pods", "693-738", HALF_POD, [m(RESTRICTED, ONE, EMPTY, ONE)],
          {"gpu": {"0": g(175, 14 * GI, 175), "1": g(150, 12 * GI, 150)}}, HALF, EMPTY, want_minors={"gpu": [1]}),
    tcase("reservation_ignored_pod", "739-793", HALF_POD, [m(RESTRICTED, ONE, P75, P25_1)],
          {"gpu": {"0": g(175, 14 * GI, 175), "1": g(100, 8 * GI, 100)}}, ONE, P75, ignored=True,
          want_minors={"gpu": [1]}),
    tcase("reservation_ignored_pod_fails", "794-837", HALF_POD, [m(RESTRICTED, ONE, ONE, EMPTY)],
          {"gpu": {"0": g(200, 16 * GI, 200), "1": g(200, 16 * GI, 200)}}, ONE, ONE, ignored=True, want_code=2,
          want_reason="gpu"),
]

score_devices = {"gpu": {"0": g(100, 16 * GI, 100)}, "rdma": {"0": 100}}
U25 = {"0": g(25, 4 * GI, 25)}


def scase(name, lines, pod, reserved, policy, used, strategy="least", basic=EMPTY, want=0, want_normalize=None):
    # the reserve pod's allocation is added to the cache's used (updatePod)
    u = {"gpu": dict(used.get("gpu", {}))}
    for mi, v in reserved["gpu"].items():
        old = u["gpu"].get(mi)
        u["gpu"][mi] = v if old is None else [a + b for a, b in zip(old, v)]
    return {"name": name, "source": f"{ST}:{lines}", "devices": score_devices, "used": u, "pod": pod,
            "matched": [m(policy, reserved, EMPTY, reserved)], "basic": basic, "matched_allocatable": reserved,
            "matched_allocated": EMPTY, "strategy": strategy, "want_score": want, "want_normalize": want_normalize}


R50_12 = {"gpu": {"0": g(50, 12 * GI, 50)}}
R50_8 = {"gpu": {"0": g(50, 8 * GI, 50)}}
R75_12 = {"gpu": {"0": g(75, 12 * GI, 75)}}
POD_RATIO = {"gpu_core": 50, "gpu_memory_ratio": 50}
POD_MEM = {"gpu_core": 50, "gpu_memory": 8 * GI}
PRE25 = {"gpu": U25}
score_cases = [
    scase("default_1", "738-768", POD_RATIO, R50_12, DEFAULT, {"gpu": U25}, want=50),
    scase("default_2", "769-799", POD_MEM, R50_12, DEFAULT, {"gpu": U25}, want=50),
    scase("default_most_1", "800-831", POD_RATIO, R50_8, DEFAULT, {"gpu": U25}, "most", want=50),
    scase("default_most_2", "832-863", POD_MEM, R50_8, DEFAULT, {"gpu": U25}, "most", want=50),
    scase("aligned_least", "864-898", POD_RATIO, R50_8, ALIGNED, {"gpu": U25}, "least", want=50),
    scase("aligned_most", "899-933", POD_RATIO, R50_8, ALIGNED, {"gpu": U25}, "most", want=50),
    scase("restricted_least", "934-968", POD_RATIO, R50_8, RESTRICTED, {}, "least", want=25),
    scase("restricted_most", "969-1003", POD_RATIO, R50_8, RESTRICTED, {}, "most", want=75),
    scase("aligned_preemptible", "1004-1048", POD_RATIO, R75_12, ALIGNED, {"gpu": U25}, basic=PRE25, want=75),
    scase("aligned_preemptible_2", "1049-1101", POD_RATIO, R75_12, ALIGNED, {"gpu": U25}, basic=PRE25, want=75),
    scase("restricted_multi_resources_most", "1102-1160", dict(POD_RATIO, rdma=20), R50_8, RESTRICTED,
          {"gpu": {"0": g(50, 8 * GI, 50)}}, "most", want=95, want_normalize=100),
]

nominate_devices = {"gpu": {"1": g(100, 8 * GI, 100), "2": g(100, 8 * GI, 100)}}
R1 = {"gpu": {"1": g(100, 8 * GI, 100)}}
nominate_cases = [
    {"name": "filter_nominate_reservation_fits", "source": f"{PT}:2681-2771", "devices": nominate_devices,
     "used": R1, "pod": {"koord_gpu": 100}, "matched": [m(DEFAULT, R1, EMPTY, R1)], "basic": EMPTY,
     "matched_allocatable": R1, "matched_allocated": EMPTY, "required": True, "ignored": False, "want_code": 0,
     "want_minors": {"gpu": [1]}, "want_reason": None},
    {"name": "filter_nominate_reservation_owned_out", "source": f"{PT}:2772-2800", "devices": nominate_devices,
     "used": {"gpu": {"1": g(200, 16 * GI, 200), "2": g(100, 8 * GI, 100)}}, "pod": {"koord_gpu": 100},
     "matched": [m(DEFAULT, R1, R1, EMPTY)], "basic": EMPTY, "matched_allocatable": R1, "matched_allocated": R1,
     "required": True, "ignored": False, "want_code": 2, "want_minors": None, "want_reason": "rsv"},
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "ds_reservation.json"), "w") as f:
        json.dump({"source": "make_ds_rsv_fixtures.py",
                   "cases": {"try": try_cases + nominate_cases, "score": score_cases}}, f,
                  indent=1)
