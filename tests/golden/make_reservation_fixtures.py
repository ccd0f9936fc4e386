"""Transcription of the reference's reservation restore test into
tests/golden/reservations.json.  Same rules as make_fixtures.py: the Go tests cannot run here; each case
restates one test's objects and expectations by hand.  Only data is written.

  * pkg/scheduler/plugins/reservation/transformer_test.go:40-368 TestRestoreReservation: a 32C/64Gi node with
    pod-1 (4C8Gi), pod-2 (8C16Gi), the reserve pods of reservation12C24G (AllocateOnce false, one assigned pod
    4C8Gi) and reservation8C16G (no assigned pod), and the assigned pod 4C8Gi: NodeInfo.Requested 36C/72Gi
    (:285-289).  BeforePreFilter of a pod that matches only reservation8C16G records the node's requested after
    the unmatched restore, podRequested = 32C/64Gi (:330-333) -- what every pod matching no reservation sees:
    restoreUnmatchedReservations (transformer.go:447-473) swaps the 12C24G reserve pod for an 8C16Gi one.

  * pkg/scheduler/plugins/reservation/scoring_test.go:40-284 TestScore: one 16C/128Gi node, the pod's matched
    reservations reservation4C8G / reservation2C4G (optionally with allocated resources); PreScore + Score
    (before NormalizeScore): no reservation 0, a zero-request pod 0 (no shared resource name: not nominated), 2C4Gi
    into 4C8G 50, into a 2C4G holding 2C3Gi 0, both reservations 100 (the better ScoreReservation is nominated).
  * scoring_test.go:286-461 TestScoreWithOrder: four nodes without allocatable, a 4C8G reservation on each, the
    one on test-node-4 labelled reservation-order 123456; a 4C8Gi pod: test-node-4 is preferredNode and scores
    mostPreferredScore 1000, the others MaxNodeScore.
  * nominator_test.go:40-356 TestNominateReservation on a node without allocatable: no reservation -> nil, the
    reservation-order label wins (100), an allocated-out 2C4G loses to 4C8G, 2C4G (score 100) beats 4C8G (50).
  * plugin_test.go:788-1342 Test_filterWithReservations (cpu / memory cases; a 32C/32Gi node whose NodeInfo after
    the unmatched restore -- podRequested -- is 30C/24Gi or 32C/24Gi, one matched 6C reservation, a reservation
    affinity): Aligned 8C8Gi fits (8 <= 32 - (30 - 6)), not at 32C; Restricted 6C8Gi fits, 8C8Gi exceeds the
    reservation's 6C.
  The tests write the cycle state by hand (no restore ran): NodeInfo holds no reserve pods and fitsNode's
  podRequested / rAllocated are empty, so the cases' nodes have requested 0; nodes are indexed in test order.

Run:  python tests/golden/make_reservation_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GI = 2**30
SRC = "pkg/scheduler/plugins/reservation/transformer_test.go"

cases = [{
    "name": "restore_unmatched_reservation",
    "source": f"{SRC}:40-368",
    "node": {"allocatable": [32000, 64 * GI], "requested": [36000, 72 * GI]},
    "reservations": [
        {"name": "reservation12C24G", "available": True, "allocate_once": False, "allocated_pods": 1,
         "allocatable": [12000, 24 * GI], "allocated": [4000, 8 * GI]},
        {"name": "reservation8C16G", "available": True, "allocate_once": False, "allocated_pods": 0,
         "allocatable": [8000, 16 * GI], "allocated": [0, 0]},
    ],
    "want_requested": [32000, 64 * GI],
}]

SC = "pkg/scheduler/plugins/reservation/scoring_test.go"
R4C8G = {"allocatable": [4000, 8 * GI], "allocated": [0, 0], "order": 0}
R2C4G = {"allocatable": [2000, 4 * GI], "allocated": [0, 0], "order": 0}


def score_case(name, lines, pod, resv, want, nodes=1, alloc=(16000, 128 * GI), nominated=None, src=SC):
    """resv: [(node, reservation)]; want: the Score of each node (None: not asserted); nominated: per node the
    index of the reservation NominateReservation returns, -1 = nil (None: not asserted)"""
    requested = [[0, 0] for _ in range(nodes)]  # the tests build the state by hand: no reserve pods in NodeInfo
    return {"name": name, "source": f"{src}:{lines}", "nodes": [{"allocatable": list(alloc), "requested": q}
                                                               for q in requested],
            "reservations": [dict(r, node=n) for n, r in resv], "pod": pod, "want_score": want,
            "want_nominated": nominated}


score_cases = [
    score_case("no_reservation_matched", "136-139", [0, 0], [], [0]),
    score_case("matched_zero_request_pod", "140-148", [0, 0], [(0, R2C4G)], [0]),
    score_case("matched_4c8g_pod_2c4g", "149-172", [2000, 4 * GI], [(0, R4C8G)], [50]),
    score_case("allocated_2c4g_pod_2c4g", "173-202", [2000, 4 * GI],
               [(0, dict(R2C4G, allocated=[2000, 3 * GI]))], [0]),
    score_case("multi_matched_pod_2c4g", "203-226", [2000, 4 * GI], [(0, R4C8G), (0, R2C4G)], [100]),
    score_case("preferred_by_order", "286-461", [4000, 8 * GI],
               [(0, R4C8G), (1, R4C8G), (2, R4C8G), (3, dict(R4C8G, order=123456))], [100, 100, 100, 1000],
               nodes=4, alloc=(0, 0)),
]
NM = "pkg/scheduler/plugins/reservation/nominator_test.go"
# TestNominateReservation (nominator_test.go:40-356): a node without allocatable; NominateReservation's choice.
# The "preferred reservation" pair is not Available: ReservationRequests falls back to the template (2C4Gi).
score_cases += [
    score_case("nominate_node_without_reservations", "121-125", [0, 0], [], None, alloc=(0, 0), nominated=[-1], src=NM),
    score_case("nominate_preferred_reservation", "126-226", [2000, 4 * GI],
               [(0, dict(R2C4G, order=100)), (0, R2C4G)], None, alloc=(0, 0), nominated=[0], src=NM),
    score_case("nominate_allocated_reservation", "227-252", [2000, 4 * GI],
               [(0, R4C8G), (0, dict(R2C4G, allocated=[2000, 4 * GI]))], None, alloc=(0, 0), nominated=[0], src=NM),
    score_case("nominate_matched_reservations", "253-275", [2000, 4 * GI], [(0, R4C8G), (0, R2C4G)], None,
               alloc=(0, 0), nominated=[1], src=NM),
]

PT = "pkg/scheduler/plugins/reservation/plugin_test.go"
ALIGNED, RESTRICTED = 1, 2
filter_cases = [
    {"name": n, "source": f"{PT}:{l}", "node": {"allocatable": [32000, 32 * GI], "requested": [req, 24 * GI]},
     "reservation": {"allocatable": [6000, 0], "allocated": [0, 0], "allocate_policy": pol}, "pod": pod, "want": w}
    for n, l, req, pol, pod, w in (
        ("aligned_fits_node", "878-924", 30000, ALIGNED, [8000, 8 * GI], True),
        ("aligned_insufficient_cpu_by_node", "925-971", 32000, ALIGNED, [8000, 8 * GI], False),
        ("restricted_with_affinity_fits", "1019-1065", 30000, RESTRICTED, [6000, 8 * GI], True),
        ("restricted_insufficient_cpu", "1117-1163", 30000, RESTRICTED, [8000, 8 * GI], False))]

if __name__ == "__main__":
    with open(os.path.join(HERE, "reservation_filters.json"), "w") as f:
        json.dump({"source": "make_reservation_fixtures.py", "cases": filter_cases}, f, indent=1)
    with open(os.path.join(HERE, "reservation_scores.json"), "w") as f:
        json.dump({"source": "make_reservation_fixtures.py", "cases": score_cases}, f, indent=1)
    with open(os.path.join(HERE, "reservations.json"), "w") as f:
        json.dump({"source": "make_reservation_fixtures.py", "cases": cases}, f, indent=1)
    print(len(cases), "cases")
