"""Transcription of the reference's Test_filterWithReservations cases that read a reservation's allocatable beyond
cpu / memory (the "pods" cap, the node-reservation annotation's reserved part, batch scalar requests) into
tests/golden/reservation_filters_general.json.  Same rules as make_fixtures.py: the Go tests cannot run here; each
case restates one test's objects and expectations by hand.  Only data is written.

  * pkg/scheduler/plugins/reservation/plugin_test.go:788-872: testRInfo is a Restricted reservation with
    status.allocatable cpu 7 / pods 2, the annotation node-reservation {"resources": {"cpu": "1"}} (rInfo.Reserved,
    reservation_info.go:88) and two assigned pods of 1 cpu each (allocated cpu 2, two allocated pods); the node has
    allocatable cpu 32 / memory 32Gi / pods 100 / kubernetes.io/batch-cpu 7500 / kubernetes.io/batch-memory 10Gi.
  * the cases (the test writes the cycle state by hand: podRequested, rAllocated, hasAffinity):
      :973-1018    Restricted cpu 6, 6C8Gi pod, no affinity -> filterWithReservations is not required: Success
      :1066-1116  Restricted cpu 6, batch-cpu 6000 / batch-memory 8Gi pod, affinity, podRequested 30C/24Gi with
                  batch 1500 / 2Gi, rAllocated 6C -> the masked requests are zero, the node fits: Success
      :1164-1189  testRInfo, 3C pod, affinity, rAllocated 2C -> "Reservation(s) Too many pods"
      :1190-1241  Restricted cpu 6, batch-cpu 8000 / batch-memory 8Gi pod, affinity, rAllocated 2C ->
                  "Insufficient kubernetes.io/batch-cpu by node" (8000 > 7500 - 1500)
      :1242-1292  the same pod without an affinity -> not required: Success
      :1293-1342  Restricted cpu 6 with node-reservation cpu 2, 6C8Gi pod, affinity -> "Reservation(s) Insufficient
                  cpu" (6 > 6 - 2)
Encoding: cpu in milli, memory in bytes; scalar names by resource id (batch-cpu 2, batch-memory 3); `want`: 0
Success, 1 a node insufficiency, 2 a reservation reason (or_rsv_filter_with).

Run:  python tests/golden/make_rsv_general_fixtures.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GI = 2**30
PT = "pkg/scheduler/plugins/reservation/plugin_test.go"
BATCH_CPU, BATCH_MEM = 2, 3
NODE = {"allocatable": [32000, 32 * GI], "allowed_pods": 100,
        "scalars": {str(BATCH_CPU): 7500, str(BATCH_MEM): 10 * GI}}
R6 = {"policy": 2, "allocatable": [6000, 0], "allocated": [0, 0], "reserved": [0, 0], "allocated_pods": 0,
      "entries": []}
TEST_R = {"policy": 2, "allocatable": [7000, 0], "allocated": [2000, 0], "reserved": [1000, 0], "allocated_pods": 2,
          "entries": [{"id": -1, "allocatable": 2, "allocated": 0, "reserved": 0}]}
R6_RESERVED = dict(R6, reserved=[2000, 0])
PR_30 = {"0": 30000, "1": 24 * GI}
PR_30_BATCH = dict(PR_30, **{str(2 + BATCH_CPU): 1500, str(2 + BATCH_MEM): 2 * GI})


def case(name, lines, r, pod, scalars, pr, ra, affinity, want):
    return {"name": name, "source": f"{PT}:{lines}", "node": NODE, "reservation": r,
            "pod": {"requests": pod, "scalars": scalars}, "pod_requested": pr, "r_allocated": ra,
            "required": affinity, "affinity": affinity, "want": want}


cases = [
    case("restricted_no_affinity_not_required", "973-1018", R6, [6000, 8 * GI], {}, PR_30, {"0": 0}, False, 0),
    case("restricted_matched_requests_zero_with_affinity", "1066-1116", R6, [0, 0],
         {str(BATCH_CPU): 6000, str(BATCH_MEM): 8 * GI}, PR_30_BATCH, {"0": 6000}, True, 0),
    case("restricted_exceeding_max_pods", "1164-1189", TEST_R, [3000, 0], {}, PR_30, {"0": 2000}, True, 2),
    case("restricted_unmatched_scalar_insufficient_by_node", "1190-1241", R6, [0, 0],
         {str(BATCH_CPU): 8000, str(BATCH_MEM): 8 * GI}, PR_30_BATCH, {"0": 2000}, True, 1),
    case("restricted_scalars_without_affinity_not_required", "1242-1292", R6, [0, 0],
         {str(BATCH_CPU): 8000, str(BATCH_MEM): 8 * GI}, PR_30_BATCH, {"0": 6000}, False, 0),
    case("restricted_insufficient_due_to_reserved", "1293-1342", R6_RESERVED, [6000, 8 * GI], {}, PR_30, {"0": 0},
         True, 2),
]

if __name__ == "__main__":
    with open(os.path.join(HERE, "reservation_filters_general.json"), "w") as f:
        json.dump({"source": "make_rsv_general_fixtures.py", "cases": cases}, f, indent=1)
