"""Transcription of the reference's reservation restore test into
tests/golden/reservations.json.  Same rules as make_fixtures.py: the Go tests cannot run here; each case
restates one test's objects and expectations by hand.  Only data is written.

  * pkg/scheduler/plugins/reservation/transformer_test.go:40-368 TestRestoreReservation: a 32C/64Gi node with
    pod-1 (4C8Gi), pod-2 (8C16Gi), the reserve pods of reservation12C24G (AllocateOnce false, one assigned pod
    4C8Gi) and reservation8C16G (no assigned pod), and the assigned pod 4C8Gi: NodeInfo.Requested 36C/72Gi
    (:285-289).  BeforePreFilter of a pod that matches only reservation8C16G records the node's requested after
    the unmatched restore, podRequested = 32C/64Gi (:330-333) -- what every pod matching no reservation sees:
    restoreUnmatchedReservations (transformer.go:447-473) swaps the 12C24G reserve pod for an 8C16Gi one.

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

if __name__ == "__main__":
    with open(os.path.join(HERE, "reservations.json"), "w") as f:
        json.dump({"source": "make_reservation_fixtures.py", "cases": cases}, f, indent=1)
    print(len(cases), "cases")
