"""Replay anatomy: shader cycles per pod of each phase of k_resolve's sequential replay, from the
diagnostic build (make -C koordinator_amd/csrc prof -> libkoordeval_prof.so, -DKE_PROF_REPLAY).

usage: KOORDEVAL_LIB=koordinator_amd/libkoordeval_prof.so python tools/replay_phases.py [--nodes N --pods P]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, synth  # noqa: E402

PHASES = ["best_unchanged", "row_fetch_issue", "re_evaluation", "re_eval_max", "decision_adopt", "reserve",
          "next_changed_flags"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=5_000)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--ds", type=float, default=0.0, help="C5 shape: DeviceShare pods (this fraction) on 8 GPU + 2 RDMA nodes")
    a = ap.parse_args()
    cl = synth.make_cluster(a.nodes, synth.BASE_SEED + a.config)
    pods = synth.make_pods(a.pods, synth.BASE_SEED + 100 + a.config)
    ev = Evaluator(synth.config(a.nodes))
    synth.load_into(ev, cl)
    if a.ds > 0:
        pods = synth.make_ds_pods(a.pods, synth.BASE_SEED + 105, device_fraction=a.ds)
        synth.load_devices(ev, synth.make_devices(a.nodes, synth.BASE_SEED + 55))
    ev.eval(pods[:0], synth.T0)
    cyc = np.zeros(8)
    ev.lib.ke_debug_replay_phases(ev.h, cyc.ctypes.data_as(C.c_void_p))  # reset
    ev.schedule(pods, synth.T0)
    ev.lib.ke_debug_replay_phases(ev.h, cyc.ctypes.data_as(C.c_void_p))
    ks = ev.kernel_stats()
    out = {"lib": os.environ.get("KOORDEVAL_LIB"), "nodes": a.nodes, "pods": int(cyc[7]),
           "cycles_per_pod": dict(zip(PHASES, cyc[:7].round(1).tolist())), "total_cycles_per_pod": float(cyc[:7].sum()),
           "resolve_replay_ms_per_batch": ks["resolve_replay_ms"], "rows_changed_per_batch": ks["rows_changed"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
