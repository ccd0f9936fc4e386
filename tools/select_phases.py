"""k_select anatomy: shader cycles per wave of each phase of the top-k selection, from the diagnostic build
(make -C koordinator_amd/csrc prof -> libkoordeval_prof.so, -DKE_PROF_REPLAY), on the C3 queue.

usage: KOORDEVAL_LIB=koordinator_amd/libkoordeval_prof.so python tools/select_phases.py [--pipeline 0|1]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, synth  # noqa: E402

PHASES = ["prologue_pass1_loads", "pass1_reduce", "pass2_histogram", "pass3_select", "sort_count",
          "drain_parts_done", "merge_publish"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=12_800)
    ap.add_argument("--pipeline", type=int, default=1)
    a = ap.parse_args()
    cl = synth.make_cluster(a.nodes, synth.BASE_SEED + 3)
    pods = synth.make_pods(a.pods, synth.BASE_SEED + 103)
    ev = Evaluator(synth.config(a.nodes))
    synth.load_into(ev, cl)
    ev.lib.ke_set_pipeline(ev.h, int(a.pipeline))
    ev.eval(pods[:0], synth.T0)
    cyc = np.zeros(8)
    ev.lib.ke_debug_kernel_phases(ev.h, 3, cyc.ctypes.data_as(C.c_void_p))  # reset
    ev.schedule(pods, synth.T0)
    ev.lib.ke_debug_kernel_phases(ev.h, 3, cyc.ctypes.data_as(C.c_void_p))
    ks = ev.kernel_stats()
    out = {"lib": os.environ.get("KOORDEVAL_LIB"), "pipeline": a.pipeline, "waves": int(cyc[7]),
           "cycles_per_wave": dict(zip(PHASES, cyc[:7].round(1).tolist())), "total": float(cyc[:7].sum()),
           "select_ms_per_batch": ks.get("select_ms"), "eval_ms_per_batch": ks.get("eval_ms")}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
