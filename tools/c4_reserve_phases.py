"""Anatomy of k_cpuset_reserve on the C4 workload: shader cycles per pod of each phase, from the diagnostic
build (make -C koordinator_amd/csrc prof -> libkoordeval_prof.so, -DKE_PROF_REPLAY).

usage: KOORDEVAL_LIB=koordinator_amd/libkoordeval_prof.so python tools/c4_reserve_phases.py [--nodes N --pods P]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, synth  # noqa: E402

PHASES = ["select_admit", "cs_old", "cpuset_allocate", "row_record", "commit", "numa_reserve", "ds_out"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=256)
    a = ap.parse_args()
    cl, zones, tables = synth.make_c4_cluster(a.nodes, synth.BASE_SEED + 4)
    pods = synth.make_c4_pods(a.pods, synth.BASE_SEED + 104)
    ev = Evaluator(synth.config(a.nodes))
    synth.load_into(ev, cl)
    synth.load_numa(ev, zones)
    synth.load_cpus(ev, tables)
    ev.eval(pods[:0], synth.T0)
    cyc = np.zeros(8)
    ev.lib.ke_debug_kernel_phases(ev.h, 2, cyc.ctypes.data_as(C.c_void_p))  # reset
    ev.schedule(pods, synth.T0)
    ev.lib.ke_debug_kernel_phases(ev.h, 2, cyc.ctypes.data_as(C.c_void_p))
    print(json.dumps({"pods": int(cyc[7]), "cycles_per_pod": dict(zip(PHASES, cyc[:7].round(1).tolist())),
                      "total_cycles_per_pod": float(cyc[:7].sum())}))


if __name__ == "__main__":
    main()
