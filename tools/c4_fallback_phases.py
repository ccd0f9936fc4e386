"""Anatomy of k_numa_fallback on the C4 workload: shader cycles per deferred pair of the first listing step
(one- and two-zone hints + search), the later steps, and the BestEffort merge, from the diagnostic build
(make -C koordinator_amd/csrc prof).  usage: KOORDEVAL_LIB=koordinator_amd/libkoordeval_prof.so python
tools/c4_fallback_phases.py"""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, synth  # noqa: E402

N, P = 50_000, 128
cl, zones, tables = synth.make_c4_cluster(N, synth.BASE_SEED + 4)
pods = synth.make_c4_pods(P, synth.BASE_SEED + 104)
ev = Evaluator(synth.config(N))
synth.load_into(ev, cl)
synth.load_numa(ev, zones)
synth.load_cpus(ev, tables)
ev.eval(pods[:0], synth.T0)
cyc = np.zeros(8)
ev.lib.ke_debug_kernel_phases(ev.h, 1, cyc.ctypes.data_as(C.c_void_p))
ev.schedule(pods, synth.T0)
ev.lib.ke_debug_kernel_phases(ev.h, 1, cyc.ctypes.data_as(C.c_void_p))
print(json.dumps({"units": int(cyc[7]), "cycles_per_unit": dict(zip(["step0_search", "later_steps", "best_effort_merge", "setup", "step0_list", "-", "-"],
                                                                  cyc[:7].round(1).tolist()))}))
