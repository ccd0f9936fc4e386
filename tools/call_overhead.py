"""Where the per-call time of the bench workload goes: the ke_schedule call's wall time (Python clock around the
ctypes call) against the library's own host phases (ke_last_host_stats) and the device window, and the Python time
between calls.  Usage: python tools/call_overhead.py [--steps K] [--pods-per-call P]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--pods-per-call", type=int, default=5000)
    ap.add_argument("--stats", action="store_true", help="the bench loop's per-call statistics calls too")
    a = ap.parse_args()
    N = 50000
    cl = synth.make_cluster(N, synth.BASE_SEED + 3)
    pods = synth.make_pods(a.steps * a.pods_per_call, synth.BASE_SEED + 103)
    ev = Evaluator(synth.config(N, pod_batch=64))
    synth.load_into(ev, cl)
    ev.eval(pods[:0], synth.T0)
    ev.set_profiling(0)
    ev.schedule(pods[:a.pods_per_call], synth.T0)  # warm the call path (its pods are scheduled again below)
    ev.close()
    ev = Evaluator(synth.config(N, pod_batch=64))
    synth.load_into(ev, cl)
    ev.eval(pods[:0], synth.T0)
    ev.set_profiling(0)
    call, between, host = [], [], []
    t_end = time.perf_counter()
    t0 = t_end
    for s in range(a.steps):
        t1 = time.perf_counter()
        between.append(t1 - t_end)
        ev.schedule(pods[s * a.pods_per_call:(s + 1) * a.pods_per_call], synth.T0)
        t2 = time.perf_counter()
        call.append(t2 - t1)
        host.append(ev.host_stats())
        if a.stats:
            ev.stats()
            ev.pod_latencies(a.pods_per_call)
            ev.kernel_stats()
        t_end = time.perf_counter()
    total = time.perf_counter() - t0
    hs = {k: float(np.mean([h[k] for h in host])) for k in host[0]}
    out = {"ms_per_step": total / a.steps * 1e3, "call_ms": float(np.mean(call)) * 1e3,
           "between_calls_ms": float(np.mean(between)) * 1e3, "host_phases_ms": hs,
           "host_phases_sum_ms": sum(hs.values()),
           "unaccounted_in_call_ms": float(np.mean(call)) * 1e3 - sum(hs.values())}
    print(json.dumps(out))
    ev.close()


if __name__ == "__main__":
    main()
