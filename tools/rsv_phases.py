"""Fixed costs of the reservation-matched path (tools/rsv_bench.py's workload): the wall time of one ke_schedule
call of 30 plain pods, of one matched pod, and of the two in one call, with the library's host phases.
Usage: python tools/rsv_phases.py [--reps 40]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, abi, synth  # noqa: E402
from tools.rsv_bench import reservations  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    N = 50_000
    cl = synth.make_cluster(N, synth.BASE_SEED + 3)
    rs = reservations(cl, 0.1, synth.BASE_SEED + 61)
    groups = np.arange(len(rs)) // 25
    pods = synth.make_pods(a.reps * 31 * 5 + 31, synth.BASE_SEED + 62)
    cpuset = np.isin(pods["qos_class"], [abi.QOS_LSE, abi.QOS_LSR]) & (pods["priority_class"] == abi.PRIORITY_PROD)
    elig = np.flatnonzero((pods["numa_topology_policy"] == 0) & (pods["requests"][:, 2:] == 0).all(1)
                          & (pods["has_other_requests"] == 0) & (pods["device_requests"] == 0).all(1) & ~cpuset)
    ev = Evaluator(synth.config(N))
    synth.load_into(ev, cl)
    ev.reservations_load(rs)
    ev.schedule(pods[:0], synth.T0)
    rng = np.random.default_rng(5)
    out = {}
    names = ["checks", "refresh", "upload", "setup", "enqueue", "wait", "stats", "mirror"]
    cur = 0
    for kind in ("plain30", "matched1", "plain30+matched1", "plain30", "matched1"):
        ts, hs = [], []
        for r in range(a.reps):
            q = pods[cur:cur + 31].copy()
            cur += 31
            m = [[] for _ in range(31)]
            if kind != "plain30":
                q[30] = pods[elig[rng.integers(len(elig))]]
                q["pod_key"][30] += 10**9 + cur
                q["uid"][30] += 10**9 + cur
                q["reservation_matched"][30] = abi.RSV_MATCHED
                m[30] = np.flatnonzero(groups == rng.integers(0, groups.max() + 1)).tolist()
            if kind == "matched1":
                q, m = q[30:], m[30:]
            elif kind == "plain30":
                q, m = q[:30], None
            t0 = time.perf_counter()
            ev.schedule(q, synth.T0, matches=m)
            ts.append(time.perf_counter() - t0)
            hs.append(list(ev.host_stats().values()))
        k = kind + ("_2" if kind in out else "")
        out[k] = {"ms": float(np.median(ts)) * 1e3, "host_ms": dict(zip(names, np.median(hs, 0).round(4).tolist()))}
    print(json.dumps(out))
    ev.close()


if __name__ == "__main__":
    main()
