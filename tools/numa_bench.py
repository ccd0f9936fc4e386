"""NUMA topology-policy workload (BASELINE config 4 without cpuset pods): throughput and latency.

N synthetic nodes with `--zones` NUMA zones each (policy mix None/BestEffort/Restricted/SingleNUMANode
10/30/30/30 %), the config-2 pod mix of which `--pod-policy` also carry a numa-topology-spec.  Every
pod is scheduled in queue order with NUMA Reserve between pods.  Prints one JSON line: evals/s, p99
per-batch latency, eval-kernel time per batch, and the oracle on the host's cores for a bounded
prefix of the same queue (cpu_baseline).  Usage: python tools/numa_bench.py [--nodes 50000] ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from koordinator_amd import Evaluator, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=10_240)
    ap.add_argument("--zones", type=int, default=8)
    ap.add_argument("--pod-policy", type=float, default=0.2)
    ap.add_argument("--status", type=float, default=0.1, help="fraction of zones single / shared (cpuset pods)")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    N, P, K = a.nodes, a.pods, a.steps
    cl = synth.make_cluster(N, synth.BASE_SEED + 4, amplified_fraction=0.3)
    zones = synth.make_numa(cl, synth.BASE_SEED + 44, zone_counts=(a.zones,), status_fraction=a.status)
    pods = synth.make_numa_pods(P, synth.BASE_SEED + 104, policy_fraction=a.pod_policy)
    cfg = synth.config(N)

    def fresh():
        ev = Evaluator(cfg)
        synth.load_into(ev, cl)
        synth.load_numa(ev, zones)
        return ev

    ew = fresh()  # warm-up context: kernels loaded, code paths exercised
    ew.schedule(synth.make_numa_pods(256, synth.BASE_SEED + 204, policy_fraction=a.pod_policy), synth.T0)
    ew.close()
    ev = fresh()
    ev.eval(pods[:0], synth.T0)  # rows + NUMA rows resident in HBM
    ev.set_profiling(4)
    sl = P // K
    lat, evm, samples, deferred = [], 0.0, 0, 0
    t0 = time.perf_counter()
    for s in range(K):
        ev.schedule(pods[s * sl:(s + 1) * sl], synth.T0)
        _, per_batch = ev.stats()
        lat.extend(per_batch.tolist())
        ks = ev.kernel_stats()
        evm += ks["eval_ms"] * ks["samples"]
        samples += ks["samples"]
        deferred += ev.numa_deferred()
    dt = time.perf_counter() - t0
    ev.close()
    out = {"workload": f"{N} nodes x {a.zones} NUMA zones, {K * sl} pods ({a.pod_policy:.0%} with a pod NUMA policy)",
           "value": K * sl * N / dt, "unit": "pod-node evals/s", "ms_per_pod": dt / (K * sl) * 1e3,
           "p99_batch_latency_ms": float(np.percentile(lat, 99)), "p50_batch_latency_ms": float(np.percentile(lat, 50)),
           "eval_kernel_ms_per_batch": evm / max(samples, 1), "deferred_pairs": deferred}
    if not a.no_cpu_baseline:
        from oracle.binding import Oracle  # checker / baseline only

        o = Oracle(cfg, N)
        synth.load_into(o, cl)
        synth.load_numa(o, zones)
        t = time.perf_counter()
        o.schedule(pods[:8], synth.T0, n_threads=a.cpu_threads)
        per_pod = max((time.perf_counter() - t) / 8, 1e-6)
        n = int(min(P - 8, max(8, a.cpu_seconds / per_pod)))
        t = time.perf_counter()
        o.schedule(pods[8:8 + n], synth.T0, n_threads=a.cpu_threads)
        cdt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": n * N / cdt, "unit": "pod-node evals/s", "cores": a.cpu_threads, "kind": "port",
                               "sample": f"oracle scheduling pods 8..{8 + n} of the same queue, {cdt:.1f} s"}
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
