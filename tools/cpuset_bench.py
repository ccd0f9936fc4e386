"""BASELINE config 4 — NUMA-aware cpuset binding (8 NUMA nodes per host, LSR/LSE pods, topology-hint
scoring): throughput and per-pod latency.

N synthetic nodes with `--zones` NUMA zones each and a consistent CPU table (synth.make_numa_cpus:
policies None/BestEffort/Restricted/SingleNUMANode 10/30/30/30 %, earlier cpusets with RefCount /
exclusivity, node CPU bind policies on 20 % of the nodes); the queue (synth.make_numa_cpuset_pods)
is 60 % LSR/LSE koord-prod binding pods with ResourceSpec bind / exclusive policies, 20 % of all pods
with their own NUMA topology spec.  Every pod is scheduled in queue order: with node CPU bind
policies present every cpu-requesting pod may bind, so each is its own batch (eval over all nodes,
select, the accumulator Reserve).  Prints one JSON line; the oracle schedules a bounded prefix of
the same queue on the host's cores (cpu_baseline).  Usage: python tools/cpuset_bench.py [--nodes 50000]
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
    ap.add_argument("--pods", type=int, default=4096)
    ap.add_argument("--zones", type=int, default=8)
    ap.add_argument("--cpuset", type=float, default=0.6, help="fraction of LSR/LSE binding pods")
    ap.add_argument("--pod-policy", type=float, default=0.2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--survey", action="store_true", help="SURVEY.md §8d C4 spec: 128-CPU 2x4x8x2 hosts, "
                    "policies 40/30/30, LSR/LSE pods cpu {2,4,8,16} with the FullPCPUs default")
    ap.add_argument("--policy-weights", default="", help="with --survey: None,BestEffort,Restricted,SingleNUMANode "
                    "weights (default 0,0.3,0.3,0.4)")
    a = ap.parse_args()
    N, P, K = a.nodes, a.pods, a.steps
    if a.survey:
        pw = tuple(float(x) for x in a.policy_weights.split(",")) if a.policy_weights else (0.0, 0.3, 0.3, 0.4)
        cl, zones, tables = synth.make_c4_cluster(N, synth.BASE_SEED + 4, policy_weights=pw)
        pods = synth.make_c4_pods(P, synth.BASE_SEED + 104)
    else:
        cl = synth.make_cluster(N, synth.BASE_SEED + 6, amplified_fraction=0.3)
        zones, tables = synth.make_numa_cpus(cl, synth.BASE_SEED + 66, zone_counts=(a.zones,))
        pods = synth.make_numa_cpuset_pods(P, synth.BASE_SEED + 106, cpuset_fraction=a.cpuset,
                                           policy_fraction=a.pod_policy)
    cfg = synth.config(N)

    def load(h):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tables)
        return h

    ew = load(Evaluator(cfg))  # warm-up context: kernels loaded, code paths exercised
    ew.schedule(pods[:64], synth.T0)
    ew.close()
    ev = load(Evaluator(cfg))
    ev.eval(pods[:0], synth.T0)  # rows, NUMA rows and CPU tables resident in HBM
    ev.set_profiling(8)
    sl = P // K
    lat, ks_acc, samples, placed, cpusets, deferred = [], {"eval_ms": 0.0, "select_ms": 0.0, "resolve_ms": 0.0}, 0, 0, 0, 0
    t0 = time.perf_counter()
    for s in range(K):
        chosen, _ = ev.schedule(pods[s * sl:(s + 1) * sl], synth.T0)
        placed += int((chosen >= 0).sum())
        cpusets += int(np.any(ev.last_cpusets != 0, axis=1).sum())
        _, per_batch = ev.stats()
        lat.extend(per_batch.tolist())
        ks = ev.kernel_stats()
        for key in ("eval_ms", "select_ms"):  # HIP-event samples
            ks_acc[key] += ks[key] * ks["samples"]
        ks_acc["resolve_ms"] += ks["resolve_ms"] * len(per_batch)  # in-kernel stamps: mean over every batch
        samples += ks["samples"]
        deferred += ev.numa_deferred()
    dt = time.perf_counter() - t0
    ev.close()
    wl = (f"C4 (SURVEY.md §8d): {N} nodes x 128 CPUs (2 sockets x 4 NUMA x 8 cores x 2 threads), {K * sl} LSR/LSE pods"
          if a.survey else f"{N} nodes x {a.zones} NUMA zones with CPU tables, {K * sl} pods "
                           f"({a.cpuset:.0%} LSR/LSE binding, {a.pod_policy:.0%} with a pod NUMA policy)")
    out = {"workload": wl,
           "value": K * sl * N / dt, "unit": "pod-node evals/s", "pods_per_s": K * sl / dt,
           "ms_per_pod": dt / (K * sl) * 1e3, "batches": len(lat),
           "p99_batch_latency_ms": float(np.percentile(lat, 99)), "p50_batch_latency_ms": float(np.percentile(lat, 50)),
           "kernel_ms_per_batch": {"eval_ms": ks_acc["eval_ms"] / max(samples, 1),
                                   "select_ms": ks_acc["select_ms"] / max(samples, 1),
                                   "resolve_ms": ks_acc["resolve_ms"] / max(len(lat), 1)},
           "placed": placed, "cpusets": cpusets, "deferred_pairs": deferred}
    if not a.no_cpu_baseline:
        from oracle.binding import Oracle  # checker / baseline only

        o = load(Oracle(cfg, N))
        t = time.perf_counter()
        o.schedule(pods[:4], synth.T0, n_threads=a.cpu_threads)
        per_pod = max((time.perf_counter() - t) / 4, 1e-6)
        n = int(min(P - 4, max(4, a.cpu_seconds / per_pod)))
        t = time.perf_counter()
        o.schedule(pods[4:4 + n], synth.T0, n_threads=a.cpu_threads)
        cdt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": n * N / cdt, "unit": "pod-node evals/s", "cores": a.cpu_threads, "kind": "port",
                               "sample": f"oracle scheduling pods 4..{4 + n} of the same queue, {cdt:.1f} s"}
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
