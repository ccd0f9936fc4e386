"""BASELINE config 5 — DeviceShare GPU/RDMA partial-device Filter + Score + ElasticQuota admission over
20k nodes: throughput and per-pod latency.  `--quota` (default on) loads a 64-leaf ElasticQuota tree
(synth.make_quota_tree) whose total is `--quota-frac` of the queue's requests; every pod with a quota
is admitted (PreFilter) and reserved (used += request) on the GPU, in queue order.

N synthetic nodes (synth.make_cluster + synth.make_devices: 8 GPUs with gpu-core 100 / ratio 100 /
192Gi and 2 RDMA NICs each, random partial usage, 5 % without a device cache entry, 2 % unhealthy
GPUs); the config-2 queue of which `--device` request devices (gpu-core = gpu-memory-ratio in
{25..800}, nvidia.com/gpu, shared gpu-memory slices, optional RDMA; synth.make_ds_pods).  Pods are
scheduled in queue order; a DeviceShare pod is its own batch (NormalizeScore needs the max over all
feasible nodes), the others run in exact speculative batches of 64.  Prints one JSON line; the oracle
schedules a bounded prefix of the same queue on the host's cores (cpu_baseline).
Usage: python tools/ds_bench.py [--nodes 20000] [--pods 4096]
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
    ap.add_argument("--nodes", type=int, default=20_000)
    ap.add_argument("--pods", type=int, default=4096)
    ap.add_argument("--device", type=float, default=0.5, help="fraction of pods with device requests")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-quota", action="store_true")
    ap.add_argument("--quota-frac", type=float, default=0.6)
    a = ap.parse_args()
    N, P, K = a.nodes, a.pods, a.steps
    cl = synth.make_cluster(N, synth.BASE_SEED + 5)
    devices = synth.make_devices(N, synth.BASE_SEED + 55)
    pods = synth.make_ds_pods(P, synth.BASE_SEED + 105, device_fraction=a.device)
    cfg = synth.config(N)
    quotas = None
    if not a.no_quota:
        tc = int(pods["requests"][:, 0].sum() * a.quota_frac)
        tm = int(pods["requests"][:, 1].sum() * a.quota_frac)
        quotas = synth.make_quota_tree(synth.BASE_SEED + 305, 64, 8, tc, tm)
        pods = synth.assign_quotas(pods, quotas, synth.BASE_SEED + 306)
        qargs = synth.quota_args(tc, tm)

    def load(h):
        synth.load_into(h, cl)
        synth.load_devices(h, devices)
        if quotas is not None:
            h.quotas_load(qargs, quotas)
        return h

    ew = load(Evaluator(cfg))  # warm-up context
    ew.schedule(synth.make_ds_pods(128, synth.BASE_SEED + 205, device_fraction=a.device), synth.T0)
    ew.close()
    ev = load(Evaluator(cfg))
    ev.eval(pods[:0], synth.T0)
    ev.set_profiling(8)
    sl = P // K
    lat, ks_acc, samples, placed, with_dev = [], {"eval_ms": 0.0, "select_ms": 0.0, "resolve_ms": 0.0}, 0, 0, 0
    hs = []
    cuts = 0
    t0 = time.perf_counter()
    for s in range(K):
        chosen, _ = ev.schedule(pods[s * sl:(s + 1) * sl], synth.T0)
        placed += int((chosen >= 0).sum())
        with_dev += int((ev.last_device_allocations != 0).sum())
        _, per_batch = ev.stats()
        lat.extend(per_batch.tolist())
        ks = ev.kernel_stats()
        for key in ("eval_ms", "select_ms"):  # HIP-event samples
            ks_acc[key] += ks[key] * ks["samples"]
        ks_acc["resolve_ms"] += ks["resolve_ms"] * len(per_batch)  # in-kernel stamps: mean over every batch
        samples += ks["samples"]
        hs.append(ev.host_stats())
        cuts += ev.ds_cuts()
    dt = time.perf_counter() - t0
    ev.close()
    out = {"workload": f"{N} nodes x (8 GPU + 2 RDMA), {K * sl} pods ({a.device:.0%} with device requests)"
                       + ("" if quotas is None else f", ElasticQuota tree of 64 leaves (total {a.quota_frac:.0%} of requests)"),
           "value": K * sl * N / dt, "unit": "pod-node evals/s", "pods_per_s": K * sl / dt,
           "ms_per_pod": dt / (K * sl) * 1e3, "batches": len(lat),
           "p99_batch_latency_ms": float(np.percentile(lat, 99)), "p50_batch_latency_ms": float(np.percentile(lat, 50)),
           "kernel_ms_per_batch": {"eval_ms": ks_acc["eval_ms"] / max(samples, 1),
                                   "select_ms": ks_acc["select_ms"] / max(samples, 1),
                                   "resolve_ms": ks_acc["resolve_ms"] / max(len(lat), 1)},
           "placed": placed, "device_allocations": with_dev, "ds_batch_cuts": cuts,
           "host_ms_per_step": {k: float(np.mean([h[k] for h in hs])) for k in hs[0]} if hs else None}
    if not a.no_cpu_baseline:
        from oracle.binding import Oracle  # checker / baseline only

        o = load(Oracle(cfg, N))
        t = time.perf_counter()
        o.schedule(pods[:16], synth.T0, n_threads=a.cpu_threads)
        per_pod = max((time.perf_counter() - t) / 16, 1e-6)
        n = int(min(P - 16, max(16, a.cpu_seconds / per_pod)))
        t = time.perf_counter()
        o.schedule(pods[16:16 + n], synth.T0, n_threads=a.cpu_threads)
        cdt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": n * N / cdt, "unit": "pod-node evals/s", "cores": a.cpu_threads, "kind": "port",
                               "sample": f"oracle scheduling pods 16..{16 + n} of the same queue, {cdt:.1f} s"}
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
