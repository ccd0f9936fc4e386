"""NodeResourcesFitPlus + ScarceResourceAvoidance in the fused pass: the cost of the two
extra Score plugins on the config-3 workload shape.

The same synthetic cluster and queue (synth.make_cluster / make_pods, the resource tables of
synth.make_node_resources, the pods' requested names / FitPlus requests of synth.add_pod_xres) scheduled twice:
the default profile (LoadAware + NodeNUMAResource, pipelined fast replay) and the profile with FitPlus (cpu,
memory, batch-cpu LeastAllocated; GPUs MostAllocated w2) and SRA (GPUs, a scarce device) at weight 1, which runs
on the zone-aware path.  The placements of the ext run are checked against the oracle on a
bounded prefix.  Prints one JSON line.  Usage: python tools/ext_bench.py [--nodes 50000 --pods 10240]
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


def run(cfg, cl, tables, pods, steps):
    def fresh():
        ev = Evaluator(cfg)
        synth.load_into(ev, cl)
        synth.load_node_resources(ev, tables)
        return ev

    ew = fresh()
    ew.schedule(pods[:256], synth.T0)  # warm-up: kernels loaded, paths exercised
    ew.close()
    ev = fresh()
    ev.eval(pods[:0], synth.T0)
    sl = len(pods) // steps
    lat = []
    t0 = time.perf_counter()
    for s in range(steps):
        ev.schedule(pods[s * sl:(s + 1) * sl], synth.T0)
        _, per_batch = ev.stats()
        lat.extend(per_batch.tolist())
    dt = time.perf_counter() - t0
    ev.close()
    n = steps * sl
    return {"value": n * cl.n_nodes / dt, "ms_per_pod": dt / n * 1e3, "p99_batch_latency_ms": float(np.percentile(lat, 99))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=10_240)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--check-pods", type=int, default=256, help="oracle parity prefix of the ext run (0 = off)")
    a = ap.parse_args()
    cl = synth.make_cluster(a.nodes, synth.BASE_SEED + 3)
    tables = synth.make_node_resources(cl, synth.BASE_SEED + 33)
    pods = synth.add_pod_xres(synth.make_pods(a.pods, synth.BASE_SEED + 103), synth.BASE_SEED + 133)
    base = run(synth.config(a.nodes), cl, tables, pods, a.steps)
    ext_cfg = synth.ext_config(synth.config(a.nodes))
    ext = run(ext_cfg, cl, tables, pods, a.steps)
    out = {"workload": f"{a.nodes} nodes x {a.pods} pods (config-3 shape) with node resource tables",
           "unit": "pod-node evals/s", "default_profile": base, "fitplus_sra_profile": ext,
           "ext_cost": base["value"] / ext["value"]}
    if a.check_pods:
        from oracle.binding import Oracle  # checker only

        ev, o = Evaluator(ext_cfg), Oracle(ext_cfg, a.nodes)
        for h in (ev, o):
            synth.load_into(h, cl)
            synth.load_node_resources(h, tables)
        c1, s1 = ev.schedule(pods[:a.check_pods], synth.T0)
        c0, s0 = o.schedule(pods[:a.check_pods], synth.T0, n_threads=16)
        out["oracle_prefix_equal"] = bool(np.array_equal(c1, c0) and np.array_equal(s1, s0))
        out["oracle_prefix_pods"] = a.check_pods
    print(json.dumps(out))


if __name__ == "__main__":
    main()
