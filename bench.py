"""Benchmark: pod-node Filter+Score evaluations/s and p99 per-pod scheduling latency (BASELINE.json).

Workload (BASELINE.json configs[2]): 50k synthetic nodes x 100k pending pods, LoadAwareScheduling +
NodeNUMAResource with v1beta3 default args, every pod scheduled in queue order with Reserve between
pods (bit-exact with one-pod-at-a-time scheduling).  One step = scheduling one slice of the queue
(queue / steps pods) against all nodes; `value` = pods x nodes evaluated per second over the timed
steps.  The node state is resident in HBM before the timed region starts.

cpu_baseline: the oracle (C restatement of the Go plugins, oracle/) scheduling a prefix of the same
queue on the host's cores (16 threads = the upstream scheduler's Parallelism) for ~10 s of work.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from koordinator_amd import Evaluator, abi, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
DEVPOD_BYTES = 40


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, choices=(2, 3),
                    help="BASELINE.json config: 3 = 50k x 100k (the metric's workload), 2 = 5k x 10k")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--pods", type=int, default=None)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target host time of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="one-stream schedule (A/B of the pipelined one)")
    ap.add_argument("--profile-every", type=int, default=8, help="HIP-event-sample every n-th batch (0 = off)")
    ap.add_argument("--stream-nodes", type=int, default=4_000_000,
                    help="B=1 streaming sweep size (N*row > 512 MB, past the 256 MB Infinity Cache); 0 = skip")
    return ap.parse_args()


def eval_bytes(n_nodes, b):
    """algorithmic bytes of one eval-kernel launch: the node SoA once, the pod batch, the score output"""
    return n_nodes * abi.load_library().ke_row_bytes() + b * DEVPOD_BYTES + b * n_nodes * 2


def pmc_traffic(n_nodes, b):
    """HBM bytes per k_eval_batch launch from the committed rocprofv3 PMC passes (tools/pmc_summary.py)
    for this exact workload shape; None when no pass covers it."""
    f = os.path.join(ROOT, "profiles", "r01", "pmc_eval_traffic.json")
    if not os.path.exists(f):
        return None, None
    d = json.load(open(f))
    e = d["shapes"].get(f"nodes{n_nodes}pods{b}", {})
    return e.get("traffic_bytes"), d["source"] if "traffic_bytes" in e else None


def cpu_baseline(cl, pods, cfg, seconds, threads):
    from oracle.binding import Oracle  # checker / baseline only

    o = Oracle(cfg, cl.n_nodes)
    synth.load_into(o, cl)
    # calibrate on a small prefix, then time a prefix worth ~`seconds`
    t = time.perf_counter()
    o.schedule(pods[:64], synth.T0, n_threads=threads)
    per_pod = max((time.perf_counter() - t) / 64, 1e-6)
    n = int(min(len(pods) - 64, max(16, seconds / per_pod)))
    t = time.perf_counter()
    o.schedule(pods[64:64 + n], synth.T0, n_threads=threads)
    dt = time.perf_counter() - t
    return {"value": n * cl.n_nodes / dt, "unit": "pod-node evals/s", "cores": threads, "kind": "port",
            "sample": f"oracle (C restatement of the Go plugins) scheduling pods 64..{64 + n} of the same queue "
                      f"against all {cl.n_nodes} nodes, {threads} threads, {dt:.1f} s"}


def stream_sweep(n_nodes, cfg_batch):
    """B=1 HBM streaming measurement of the eval kernel over a SoA far larger than the MALL."""
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + 9, max_pods_per_node=0)
    ev = Evaluator(synth.config(n_nodes, pod_batch=cfg_batch))
    synth.load_into(ev, cl)
    pod = synth.make_pods(1, synth.BASE_SEED + 99)
    ms = ev.bench_eval_kernel(pod, synth.T0, iters=20)
    by = eval_bytes(n_nodes, 1)
    ev.close()
    return {"nodes": n_nodes, "pods_per_launch": 1, "avg_ms": ms, "bytes_per_launch": by,
            "achieved": by / ms / 1e6, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": by / ms / 1e6 / HBM_PEAK_GBS}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} needs {a.gpus} ranks (torch.distributed.run --nproc-per-node {a.gpus}); "
                         f"WORLD_SIZE={world}")
    import torch
    import torch.distributed as dist

    from koordinator_amd import shard

    if world > 1:  # control plane only (RCCL id broadcast, barriers, max-over-ranks); data path = RCCL in libkoordeval
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    N = a.nodes or synth.CONFIGS[a.config]["nodes"]
    P = a.pods or synth.CONFIGS[a.config]["pods"]
    K, W = a.steps, a.warmup
    cl = synth.make_cluster(N, synth.BASE_SEED + a.config)
    pods = synth.make_pods(P, synth.BASE_SEED + 100 + a.config)
    cfg = synth.config(N, pod_batch=a.batch)
    cfg.device_ordinal = local_rank
    slice_len = P // K

    # warmup on a throwaway context (same cluster, different pods) so the timed job starts pristine
    if W > 0:
        ew = Evaluator(cfg)
        synth.load_into(ew, cl)
        shard.init_node_sharding(ew, rank, world)
        wp = synth.make_pods(W * slice_len, synth.BASE_SEED + 203)
        for w in range(W):
            ew.schedule(wp[w * slice_len:(w + 1) * slice_len], synth.T0)
        ew.close()

    ev = Evaluator(cfg)
    synth.load_into(ev, cl)
    shard.init_node_sharding(ev, rank, world)
    lo, hi = ev.shard_range()
    ev.eval(pods[:0], synth.T0)  # derive + upload every node row: state resident in HBM
    ev.set_profiling(a.profile_every)
    ev.set_pipeline(not a.no_pipeline)
    lat, evm, sel, fix, res, samples, rsplit, npipe, enq, hof = [], [], [], [], [], 0, [], 0, [], []
    placed = 0
    barrier()
    t0 = time.perf_counter()
    for s in range(K):
        chosen, _ = ev.schedule(pods[s * slice_len:(s + 1) * slice_len], synth.T0)
        placed += int((chosen >= 0).sum())
        _, per_batch = ev.stats()
        lat.extend(per_batch.tolist())
        ks = ev.kernel_stats()
        evm.append(ks["eval_ms"] * ks["samples"])
        sel.append(ks["select_ms"] * ks["samples"])
        res.append(ks["resolve_ms"])
        fix.append(ks["fixup_ms"])
        npipe += ks["pipelined_batches"]
        enq.append(ks["enqueue_ms"])
        hof.append(ks["handoff_ms"])
        samples += ks["samples"]
        rsplit.append((ks["resolve_prologue_ms"], ks["resolve_replay_ms"]))
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    evals = K * slice_len * N
    eval_ms = sum(evm) / max(samples, 1)
    by = eval_bytes(hi - lo, a.batch)
    traffic, traffic_src = pmc_traffic(hi - lo, a.batch)
    out = {
        "metric": "pod-node Filter+Score evals/sec + p99 per-pod sched latency @50k nodes",
        "value": evals / dt,
        "unit": "pod-node evals/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": dt / K * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": f"synthetic (BASELINE.md generator, seed 20251015+{a.config})",
        "config": {"workload": synth.CONFIGS[a.config]["name"], "baseline_config": a.config, "nodes": N, "pods": K * slice_len,
                   "pods_per_batch": a.batch, "plugins": "LoadAwareScheduling+NodeNUMAResource",
                   "args": "v1beta3 defaults, NodeMetricExpirationSeconds=3600",
                   "parallelism": f"node-shard x{world}" + (" (RCCL all-gather of per-shard top-k)" if world > 1 else ""),
                   "nodes_per_rank": hi - lo},
        "p99_pod_latency_ms": float(np.percentile(lat, 99)) if lat else None,
        "p50_pod_latency_ms": float(np.percentile(lat, 50)) if lat else None,
        "pods_placed": placed,
        "kernel_ms": {"eval": eval_ms, "select": sum(sel) / max(samples, 1), "fixup": float(np.mean(fix)), "handoff": float(np.mean(hof)),
                      "resolve": float(np.mean(res)), "pipelined_batches": npipe,
                      "host_enqueue_ms_per_step": float(np.mean(enq)),
                      "resolve_prologue": float(np.mean([x[0] for x in rsplit])),
                      "resolve_replay": float(np.mean([x[1] for x in rsplit])), "samples": samples,
                      "note": "per batch; 'select' includes the all-gather + merge when sharded"},
        "roofline": {"bound": "hbm", "kernel": "k_eval_batch", "achieved": by / eval_ms / 1e6 if eval_ms else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (by / eval_ms / 1e6 / HBM_PEAK_GBS) if eval_ms else None, "traffic": traffic,
                     "traffic_source": traffic_src, "bytes_per_launch": by},
    }
    ev.close()
    if world == 1 and a.stream_nodes > 0:
        out["stream_roofline"] = stream_sweep(a.stream_nodes, a.batch)
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cl, pods, cfg, a.cpu_seconds, a.cpu_threads)
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
