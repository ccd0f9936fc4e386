"""Benchmark: pod-node Filter+Score evaluations/s and p99 per-pod scheduling latency (BASELINE.json).

Workload (BASELINE.json configs[2]): 50k synthetic nodes x 100k pending pods, LoadAwareScheduling +
NodeNUMAResource with v1beta3 default args, every pod scheduled in queue order with Reserve between
pods (bit-exact with one-pod-at-a-time scheduling).  One step = scheduling one slice of the queue
(queue / steps pods) against all nodes; `value` = pods x nodes evaluated per second over the timed
steps.  The node state is resident in HBM before the timed region starts.

roofline: the per-batch pipeline.  The critical path is the Reserve chain (k_resolve_run,
one workgroup, per-batch time from in-kernel s_memrealtime stamps); eval and select run beside it on two
alternating eval streams (k_fixup too with --pipeline-fixup).  `roofline.achieved` = SURVEY.md §8(d)'s algorithmic bytes of a batch (N*S_row +
B*S_pod + B*k*12) over that critical path; `roofline.replay` the replay's own bytes, `roofline.kernels`
every kernel of a batch and `roofline.end_to_end` the whole step, each against 8 TB/s.
`traffic` = HBM bytes from a prior rocprofv3 PMC pass of this workload (profiles/r06/pmc_bench.json).

cpu_baseline: the oracle (C restatement of the Go plugins, oracle/) scheduling a prefix of the same
queue on the host's cores at 1 thread, 16 threads (upstream Parallelism) and every usable core.
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
KMAX, KSTALE = 64, 128  # candidate list lengths (ke_kernels.hip)
CAND_BYTES = 4
# replay records (ke_kernels.hip RecWord, NUM_RW = 26 int64 words per node)
REC_READ = 25 * 8   # words a fetch loads (all but RW_PAD)
REC_DYN = 11 * 8    # Reserve-dependent words a changed node writes back (rec_store_dyn)
REC_FULL = 26 * 8   # the full record of a changed node in the hand-off list k_fixup reads
ROW_PATCH = 10 * 8  # SoA int64 fields a Reserve writes back (fh 4, sa 4, NodeInfo.Requested 2)
OUT_BYTES = 4 + 4 + 8  # chosen, score, device allocation per pod


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
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="host time of each CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="one-stream schedule (A/B of the pipelined one)")
    ap.add_argument("--pipeline-fixup", action="store_true",
                    help="pipelined with exact lists from k_fixup (ke_set_pipeline 2, the round-3 schedule)")
    ap.add_argument("--profile-every", type=int, default=8, help="HIP-event-sample every n-th batch (0 = off)")
    ap.add_argument("--sync", action="store_true", help="one ke_schedule call per step (no submit-ahead)")
    ap.add_argument("--stream-nodes", type=int, default=4_000_000,
                    help="B=1 streaming sweep size (N*row > 512 MB, past the 256 MB Infinity Cache); 0 = skip")
    return ap.parse_args()


def sizes():
    lib = abi.load_library()
    return lib.ke_row_bytes(), lib.ke_pod_record_bytes()


REC_EVAL = 13 * 16  # the replay record k_eval_plain reads per node (13 16-byte loads)


def eval_kernel(b):
    """the eval kernel a plain batch of b pods launches (ke_kernels.hip use_record_eval)"""
    return "k_eval_plain" if b > 2 else "k_eval_batch"


def eval_bytes(n_nodes, b):
    """algorithmic bytes of one eval-kernel launch: per node the SoA row (k_eval_batch) or the replay record
    (k_eval_plain), the pod batch, the score output"""
    row, pod = sizes()
    return n_nodes * (REC_EVAL if b > 2 else row) + b * pod + b * n_nodes * 2


def batch_bytes(n_nodes, b, fetched, changed, pipelined, fixup=False):
    """algorithmic bytes per batch of each kernel: every input read once, every output
    written once; `fetched` = replay records of best unchanged candidates, `changed` = nodes a batch Reserved"""
    row, pod = sizes()
    L = KSTALE if pipelined else KMAX
    return {
        eval_kernel(b): eval_bytes(n_nodes, b),
        "k_select": b * n_nodes * 2 + b * (L + 1) * CAND_BYTES,
        "k_fixup": (b * ((L + 1) * CAND_BYTES + pod + (KMAX + 1) * CAND_BYTES) + changed * REC_FULL) if fixup else 0,
        "k_resolve": b * ((KMAX + 1) * CAND_BYTES + pod + OUT_BYTES) + fetched * REC_READ
                     + changed * (ROW_PATCH + REC_DYN + (REC_FULL if fixup else 0)),
    }


def pmc_traffic(tag):
    """HBM bytes per launch by kernel from the committed PMC passes (tools/pmc_bench.sh, summarised by
    tools/pmc_summary.py into profiles/<round>/pmc_bench.json, the newest) of this workload.  Counter collection serialises
    dispatches, which the persistent Reserve chain (and the eval streams' kernels that wait on its flags: k_handoff,
    k_fixlist) cannot run under, so the passes run the one-stream schedule (tag suffix _serial): its k_eval_plain /
    k_select / k_resolve launches do the same work per batch; k_fixlist moves <= 64 records + 64 x 256 keys per
    batch (about 64 KB)."""
    f = next((x for x in (os.path.join(ROOT, "profiles", r, "pmc_bench.json") for r in ("r06", "r05")) if os.path.exists(x)),
             None)  # (the newest round's passes)
    if f is None:
        return {}, None
    d = json.load(open(f))
    w = d.get("workloads", {})
    key = tag if tag in w else (tag + "_serial" if tag + "_serial" in w else None)
    if key is None:
        return {}, None
    e = {k: {x: v[x] for x in ("traffic_bytes", "valu_busy", "wave_issue_stall_share", "wave_wait_share") if x in v}
         for k, v in w[key].items() if isinstance(v, dict) and "traffic_bytes" in v}
    return e, f"PMC passes {key} ({d.get('source')})"


def host_info():
    """CPU model, the affinity mask and the cgroup CPU quota (cpu.max) -- the box shares its host, so the
    quota, not nproc, is the number of cores a process can keep busy."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = affinity if quota is None else max(1, min(affinity, int(quota)))
    return {"nproc": affinity, "cpu_count": os.cpu_count(), "cgroup_cpus": quota, "usable": usable, "model": model}


def cpu_baseline(cl, pods, cfg, seconds):
    """The oracle scheduling consecutive prefixes of the queue at 1, 16 and every usable thread."""
    from oracle.binding import Oracle  # checker / baseline only

    info = host_info()
    o = Oracle(cfg, cl.n_nodes)
    synth.load_into(o, cl)
    rates, pos = {}, 0
    for threads in sorted({1, 16, info["usable"]}):
        o.schedule(pods[pos:pos + 4], synth.T0, n_threads=threads)  # thread pool warm-up
        pos += 4
        p0, dt, chunk = pos, 0.0, 8  # doubling chunks of the queue until ~`seconds` of work
        while dt < seconds and pos < len(pods):
            n = min(chunk, len(pods) - pos)
            t = time.perf_counter()
            o.schedule(pods[pos:pos + n], synth.T0, n_threads=threads)
            dt += time.perf_counter() - t
            pos += n
            chunk *= 2
        rates[str(threads)] = {"value": (pos - p0) * cl.n_nodes / dt, "pods": [p0, pos], "seconds": dt}
    best = max(rates, key=lambda k: rates[k]["value"])
    return {"value": rates[best]["value"], "unit": "pod-node evals/s", "cores": int(best), "kind": "port",
            "host": info, "rates_by_threads": rates,
            "sample": f"oracle (C restatement of the Go plugins) scheduling consecutive prefixes of the same queue "
                      f"against all {cl.n_nodes} nodes at 1 / 16 / {info['usable']} threads (all usable cores: "
                      f"cgroup quota {info['cgroup_cpus']}, affinity {info['nproc']}) (~{seconds:.0f} s each); "
                      f"value = the fastest ({best} threads)"}


def c3_parity(chosen, score, n_nodes, n_pods, config):
    """The timed run's placements and scores against the oracle's full-queue fixture (tests/golden/
    make_c3_fixture.py: the oracle scheduled the same 100k-pod queue on the same 50k-node cluster), compared after
    the timed region.  Only for the default config-3 workload (other sizes have no fixture)."""
    f = os.path.join(ROOT, "tests", "golden", "c3_placements.npz")
    if config != 3 or not os.path.exists(f):
        return "unchecked (no fixture for this workload)"
    g = np.load(f)
    if int(g["nodes"]) != n_nodes:
        return "unchecked (no fixture for this workload)"
    if n_pods != int(g["pods"]):  # synth.make_pods of another length is another queue, not a prefix
        return f"unchecked (the fixture holds the {int(g['pods'])}-pod queue; this run's queue has {n_pods})"
    m = n_pods
    ok = (chosen[:m] == g["chosen"][:m]) & (score[:m] == g["score"][:m].astype(np.int32))
    if ok.all():
        return f"bit-exact {m}/{int(g['pods'])} (placements + scores vs the oracle fixture)"
    bad = np.flatnonzero(~ok)
    return f"MISMATCH {len(bad)}/{m} (first at pod {int(bad[0])})"


def alg_batch_bytes(n_nodes, b):
    """SURVEY.md §8(d) algorithmic bytes of one B-pod batch: the node SoA row once (S_row = ke_row_bytes()),
    the pod records (S_pod = ke_pod_record_bytes()) and the top-k out (B * k * 12 B, k = KMAX)."""
    row, pod = sizes()
    return n_nodes * row + b * pod + b * KMAX * 12


def roofline(n_nodes, b, ks, dt_step, batches_per_step, pipelined, tag, fixup=False):
    """§8(d) roofline of a batch over its critical path (the Reserve chain: replay + hand-off per batch), with
    the replay's own bytes, the per-kernel and the end-to-end fractions as sub-fields."""
    by = batch_bytes(n_nodes, b, ks["rows_fetched"], ks["rows_changed"], pipelined, fixup)
    ms = {eval_kernel(b): ks["eval_ms"], "k_select": ks["select_ms"], "k_fixup": ks["fixup_ms"],
          "k_resolve": ks["resolve_ms"]}
    traffic, src = pmc_traffic(tag)
    kern = {}
    for k in by:
        t = ms[k]
        ach = by[k] / t / 1e6 if t else None
        pmc = traffic.get(k, {})
        kern[k] = {"bytes_per_batch": by[k], "ms_per_batch": t, "achieved": ach,
                   "frac": ach / HBM_PEAK_GBS if ach else None, "traffic": pmc.get("traffic_bytes"),
                   "valu_busy": pmc.get("valu_busy"), "issue_stall_share": pmc.get("wave_issue_stall_share")}
    step_bytes = sum(by.values()) * batches_per_step
    dom = kern["k_resolve"]
    alg = alg_batch_bytes(n_nodes, b)
    crit_ms = ks["resolve_ms"] + (ks["handoff_ms"] if pipelined else 0.0)
    ach = alg / crit_ms / 1e6 if crit_ms else None
    pmc_sum = sum(v["traffic"] for v in kern.values() if v.get("traffic")) or None
    return {"bound": "hbm", "kernel": "k_resolve_run (the Reserve chain: the batch's critical path)",
            "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS if ach else None,
            "traffic": pmc_sum, "traffic_source": src, "bytes_per_launch": alg, "launch_ms": crit_ms,
            "batches_per_launch": batches_per_step,
            "reproduce": "k_resolve_run is one persistent launch per ke_schedule call (one call per step): achieved = "
                         "bytes_per_launch x batches_per_launch / (AverageNs of k_resolve_run in a rocprofv3 "
                         "--kernel-trace --stats CSV of the same command); the profiler slows the pipeline, so compare "
                         "with the bench line printed under it (profiles/r06/bench_under_rocprof.json)",
            "bytes_definition": "SURVEY.md §8(d) per B-pod batch: N*S_row + B*S_pod + B*k*12 "
                                f"(S_row {sizes()[0]}, S_pod {sizes()[1]}, k {KMAX}); time = replay + hand-off per batch "
                                "(in-kernel s_memrealtime); traffic = PMC HBM bytes of every kernel of a batch",
            "replay": {"bytes_per_batch": dom["bytes_per_batch"], "ms_per_batch": dom["ms_per_batch"],
                       "achieved": dom["achieved"], "frac": dom["frac"], "traffic": dom["traffic"]},
            "timing": "k_resolve / k_fixup: in-kernel s_memrealtime per batch (one persistent launch per run); "
                      "k_eval_plain / k_eval_batch / k_select: HIP events on the eval stream",
            "kernels": kern,
            "end_to_end": {"bytes_per_step": step_bytes, "ms_per_step": dt_step * 1e3,
                           "achieved": step_bytes / dt_step / 1e9, "frac": step_bytes / dt_step / 1e9 / HBM_PEAK_GBS},
            "note": "the Reserve replay is sequential (pod j sees pods < j) and latency-bound on one wave; "
                    "its HBM fraction is small by nature. The HBM gate is stream_roofline (eval kernel, B=1, "
                    "SoA past the 256 MB Infinity Cache)."}


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
    ev.set_pipeline(False if a.no_pipeline else ("fixup" if a.pipeline_fixup else True))
    lat, plat, evm, sel, samples, rsplit, npipe, hs, kss = [], [], [], [], 0, [], 0, [], []
    placed = 0
    n_batches = 0
    got_c, got_s = [], []
    barrier()
    t0 = time.perf_counter()
    # the scheduler loop hands over slice s+1 (ke_schedule_submit) before collecting slice s (ke_schedule_wait): the
    # host's argument checks, staging and launches of s+1 overlap the device's work on s (--sync: ke_schedule)
    sl = lambda s: pods[s * slice_len:(s + 1) * slice_len]  # noqa: E731
    nxt = None if a.sync or K == 0 else ev.submit(sl(0), synth.T0)
    for s in range(K):
        if a.sync:
            chosen, score = ev.schedule(sl(s), synth.T0)
        else:
            cur, nxt = nxt, (ev.submit(sl(s + 1), synth.T0) if s + 1 < K else None)
            chosen, score = ev.wait(cur)
        got_c.append(chosen)
        got_s.append(score)
        placed += int((chosen >= 0).sum())
        _, per_batch = ev.stats()
        lat.extend(per_batch.tolist())
        plat.append(ev.pod_latencies(slice_len))
        n_batches += len(per_batch)
        ks = ev.kernel_stats()
        kss.append(ks)
        evm.append(ks["eval_ms"] * ks["samples"])
        sel.append(ks["select_ms"] * ks["samples"])
        npipe += ks["pipelined_batches"]
        hs.append(ev.host_stats())
        samples += ks["samples"]
        rsplit.append((ks["resolve_prologue_ms"], ks["resolve_replay_ms"]))
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    evals = K * slice_len * N
    mean = lambda key: float(np.mean([k[key] for k in kss]))  # noqa: E731
    kagg = {"eval_ms": sum(evm) / max(samples, 1), "select_ms": sum(sel) / max(samples, 1),
            "fixup_ms": mean("fixup_ms"), "resolve_ms": mean("resolve_ms"), "handoff_ms": mean("handoff_ms"),
            "rows_fetched": mean("rows_fetched"), "rows_changed": mean("rows_changed"),
            "spec_failed": mean("spec_failed_rounds"),
            "resolve_phases": {k: float(np.mean([x["resolve_phases_ms"][k] for x in kss])) for k in kss[0]["resolve_phases_ms"]},
            "resolve_wave1": {k: float(np.mean([x["resolve_wave1_ms"][k] for x in kss])) for k in kss[0]["resolve_wave1_ms"]}}
    tag = f"config{a.config}_nodes{hi - lo}_batch{a.batch}_world{world}" + ("" if not a.no_pipeline else "_serial")
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
                   "nodes_per_rank": hi - lo, "pipelined": not a.no_pipeline,
                   "calls": "ke_schedule per step" if a.sync else "ke_schedule_submit one step ahead + ke_schedule_wait"},
        # pod dequeue (the ke_schedule call's entry: every pod of a step is dequeued then) -> its
        # node selected (its batch's Reserve end); includes host staging and the wait behind earlier batches
        "p99_pod_latency_ms": float(np.percentile(np.concatenate(plat), 99)) if plat else None,
        "p50_pod_latency_ms": float(np.percentile(np.concatenate(plat), 50)) if plat else None,
        "pods_per_call": slice_len,
        "latency_definition": "ke_last_pod_latencies: ke_schedule entry -> the pod's batch Reserve end (host clock)",
        "p99_batch_service_ms": float(np.percentile(lat, 99)) if lat else None,
        "pods_placed": placed,
        "kernel_ms": {"eval": kagg["eval_ms"], "select": kagg["select_ms"], "fixup": kagg["fixup_ms"],
                      "handoff": kagg["handoff_ms"], "resolve": kagg["resolve_ms"],
                      "resolve_prologue": float(np.mean([x[0] for x in rsplit])),
                      "resolve_replay": float(np.mean([x[1] for x in rsplit])),
                      "pipelined_batches": npipe, "batches": n_batches, "event_samples": samples,
                      "records_fetched_per_batch": kagg["rows_fetched"], "rows_changed_per_batch": kagg["rows_changed"],
                      "spec_failed_rounds_per_batch": kagg["spec_failed"],
                      "resolve_phases": kagg["resolve_phases"],
                      "resolve_wave1": kagg["resolve_wave1"],
                      "note": "per batch; 'select' includes the all-gather + merge when sharded"},
        "host_ms_per_step": {k: float(np.mean([h[k] for h in hs])) for k in hs[0]} if hs else None,
        "roofline": roofline(hi - lo, a.batch, kagg, dt / K, n_batches / K, not a.no_pipeline, tag,
                             a.pipeline_fixup and not a.no_pipeline),
    }
    ev.close()
    out["parity"] = c3_parity(np.concatenate(got_c), np.concatenate(got_s), N, K * slice_len, a.config)
    if world == 1 and a.stream_nodes > 0:
        out["stream_roofline"] = stream_sweep(a.stream_nodes, a.batch)
    if world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cl, pods, cfg, a.cpu_seconds)
        out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
