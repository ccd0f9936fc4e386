"""Quick device-time breakdown of ke_schedule on a synthetic cluster (development tool)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nodes", type=int, default=50_000)
ap.add_argument("--pods", type=int, default=10_000)
ap.add_argument("--batch", type=int, default=64)
a = ap.parse_args()
cl = synth.make_cluster(a.nodes, synth.BASE_SEED + 3)
pods = synth.make_pods(a.pods, synth.BASE_SEED + 103)
ev = Evaluator(synth.config(a.nodes, pod_batch=a.batch))
synth.load_into(ev, cl)
ev.eval(pods[:0], synth.T0)
ev.set_profiling(4)
ev.schedule(pods[:2048], synth.T0)  # warm
t = time.perf_counter()
ev.schedule(pods[2048:], synth.T0)
dt = time.perf_counter() - t
tot, per = ev.stats()
ks = ev.kernel_stats()
n = a.pods - 2048
print(json.dumps({"evals_per_s": n * a.nodes / dt, "wall_ms": dt * 1e3, "device_ms": tot,
                  "per_batch_ms": float(per.mean()), "kernels": ks}, indent=1))
