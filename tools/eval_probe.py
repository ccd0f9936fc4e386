"""Launch only the batch eval kernel (k_eval_batch) `iters` times over a synthetic SoA: the target of
the rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE per launch) behind roofline.traffic."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import Evaluator, abi, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--nodes", type=int, default=50_000)
ap.add_argument("--pods", type=int, default=64)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
cl = synth.make_cluster(a.nodes, synth.BASE_SEED + 3, max_pods_per_node=0 if a.nodes > 1_000_000 else 20)
ev = Evaluator(synth.config(a.nodes))
synth.load_into(ev, cl)
pods = synth.make_pods(a.pods, synth.BASE_SEED + 103)
ms = ev.bench_eval_kernel(pods, synth.T0, a.iters)
row = abi.load_library().ke_row_bytes()
by = a.nodes * row + a.pods * 40 + a.pods * a.nodes * 2
print(f"nodes={a.nodes} pods={a.pods} avg_ms={ms:.5f} algorithmic_bytes={by} GB/s={by / ms / 1e6:.1f}")
