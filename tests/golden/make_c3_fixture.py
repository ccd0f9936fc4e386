"""Fixture of the headline run (BASELINE.json configs[2], the workload bench.py times): the oracle (oracle/, the
C restatement of the Go plugins) schedules the whole config-3 queue -- 100,000 pods in queue order against the
50,000-node cluster of synth.make_cluster(BASE_SEED + 3), every pod seeing the Reserves of all earlier ones --
and this script stores every placement and its framework score.

  python tests/golden/make_c3_fixture.py [--threads 8]      (about 4-6 minutes on 8 cores)

bench.py compares its timed run with it after the timed region ("parity" in the bench line) and
tests/test_gpu_parity.py::test_c3_full_queue_fixture runs the queue at the driver's call size against it.
The cluster / queue generators are deterministic (numpy PCG64 streams), so the fixture pins the product's
placements to the oracle's for exactly the inputs bench.py builds."""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from koordinator_amd import synth  # noqa: E402
from oracle.binding import Oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "c3_placements.npz")


def inputs_digest(cl, pods):
    """sha256 over the node / pod records the fixture was made from (a generator change shows up here)"""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(cl.nodes).tobytes())
    h.update(np.ascontiguousarray(pods).tobytes())
    return h.hexdigest()


def build_inputs():
    c = synth.CONFIGS[3]
    cl = synth.make_cluster(c["nodes"], synth.BASE_SEED + 3)
    pods = synth.make_pods(c["pods"], synth.BASE_SEED + 100 + 3)
    return cl, pods


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--chunk", type=int, default=5000)
    a = ap.parse_args()
    cl, pods = build_inputs()
    cfg = synth.config(cl.n_nodes)
    o = Oracle(cfg, cl.n_nodes)
    synth.load_into(o, cl)
    chosen = np.empty(len(pods), np.int32)
    score = np.empty(len(pods), np.int32)
    t = time.time()
    for s in range(0, len(pods), a.chunk):  # consecutive calls: the same sequential semantics as one
        c, sc = o.schedule(pods[s:s + a.chunk], synth.T0, n_threads=a.threads)
        chosen[s:s + a.chunk], score[s:s + a.chunk] = c, sc
        print(f"{s + len(c)} pods, {time.time() - t:.0f} s", flush=True)
    np.savez_compressed(OUT, chosen=chosen, score=score.astype(np.int16), digest=np.array(inputs_digest(cl, pods)),
                        nodes=np.int64(cl.n_nodes), pods=np.int64(len(pods)), now_ns=np.int64(synth.T0))
    print(f"wrote {OUT}: placed {(chosen >= 0).sum()} of {len(pods)}")


if __name__ == "__main__":
    main()
