"""One rank of the world-2 sharded test (tests/test_gpu_shard_gloo.py): a gloo process group on 127.0.0.1, an
Evaluator on cuda:0 whose node shard exchanges its candidate lists / maxima / Reservation-pick words with the other
rank through libkoordeval's host-collective hook (ke_shard_init_host), three queues -- plain, DeviceShare and
reservation-matched DeviceShare -- each compared with this rank's oracle.  argv: rank world port out.json"""
import json
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__)), os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import ds_rsv_cases as dc  # noqa: E402
from koordinator_amd import Evaluator, abi, shard, synth  # noqa: E402
from oracle.binding import Oracle  # noqa: E402


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    coll = shard.gloo_collective()
    res = {}

    def run(name, ev, o, pods, matches=None):
        ev.shard_init_host(rank, world, coll)
        c1, s1 = ev.schedule(pods, synth.T0, matches=matches)
        c0, s0 = o.schedule(pods, synth.T0, matches=matches)
        ok = bool(np.array_equal(c1, c0) and np.array_equal(s1, s0))
        a1, a0 = ev.last_allocations(), o.last_allocations()
        ok = ok and bool(np.array_equal(a1["device_minors"], a0["device_minors"]))
        ok = ok and bool(np.array_equal(a1["reservation"], a0["reservation"]))
        lo, hi = ev.shard_range()
        res[name] = {"ok": ok, "placed": int((c1 >= 0).sum()), "range": [lo, hi],
                     "into_rsv": int((a1["reservation"] > 0).sum()), "chosen_sum": int(c1.sum())}

    n = 1200  # > 2 shards of 512-aligned ranges
    cl = synth.make_cluster(n, synth.BASE_SEED + 8101)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
    run("plain", ev, o, synth.make_pods(600, synth.BASE_SEED + 8102))
    ev.close()

    devs = synth.make_devices(n, synth.BASE_SEED + 8103)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_devices(h, devs)
    run("deviceshare", ev, o, synth.make_ds_pods(300, synth.BASE_SEED + 8104))
    ev.close()

    (ev, o), pods, matches, rs = dc.setup(lambda c, m: [Evaluator(c), Oracle(c, m)], n, 8105, 300, affinity=0.3)
    run("reservations", ev, o, pods, matches)
    ev.close()

    # both ranks agree (each rank replays every Reserve identically)
    mine = [res[k]["chosen_sum"] for k in sorted(res)]
    allv = [None] * world
    dist.all_gather_object(allv, mine)
    res["ranks_agree"] = all(v == allv[0] for v in allv)
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()
    return 0 if res["ranks_agree"] and all(r["ok"] for k, r in res.items() if k != "ranks_agree") else 1


if __name__ == "__main__":
    sys.exit(main())
