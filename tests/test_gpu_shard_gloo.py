"""The sharded protocol across two real processes: two ranks on one GPU, each with its own
libkoordeval context evaluating half of the nodes, exchange the per-batch candidate lists (all-gather), DeviceShare's
NormalizeScore max and the staged Reservation pick's words (all-reduces) through a gloo process group
(ke_shard_init_host) -- plain, DeviceShare and reservation-matched DeviceShare queues bit-exact with the oracle on
every rank, and the ranks agree.  (The RCCL transport of the same exchange runs in loopback and 1-rank tests; the
multi-GPU RCCL path is the driver's scaling run.)"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_world2_gloo_sharded_schedule(gpu, tmp_path):
    port = _free_port()
    procs, outs = [], []
    for r in range(2):
        out = tmp_path / f"rank{r}.json"
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "shard_gloo_worker.py"), str(r), "2",
                                       str(port), str(out)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=170)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for r, p in enumerate(procs):
        assert p.returncode == 0, logs[r][-3000:]
    res = [json.loads(o.read_text()) for o in outs]
    for r in res:
        assert r["ranks_agree"]
        for k in ("plain", "deviceshare", "reservations"):
            assert r[k]["ok"] and r[k]["placed"] > 0, (k, r[k])
    assert res[0]["plain"]["range"] != res[1]["plain"]["range"]  # each rank evaluated its own shard
    assert res[0]["reservations"]["into_rsv"] > 0
