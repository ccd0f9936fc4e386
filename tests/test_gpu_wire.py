"""VERDICT r02 item 7 (§8f rank 1 closure): a cluster built only from decoded wire-format objects (Node,
NodeMetric, NodeResourceTopology, Device, bound Pods; tests/wire.py) is scheduled on the GPU path and by the
oracle from the same decoded structs, bit-exact: placements, scores, cpusets, NUMA allocations, device minors,
every node's state afterwards and the replay records."""
import numpy as np
import pytest

import wire
from koordinator_amd import Evaluator, synth
from oracle.binding import Oracle
from test_gpu_release import assert_same_schedule

pytestmark = pytest.mark.gpu
NOW = wire.T0 * 10**9


@pytest.mark.parametrize("seed,devices,numa", [(7, True, True), (8, False, True), (9, True, False)])
def test_schedule_from_decoded_objects(gpu, seed, devices, numa):
    n = 300
    objs = wire.make_objects(n, 1500, 700, seed, devices=devices, numa=numa)
    cfg = synth.config(n)
    ev, o = Evaluator(cfg), Oracle(cfg, n)
    pods = wire.ingest([ev, o], objs, NOW)
    c1, s1 = ev.schedule(pods, NOW)
    c0, s0 = o.schedule(pods, NOW)
    assert_same_schedule(ev, o, c1, s1, c0, s0)
    assert int((c1 >= 0).sum()) > len(pods) // 2
    for i in range(n):
        n1, c_1, z1, d1 = ev.node_state(i)
        n0, c_0, z0, d0 = o.node_state(i)
        assert list(n1.requested) == list(n0.requested), i
        assert np.array_equal(z1["allocated"], z0["allocated"]), i
        assert np.array_equal(d1["used"], d0["used"]), i
    assert ev.check_records(NOW) == 0
    probe = wire.ingest([], wire.make_objects(4, 0, 40, seed + 100, devices=devices, numa=numa), NOW)
    a, b = ev.eval(probe, NOW), o.eval(probe, NOW)
    for k in ("status", "reason", "la", "numa", "ds", "total", "best"):
        assert np.array_equal(a[k], b[k]), k
