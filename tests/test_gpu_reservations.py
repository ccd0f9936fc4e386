"""Reservations on the GPU (first part): with a reservation cache loaded, every pod that
matches no reservation is evaluated against the restored NodeInfo (restoreUnmatchedReservations,
transformer.go:447-473) -- NodeNUMAResource's amplified-cpu Filter and Score and NodeResourcesFitPlus read it --
bit-exact with the oracle on eval matrices and schedules, and again after the reservation set changes."""
import numpy as np
import pytest

from koordinator_amd import abi, synth
from test_gpu_cpuset import assert_eval_equal
from test_gpu_ext import _cluster, _schedule_equal

pytestmark = pytest.mark.gpu


def _reservations(cl, seed, frac=0.4):
    rng = np.random.default_rng(seed)
    rs = []
    for i in range(cl.n_nodes):
        if rng.random() >= frac:
            continue
        for _ in range(int(rng.integers(1, 3))):
            r = abi.Reservation()
            r.node = i
            r.available = int(rng.random() < 0.95)
            r.allocate_once = int(rng.random() < 0.2)
            r.allocated_pods = int(rng.choice([0, 1, 1, 2]))
            for k in range(abi.NRES):
                a = int(cl.nodes["requested"][i, k]) // int(rng.integers(2, 6))
                a = a // 1000 * 1000 if k == 0 else a
                r.allocatable[k] = a
                r.allocated[k] = int(rng.choice([0, a // 2, a, a + (1000 if k == 0 else 2**30)]))
            rs.append(r)
    return rs


def test_reservation_restore_schedule_parity(gpu):
    ev, o, tables = _cluster(500, 941, cpus=True)
    cl = synth.make_cluster(500, synth.BASE_SEED + 941, amplified_fraction=0.2)  # _cluster's nodes
    rs = _reservations(cl, 942)
    for h in (ev, o):
        h.reservations_load(rs)
    pods = synth.add_pod_xres(synth.make_pods(400, synth.BASE_SEED + 943), synth.BASE_SEED + 944)
    assert_eval_equal(ev.eval(pods[:48], synth.T0), o.eval(pods[:48], synth.T0))
    _schedule_equal(ev, o, pods, tables)
    for i in range(0, 500, 37):
        assert ev.node_info_requested(i) == o.node_info_requested(i), i
    # a new reservation set: the restore moves, the rows follow
    rs2 = _reservations(cl, 945, frac=0.6)
    for h in (ev, o):
        h.reservations_load(rs2)
    more = synth.add_pod_xres(synth.make_pods(200, synth.BASE_SEED + 946, key_base=9_900_000_000),
                              synth.BASE_SEED + 947)
    assert_eval_equal(ev.eval(more[:48], synth.T0), o.eval(more[:48], synth.T0))
    c1, s1 = ev.schedule(more, synth.T0)
    c0, s0 = o.schedule(more, synth.T0)
    assert np.array_equal(c1, c0) and np.array_equal(s1, s0)
    assert ev.check_records(synth.T0) == 0
