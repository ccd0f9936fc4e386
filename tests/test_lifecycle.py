"""Host-side checks of the informer lifecycle and the round-3 review fixes (no device call): node / NRT deletes in
the derived rows, the reservation `holds` refusals, the reservation-set generation, the argument checks that refuse a
matched pod before any pod is scheduled, the Reservation weight bound, and the library's build dependencies."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, synth
from koordinator_amd.evaluator import KoordEvalError
from oracle.binding import Oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NF_VALID = 1


def _rows(ev, n):
    rows = np.zeros(n, abi.ROW_DTYPE)
    ev._check(ev.lib.ke_debug_rows(ev.h, n, synth.T0, None, abi.ptr(rows)))
    return rows


def test_node_delete_rows_and_readd():
    """ke_node_delete drops NF_VALID from the node's row (every Filter path fails it) and keeps the other caches;
    ke_node_upsert brings the row back equal to the one before the delete."""
    cl = synth.make_cluster(16, synth.BASE_SEED + 1201)
    ev = Evaluator(synth.config(16))
    synth.load_into(ev, cl)
    before = _rows(ev, 16)
    assert (before["flags"] & NF_VALID).all()
    ev.delete_node(3)
    ev.delete_node(3)  # idempotent
    after = _rows(ev, 16)
    assert not after["flags"][3] & NF_VALID
    assert np.array_equal(np.delete(after, 3), np.delete(before, 3))
    ev.upsert_node(3, abi.Node.from_buffer_copy(cl.nodes[3].tobytes()))
    assert np.array_equal(_rows(ev, 16), before)  # NodeMetric and assign cache kept across the delete
    with pytest.raises(KoordEvalError) as e:
        ev.delete_node(16)
    assert e.value.code == abi.ERR_NOT_FOUND
    ev.close()


def test_node_topology_delete_clears_zones_and_cpus():
    cl = synth.make_cluster(12, synth.BASE_SEED + 1202, amplified_fraction=0.5)
    zones, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + 1203)
    ev, o = Evaluator(synth.config(12)), Oracle(synth.config(12), 12)
    for h in (ev, o):
        synth.load_into(h, cl)
        synth.load_numa(h, zones)
        synth.load_cpus(h, tabs)
        h.delete_topology(5)
    for h in (ev, o):
        node, cpus, z, _ = h.node_state(5)
        assert len(cpus) == 0 and len(z) == 0
        assert node.nrt_cpu_amplification_ratio == -2 and node.cpuset_allocated_cpus == 0
    assert ev.node_state(4)[1].shape == o.node_state(4)[1].shape
    ev.close()


@pytest.mark.parametrize("bit", [abi.RSV_HOLDS_NUMA, abi.RSV_HOLDS_CPUSET, abi.RSV_HOLDS_DEVICES,
                                 abi.RSV_OTHER_ALLOCATABLE])
def test_reservation_holds_refused(bit):
    """A reservation whose reserve pod holds a NUMA allocation, a cpuset or devices (or other allocatable names) needs
    the NUMA / DeviceShare restore the ABI does not carry: refused by ke_reservations_load (and the oracle), never
    scheduled around silently."""
    cl = synth.make_cluster(4, synth.BASE_SEED + 1204)
    ev, o = Evaluator(synth.config(4)), Oracle(synth.config(4), 4)
    for h in (ev, o):
        synth.load_into(h, cl)
    r = abi.Reservation(node=1, available=1, holds=bit)
    r.allocatable[0] = 2000
    g = ev.lib.ke_reservations_generation(ev.h)
    with pytest.raises(KoordEvalError) as e:
        ev.reservations_load([r])
    assert e.value.code == abi.ERR_UNSUPPORTED
    with pytest.raises(RuntimeError, match=f"rc={abi.ERR_UNSUPPORTED}"):
        o.reservations_load([r])
    assert ev.lib.ke_reservations_generation(ev.h) == g  # a refused load changes nothing
    r.holds = 0
    ev.reservations_load([r])
    assert ev.lib.ke_reservations_generation(ev.h) == g + 1
    r.holds = 16
    with pytest.raises(KoordEvalError) as e:
        ev.reservations_load([r])
    assert e.value.code == abi.ERR_INVALID
    ev.close()


def test_matched_refusals_precede_every_segment():
    """the refusal of a matched reservation on a NUMA-policy node is an argument check, so a queue
    with plain pods ahead of the matched one fails before the device (here absent: NO_DEVICE would come later)."""
    cl = synth.make_cluster(8, synth.BASE_SEED + 1205)
    ev = Evaluator(synth.config(8))
    synth.load_into(ev, cl)
    node = abi.Node.from_buffer_copy(cl.nodes[2].tobytes())
    node.numa_topology_policy = abi.NUMA_POLICY_RESTRICTED
    ev.upsert_node(2, node)
    ev.reservations_load([abi.Reservation(node=2, available=1), abi.Reservation(node=4, available=1)])
    pods = synth.make_pods(6, synth.BASE_SEED + 1206)
    pods["requests"][:, 2:] = 0
    pods["has_other_requests"] = 0
    pods["device_requests"] = 0
    pods["numa_topology_policy"] = 0
    pods["qos_class"] = abi.QOS_LS
    pods["reservation_matched"][4] = abi.RSV_MATCHED
    with pytest.raises(KoordEvalError) as e:
        ev.schedule(pods, synth.T0, matches=[[], [], [], [], [0, 1], []])
    assert e.value.code == abi.ERR_UNSUPPORTED
    if not ev.device:
        plain = synth.make_pods(9, synth.BASE_SEED + 1207)
        plain["reservation_matched"] = 0
        with pytest.raises(KoordEvalError) as e:  # the refused call consumed its lists: no shape error here
            ev.schedule(plain, synth.T0)
        assert e.value.code == abi.ERR_NO_DEVICE
        with pytest.raises(KoordEvalError) as e:  # without the NUMA-policy node: past the checks, no device here
            ev.schedule(pods, synth.T0, matches=[[], [], [], [], [1], []])
        assert e.value.code == abi.ERR_NO_DEVICE
    ev.close()


def test_reservation_weight_bound():
    cfg = synth.config(4)
    cfg.weight_reservation = (1 << 20) + 1
    h = C.c_void_p()
    lib = abi.load_library()
    assert lib.ke_create(C.byref(cfg), C.byref(h)) == abi.ERR_UNSUPPORTED
    cfg.weight_reservation = 1 << 20
    assert lib.ke_create(C.byref(cfg), C.byref(h)) == abi.OK
    lib.ke_destroy(h)


def test_makefile_rebuilds_kernels_on_every_header():
    """every header ke_kernels.hip includes is a prerequisite of its object (make -n -W <header>
    lists the compile without touching anything)."""
    csrc = os.path.join(ROOT, "koordinator_amd", "csrc")
    src = open(os.path.join(csrc, "ke_kernels.hip")).read()
    local = [ln.split('"')[1] for ln in src.splitlines() if ln.startswith('#include "')]
    assert "ke_merge.h" in local
    for hdr in local:
        out = subprocess.run(["make", "-n", "-C", csrc, "-W", hdr.split("/")[-1] if "/" not in hdr else hdr],
                             capture_output=True, text=True)
        assert "ke_kernels.hip" in out.stdout, (hdr, out.stdout[-500:], out.stderr[-500:])
