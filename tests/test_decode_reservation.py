"""Reservation CRD decoder (ke_decode_reservation, SURVEY.md §8f ranks 1 + 3): the object as the reservation cache
builds its ReservationInfo (frameworkext/reservation_info.go:87-130) -- availability, ReservationRequests
(util/reservation/reservation.go:393-404), the Restricted options' ResourceNames (:637-654), rInfo.Reserved
(util/node.go:85-120), allocateOnce's default, the order label -- and the reserve pod's holdings from its
device-allocated / resource-status annotations, so no caller flag decides what scoreReservation / fitsReservation
read.  Host-only: no device needed."""
import json

import numpy as np
import pytest

from koordinator_amd import abi, decode
from koordinator_amd.decode import DecodeError

NAMES = [None] * 16
for i, n in {2: "ephemeral-storage", 10: "koordinator.sh/gpu-core", 11: "koordinator.sh/gpu-memory-ratio",
             12: "koordinator.sh/gpu-memory", 13: "koordinator.sh/rdma"}.items():
    NAMES[i] = n
GI = 2**30


def gpu_reservation(**kw):
    alloc = {"cpu": "4", "memory": "8Gi", "koordinator.sh/gpu-core": "100", "koordinator.sh/gpu-memory-ratio": "100",
             "koordinator.sh/gpu-memory": "80Gi", "koordinator.sh/rdma": "50", "pods": "4"}
    r = {"apiVersion": "scheduling.koordinator.sh/v1alpha1", "kind": "Reservation",
         "metadata": {"name": "r1", "uid": "8b1d6c3e-0000-4000-8000-000000000001",
                      "labels": {"scheduling.koordinator.sh/reservation-order": "7"},
                      "annotations": {
                          "scheduling.koordinator.sh/device-allocated": json.dumps({
                              "gpu": [{"minor": 3, "resources": {"koordinator.sh/gpu-core": "100",
                                                                 "koordinator.sh/gpu-memory": "80Gi",
                                                                 "koordinator.sh/gpu-memory-ratio": "100"}}],
                              "rdma": [{"minor": 1, "resources": {"koordinator.sh/rdma": "50"}}]}),
                          "scheduling.koordinator.sh/resource-status": json.dumps({
                              "cpuset": "0-3", "numaNodeResources": [{"node": 1, "resources": {"cpu": "4", "memory": "8Gi"}}]})}},
         "spec": {"allocatePolicy": "Aligned", "template": {"spec": {"containers": [{"resources": {"requests": alloc}}]}},
                  "owners": [{"labelSelector": {"matchLabels": {"app": "x"}}}]},
         "status": {"phase": "Available", "nodeName": "node-7", "allocatable": alloc,
                    "allocated": {"cpu": "1", "memory": "2Gi", "koordinator.sh/gpu-core": "50"},
                    "currentOwners": [{"name": "p1", "namespace": "default", "uid": "u1"}]}}
    for k, v in kw.items():
        r[k] = v
    return r


def test_gpu_reservation_decodes_allocatable_and_holdings():
    r, a, res, node = decode.decode_reservation(gpu_reservation(), NAMES)
    assert node == "node-7" and r.node == -1 and r.available == 1 and r.allocate_once == 1
    assert r.allocate_policy == abi.RSV_POLICY_ALIGNED and r.order == 7 and r.allocated_pods == 1 and r.uid != 0
    assert list(r.allocatable) == [4000, 8 * GI] and list(r.allocated) == [1000, 2 * GI]
    got = {int(e["id"]): (int(e["allocatable"]), int(e["allocated"])) for e in res}
    assert got == {abi.RSV_RES_PODS: (4, 0), 10: (100, 50), 11: (100, 0), 12: (80 * GI, 0), 13: (50, 0)}
    assert r.holds == abi.RSV_HOLDS_NUMA | abi.RSV_HOLDS_CPUSET | abi.RSV_HOLDS_DEVICES | abi.RSV_OTHER_ALLOCATABLE
    assert int(a["device_minors"]) == (1 << 3) | (1 << 17)
    assert list(a["device"][abi.DEV_GPU, 3]) == [100, 80 * GI, 100] and a["device"][abi.DEV_RDMA, 1, 0] == 50
    assert int(a["cpuset"][0]) == 0xF and a["numa"][2] == 4000 and a["numa"][3] == 8 * GI
    assert not a["owner_device"].any() and not a["owner_cpuset"].any()


def test_decoded_reservation_loads():
    """the decoded record, its holdings and entries are what ke_reservations_load_full accepts"""
    from koordinator_amd import Evaluator, synth
    r, a, res, _ = decode.decode_reservation(gpu_reservation(), NAMES)
    r.node = 0
    ev = Evaluator(synth.config(4))
    synth.load_into(ev, synth.make_cluster(4, synth.BASE_SEED + 17))
    ev.reservations_load([r], np.array([a]), [res])
    assert {int(e["id"]) for e in ev.reservation_resources_get(0)} == {int(e["id"]) for e in res}
    ev.close()


def test_restricted_options_and_node_reservation():
    obj = gpu_reservation()
    obj["spec"]["allocatePolicy"] = "Restricted"
    obj["metadata"]["annotations"]["scheduling.koordinator.sh/reservation-restricted-options"] = json.dumps(
        {"resources": ["cpu", "koordinator.sh/gpu-core"]})
    obj["metadata"]["annotations"]["node.koordinator.sh/reservation"] = json.dumps(
        {"resources": {"memory": "1Gi", "koordinator.sh/rdma": "10"}, "reservedCPUs": "0-1"})
    r, a, res, _ = decode.decode_reservation(obj, NAMES)
    assert r.allocate_policy == abi.RSV_POLICY_RESTRICTED
    assert r.names_excluded == 1 << abi.RES_MEMORY  # memory left out of ResourceNames
    assert list(r.allocated) == [1000, 0]  # Mask(owners' requests, ResourceNames)
    assert list(r.reserved) == [2000, GI]  # |reservedCPUs| overrides the cpu quantity
    ex = {int(e["id"]): (int(e["excluded"]), int(e["reserved"])) for e in res}
    assert ex[10] == (0, 0) and ex[13] == (1, 10) and ex[abi.RSV_RES_PODS] == (1, 0)
    # an options list naming none of the allocatable names keeps them all (GetReservationRestrictedResources)
    obj["metadata"]["annotations"]["scheduling.koordinator.sh/reservation-restricted-options"] = json.dumps(
        {"resources": ["example.com/none"]})
    r, _, res, _ = decode.decode_reservation(obj, NAMES)
    assert r.names_excluded == 0 and not res["excluded"].any()
    # a malformed one is a ParseError: the reservation takes no part
    obj["metadata"]["annotations"]["scheduling.koordinator.sh/reservation-restricted-options"] = "{"
    r, *_ = decode.decode_reservation(obj, NAMES)
    assert r.available == 0


def test_pending_reservation_reads_its_template():
    obj = gpu_reservation()
    obj["status"] = {"phase": "Pending"}
    obj["spec"]["allocateOnce"] = False
    obj["spec"]["template"]["spec"]["containers"] = [{"resources": {"requests": {"cpu": "2", "memory": "1Gi"}}},
                                                     {"resources": {"requests": {"cpu": "500m"}}}]
    r, _, res, node = decode.decode_reservation(obj, NAMES)
    assert r.available == 0 and node == "" and r.allocate_once == 0
    assert list(r.allocatable) == [2500, GI] and len(res) == 0 and not (r.holds & abi.RSV_OTHER_ALLOCATABLE)


@pytest.mark.parametrize("mutate,code", [
    (lambda o: o["status"]["allocatable"].update({"example.com/foo": "1"}), abi.ERR_UNSUPPORTED),  # no resource id
    (lambda o: o["spec"].update({"allocatePolicy": "Greedy"}), abi.ERR_UNSUPPORTED),
    (lambda o: o["metadata"]["annotations"].update({"scheduling.koordinator.sh/device-allocated": "{"}), abi.ERR_INVALID),
    (lambda o: o["metadata"]["annotations"].update({"scheduling.koordinator.sh/device-allocated":
                                                    json.dumps({"npu": [{"minor": 0, "resources": {}}]})}),
     abi.ERR_UNSUPPORTED),
    (lambda o: o["metadata"]["annotations"].update({"scheduling.koordinator.sh/resource-status":
                                                    json.dumps({"cpuset": "3-1"})}), abi.ERR_INVALID),
    (lambda o: o["spec"].update({"allocateOnce": "yes"}), abi.ERR_INVALID),
], ids=["unnamed-resource", "policy", "device-json", "device-type", "cpuset", "allocate-once"])
def test_reservation_decode_refusals(mutate, code):
    obj = gpu_reservation()
    mutate(obj)
    with pytest.raises(DecodeError) as e:
        decode.decode_reservation(obj, NAMES)
    assert e.value.code == code
