"""DeviceShare hints on the oracle, pinned by the reference's own tests
(tests/golden/ds_hints.json): TestAutopilotAllocator's VF / joint GPU+RDMA / well-planned cases and
DefaultDeviceHandler's ApplyForAll / RequestsAsCount / DeviceLevel cases.  The GPU path is compared with the
oracle on the same objects in tests/test_gpu_ds_hints.py."""
import numpy as np
import pytest

import cases
import ds_hint_cases as dh
from koordinator_amd import abi, model
from oracle.binding import Oracle


@pytest.mark.parametrize("case", [c for c in dh.HINTS if c["kind"] == "autopilot"], ids=lambda c: c["name"])
def test_autopilot_allocator(lib, case):
    o = Oracle(abi.default_config(1), 1)
    dh.node_cluster(o)
    dh.build(o, case)
    pod, hint = dh.pod_and_hints(case)
    o.set_pod_device_hints([hint])
    st, reason, out, vf = o.ds_allocate(pod, 0)  # Allocate outside Reserve, no scorer (the test's allocator)
    assert st == 0, (case["source"], reason)
    gpu = [m for m in range(16) if (out[0] >> m) & 1]
    assert gpu == case["want"]["gpu"], case["source"]
    rdma = [[m, int(vf[0][m])] for m in range(16) if (out[1] >> m) & 1]
    want = [[m, dh.vf_rank(case["device"], m, bus)] for m, bus in case["want"]["rdma"]]
    assert rdma == want, case["source"]


@pytest.mark.parametrize("case", [c for c in dh.HINTS if c["kind"] == "handler"], ids=lambda c: c["name"])
def test_default_device_handler(lib, case):
    o = Oracle(abi.default_config(1), 1)
    dh.node_cluster(o)
    dh.build(o, case)
    pod, hint = dh.pod_and_hints(case)
    o.set_pod_device_hints([hint])
    st, reason, out, vf = o.ds_allocate(pod, 0)
    w = case["want"]
    if not w["ok"]:
        assert st == abi.CODE_UNSCHEDULABLE_AND_UNRESOLVABLE and reason == abi.REASON_DS_INSUFFICIENT_RDMA
        return
    assert st == 0 and bin(int(out[1])).count("1") == w["count"], case["source"]
    c, s = o.schedule([pod], cases.NOW)  # Reserve: each allocated device's used grows by the per-device amount
    assert c[0] == 0
    _, _, _, devs = o.node_state(0)
    used = [int(d["used"][0]) for d in devs if d["type"] == abi.DEV_RDMA and d["has_used"][0]]
    assert used == [w["per_device"]] * w["count"], case["source"]


def test_hints_decode_like_the_model(lib):
    from koordinator_amd import decode
    doc = {"metadata": {"name": "p", "namespace": "n", "annotations": {
        "scheduling.koordinator.sh/device-allocate-hint":
            '{"rdma":{"selector":{"matchLabels":{"type":"fakeW"}},"vfSelector":{"matchExpressions":[{"key":"type",'
            '"operator":"In","values":["general","fakeG"]}]},"allocateStrategy":"RequestsAsCount",'
            '"exclusivePolicy":"DeviceLevel"},"npu":{"selector":{}}}',
        "scheduling.koordinator.sh/device-joint-allocate": '{"deviceTypes":["gpu","rdma"],"requiredScope":"SamePCIe"}'}},
        "spec": {"containers": [{"resources": {"requests": {"nvidia.com/gpu": "1", "koordinator.sh/rdma": "1"}}}]}}
    got = decode.decode_pod_device_hints(doc)
    want = model.make_device_hints({"rdma": {"selector": {"matchLabels": {"type": "fakeW"}},
                                             "vfSelector": {"matchExpressions": [{"key": "type", "operator": "In",
                                                                                  "values": ["general", "fakeG"]}]},
                                             "allocateStrategy": "RequestsAsCount", "exclusivePolicy": "DeviceLevel"},
                                    "npu": {"selector": {}}},
                                   {"deviceTypes": ["gpu", "rdma"], "requiredScope": "SamePCIe"})
    assert bytes(got) == bytes(want)
    assert decode.decode_pod_device_hints({"metadata": {"name": "x"}}) is None
    bad = {"metadata": {"annotations": {"scheduling.koordinator.sh/device-allocate-hint":
                                        '{"rdma":{"selector":{"matchExpressions":[{"key":"a","operator":"In"}]}}}'}}}
    assert decode.decode_pod_device_hints(bad).invalid == 1  # In without values: LabelSelectorAsSelector fails
    w, k = decode.decode_device_flags({"metadata": {"labels": {"node.koordinator.sh/secondary-device-well-planned": "true"}}},
                                      {"metadata": {"labels": {"node.koordinator.sh/gpu-vendor": "nvidia",
                                                               "node.koordinator.sh/gpu-model": "A100"}}})
    assert w and k == decode.label_id("nvidia-A100")


@pytest.mark.parametrize("case", [c for c in dh.HINTS if c["kind"] == "numa_hints"], ids=lambda c: c["name"])
def test_numa_hints_with_device_hints(lib, case):
    o = Oracle(abi.default_config(1), 1)
    dh.node_cluster(o)
    dh.build(o, case)
    pod, hint = dh.pod_and_hints(case)
    o.set_pod_device_hints([hint])
    st, reason, none, copies, hints = o.ds_numa_hints(pod, 0)
    assert st == 0 and not none, (case["source"], reason)
    assert copies == case["want"]["copies"], case["source"]
    assert [list(h) for h in hints] == case["want"]["hints"], case["source"]
