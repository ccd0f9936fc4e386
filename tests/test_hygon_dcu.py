"""Hygon DCU requests (dcu.com/gpu): a GPU request converted like nvidia.com/gpu / amd.com/gpu -- gpu-core =
gpu-memory-ratio = 100 x the count (ConvertDeviceRequest, deviceshare/utils.go:190-212; ValidDeviceResourceCombinations
HygonDCU: DefaultTrue, :91).  The reference's tests hold no DCU vector, so parity rests on that equivalence: a queue
whose whole-GPU requests name dcu.com/gpu schedules exactly as the same queue naming nvidia.com/gpu (oracle here, the
product on the GPU), and a DCU request mixed with another GPU name is invalid (no combination entry)."""
import numpy as np
import pytest

from koordinator_amd import Evaluator, abi, decode, synth
from oracle.binding import Oracle

NV, AMD, DCU = abi.PDR["nvidia.com/gpu"], abi.PDR["amd.com/gpu"], abi.PDR["dcu.com/gpu"]


def _cluster(n, seed):
    cl = synth.make_cluster(n, seed)
    devices = synth.make_devices(n, seed + 50)
    return cl, devices


def _renamed(pods, to, every=1):
    """the queue with every `every`-th whole-GPU (nvidia.com/gpu) request moved to the name `to`"""
    out = pods.copy()
    idx = np.flatnonzero(out["device_requests"][:, NV] > 0)[::every]
    out["device_requests"][idx, to] = out["device_requests"][idx, NV]
    out["device_requests"][idx, NV] = 0
    return out, idx


def _load(h, cl, devices):
    synth.load_into(h, cl)
    synth.load_devices(h, devices)
    return h


def test_dcu_schedules_like_nvidia_gpu_oracle(lib):
    n, p = 300, 160
    cl, devices = _cluster(n, synth.BASE_SEED + 901)
    pods = synth.make_ds_pods(p, synth.BASE_SEED + 902, device_fraction=0.7)
    cfg = synth.config(n)
    dcu, idx = _renamed(pods, DCU)
    assert len(idx) >= 10
    mixed, _ = _renamed(pods, AMD, every=2)
    mixed, _ = _renamed(mixed, DCU)
    res = []
    for q in (pods, dcu, mixed):
        o = _load(Oracle(cfg, n), cl, devices)
        c, s = o.schedule(q, synth.T0, n_threads=8)
        res.append((c, s, o.last_device_allocations.copy()))
    for c, s, d in res[1:]:
        assert np.array_equal(c, res[0][0]) and np.array_equal(s, res[0][1]) and np.array_equal(d, res[0][2])
    assert np.any(res[0][2][idx] != 0)  # the renamed pods took devices


def test_dcu_mixed_with_another_gpu_name_is_invalid(lib):
    n = 64
    cl, devices = _cluster(n, synth.BASE_SEED + 903)
    pods = synth.make_ds_pods(8, synth.BASE_SEED + 904, device_fraction=0.0)
    pods["device_requests"] = 0
    pods["device_requests"][0, DCU] = 1
    pods["device_requests"][1, DCU] = 1
    pods["device_requests"][1, NV] = 1
    pods["device_requests"][2, DCU] = 1
    pods["device_requests"][2, abi.PDR["koordinator.sh/gpu-core"]] = 100
    o = _load(Oracle(synth.config(n), n), cl, devices)
    e = o.eval(pods[:3], synth.T0)
    assert (e["status"][0] == abi.CODE_SUCCESS).any()
    for i in (1, 2):
        assert (e["status"][i] == abi.CODE_UNSCHEDULABLE_AND_UNRESOLVABLE).all()


def test_decoder_reads_dcu_and_refuses_npu(lib):
    doc = {"metadata": {"name": "p", "namespace": "ns", "uid": "u"},
           "spec": {"containers": [{"name": "c", "resources": {"requests": {"cpu": "1", "dcu.com/gpu": "2"}}}]}}
    p = decode.decode_pod(doc)
    assert p.device_requests[DCU] == 2 and p.has_unsupported_device_requests == 0
    doc["spec"]["containers"][0]["resources"]["requests"]["huawei.com/npu-core"] = "1"
    assert decode.decode_pod(doc).has_unsupported_device_requests == 1


@pytest.mark.gpu
def test_dcu_queue_parity(gpu):
    n, p = 2000, 256
    cl, devices = _cluster(n, synth.BASE_SEED + 905)
    pods = synth.make_ds_pods(p, synth.BASE_SEED + 906, device_fraction=0.6)
    q, idx = _renamed(pods, DCU, every=2)
    q, _ = _renamed(q, AMD)
    assert len(idx) >= 5
    cfg = synth.config(n)
    ev, o = _load(Evaluator(cfg), cl, devices), _load(Oracle(cfg, n), cl, devices)
    c1, s1 = ev.schedule(q, synth.T0)
    c0, s0 = o.schedule(q, synth.T0, n_threads=16)
    assert np.array_equal(c1, c0), np.argwhere(c1 != c0)[:5].ravel().tolist()
    assert np.array_equal(s1, s0)
    assert np.array_equal(ev.last_device_allocations, o.last_device_allocations)
    assert np.any(ev.last_device_allocations[idx] != 0)
    ev.close()
