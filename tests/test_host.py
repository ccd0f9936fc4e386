"""CPU-side tests of the product library: the C ABI loads and exports what include/koord_eval.h
declares, the binding layouts match, the host-side logic (estimator, threshold folding, validation)
matches the oracle / golden vectors, and evaluation without a device fails loudly (no CPU path)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import cases
from koordinator_amd import Evaluator, KoordEvalError, abi, model
from oracle.binding import Oracle, usage_percent

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "koord_eval.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[\w\s\*]+?\b(ke_\w+)\s*\(", src, flags=re.M)))


def test_exports_every_header_symbol(lib):
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"{n} declared in include/koord_eval.h but not exported"
        assert n in abi.EXPORTS, f"{n} not bound in koordinator_amd/abi.py"


def test_struct_layouts(lib):
    sizes = (abi.i32 * len(abi.STRUCTS))()
    assert lib.ke_abi_struct_sizes(sizes, len(abi.STRUCTS)) == len(abi.STRUCTS)
    for s, n in zip(abi.STRUCTS, sizes):
        assert C.sizeof(s) == n, s.__name__
    assert lib.ke_row_bytes() == 18 * 8 + 4


@pytest.mark.parametrize("case", cases.load("estimator.json"), ids=lambda c: c["name"])
def test_product_estimator_golden(case):
    ev = Evaluator(cases.make_cfg(case))
    est = ev.estimate_pod(cases.make_pod(case["pod"]))
    assert list(est) == [case["want"]["cpu"], case["want"]["memory"]], case["source"]


def test_product_estimator_matches_oracle_random():
    rng = np.random.default_rng(7)
    cfg = abi.default_config(1)
    cfg.loadaware.allow_customize_estimation = 1
    ev, o = Evaluator(cfg), Oracle(cfg, 1)
    for i in range(2000):
        kind = rng.integers(0, 5)
        req_cpu, req_mem = int(rng.integers(0, 64000)), int(rng.integers(0, 2**37))
        lim_cpu = req_cpu * int(rng.integers(0, 3))
        lim_mem = req_mem * int(rng.integers(0, 3))
        if kind == 0:
            p = model.make_pod(requests={"cpu": f"{req_cpu}m", "memory": str(req_mem)},
                               limits={"cpu": f"{lim_cpu}m", "memory": str(lim_mem)})
        elif kind == 1:
            p = model.make_pod(requests={"kubernetes.io/batch-cpu": str(req_cpu), "kubernetes.io/batch-memory": str(req_mem)},
                               limits={"kubernetes.io/batch-cpu": str(lim_cpu)}, priority=5500)
        elif kind == 2:
            p = model.make_pod(requests={"kubernetes.io/mid-cpu": str(req_cpu)}, priority=7500)
        elif kind == 3:
            p = model.make_pod(requests={"cpu": f"{req_cpu}m"}, priority=3500)  # koord-free
        else:
            p = model.make_pod(requests={"cpu": f"{req_cpu}m", "memory": str(req_mem)}, priority=9500,
                               custom_factors={"cpu": int(rng.integers(1, 200))})
        assert list(ev.estimate_pod(p)) == list(o.estimate_pod(p))


def test_threshold_fold_is_exact():
    """U*(total,thr) from the product = the last `used` the reference's f64 rounding accepts."""
    rng = np.random.default_rng(3)
    lib = abi.load_library()
    totals = [1, 3, 7, 100, 96000, 128000, 2**30, 512 * 2**30, 1024 * 2**30 + 12345] + \
             [int(x) for x in rng.integers(1, 2**44, 200)]
    for total in totals:
        for thr in [1, 5, 50, 65, 80, 95, 99, 100, int(rng.integers(1, 101))]:
            u = lib.ke_debug_usage_bound(total, thr)
            assert usage_percent(u, total) <= thr < usage_percent(u + 1, total), (total, thr, u)


def test_eval_without_device_fails_loudly(lib):
    if lib.ke_device_available():
        pytest.skip("device present")
    ev = Evaluator(abi.default_config(4))
    ev.upsert_node(0, model.make_node(allocatable={"cpu": "8", "memory": "8Gi"}))
    with pytest.raises(KoordEvalError) as e:
        ev.eval([model.make_pod(requests={"cpu": "1"})], cases.NOW)
    assert e.value.code == abi.ERR_NO_DEVICE
    with pytest.raises(KoordEvalError):
        ev.schedule([model.make_pod(requests={"cpu": "1"})], cases.NOW)


def test_unsupported_inputs_are_rejected():
    ev = Evaluator(abi.default_config(4))
    ev.upsert_node(0, model.make_node(allocatable={"cpu": "8", "memory": "8Gi"}))
    n = model.make_node(allocatable={"cpu": "8"})
    n.cpu_bind_policy = 5
    with pytest.raises(KoordEvalError) as e:
        ev.upsert_node(1, n)
    assert e.value.code == abi.ERR_INVALID
    n.cpu_bind_policy = abi.NODE_CPU_BIND_FULL_PCPUS_ONLY  # cpuset binding forced by the node: accepted
    ev.upsert_node(1, n)
    n.cpu_bind_policy = 0
    n.numa_topology_policy = 7
    with pytest.raises(KoordEvalError) as e:
        ev.upsert_node(1, n)
    assert e.value.code == abi.ERR_INVALID
    # a NUMA-policy node is accepted (DeviceShare pods meet it as a second NUMA hint provider)
    n.numa_topology_policy = abi.NUMA_POLICY_RESTRICTED
    ev.upsert_node(1, n)
    bad_spec = model.make_pod(requests={"cpu": "2"})
    bad_spec.has_resource_spec = 1
    with pytest.raises(KoordEvalError) as e:
        ev.eval([bad_spec], cases.NOW)
    assert e.value.code == abi.ERR_UNSUPPORTED
    # CPU tables: ids unique and in range; a regular topology (same CPUs per core, one socket / NUMA
    # node per core)
    topo = [(c, c // 2, 0, 0) for c in range(8)]
    ev.set_cpus(0, model.make_cpus(topo))
    with pytest.raises(KoordEvalError) as e:
        ev.set_cpus(0, model.make_cpus(topo + [(3, 1, 0, 0)]))
    assert e.value.code == abi.ERR_INVALID
    with pytest.raises(KoordEvalError) as e:
        ev.set_cpus(0, model.make_cpus(topo + [(8, 4, 0, 0)]))
    assert e.value.code == abi.ERR_UNSUPPORTED
    with pytest.raises(KoordEvalError) as e:
        ev.set_cpus(0, model.make_cpus([(0, 0, 0, 0), (1, 0, 1, 0)]))
    assert e.value.code == abi.ERR_UNSUPPORTED
    ev.set_cpus(0, model.make_cpus([]))
    # zones: ids ascending, cpuset CPUs only inside an allocation entry
    z = model.make_zones([{"id": 1, "cpu": "4"}, {"id": 0, "cpu": "4"}])
    with pytest.raises(KoordEvalError) as e:
        ev.set_numa(1, z)
    assert e.value.code == abi.ERR_INVALID
    z = model.make_zones([{"id": 0, "cpu": "4", "cpuset_cpus": 2}])
    with pytest.raises(KoordEvalError) as e:
        ev.set_numa(1, z)
    assert e.value.code == abi.ERR_INVALID
    bad = abi.default_config(4)
    bad.abi_version = 99
    with pytest.raises(KoordEvalError):
        Evaluator(bad)


def _unsupported(fn, *args):
    with pytest.raises(KoordEvalError) as e:
        fn(*args)
    assert e.value.code == abi.ERR_UNSUPPORTED, str(e.value)


GPU2 = {"nvidia.com/gpu": "2"}


@pytest.mark.parametrize("kind", ["gpu_vf", "gpu_secondary", "three_types", "bad_index"])
def test_unmodelled_device_hints_are_refused(kind):
    """The DeviceShare hint paths outside the modelled allocator fail loudly: a VFSelector on the gpu type
    (defaultAllocateDevices' GPU VFs), a joint allocation with the gpu type after the primary or over three
    types (device_allocator.go:205-300), and a hint index outside the table."""
    ev = Evaluator(abi.default_config(4))
    ev.upsert_node(0, model.make_node(allocatable={"cpu": "8", "memory": "8Gi"}))
    req = dict(GPU2, **{"koordinator.sh/rdma": "1"})
    hints, joint = {}, None
    if kind == "gpu_vf":
        hints = {"gpu": {"vfSelector": {}}}
    elif kind == "gpu_secondary":
        joint = {"deviceTypes": ["rdma", "gpu"]}
    elif kind == "three_types":
        req["koordinator.sh/fpga"] = "1"
        joint = {"deviceTypes": ["gpu", "rdma", "fpga"]}
    pod = model.make_pod(requests=req, device_hints=hints)
    ev.set_pod_device_hints([model.make_device_hints(hints, joint)])
    pod.device_hint = 5 if kind == "bad_index" else 1
    with pytest.raises(KoordEvalError) as e:
        ev.schedule([pod], cases.NOW)
    assert e.value.code == (abi.ERR_INVALID if kind == "bad_index" else abi.ERR_UNSUPPORTED), str(e.value)


def test_joint_allocate_of_one_requested_type_is_dropped():
    """parsePodDeviceShareExtensions keeps only requested types without an ApplyForAll hint (utils.go:428-441):
    a joint spec naming only unrequested types carries nothing."""
    pod = model.make_pod(requests=GPU2, device_joint_allocate={"deviceTypes": ["rdma"]})
    assert pod.device_joint_allocate == 0
    pod = model.make_pod(requests=GPU2, device_hints={"gpu": {"requiredTopologyScope": "PCIe"}})
    assert pod.device_hints == 0 and pod.gpu_required_topology_scope == abi.SCOPE_PCIE


@pytest.mark.parametrize("which", ["loadaware", "numa", "deviceshare"])
def test_args_with_other_resource_keys_are_refused(which):
    """pkg/scheduler/apis/config/types.go:31-125: the args are maps; keys beyond the modelled ones fail."""
    cfg = abi.default_config(4)
    getattr(cfg, which).has_other_keys = 1
    _unsupported(Evaluator, cfg)


def test_gpu_partition_tables_validated():
    ev = Evaluator(abi.default_config(4))
    ev.upsert_node(0, model.make_node(allocatable={"cpu": "8", "memory": "8Gi"}))
    has, honor, parts = model.gpu_partition_state(node_labels={"node.koordinator.sh/gpu-model": "H800"})
    assert has and not honor and len(parts) == 15
    ev.set_gpu_partitions(0, has, honor, parts)
    ev.set_gpu_partitions(1, has, True, parts)  # same table: interned once
    ev.set_gpu_partitions(2, True, False, None)  # empty table: indexer present, every count unsupported
    big = model.make_gpu_partitions({1: [[m] for m in range(13)]})  # 13 in one group: Go's sort is unstable
    _unsupported(ev.set_gpu_partitions, 0, True, False, big)
    bad = model.make_gpu_partitions({1: [[16]]})
    with pytest.raises(KoordEvalError) as e:
        ev.set_gpu_partitions(0, True, False, bad)
    assert e.value.code == abi.ERR_INVALID
    assert model.gpu_partition_state(node_labels={"node.koordinator.sh/gpu-model": "A100"})[0] is False


def test_host_rows_fold_loadaware_terms():
    """The row the host derives for a golden case reproduces the Go score arithmetic."""
    case = [c for c in cases.load("loadaware_score.json") if c["name"] == "score load node"][0]
    ev = Evaluator(cases.make_cfg(case))
    pod = cases.setup_loadaware(ev, case)
    _, rows = ev.debug_rows(cases.NOW, device=False)
    f = rows[0]["f"]
    est = ev.estimate_pod(pod)
    cap = f[9:11]
    sa_np = f[5:7]
    s = [((sa_np[r] - est[r]) * 100) // cap[r] for r in range(2)]
    assert (s[0] + s[1]) // 2 == case["want"]["score"]
