"""Pin the oracle: every known-answer vector transcribed from the reference's Go tests
(tests/golden/) must come out of the CPU restatement unchanged."""
import numpy as np
import pytest

import cases
from oracle.binding import Oracle

LA_FILTER = cases.load("loadaware_filter.json")
LA_SCORE = cases.load("loadaware_score.json")
EST = cases.load("estimator.json")
NUMA = cases.load("numa.json")


@pytest.mark.parametrize("case", LA_FILTER, ids=[c["name"] for c in LA_FILTER])
def test_loadaware_filter(case):
    o = Oracle(cases.make_cfg(case), 1)
    pod = cases.setup_loadaware(o, case)
    code, reason = o.la_filter(pod, 0, cases.NOW)
    assert (code, reason) == (case["want"]["code"], case["want"]["reason"]), case["source"]


@pytest.mark.parametrize("case", LA_SCORE, ids=[c["name"] for c in LA_SCORE])
def test_loadaware_score(case):
    o = Oracle(cases.make_cfg(case), 1)
    pod = cases.setup_loadaware(o, case)
    assert o.la_score(pod, 0, cases.NOW) == case["want"]["score"], case["source"]


@pytest.mark.parametrize("case", EST, ids=[c["name"] for c in EST])
def test_estimator(case):
    o = Oracle(cases.make_cfg(case), 1)
    est = o.estimate_pod(cases.make_pod(case["pod"]))
    assert list(est) == [case["want"]["cpu"], case["want"]["memory"]], case["source"]


@pytest.mark.parametrize("case", NUMA, ids=[c["name"] for c in NUMA])
def test_numa(case):
    nodes = cases.make_numa_nodes(case)
    o = Oracle(cases.make_cfg(case, len(nodes)), len(nodes))
    for i, n in enumerate(nodes):
        o.upsert_node(i, n)
    pod = cases.make_pod(case["pod"])
    if case["op"] == "score":
        got = [o.numa_score(pod, i) for i in range(len(nodes))]
        assert got == case["want"]["scores"], case["source"]
    else:
        code, reason = o.numa_filter(pod, 0)
        assert (code, reason) == (case["want"]["code"], case["want"]["reason"]), case["source"]


# ---- DeviceShare ---------------------------------------------------------------------------------
DS = cases.load("deviceshare.json")
TYPES = {"gpu": 0, "rdma": 1, "fpga": 2}


@pytest.mark.parametrize("case", DS, ids=[c["name"] for c in DS])
def test_deviceshare(case):
    from koordinator_amd import abi, model
    from oracle.binding import normalize_scores

    op, want = case["op"], case["want"]
    if op == "normalize":
        assert list(normalize_scores(case["raw"])) == want["scores"], case["source"]
        return
    o = Oracle(cases.ds_cfg(case), 1)
    if op == "score_device":
        r = o.ds_score_device(abi.DEV_GPU, cases.rl3(abi.DEV_GPU, case["request"]),
                              cases.rl3(abi.DEV_GPU, case["total"]), cases.rl3(abi.DEV_GPU, case["free"]))
        assert r == want["score"], case["source"]
        return
    if op == "prefilter":
        code, skip, cnt, req, has = o.ds_prefilter(cases.ds_pod(case))
        assert (code, skip) == (want["code"], want["skip"]), case["source"]
        for tname, t in TYPES.items():
            exp = want["per"].get(tname)
            assert cnt[t] == (exp[0] if exp else 0), (case["source"], tname)
            if exp:
                vals, hs = cases.rl3(t, exp[1])
                assert list(has[t]) == hs and [int(v) for v, h in zip(req[t], hs) if h] == [v for v, h in zip(vals, hs) if h]
        return
    pod = cases.setup_ds(o, case)
    code, reason = o.ds_filter(pod, 0)
    if op == "filter":
        assert (code, reason) == (want["code"], want["reason"]), case["source"]
    else:  # Score (TestScore calls Score directly; a Prepare error shows up as Filter's status)
        assert (code, reason) == (want["code"], want["reason"]), case["source"]
        assert o.ds_score(pod, 0) == want["score"], case["source"]


# ---- NUMA topology policies ----------------------------------------------------------------------
NUMA_POLICY = cases.load("numa_policy.json")
POLICY_ID = {"BestEffort": 1, "Restricted": 2, "SingleNUMANode": 3}


def _mask(bits):
    return 0 if bits is None else sum(1 << b for b in bits)


def _lists(providers):
    """filterProvidersHints input: the providers' maps in sorted resource order."""
    out = []
    for p in providers:
        if p is None or len(p) == 0:
            out.append((1, []))
            continue
        for res in sorted(p):
            hints = p[res]
            if hints is None:
                out.append((1, []))
            elif len(hints) == 0:
                out.append((2, []))
            else:
                out.append((0, [(_mask(b), pref, 0) for b, pref in hints]))
    return out


NUMA_MERGE = [c for c in NUMA_POLICY if c["op"] == "merge"]


@pytest.mark.parametrize("case", NUMA_MERGE, ids=[c["name"] for c in NUMA_MERGE])
def test_numa_policy_merge(case):
    from oracle.binding import topology_merge
    admit, mask, pref, _, _ = topology_merge(POLICY_ID[case["policy"]], _mask(case["numa_nodes"]),
                                             _lists(case["providers"]))
    want = case["want"]
    assert (mask, pref, admit) == (_mask(want["bits"]), want["preferred"], want["admit"]), case["source"]


NUMA_PATH = [c for c in NUMA_POLICY if c["op"] not in ("merge", "exclusive")]
NUMA_EXCL = [c for c in NUMA_POLICY if c["op"] == "exclusive"]


@pytest.mark.parametrize("case", NUMA_EXCL, ids=[c["name"] for c in NUMA_EXCL])
def test_numa_exclusive_policy(case):
    import numpy as np
    from oracle.binding import load
    from koordinator_amd import abi, model
    st = np.array([{"idle": 0, "single": 1, "shared": 2}[x] for x in case["status"]], np.uint8)
    excl = {"Preferred": abi.NUMA_EXCLUSIVE_PREFERRED, "Required": abi.NUMA_EXCLUSIVE_REQUIRED}[case["exclusive"]]
    got = load().or_numa_exclusive_ok(sum(1 << b for b in case["bits"]), excl, abi.ptr(st), len(st))
    assert bool(got) == case["want"]["ok"], case["source"]


@pytest.mark.parametrize("case", NUMA_PATH, ids=[f'{c["op"]}: {c["name"]}' for c in NUMA_PATH])
def test_numa_policy_path(case):
    """Non-cpuset pods under a NUMA topology policy against the reference's own vectors."""
    o = Oracle(cases.numa_case_cfg(case), 1)
    pod = cases.setup_numa_case(o, case)
    want = case["want"]
    if case["op"] == "affinity":  # Filter succeeds; Reserve allocates on exactly the stored affinity
        chosen, _ = o.schedule([pod], cases.NOW)
        assert chosen[0] == 0
        alloc = o.last_numa_allocations[0].reshape(8, 2)
        assert [z for z in range(8) if alloc[z].any()] == want["bits"], case["source"]
    elif case["op"] == "distribute":
        ok, out = o.numa_distribute(0, pod, sum(1 << b for b in case["hint"]))
        assert ok == want["ok"], case["source"]
        if ok:
            got = {str(z): out[2 * z: 2 * z + 2].tolist() for z in range(8) if out[2 * z: 2 * z + 2].any()}
            assert got == {z: cases.quantity_vec(rl) for z, rl in want["alloc"].items()}, case["source"]
    elif case["op"] == "hints":
        hints = o.numa_hints(0, pod, cases.NUMA_POLICY_ID[case["policy"]])
        names = {"cpu": 0, "memory": 1}
        want_h = {names[k]: [(sum(1 << b for b in bits), pref) for bits, pref in v] for k, v in want["hints"].items()}
        assert {r: [(m, p) for m, p, _ in h] for r, h in hints.items()} == want_h, case["source"]
    else:  # available: the largest request a single zone can take (tryBestToDistributeEvenly on {zone})
        for z, rl in enumerate(want["available"]):
            for key, q in zip(("cpu", "memory"), cases.quantity_vec(rl)):
                for amount, fits in ((q, True), (q + 1, False)):
                    p = cases.make_pod({"requests": {key: f"{amount}m" if key == "cpu" else str(amount)}})
                    ok, _ = o.numa_distribute(0, p, 1 << z)
                    assert ok == fits, (case["source"], z, key, amount)


# ---- CPU accumulator ---------------------------------------------------------------------------
CPU_ACC = cases.load("cpu_accumulator.json")


def _take(rows, max_ref, available, ref, excl_arr, needed, bind, excl, most, preferred):
    import numpy as np
    from oracle.binding import load
    from koordinator_amd import abi, model
    cpus = np.ascontiguousarray(rows, np.int32).ravel()
    out = np.zeros(4, np.uint64)
    pref = None if preferred is None else cases.cpu_bits(preferred)
    rc = load().or_take_cpus(abi.ptr(cpus), len(rows), max_ref, abi.ptr(cases.cpu_bits(available)), abi.ptr(ref),
                             abi.ptr(excl_arr), needed, bind, excl, most, None if pref is None else abi.ptr(pref),
                             abi.ptr(out))
    return rc, cases.bits_cpus(out)


@pytest.mark.parametrize("case", CPU_ACC, ids=[c["name"] for c in CPU_ACC])
def test_cpu_accumulator(case):
    import numpy as np
    rows = cases.test_topology(*case["topology"], core_shift=case.get("core_shift", False))
    all_cpus = [r[0] for r in rows]
    most = 1 if case["strategy"] == "MostAllocated" else 0
    if case["op"] == "spread":
        from oracle.binding import load
        from koordinator_amd import abi
        out = np.zeros(256, np.int32)
        cpus = np.ascontiguousarray(rows, np.int32).ravel()
        n = load().or_spread_order(abi.ptr(cpus), len(rows), abi.ptr(cases.cpu_bits(all_cpus)), most, abi.ptr(out))
        assert out[:n].tolist() == case["want"], case["source"]
        return
    if case["op"] == "take":
        allocated = cases.parse_cpuset(case["allocated"])
        ref = np.full(256, -1, np.int32)
        excl_arr = np.zeros(256, np.int32)
        for c in allocated:
            ref[c] = 0
            excl_arr[c] = cases.CPU_EXCL_ID[case["alloc_excl"]]
        available = [c for c in all_cpus if c not in allocated]
        pref = None if case["preferred"] is None else cases.parse_cpuset(case["preferred"])
        rc, got = _take(rows, case["max_ref"], available, ref, excl_arr, case["needed"], cases.BIND_ID[case["bind"]],
                        cases.CPU_EXCL_ID[case["excl"]], most, pref)
        assert rc == 0 and got == cases.parse_cpuset(case["want"]), (case["source"], got)
        return
    # sequence: NodeAllocation.getAvailableCPUs / addCPUs(PCPULevel) between the pods
    ref = np.zeros(256, np.int32)
    for needed, bind, want in case["steps"]:
        available = [c for c in all_cpus if ref[c] < case["max_ref"]]
        alloc_ref = np.where(ref > 0, ref, -1).astype(np.int32)
        excl_arr = np.where(ref > 0, 1, 0).astype(np.int32)
        rc, got = _take(rows, case["max_ref"], available, alloc_ref, excl_arr, needed, cases.BIND_ID[bind], 0, most,
                        None)
        assert rc == 0 and got == cases.parse_cpuset(want), (case["source"], needed, got)
        for c in got:
            ref[c] += 1
    if "final_available" in case:
        assert [c for c in all_cpus if ref[c] < case["max_ref"]] == cases.parse_cpuset(case["final_available"])


# ---- cpuset pods (NUMA policy None) --------------------------------------------------------------
CPUSET = cases.load("cpuset.json")


@pytest.mark.parametrize("case", CPUSET, ids=[f'{c["op"]}: {c["name"]}' for c in CPUSET])
def test_cpuset_plugin(case):
    from koordinator_amd import abi, model
    o = Oracle(abi.default_config(1), 1)
    pod = cases.setup_cpuset_case(o, case)
    if case["op"] == "filter":
        r = o.eval([pod], cases.NOW)
        assert (int(r["status"][0, 0]), int(r["reason"][0, 0])) == (case["want"]["code"], case["want"]["reason"]), \
            case["source"]
        return
    chosen, _ = o.schedule([pod], cases.NOW)
    if case["want"]["fails"]:
        assert chosen[0] == -1, case["source"]
        return
    assert chosen[0] == 0, case["source"]
    assert cases.bits_cpus(o.last_cpusets[0]) == cases.parse_cpuset(case["want"]["cpuset"]), case["source"]


# ---- cpusets under NUMA topology policies ----------------------------------------------------------
NUMA_CPUSET = cases.load("numa_cpuset.json")


@pytest.mark.parametrize("exact", [False, True], ids=["counts", "accumulator"])
@pytest.mark.parametrize("case", NUMA_CPUSET, ids=[f'{c["op"]}: {c["name"]}' for c in NUMA_CPUSET])
def test_numa_cpuset(case, exact):
    """Allocate with a hint, BestEffort hint lists and Filter + Score of binding pods against the
    reference's vectors; `exact` runs hints / admit through the CPU accumulator itself instead of the
    count reduction (both must agree with the reference)."""
    from koordinator_amd import abi, model
    if case["op"] == "node_score":
        cfg = abi.default_config(len(case["nodes"]))
        cfg.numa.strategy = abi.STRATEGY_MOST_ALLOCATED
        o = Oracle(cfg, len(case["nodes"]))
        o.set_exact_cpusets(exact)
        pod = cases.setup_numa_score_case(o, case)
        r = o.eval([pod], cases.NOW)
        assert list(r["status"][0]) == [abi.CODE_SUCCESS] * len(case["nodes"]), case["source"]
        assert [int(x) for x in r["numa"][0]] == case["want"]["scores"], case["source"]
        return
    o = Oracle(abi.default_config(1), 1)
    o.set_exact_cpusets(exact)
    pod = cases.setup_numa_cpuset_case(o, case)
    if case["op"] == "allocate":
        mask = sum(1 << b for b in case["hint"])
        got = o.numa_allocate(0, pod, mask)
        if case["want"]["error"]:
            assert got is None, case["source"]
            return
        assert got is not None, case["source"]
        out, cpus = got
        assert cases.bits_cpus(cpus) == cases.parse_cpuset(case["want"]["cpuset"]), case["source"]
        want = np.zeros(16, np.int64)
        for zid, res in case["want"]["numa"].items():
            want[2 * int(zid)] = model.milli_value(res["cpu"])
        assert list(out) == list(want), case["source"]
        return
    hints = o.numa_hints(0, pod, abi.NUMA_POLICY_BEST_EFFORT)
    want = [(sum(1 << b for b in h["bits"]), h["preferred"]) for h in case["want"]["cpu"]]
    assert [(m, p) for m, p, _ in hints.get(0, [])] == want, case["source"]
    assert 1 not in hints, case["source"]


# ---- DeviceShare GPUAllocator: partitions, topology scopes, shared GPUs -------------------------------
GPU_ALLOC = cases.load("gpu_allocator.json")


def gpu_alloc_setup(handle, case, node=0):
    """Node `node` gets the case's GPUs and partition state; returns the pod (cases.py conventions)."""
    from koordinator_amd import model
    handle.upsert_node(node, model.make_node(allocatable={"cpu": "96", "memory": "512Gi"}))
    handle.set_devices(node, model.make_devices(case["devices"]))
    has_table, honor, parts = model.gpu_partition_state(node_labels=case["node_labels"])
    handle.set_gpu_partitions(node, has_table, honor, parts)
    return model.make_pod(requests=dict(case["pod"]["requests"]), device_hints=case["pod"]["device_hints"])


def gpu_alloc_cfg(case, n_nodes=1):
    from koordinator_amd import abi
    cfg = cases.ds_cfg(case, n_nodes)
    if case.get("weights"):
        cfg.deviceshare.weights[:] = [abi.ABSENT if w is None else w for w in case["weights"]]
    return cfg


@pytest.mark.parametrize("case", GPU_ALLOC, ids=[c["name"] for c in GPU_ALLOC])
def test_gpu_allocator(case):
    o = Oracle(gpu_alloc_cfg(case), 1)
    pod = gpu_alloc_setup(o, case)
    want = case["want"]
    assert o.ds_filter(pod, 0) == (want["code"], want["reason"]), case["source"]
    if want["code"] == 0:
        mask = o.ds_reserve(pod, 0)
        assert [m for m in range(16) if mask >> m & 1] == want["minors"], case["source"]


# ---- DeviceShare as a NUMA hint provider (topology_hint.go) --------------------------------------------
DS_NUMA = cases.load("ds_numa.json")


@pytest.mark.parametrize("case", DS_NUMA, ids=[c["name"] for c in DS_NUMA])
def test_ds_numa_hints(case):
    from koordinator_amd import abi, model
    o = Oracle(abi.default_config(1), 1)
    o.upsert_node(0, model.make_node(allocatable={"cpu": "96", "memory": "512Gi"}))
    o.set_devices(0, model.make_devices(case["devices"]))
    pod = model.make_pod(requests=dict(case["pod"]["requests"]))
    want = case["want"]
    if case["op"] == "allocate":
        st, _ = o.ds_numa_allocate(pod, 0, case["affinity"])
        assert st == want["code"], case["source"]
        return
    st, reason, none, copies, hints = o.ds_numa_hints(pod, 0)
    assert (st, reason if st else 0) == (want["code"], want["reason"]), case["source"]
    if not st:
        assert not none and copies == want["copies"], case["source"]
        assert [list(h) for h in hints] == want["hints"], case["source"]
