"""Oracle self-check for cpusets under NUMA topology policies: the hint / admit feasibility of a
binding pod reduced to CPU counts (oracle.c cpuset_fits_cs) against running the CPU
accumulator itself per hint (cpuset_allocate_cs, the reference's shape), on config-4 style clusters.
Both are pinned by the reference vectors in test_oracle_golden.py::test_numa_cpuset."""
import numpy as np
import pytest

from koordinator_amd import abi, synth
from oracle.binding import Oracle


def pair(n_nodes, seed, **kw):
    cl = synth.make_cluster(n_nodes, synth.BASE_SEED + seed, amplified_fraction=0.3)
    zs, tabs = synth.make_numa_cpus(cl, synth.BASE_SEED + seed + 1, **kw)
    cfg = synth.config(n_nodes)
    # no LoadAware thresholds: every node reaches the NodeNUMAResource filter
    cfg.loadaware.usage_thresholds[:] = [abi.ABSENT, abi.ABSENT]
    out = []
    for exact in (False, True):
        o = Oracle(cfg, n_nodes)
        o.set_exact_cpusets(exact)
        synth.load_into(o, cl)
        synth.load_numa(o, zs)
        synth.load_cpus(o, tabs)
        out.append(o)
    return out


@pytest.mark.parametrize("seed,kw", [(311, {}), (321, {"zone_counts": (8,), "max_ref_choices": (2, 3)}),
                                     (331, {"bind_weights": (0.2, 0.4, 0.4), "policy_weights": (0, 1, 1, 1)})])
def test_count_reduction_matches_accumulator(seed, kw):
    a, b = pair(64, seed, **kw)
    pods = synth.make_numa_cpuset_pods(40, synth.BASE_SEED + seed + 2)
    ea, eb = a.eval(pods, synth.T0), b.eval(pods, synth.T0)
    for k in ("status", "reason", "la", "numa", "total", "best"):
        assert np.array_equal(ea[k], eb[k]), k
    assert np.any(ea["status"] == abi.CODE_SUCCESS)
    ca, sa = a.schedule(pods, synth.T0)
    cb, sb = b.schedule(pods, synth.T0)
    assert np.array_equal(ca, cb) and np.array_equal(sa, sb)
    assert np.array_equal(a.last_cpusets, b.last_cpusets)
    assert np.array_equal(a.last_numa_allocations, b.last_numa_allocations)
    assert np.any(a.last_cpusets != 0)
