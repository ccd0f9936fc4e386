"""Debug helper: schedule the DS+NUMA parity queue pod by pod on the device and the oracle; at the first
difference print the pod, both results and the eval rows of the chosen nodes."""
import sys
import numpy as np
sys.path[:0] = [".", "tests"]
from koordinator_amd import abi, synth
from test_gpu_ds_numa import _both, _cpuset_ds_pods

name = sys.argv[1] if len(sys.argv) > 1 else "zones-2-4-8"
if name == "cpuset":
    ev, o = _both(120, 721, cpus=True, zone_counts=(2, 4))
    pods = _cpuset_ds_pods(200, 722)
else:
    kw = {"zones-2-4-8": {}, "alignment-disabled": {"disable": True}}[name]
    ev, o = _both(96, 711, **kw)
    pods = synth.make_ds_numa_pods(240, synth.BASE_SEED + 712)
for p in range(len(pods)):
    one = pods[p:p + 1]
    a, b = ev.eval(one, synth.T0), o.eval(one, synth.T0)
    evdiff = [k for k in ("status", "reason", "la", "numa", "total", "best") if not np.array_equal(a[k], b[k])]
    c1, s1 = ev.schedule(one, synth.T0)
    c0, s0 = o.schedule(one, synth.T0)
    same = (c1[0] == c0[0] and s1[0] == s0[0] and ev.last_device_allocations[0] == o.last_device_allocations[0]
            and np.array_equal(ev.last_numa_allocations, o.last_numa_allocations)
            and np.array_equal(ev.last_cpusets, o.last_cpusets))
    if evdiff or not same:
        pod = pods[p]
        print("pod", p, "evdiff", evdiff, "flags pol", pod["numa_topology_policy"], "excl", pod["numa_exclusive"],
              "req", pod["requests"][:2].tolist(), "qos", pod["qos_class"], "prio", pod["priority_class"],
              "dreq", {k: int(pod["device_requests"][v]) for k, v in abi.PDR.items() if pod["device_requests"][v]})
        print("device chosen", c1[0], s1[0], hex(int(ev.last_device_allocations[0])), ev.last_numa_allocations[0].tolist(),
              ev.last_cpusets[0].tolist())
        print("oracle chosen", c0[0], s0[0], hex(int(o.last_device_allocations[0])), o.last_numa_allocations[0].tolist(),
              o.last_cpusets[0].tolist())
        for n in {int(c1[0]), int(c0[0])} - {-1}:
            print(" node", n, {k: (int(a[k][0, n]), int(b[k][0, n])) for k in ("status", "reason", "la", "numa", "ds", "total")
                                if k in a})
        break
else:
    print("all equal")
