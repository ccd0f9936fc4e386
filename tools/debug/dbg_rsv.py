import sys; sys.path.insert(0,'tests'); sys.path.insert(0,'.')
import numpy as np
import test_gpu_reservation_holdings as t
from koordinator_amd import synth, abi
ev,o,pods,matches,rs = t.cpuset_matched_setup(300, 1363, 300, 0.3, 0.4)
c1,s1 = ev.schedule(pods, synth.T0, matches=matches)
c0,s0 = o.schedule(pods, synth.T0, matches=matches)
bad = np.flatnonzero((c1!=c0)|(s1!=s0))
print("bad", bad[:10].tolist())
for p in bad[:3]:
    print("pod", p, "ev", c1[p], s1[p], "or", c0[p], s0[p], "rm", pods["reservation_matched"][p], "match", matches[p])
    print("  cpu", pods["requests"][p][:2], "qos", pods["qos_class"][p], "bind", pods["cpu_bind_required"][p], pods["cpu_bind_preferred"][p])
    for r in matches[p]:
        n = rs["node"][r]
        print("   r", r, "node", n, "holds", rs["holds"][r], "pol", rs["allocate_policy"][r], "avail", rs["available"][r], "ap", rs["allocated_pods"][r], "alloc", rs["allocatable"][r], rs["allocated"][r])
    a1 = ev.last_allocations(); a0 = o.last_allocations()
    print("  rsv", a1["reservation"][p], a0["reservation"][p])
p0 = int(bad[0])
ev,o,pods,matches,rs = t.cpuset_matched_setup(300, 1363, 300, 0.3, 0.4)
ev.schedule(pods[:p0], synth.T0, matches=matches[:p0]); o.schedule(pods[:p0], synth.T0, matches=matches[:p0])
nodes = sorted(set(int(rs["node"][r]) for r in matches[p0]))
for n in nodes:
    a = ev.node_state(n)[0]; b = o.node_state(n)[0]
    print("node", n, "pods ev/or", a.pod_count, b.pod_count, "allowed", a.allowed_pods, "req", list(a.requested), list(b.requested))
c1,s1 = ev.schedule(pods[p0:p0+1], synth.T0, matches=[matches[p0]])
c0,s0 = o.schedule(pods[p0:p0+1], synth.T0, matches=[matches[p0]])
print("alone", c1, s1, c0, s0)
e1 = ev.eval(pods[p0:p0+1], synth.T0) if False else None
