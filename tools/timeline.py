"""Per-queue kernel timeline from a rocprofv3 --kernel-trace CSV: average duration of each kernel and the average
idle gap before it on its queue (launch / dependency latency), over the dispatches of the steady state.

usage: python tools/timeline.py <kernel_trace.csv> [--skip N]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 200
    rows = list(csv.DictReader(open(path)))
    if not rows:
        print("empty trace")
        return
    qkey = next(k for k in ("Stream_Id", "Queue_Id", "Queue_ID") if k in rows[0])
    by_q = defaultdict(list)
    for r in rows:
        by_q[r[qkey]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60]))
    for q, ks in sorted(by_q.items()):
        ks.sort()
        ks = ks[skip:] if len(ks) > 2 * skip else ks
        dur, gap, n = defaultdict(float), defaultdict(float), defaultdict(int)
        for i, (s, e, name) in enumerate(ks):
            dur[name] += e - s
            n[name] += 1
            if i:
                gap[name] += max(0, s - ks[i - 1][1])
        span = (ks[-1][1] - ks[0][0]) / 1e3
        print(f"queue {q}: {len(ks)} dispatches over {span:.1f} us")
        for name in sorted(n, key=lambda x: -dur[x]):
            print(f"  {name:60s} n={n[name]:6d} avg {dur[name] / n[name] / 1e3:8.2f} us  gap before {gap[name] / n[name] / 1e3:7.2f} us")


if __name__ == "__main__":
    main()
