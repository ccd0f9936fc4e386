"""Timeline summary of a rocprofv3 --kernel-trace CSV (tools/gpu_round2.sh): per kernel the launch count
and mean duration, per stream the busy time and the idle gaps between consecutive kernels, and how
much of the Reserve chain's time (k_fixup + k_resolve) overlaps the eval stream's kernels — the
evidence that the pipelined schedule runs batch b's eval/select concurrently with batch b-1's replay.

usage: python tools/timeline.py <kernel_trace.csv> [--json out.json]
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:60]


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append({"name": short(r["Kernel_Name"]), "q": r.get("Stream_Id") or r.get("Queue_Id"),
                         "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"])})
    rows.sort(key=lambda r: r["t0"])
    return rows


def summarize(rows, window=None):
    if window:  # the timed region: the longest run of k_resolve launches
        rows = [r for r in rows if window[0] <= r["t0"] <= window[1]]
    per = defaultdict(list)
    for r in rows:
        per[r["name"]].append(r["t1"] - r["t0"])
    kernels = {k: {"calls": len(v), "mean_us": sum(v) / len(v) / 1e3} for k, v in per.items()}
    streams = defaultdict(list)
    for r in rows:
        streams[r["q"]].append(r)
    st = {}
    for q, rs in streams.items():
        busy = sum(r["t1"] - r["t0"] for r in rs)
        gaps = [max(0, b["t0"] - a["t1"]) for a, b in zip(rs, rs[1:])]
        names = sorted({r["name"] for r in rs})
        st[str(q)] = {"kernels": len(rs), "busy_ms": busy / 1e6, "span_ms": (rs[-1]["t1"] - rs[0]["t0"]) / 1e6,
                      "mean_gap_us": (sum(gaps) / len(gaps) / 1e3) if gaps else 0.0, "names": names}
    # idle time between consecutive kernels of one stream, by (previous kernel -> next kernel)
    pair = defaultdict(list)
    for q, rs in streams.items():
        for a, b in zip(rs, rs[1:]):
            pair[f"{a['name']} -> {b['name']}"].append(max(0, b["t0"] - a["t1"]))
    gaps = {k: {"n": len(v), "mean_us": sum(v) / len(v) / 1e3, "p50_us": sorted(v)[len(v) // 2] / 1e3}
            for k, v in pair.items() if len(v) >= 10}
    # overlap: time during which a resolve-chain kernel and an eval-chain kernel both run
    res = [(r["t0"], r["t1"]) for r in rows if r["name"].startswith(("k_resolve", "k_fixup"))]
    evs = [(r["t0"], r["t1"]) for r in rows if r["name"].startswith(("k_eval_batch", "k_select", "k_merge"))]
    ov, j = 0, 0
    for a0, a1 in res:
        while j < len(evs) and evs[j][1] < a0:
            j += 1
        k = j
        while k < len(evs) and evs[k][0] < a1:
            ov += max(0, min(a1, evs[k][1]) - max(a0, evs[k][0]))
            k += 1
    ev_busy = sum(b - a for a, b in evs)
    res_busy = sum(b - a for a, b in res)
    span = (rows[-1]["t1"] - rows[0]["t0"]) if rows else 0
    return {"kernels": kernels, "streams": st, "gaps": gaps, "span_ms": span / 1e6,
            "reserve_chain_busy_ms": res_busy / 1e6, "eval_chain_busy_ms": ev_busy / 1e6,
            "eval_chain_overlapped_frac": ov / ev_busy if ev_busy else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = load(a.csv)
    window = None
    s = summarize(rows, window)
    print(json.dumps(s, indent=1))
    if a.json:
        json.dump(s, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
