#!/bin/bash
# C4 kernel times per evaluator build (ablation / A-B): rocprofv3 --stats of tools/cpuset_bench.py --survey.
# usage (GPU box): tools/abl_c4.sh name...   (koordinator_amd/<name>.so)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  D=$R/gpurun_out/abl/$L
  mkdir -p "$D"
  KOORDEVAL_LIB=$R/koordinator_amd/$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- \
    python3 "$R/tools/cpuset_bench.py" --survey --pods 256 --steps 1 --no-cpu-baseline ${C4_ARGS:-} > "$D/out.log" 2>&1 || { tail -5 "$D/out.log"; exit 1; }
  python3 - "$D" "$L" <<'PY'
import csv, json, sys
d, name = sys.argv[1], sys.argv[2]
rows = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(d + "/run_kernel_stats.csv"))}
line = [l for l in open(d + "/out.log") if l.startswith("{")][-1]
print(name, "ms_per_pod", round(json.loads(line)["ms_per_pod"], 3), {k: round(v, 1) for k, v in rows.items() if v > 20})
PY
done
