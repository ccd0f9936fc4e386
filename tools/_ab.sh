#!/bin/bash
# A/B of an env switch on the bench line, alternated on one box: _ab.sh OUT VAR v1 v2 [bench args...]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/$1; VAR=$2; A=$3; B=$4; shift 4
mkdir -p $O
for r in 1 2; do for v in $A $B; do
  env $VAR=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
  env $VAR=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync "$@" > $O/s_${v}_$r.json 2> $O/s_${v}_$r.err || exit 1
  echo "$v $r $(python3 -c "import json;a=json.load(open('$O/b_${v}_$r.json'));b=json.load(open('$O/s_${v}_$r.json'));print(round(a['value']/1e9,2),round(b['value']/1e9,2))")"
done; done
echo done
