#!/bin/bash
# Build the evaluator library of a git revision (or the working tree: "WT") into koordinator_amd/<name>.so
# for same-box A/B runs (KOORDEVAL_LIB=koordinator_amd/<name>.so python bench.py ...).
# usage: tools/ab_build.sh <rev|WT> <name> [extra CXXFLAGS]
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2; EXTRA=${3:-}
W=$(mktemp -d /tmp/ab.XXXXXX)
if [[ $REV == WT ]]; then
  cp -r "$R/koordinator_amd/csrc" "$W/csrc"; mkdir -p "$W/include"; cp "$R/include/koord_eval.h" "$W/include/"
else
  git -C "$R" archive "$REV" koordinator_amd/csrc include | tar -x -C "$W"
  mv "$W/koordinator_amd/csrc" "$W/csrc"
fi
mkdir -p "$W/x"; mv "$W/csrc" "$W/x/csrc"; mv "$W/include" "$W/include_"; mkdir -p "$W/include"; cp "$W/include_/koord_eval.h" "$W/include/"
rm -rf "$W/x/csrc/build" "$W/x/csrc/build_prof"
make -s -C "$W/x/csrc" -j8 OUT="$R/koordinator_amd/$NAME.so" CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w $EXTRA" > /dev/null
rm -rf "$W"
echo "built koordinator_amd/$NAME.so from $REV"
