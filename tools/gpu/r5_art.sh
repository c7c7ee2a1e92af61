#!/bin/bash
# Round-5 artifacts: per config PMC traffic (-> profiles/r05_<cfg>_pmc.json), the bench line and
# the rocprofv3 kernel stats of the same command (tools/gpu/artifacts.sh), SQ passes when SQ=1.
# usage: [SQ=1] bash tools/gpu/r5_art.sh C3 [C2 ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in "$@"; do
  bash tools/gpu/artifacts.sh r5$c $c r05 || exit 1
  if [ "${SQ:-0}" = "1" ]; then bash tools/gpu/sqpass.sh $c r05 || exit 1; fi
done
