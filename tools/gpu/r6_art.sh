#!/bin/bash
# Round-6 artifacts: per config PMC traffic (-> profiles/r06_<cfg>_pmc.json), the bench line and the
# rocprofv3 kernel stats of the same command (tools/gpu/artifacts.sh), SQ passes when SQ=1.
# usage: [SQ=1] bash tools/gpu/r6_art.sh C3 [C2 ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in "$@"; do
  bash tools/gpu/artifacts.sh r6$c $c r06 || exit 1
  if [ "${SQ:-0}" = "1" ]; then bash tools/gpu/sqpass.sh $c r06 || exit 1; fi
done
