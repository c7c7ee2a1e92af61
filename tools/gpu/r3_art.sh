# round 3 artifacts: per config PMC traffic (-> profiles/r03_<cfg>_pmc.json), the bench line
# (CPU baseline for C2) and the rocprofv3 kernel stats of the same command; SQ counters for C2.
# usage: bash tools/gpu/r3_art.sh C2 [C3 ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in "$@"; do
  bash tools/gpu/artifacts.sh r3$c $c r03 || exit 1
done
if [ "${SQ:-0}" = "1" ]; then bash tools/gpu/sqpass.sh C2 r03 || exit 1; fi
