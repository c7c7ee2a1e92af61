# round artifacts for C2 (PMC traffic, bench line with CPU baseline, kernel stats) + SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/artifacts.sh f2 C2 r02 || exit 1
bash tools/gpu/sqpass.sh C2 r02 || exit 1
