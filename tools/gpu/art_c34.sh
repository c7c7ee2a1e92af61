# round artifacts for C3 and C4 (PMC traffic, bench line, kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in C3 C4; do bash tools/gpu/artifacts.sh h$c $c r02 || exit 1; done
