set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in C4 C5; do bash tools/gpu/artifacts.sh r02_$c $c r02 || exit 1; done
bash tools/gpu/sqpass.sh C3 r02 || exit 1
