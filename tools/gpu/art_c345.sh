# full GPU tests, then round artifacts for C3, C4, C5 (PMC traffic, bench line, kernel stats)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/t_art.log 2>&1 || { tail -40 gpurun_out/t_art.log; exit 1; }
tail -1 gpurun_out/t_art.log
for c in C3 C4 C5; do bash tools/gpu/artifacts.sh g$c $c r02 || exit 1; done
