# round 3: kernel-argument integrity of captured graphs across replays (never faults)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3split
timeout -k 10 120 python -u tools/probe/kernarg_probe.py 2>&1 | tee gpurun_out/r3split/kernarg.log
