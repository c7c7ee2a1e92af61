set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for S in 2 3 4; do
  echo "== stages $S"
  IMGCAP_GLDS_STAGES=$S timeout -k 10 300 python tools/microbench.py probe > gpurun_out/probe_s$S.log 2>&1 || { tail -20 gpurun_out/probe_s$S.log; exit 1; }
  grep probe gpurun_out/probe_s$S.log
done
