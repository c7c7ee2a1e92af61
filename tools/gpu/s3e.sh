set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/brk.sh s3e C2 > gpurun_out/brk_s3e_out.txt 2>&1 || { tail -20 gpurun_out/brk_s3e_out.txt; exit 1; }
head -30 gpurun_out/brk_s3e_out.txt
DIAG_EAGER=1 timeout -k 10 240 python -u tools/probe/capture_diag.py C4 side graph > gpurun_out/capdiag2.log 2>&1; rc=$?
grep -v "^frame" gpurun_out/capdiag2.log | grep -v Warn | head -24
exit $rc
