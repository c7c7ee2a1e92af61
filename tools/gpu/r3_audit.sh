# round 3: new trainer / LSTM robustness tests, then the replay-time pointer audit of the
# captured schedules (C5 sequential, C4 sequential, C2 pipelined)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
O=gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_train_step_gpu.py "tests/test_transformer_gpu.py::test_transformer_vocab_past_fused_ce_limit_vs_oracle" tests/test_lstm_gpu.py > $O/t_a.log 2>&1 || { tail -40 $O/t_a.log; exit 1; }
tail -3 $O/t_a.log
timeout -k 10 300 python -u tools/probe/replay_audit.py C5 --steps 12 > $O/audit_C5.log 2>&1; rc=$?; tail -25 $O/audit_C5.log; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit 1
timeout -k 10 200 python -u tools/probe/replay_audit.py C4 --steps 8 > $O/audit_C4.log 2>&1; rc=$?; tail -12 $O/audit_C4.log; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit 1
timeout -k 10 200 python -u tools/probe/replay_audit.py C2 --steps 8 --pipeline > $O/audit_C2.log 2>&1; rc=$?; tail -12 $O/audit_C2.log
