set -o pipefail
# stream priorities for the pipelined capture (IMGCAP_PIPE_PRIO, since removed): C3 A/B -- DESIGN 2b
O=gpurun_out/r5prio; rm -rf $O; mkdir -p $O
for r in 1 2; do for v in 1 0; do
  IMGCAP_PIPE_PRIO=$v timeout -k 10 300 python -u bench.py --config C3 --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > $O/b.txt 2>$O/b.err || { tail -20 $O/b.err; exit 1; }
  echo "C3 prio=$v $(python -c "import json; d=json.loads(open('$O/b.txt').read().strip().splitlines()[-1]); print(round(d['value']), d['ms_per_step'])")"
done; done
