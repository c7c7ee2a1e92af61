# build + run MLP kernel variants (GPU box): bash tools/kbench/run_mlp.sh "TAG:FLAGS" ...
set -e
cd $GRAFT_REPO_ROOT/tools/kbench
for v in "$@"; do
  tag=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics $flags -DMLP_TAG="\"$tag\"" mlp_bench.hip -o /tmp/mlp_$tag 2>/dev/null
  timeout -k 5 60 /tmp/mlp_$tag
done
