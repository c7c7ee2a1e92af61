set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/kbench/run_mlp.sh "stamps:-DMLP_STAMPS" 2>&1
