# (historical) A/B of the split pipeline graphs on CU-masked streams.  The masking hook was removed
# after this sweep (C2 2,170-3,010 img/s vs 8,480 for the default two-branch graph; see DESIGN.md
# section 5); the CU-mask overlap probe itself stays in tools/microbench.py (cumask).
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/microbench.py cumask
