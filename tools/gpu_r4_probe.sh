set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u tools/graph_fwd_probe.py 1,3 2>&1 | grep -a "variant\|Error" || true
