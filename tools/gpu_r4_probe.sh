set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/graph_fwd_probe3.py > $OUT/probe3.txt 2>&1; head -60 $OUT/probe3.txt
