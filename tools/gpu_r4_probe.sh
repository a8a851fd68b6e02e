set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/graph_fwd_probe2.py > $OUT/probe2.txt 2>&1; head -60 $OUT/probe2.txt
