# round-5 final GPU call: full GPU suite, wavefront A/B, closing pass (PMC, bench line, trace), other configs
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r5final}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 120 python -u tools/lstm2_bwd_bench.py 10 > $O/lstm2_bwd_tool.txt 2>&1 || exit 1
bash tools/ab_replay.sh $TAG "AVC_LSTM2_DB=1" "AVC_LSTM2_DB=0" || exit 1
bash tools/gpu_close.sh $TAG/close r5 || exit 1
bash tools/gpu_configs.sh $TAG || exit 1
