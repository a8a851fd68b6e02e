set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
for envv in "X=0" "AVC_LSTM_NO_PERSIST=1" "AVC_RING=0" "AVC_FOLD=0" "AVC_CONV0_FOLD=0" "AVC_LSTM2_OFF=1"; do
  echo "== $envv"
  env $envv timeout -k 10 120 python -u tools/graph_fwd_probe.py 1 2>&1 | grep -a "variant\|Error" || true
done
