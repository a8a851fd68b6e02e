# full GPU suite + one C2 A/B -> gpurun_out/$1
set -o pipefail
O=gpurun_out/${1:-r5full}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
bash tools/ab_replay.sh ${1:-r5full} "AVC_HALO_SPLIT=1" "AVC_HALO_SPLIT=0"
