set -e
export TMPDIR=/tmp
O=gpurun_out/r5tt2
mkdir -p $O
TT_SWEEP=1 timeout -k 10 120 python -u tools/tt_bench.py > $O/base.txt 2>&1
TT_SWEEP=1 AVC_TT_ABL=1 timeout -k 10 120 python -u tools/tt_bench.py > $O/abl.txt 2>&1
