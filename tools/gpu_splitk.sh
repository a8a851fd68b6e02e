# round 5: TT split-K reduction without atomics -- tests, microbench, C2 A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5sk}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "tt or split" > $O/t_kernels.txt 2>&1
TT_SWEEP=1 timeout -k 10 120 python -u tools/tt_bench.py > $O/tt_fix.txt 2>&1
TT_SWEEP=1 AVC_TT_SPLITK=0 timeout -k 10 120 python -u tools/tt_bench.py > $O/tt_atomic.txt 2>&1
bash tools/ab_replay.sh ${1:-r5sk} "AVC_TT_SPLITK=6" "AVC_TT_SPLITK=0"
