# Kernel traces of the recorded C2 step with and without the weight-gradient side stream, paired:
#   gpurun -- bash tools/gpu_contention.sh <tag>     -> gpurun_out/<tag>/contention.txt
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/pa -o run -- python3 $R/tools/contention_trace.py 8 > $OUT/a.log 2>&1 || exit 1
AVC_ABLATE_WGRAD=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/pb -o run -- python3 $R/tools/contention_trace.py 8 > $OUT/b.log 2>&1 || exit 1
A=$(find $OUT/pa -name "run_kernel_trace.csv" | head -1)
B=$(find $OUT/pb -name "run_kernel_trace.csv" | head -1)
cp $A $OUT/trace_side.csv; cp $B $OUT/trace_noside.csv
python3 $R/tools/contention_diff.py $A $B 3 > $OUT/contention.txt
grep ms/step $OUT/a.log $OUT/b.log >> $OUT/contention.txt
rm -rf $OUT/pa $OUT/pb
