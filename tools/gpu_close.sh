# Round closing pass in one GPU call -> gpurun_out/$1: HBM PMC passes (FETCH_SIZE / WRITE_SIZE) and the MFMA counter
# pass over the C2 bench (their summaries copied into this tree's profiles/ as r5_* first, so the bench line reads
# them), the LSTM step timeline, the default bench line (roofline + cpu_baseline), and a kernel-trace profile with
# its step breakdown.   gpurun --timeout 1200 -- bash tools/gpu_close.sh <tag> <round-prefix>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-close}
PFX=${2:-r5}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1 &&
python3 $R/tools/pmc_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) \
    $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) $OUT/pmc_traffic.json || exit 1
cp $OUT/pmc_traffic.json $R/profiles/${PFX}_pmc_traffic.json
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/mfma -o run -- python3 $R/bench.py --steps 3 --warmup 2 \
    --no-cpu-baseline --no-kernel-timing > $OUT/mfma.log 2>&1 || exit 1
python3 $R/tools/pmc_mfma.py $(find $OUT/mfma -name "*counter_collection.csv" | head -1) $OUT/pmc_mfma_step.json 30 \
    > $OUT/pmc_mfma_step.txt || exit 1
cp $OUT/pmc_mfma_step.json $R/profiles/${PFX}_pmc_mfma_step.json
timeout -k 10 120 python3 $R/tools/lstm_trace.py > $OUT/lstm_trace.txt 2>&1 || exit 1
timeout -k 10 120 python3 $R/tools/lstm2_bwd_bench.py 10 > $OUT/lstm2_bwd_bench.txt 2>&1 || exit 1
timeout -k 10 400 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
CSV=$(find $OUT/prof -name "run_kernel_trace.csv" | head -1)
python3 $R/tools/step_breakdown.py $CSV 30 > $OUT/step_breakdown.txt
cp $(find $OUT/prof -name "run_kernel_stats.csv" | head -1) $OUT/kernel_stats.csv
head -5 $OUT/step_breakdown.txt
