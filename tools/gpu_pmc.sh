# one MFMA / wait / LDS counter pass over the C2 bench (and the TT microbenchmark) -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/step -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-timing > $OUT/step.log 2>&1 || exit 1
F=$(find $OUT/step -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_mfma.py $F $OUT/step_mfma.json 30 > $OUT/step_mfma.txt
timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $OUT/tt -o run -- python3 $R/tools/tt_bench.py > $OUT/tt.log 2>&1 || exit 1
F=$(find $OUT/tt -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_mfma.py $F $OUT/tt_mfma.json 30 > $OUT/tt_mfma.txt
