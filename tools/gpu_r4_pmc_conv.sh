# PMC passes over the conv / projection microbenchmark (tools/ring_ab.py --only conv) -> gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/ring_ab.py --only conv --reps 5 --rounds 1 --configs ${2:-old,halo,auto,halo-loads,halo-math,halo-contig}"
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/p1 -o run -- $CMD > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/p2 -o run -- $CMD > $OUT/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- $CMD > $OUT/p3.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum --output-format csv -d $OUT/p4 -o run -- $CMD > $OUT/p4.log 2>&1 || true
F=$(find $OUT/p1 -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_mfma.py $F $OUT/p1.json 30 > $OUT/p1.txt
