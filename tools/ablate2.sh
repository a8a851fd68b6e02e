cd $GRAFT_REPO_ROOT
for cfg in "1 1" "0 1" "1 0" "0 0"; do set -- $cfg
  echo "AVC_PACK_BATCH=$1 AVC_CONV_DW_DIRECT=$2"
  AVC_PACK_BATCH=$1 AVC_CONV_DW_DIRECT=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c150-230
done
