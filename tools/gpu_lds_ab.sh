# round 5: LDS footprint A/B of the main-stream GEMMs (room for a side-stream workgroup beside them)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5lds}
mkdir -p $O
AVC_CU_NST=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py -k "utt or conv" > $O/t.txt 2>&1
for i in 1 2; do
  for cfg in "AVC_RING_NST128=3" "AVC_RING_NST128=4"; do
    env $cfg timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > /tmp/o.json 2>/dev/null
    echo "C2 $cfg $(grep -o 'ms_per_step": [0-9.]*' /tmp/o.json)" >> $O/ab.txt
  done
  for cfg in "AVC_CU_NST=2" "AVC_CU_NST=3"; do
    env $cfg timeout -k 10 120 python bench.py --disc --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > /tmp/o.json 2>/dev/null
    echo "C5 $cfg $(grep -o 'ms_per_step": [0-9.]*' /tmp/o.json)" >> $O/ab.txt
  done
  for cfg in "AVC_CU_NST=2 AVC_RING_NST128=3" "AVC_CU_NST=3 AVC_RING_NST128=4"; do
    env $cfg timeout -k 10 200 python bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > /tmp/o.json 2>/dev/null
    echo "C4 $cfg $(grep -o 'ms_per_step": [0-9.]*' /tmp/o.json)" >> $O/ab.txt
  done
done
cat $O/ab.txt
