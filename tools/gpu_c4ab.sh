set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5c4}
mkdir -p $O
for i in 1 2; do
  for m in "--eager" "--replay"; do
    timeout -k 10 200 python bench.py --model MetaConv $m --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing > /tmp/o.json 2>/dev/null
    echo "C4 $m $(grep -o 'ms_per_step": [0-9.]*' /tmp/o.json) $(grep -o '"launch": "[a-z]*"' /tmp/o.json)" >> $O/ab.txt
    timeout -k 10 120 python bench.py --disc $m --steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing > /tmp/o.json 2>/dev/null
    echo "C5 $m $(grep -o 'ms_per_step": [0-9.]*' /tmp/o.json) $(grep -o '"launch": "[a-z]*"' /tmp/o.json)" >> $O/ab.txt
  done
done
cat $O/ab.txt
